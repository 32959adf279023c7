"""teacher.collect_reward (reference teacher.py:39-62, with the record semantics of the runnable
lstm_train.py:113-135 warm-up): the batched collector against the reference-shaped driver's
own teacher phase, env by env against one-env collections, and through the page store."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_one_env_equals_the_lstm_driver_warm_up():
    """n_envs = 1: the same records, bit for bit, as lstm_train.train's teacher phase (its
    first warmup_episodes + 1 episodes), the reward column carried over each reset."""
    from reacherdistilation_amd import lstm_train, teacher
    _, dl, _ = lstm_train.train(episodes=4, warmup_episodes=2, log=lambda *a: None)
    dc = teacher.collect_reward(3, n_envs=1, seed=0, device=DEV)
    torch.cuda.synchronize()
    assert dc.num_episodes() == 3 and dc.lens[:3] == [50, 50, 50]
    assert torch.equal(dc.ring[:3], dl.ring[:3])
    r = dc.ring[:3].cpu().numpy()
    # record k holds the reward of step k - 1: the first episode starts at 0, the next one carries
    # the previous episode's last reward over the reset
    assert r[0, 0, 11] == 0 and r[1, 0, 11] != 0 and np.all(r[..., 16:] == 0)


def test_env_i_is_the_one_env_collection_with_seed_plus_i():
    """Batched lockstep envs: env i's episodes equal a one-env collection seeded seed + i (the
    teacher's row-independent forward, independent envs); a partial last round is dropped."""
    from reacherdistilation_amd import teacher
    n, rounds = 3, 2
    db = teacher.collect_reward(n * rounds - 1, n_envs=n, seed=5, device=DEV)
    assert db.num_episodes() == n * rounds - 1
    for i in range(n):
        d1 = teacher.collect_reward(rounds, n_envs=1, seed=5 + i, device=DEV)
        for r in range(rounds):
            e = r * n + i
            if e < n * rounds - 1:
                assert torch.equal(db.ring[e], d1.ring[r]), (i, r)


def test_pages_hold_the_collected_episodes(tmp_path):
    """With a page store: full pages of MAX_CAPACITY episodes, in the reference's page format,
    whose records read back equal to the ring's (f32 -> page f64 -> f32)."""
    from reacherdistilation_amd import teacher
    from reacherdistilation_amd.config import MAX_CAPACITY
    from reacherdistilation_amd.pages import episodes_to_records, read_page
    d = teacher.collect_reward(2 * MAX_CAPACITY + 3, n_envs=8, seed=1, device=DEV, store_dir=str(tmp_path))
    assert d.num_episodes() == 2 * MAX_CAPACITY + 3
    pages = d.store.sorted_pages()
    assert len(pages) == 2
    rec = np.concatenate([episodes_to_records(read_page(p)) for p in pages])
    assert rec.shape == (2 * MAX_CAPACITY, 50, 21)
    assert np.array_equal(rec.astype(np.float32), d.ring[:2 * MAX_CAPACITY].cpu().numpy())


def test_large_batch_collection_feeds_the_training_windows():
    """4,096 envs, one round: every record finite, the teacher-stepped flag 't', and the
    dataset's training windows drawn from them."""
    from reacherdistilation_amd import teacher
    d = teacher.collect_reward(4096, n_envs=4096, seed=2, device=DEV)
    r = d.ring[:4096]
    assert d.num_episodes() == 4096 and bool(torch.isfinite(r).all())
    assert float(r[..., 20].abs().sum()) == 0.0
    (ob, t, prev, prew), = list(d.training_batches())[:1]
    assert ob.shape == (10, 20, 11) and bool(torch.isfinite(t).all())

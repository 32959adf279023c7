"""BASELINE config 1 -- one Reacher-v2 episode + one MSE distillation step, the reference's
single-env path (mlp_train.py:120-161) -- through the MI355X path, against the oracles:
the episode's observations vs the C f64 env oracle driven by the same actions (obs atol 5e-5
+ rtol 1e-4), the teacher actions vs policy_np, and the student after one
TF1 Adam step on the episode's 50 observations vs policy_np + AdamTF1 (1e-6 where the
gradient is not ~0; a first Adam step is ~lr*sign(g))."""
import numpy as np
import pytest
import torch

from oracle import policy_np as pn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_one_episode_and_one_mse_step(oracle_c):
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    from reacherdistilation_amd.env import make_mujoco_env
    env = make_mujoco_env("Reacher-v2", 0, device=DEV)
    tr = DistillTrainer(DistillConfig(n_envs=64, loss="mse", lr=1e-3), device=DEV)
    ob = env.reset()
    obs, acts = [], []
    for k in range(50):
        t, _ = tr.forward(torch.tensor(ob, dtype=torch.float32).view(1, 11))
        a = t[0, :2].cpu().numpy()
        ft = pn.forward(*[x.astype(np.float64) for x in (tr.teacher.flat, tr.teacher.ob_mean, tr.teacher.ob_std)],
                        ob.astype(np.float32).astype(np.float64)[None])
        np.testing.assert_allclose(a, ft["mean"][0], atol=2e-5)
        obs.append(ob)
        acts.append(a)
        ob, r, done, _ = env.step(a)
        assert done == (k == 49)
    obs = np.array(obs)
    # the same actions through the C f64 oracle from the same (gym seed 0) reset
    from oracle import reacher_np as rn
    rng = rn.gym_rng(0)
    state, ob0 = oracle_c.reset(np.array([rn.reset_draw(rng)]), np.float64)
    np.testing.assert_allclose(obs[0], ob0[0], atol=1e-6)
    for k in range(49):
        o, _ = oracle_c.step(state, np.array(acts[k], np.float32)[None], np.float64)
        np.testing.assert_allclose(obs[k + 1], o[0], atol=5e-5, rtol=1e-4)
    # one MSE step on the episode's observations
    p0 = tr.student_params().cpu().numpy()
    x = torch.tensor(obs, dtype=torch.float32)
    tr.step_obs(x)
    p1 = tr.student_params().cpu().numpy()
    assert tr.counters() == (0, 1)
    ob32 = obs.astype(np.float32).astype(np.float64)
    fs = pn.forward(p0.astype(np.float64), tr.student.ob_mean.astype(np.float64),
                    tr.student.ob_std.astype(np.float64), ob32)
    ft = pn.forward(tr.teacher.flat.astype(np.float64), tr.teacher.ob_mean.astype(np.float64),
                    tr.teacher.ob_std.astype(np.float64), ob32)
    L, dmean, dls, _ = pn.loss_and_dmean(fs, ft, "mse", 50)
    g = pn.backward(p0.astype(np.float64), fs, dmean, dls)
    opt = pn.AdamTF1(pn.P_TOT, lr=1e-3)
    ref = p0.copy()
    opt.step(ref, g.astype(np.float32))
    strong = np.abs(g) > 1e-3 * np.abs(g).max()
    np.testing.assert_allclose(p1[strong], ref[strong], atol=1e-6, rtol=0)
    assert tr.metrics(1)[0, 1] == pytest.approx(L, rel=1e-4)


def test_reference_shaped_driver_runs():
    """mlp_train.train: teacher warm-up episodes, then DAgger episodes with dataset-window
    training steps; the per-episode loss is finite and the counters agree."""
    from reacherdistilation_amd import mlp_train
    tr, ds, losses = mlp_train.train(episodes=5, warmup_episodes=2, loss="mse", lr=1e-3, log=lambda *a: None)
    assert ds.num_episodes() == 5 and len(losses) == 2
    assert all(np.isfinite(losses))
    env_steps, opt_steps = tr.counters()
    assert env_steps == 0 and opt_steps == 2 * 50


def test_reference_shaped_driver_dumps_pages_and_trains_on_them(tmp_path):
    """store_dir: the driver dumps every 5 episodes (mlp_train.py:203); once data_in_memory
    holds MAX_CAPACITY episodes the page closes, and the pool refreshes (every 25 records)
    draw from data_in_memory plus the stored pages (dataset.py:164-182)."""
    from reacherdistilation_amd import mlp_train, pages
    from reacherdistilation_amd.config import MAX_CAPACITY
    tr, ds, losses = mlp_train.train(episodes=13, warmup_episodes=1, loss="mse", lr=1e-3, log=lambda *a: None,
                                     store_dir=str(tmp_path))
    assert ds.num_episodes() == 13 and len(losses) == 11 and all(np.isfinite(losses))
    assert len(ds.store.pages) == 1 and len(pages.read_page(ds.store.pages[0])) == MAX_CAPACITY
    # the last refresh (25 records into episode 13): episodes 11, 12 in memory + page 0
    assert ds.pool_pages == ds.store.pages and ds.pool_size() == MAX_CAPACITY + 2 and len(ds._mem_slots) == 3


def test_reference_shaped_driver_with_the_reference_student():
    """student="mlp": the reference's own student_mlp_graph on ob | prev_pdflat | prev_rew rows,
    kl_loss on the recorded teacher pdflat, dropout keep_prob 0.5 (reference KEEP_PROB)."""
    from reacherdistilation_amd import mlp_train
    sm, ds, losses = mlp_train.train(episodes=4, warmup_episodes=2, loss="kl", lr=1e-3, student="mlp",
                                     keep_prob=0.5, log=lambda *a: None)
    assert ds.num_episodes() == 4 and len(losses) == 1 and np.isfinite(losses[0])
    assert sm.counter() == 50
    m = sm.metrics(50)
    assert np.all(m[:, 2] == 200)   # one [10, 20] window = 200 rows per optimiser step


def test_reference_shaped_lstm_driver_runs():
    """lstm_train.train: teacher warm-up, then per env step one truncated-BPTT Adam step on a
    [10, 20] window and the student's query with the carried LSTM state."""
    from reacherdistilation_amd import lstm_train
    st, ds, losses = lstm_train.train(episodes=4, warmup_episodes=2, keep_prob=0.5, log=lambda *a: None)
    assert ds.num_episodes() == 4 and len(losses) == 1 and np.isfinite(losses[0])
    assert st.counter() == 50
    m = st.metrics(50)
    assert np.all(m[:, 2] == 200) and np.all(np.isfinite(m[:, 0]))


@pytest.mark.parametrize("student", ["policy", "mlp"])
def test_device_resident_driver_equals_the_gym_api_loop(student):
    """mlp_train.train's default loop (env I/O kept on the device, `done` from the TimeLimit
    count, losses read once per episode) writes the same records, trains the same student
    and logs the same losses as the loop through the gym-API env (numpy every step)."""
    from reacherdistilation_amd import mlp_train
    kw = dict(episodes=5, warmup_episodes=2, loss="kl", lr=1e-3, student=student, log=lambda *a: None)
    a, da, la = mlp_train.train(**kw)
    b, db, lb = mlp_train.train(gym_env=True, **kw)
    torch.cuda.synchronize()
    assert da.num_episodes() == db.num_episodes() == 5
    assert torch.equal(da.ring, db.ring)
    assert la == lb and len(la) == 2
    pa = a.params() if student == "mlp" else a.student_params()
    pb = b.params() if student == "mlp" else b.student_params()
    assert torch.equal(pa, pb)


@pytest.mark.parametrize("fn", ["train", "train_bptt"])
def test_device_resident_lstm_drivers_equal_the_gym_api_loop(fn):
    """lstm_train.train / train_bptt with the env I/O on the device write the same records,
    train the same student and log the same losses as through the gym-API env."""
    from reacherdistilation_amd import lstm_train
    kw = dict(episodes=4, warmup_episodes=2, keep_prob=0.5, log=lambda *a: None)
    a, da, la = getattr(lstm_train, fn)(**kw)
    b, db, lb = getattr(lstm_train, fn)(gym_env=True, **kw)
    torch.cuda.synchronize()
    assert da.num_episodes() == db.num_episodes() == 4
    assert torch.equal(da.ring, db.ring)
    assert la == lb and len(la) >= 1
    assert torch.equal(a.params(), b.params())

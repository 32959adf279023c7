"""DeviceDataset (reference dataset.py Dataset) semantics on CPU tensors: record layout,
prev/prew fields, training-window sampling and the test batch (reference
tests/dataset_unit_test.py checks the same windowing on its fixture)."""
import numpy as np
import pytest
import torch

from reacherdistilation_amd.dataset import DeviceDataset


def _fill(ds, episodes):
    for e in range(episodes):
        for k in range(50):
            ob = np.full(11, 100.0 * e + k)          # encodes (episode, step)
            t = np.array([e, k, -1, -2], float)
            ds.write(ob=ob, reward=0.5 * k, t_pdflat=t, stepped_with="t")
        ds.flush()


def test_training_windows_are_contiguous_episode_slices():
    ds = DeviceDataset(capacity=8, device="cpu", seed=1)
    _fill(ds, 5)
    assert ds.num_episodes() == 5 and ds.stored() == 5
    (ob, t, prev, prew), = list(ds.training_batches())
    assert ob.shape == (10, 20, 11) and t.shape == (10, 20, 4) and prev.shape == (10, 20, 4) and prew.shape == (10, 20, 1)
    code = ob[..., 0].numpy()
    ep, step = code // 100, code % 100
    assert np.all(ep == ep[0:1])                           # one episode per batch column
    assert np.all(np.diff(step, axis=0) == 1)              # consecutive steps in a window
    assert np.all(step[0] == step[0, 0]) and 0 <= step[0, 0] <= 40   # one common start
    # prev = the previous record's teacher pdflat and reward (zeros at the episode start)
    s0 = int(step[0, 0])
    exp_prev = np.where(step > 0, step - 1, 0)
    assert np.array_equal(prev[..., 1].numpy(), exp_prev.astype(np.float32))
    assert np.allclose(prew[..., 0].numpy(), np.where(step > 0, 0.5 * (step - 1), 0.0))
    assert s0 >= 0


def test_ring_overwrites_oldest_episode():
    ds = DeviceDataset(capacity=3, device="cpu")
    _fill(ds, 5)
    eps = sorted({int(x) for x in ds.ring[:, 0, 0].numpy() // 100})
    assert eps == [2, 3, 4]


def test_partial_episode_is_stored_like_the_reference():
    """flush() stores an incomplete episode with its record count (reference dataset.py:
    146-149); a training window drawn past its end raises IndexError, as the reference's
    episode[i] does; more than EPISODE_STEPS records in one episode is refused."""
    ds = DeviceDataset(capacity=3, device="cpu")
    for k in range(7):
        ds.write(ob=np.ones(11))
    ds.flush()
    assert ds.num_episodes() == 1 and ds.lens[0] == 7
    assert float(ds.ring[0, :7, :11].sum()) == 77.0 and float(ds.ring[0, 7:].abs().sum()) == 0.0
    with pytest.raises(IndexError):
        list(ds.training_batches())
    with pytest.raises(RuntimeError):
        for k in range(51):
            ds.write(ob=np.ones(11))


@pytest.mark.parametrize("length", [0, 3, 9, 12])
def test_test_batch_window(length):
    ds = DeviceDataset(device="cpu")
    for k in range(length):
        ds.write(ob=np.full(11, k + 1.0))
    tb = ds.test_batch(np.full(11, 99.0)).numpy()
    assert tb.shape == (10, 20, 11)
    assert not tb[:, :19].any()                            # only the last batch column
    col = tb[:, 19, 0]
    assert col[-1] == 99.0
    k = min(length, 9)
    assert np.array_equal(col[9 - k:9], np.arange(length - k + 1, length + 1, dtype=np.float32))
    assert not col[:9 - k].any()


@pytest.mark.parametrize("length", [0, 1, 5, 9, 30])
def test_test_windows_carry_the_prev_series(length):
    """LSTM query window: column B-1 = last T-1 records + the current step, with each step's
    prev fields (previous record's teacher pdflat / reward; the current step's = the last
    record's), zero-padded at the front; the other columns are zero."""
    ds = DeviceDataset(capacity=4, device="cpu", seed=0)
    for k in range(length):
        ds.write(ob=np.full(11, float(k)), reward=0.5 * k, t_pdflat=np.array([k, 10 + k, -1, -2], float))
    ob_w, prev_w, prew_w = ds.test_windows(np.full(11, 99.0))
    assert ob_w.shape == (10, 20, 11) and prev_w.shape == (10, 20, 4) and prew_w.shape == (10, 20, 1)
    assert not ob_w[:, :19].any() and not prev_w[:, :19].any() and not prew_w[:, :19].any()
    assert ob_w[9, 19, 0] == 99.0
    for row in range(10):
        j = length - (9 - row)          # record index of this row (j == length: the current step)
        if j < 0:
            assert not ob_w[row, 19].any() and not prev_w[row, 19].any()
            continue
        if j < length:
            assert ob_w[row, 19, 0] == j
        want_prev = j - 1               # prev = previous record's t (zeros at j = 0)
        if want_prev >= 0:
            assert prev_w[row, 19, 0] == want_prev and prev_w[row, 19, 1] == 10 + want_prev
            assert prew_w[row, 19, 0] == 0.5 * want_prev
        else:
            assert not prev_w[row, 19].any() and prew_w[row, 19, 0] == 0


def test_bptt_windows_slide_by_one_step_over_fixed_episodes():
    """backup/dataset_bbpt.py:179-193: one draw of LSTM_BATCH_SIZE episodes, then the windows
    starting at 0, 1, ..., EPISODE_STEPS - T - 1 in order, each with its prev fields."""
    ds = DeviceDataset(capacity=8, device="cpu", seed=3)
    _fill(ds, 6)
    wins = list(ds.bptt_batches())
    assert len(wins) == 40
    first_eps = None
    for i, (ob, t, prev, prew) in enumerate(wins):
        assert ob.shape == (10, 20, 11) and prev.shape == (10, 20, 4) and prew.shape == (10, 20, 1)
        code = ob[..., 0].numpy()
        ep, step = code // 100, code % 100
        assert np.all(step == (i + np.arange(10))[:, None])          # start i, consecutive steps
        first_eps = ep[0] if first_eps is None else first_eps
        assert np.array_equal(ep, np.broadcast_to(first_eps, ep.shape))   # the same episodes throughout
        assert np.array_equal(t[..., 1].numpy(), step.astype(np.float32))
        assert np.array_equal(prev[..., 1].numpy(), np.where(step > 0, step - 1, 0).astype(np.float32))
    assert list(DeviceDataset(device="cpu").bptt_batches()) == []


@pytest.mark.parametrize("cap,before,block", [(8, 0, 5), (8, 6, 5), (4, 1, 11), (5, 3, 5)])
def test_write_episodes_equals_write_and_flush(cap, before, block):
    """The batched append (teacher.collect_reward) leaves the ring, lengths, episode count and
    data_in_memory as the same episodes written record by record and flushed would, through
    ring wrap-around and blocks larger than the ring."""
    a = DeviceDataset(capacity=cap, device="cpu")
    b = DeviceDataset(capacity=cap, device="cpu")
    _fill(a, before)
    _fill(b, before)
    c = DeviceDataset(capacity=block + 1, device="cpu")
    for e in range(block):
        for k in range(50 if e % 3 else 37):            # some incomplete episodes
            c.write(ob=np.full(11, 1000.0 + 100 * e + k), reward=0.25 * k, t_pdflat=np.array([e, k, 1, 2], float))
        c.flush()
    for e in range(block):
        for k in range(c.lens[e]):
            a.write(ob=c.ring[e, k, :11], reward=c.ring[e, k, 11], t_pdflat=c.ring[e, k, 12:16])
        a.flush()
    assert b.write_episodes(c.ring[:block], c.lens[:block]) == block
    assert a.num_episodes() == b.num_episodes() == before + block
    assert torch.equal(a.ring, b.ring) and a.lens == b.lens
    assert sorted(a._mem_slots) == sorted(b._mem_slots)
    assert [a.lens[s] for s in a._mem_slots[-min(block, cap):]] == [b.lens[s] for s in b._mem_slots[-min(block, cap):]]
    with pytest.raises(ValueError):
        b.write_episodes(torch.zeros(2, 49, 21))
    b.write(ob=np.ones(11))
    with pytest.raises(RuntimeError):
        b.write_episodes(c.ring[:1])

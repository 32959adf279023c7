"""DeviceDataset on a HIP device against the reference's own fixture and its windowing test.

The reference checks its Dataset on the fixture page (tests/dataset_unit_test.py:13-94;
windowing dataset.py:179-235): the three padding cases of ob_batch_test_array, the stored
prev series, and the prev / prew test arrays.  Here the same page (rebuilt in its exact
layout from tests/golden/reacher_fixture.npz, see tests/test_pages_host.py) is loaded into a
cuda DeviceDataset and every window is compared bit for bit with numpy indexing of the
golden arrays (the device holds f32 records: compared against the golden values rounded to
f32).
"""
import numpy as np
import pytest
import torch

from reacherdistilation_amd import pages
from reacherdistilation_amd.config import EPISODE_STEPS, LSTM_BATCH_SIZE, STEPS_UNROLLED
from reacherdistilation_amd.dataset import DeviceDataset
from tests.test_pages_host import _fixture_layout_page

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
T, B = STEPS_UNROLLED, LSTM_BATCH_SIZE


@pytest.fixture
def page(golden, tmp_path):
    return _fixture_layout_page(golden, tmp_path / "fixture_layout.json")


def _f32(x):
    return np.asarray(x, np.float64).astype(np.float32)


def _write_prefix(ds, golden, e, L):
    """The reference test's `curr_episode = data_in_memory[e][:L]`: the episode's first L
    records written through the reference interface."""
    for k in range(L):
        ds.write(ob=golden["ob"][e, k], reward=float(golden["rew"][e, k]), t_pdflat=golden["t"][e, k],
                 s_pdflat=golden["s"][e, k], stepped_with="s" if golden["student"][e, k] else "t")


@pytest.mark.parametrize("L", [T - 3, T - 1, T + 5, 0, EPISODE_STEPS - 1])   # the reference's 3 cases + edges
def test_observation_test_cases_on_the_fixture(golden, L):
    ds = DeviceDataset(capacity=4, device=DEV)
    _write_prefix(ds, golden, 0, L)
    ob = np.full(11, -10.0)
    got = ds.test_batch(ob)
    assert got.device.type == "cuda"
    got = got.cpu().numpy()
    want = np.zeros((T, B, 11), np.float32)
    k = min(L, T - 1)
    want[T - 1 - k:T - 1, B - 1] = _f32(golden["ob"][0, L - k:L])
    want[T - 1, B - 1] = -10.0
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("L", [1, T - 1, T + 5, EPISODE_STEPS - 1])
def test_prev_series_of_the_test_windows_on_the_fixture(golden, L):
    """prev_pdflat_test / prev_rew_test: row i of the window holds record i's prev fields (the
    previous record's teacher pdflat and reward), the last row the last record's own."""
    ds = DeviceDataset(capacity=4, device=DEV)
    _write_prefix(ds, golden, 3, L)
    ob_w, prev_w, prew_w = ds.test_windows(np.full(11, -10.0))
    prev_w, prew_w = prev_w.cpu().numpy(), prew_w.cpu().numpy()
    t, rew = _f32(golden["t"][3]), _f32(golden["rew"][3])
    want_p = np.zeros((T, B, 4), np.float32)
    want_r = np.zeros((T, B, 1), np.float32)
    for row in range(T):
        j = L - (T - 1 - row)          # record index (j == L: the step being queried)
        if j <= 0:
            continue
        want_p[row, B - 1] = t[j - 1]
        want_r[row, B - 1, 0] = rew[j - 1]
    np.testing.assert_array_equal(prev_w, want_p)
    np.testing.assert_array_equal(prew_w, want_r)
    assert not ob_w[:, :B - 1].any()


def test_loaded_page_prev_fields_and_training_windows(golden, page):
    """A fixture page loaded onto the device: the derived prev series equals the fixture's
    stored prev wherever the previous record was teacher-stepped (the committed pdflat_at;
    the fixture's student-stepped prevs came from its commented-out variant, see
    test_pages_host), and every training window is a contiguous slice of a stored episode
    with its t / prev / prew columns."""
    ds = DeviceDataset(capacity=40, device=DEV, seed=7, epochs=3)
    assert ds.load_page(page) == 25 and ds.stored() == 25
    assert ds.ring.device.type == "cuda"
    rec = ds.ring[:25].cpu().numpy()
    np.testing.assert_array_equal(rec[..., pages.F_OB:pages.F_REW], _f32(golden["ob"]))
    np.testing.assert_array_equal(rec[..., pages.F_T:pages.F_S], _f32(golden["t"]))
    prev = ds._prev(ds.ring[:25]).cpu().numpy()
    after_t = np.zeros((25, 50), bool)
    after_t[:, 1:] = ~golden["student"][:, :-1]
    after_t[:, 0] = True
    np.testing.assert_array_equal(prev[..., :4][after_t], _f32(golden["prev"])[after_t])
    assert not prev[:, 0].any()
    ob_f, t_f, rew_f = _f32(golden["ob"]), _f32(golden["t"]), _f32(golden["rew"])
    n = 0
    for ob, t, pv, pr in ds.training_batches():
        assert ob.is_cuda and ob.shape == (T, B, 11) and pv.shape == (T, B, 4) and pr.shape == (T, B, 1)
        ob, t, pv, pr = (x.cpu().numpy() for x in (ob, t, pv, pr))
        starts = set()
        for b in range(B):
            hits = [(e, s) for e in range(25) for s in range(EPISODE_STEPS - T + 1)
                    if np.array_equal(ob_f[e, s:s + T], ob[:, b])]
            assert hits, b
            e, s = hits[0]
            starts.add(s)
            np.testing.assert_array_equal(t[:, b], t_f[e, s:s + T])
            idx = np.arange(s, s + T)
            want_p = np.where((idx > 0)[:, None], t_f[e, np.maximum(idx - 1, 0)], 0)
            want_r = np.where(idx > 0, rew_f[e, np.maximum(idx - 1, 0)], 0)
            np.testing.assert_array_equal(pv[:, b], want_p)
            np.testing.assert_array_equal(pr[:, b, 0], want_r)
        assert len(starts) == 1        # one common start per batch (dataset.py:186-187)
        n += 1
    assert n == 3

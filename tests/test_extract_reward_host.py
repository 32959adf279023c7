"""Reward extraction (reference extract_reward.py:12-48, 247-252) over pages rebuilt from the
reference fixture's 25 episodes (tests/golden/reacher_fixture.npz), split over three pages
written out of index order; the expected values repeat the reference's arithmetic (per-episode
Python float sums in record order, averages per 5 episodes, / EPISODE_STEPS)."""
import os
import shutil

import numpy as np
import pytest

from reacherdistilation_amd import extract_reward as er
from reacherdistilation_amd import pages
from reacherdistilation_amd.dataset import DeviceDataset

from tests.test_pages_host import REF_PAGE


def _episodes(golden):
    return [[{"ob": golden["ob"][e, k].tolist(), "rew": float(golden["rew"][e, k]), "t": golden["t"][e, k].tolist(),
              "s": golden["s"][e, k].tolist(), "with": "t", "prev": golden["prev"][e, k].tolist()}
             for k in range(50)] for e in range(golden["ob"].shape[0])]


def _expected(golden, per):
    ret = []
    for e in range(golden["rew"].shape[0]):
        s = 0
        for k in range(50):
            s += float(golden["rew"][e, k])
        ret.append(s)
    avg = [sum(ret[i:i + per]) / len(ret[i:i + per]) for i in range(0, len(ret), per)]
    return ret, avg, [a / 50 for a in avg]


def test_returns_and_averages_over_pages_in_index_order(golden, tmp_path):
    eps = _episodes(golden)
    for idx, lo, hi in ((2, 20, 25), (0, 0, 10), (1, 10, 20)):   # written out of order
        pages.write_page(str(tmp_path / f"dataset_{idx}.json"), eps[lo:hi])
    ret, avg, rew = _expected(golden, 5)
    assert er.ExtractReward.get_return(str(tmp_path)) == ret
    assert er.ExtractReward.get_avg_return(str(tmp_path), 5) == avg
    assert er.ExtractReward.get_avg_reward(pages.PageStore(str(tmp_path)), 5) == rew
    _, avg7, _ = _expected(golden, 7)                             # a shorter last group
    assert er.ExtractReward.get_avg_return(str(tmp_path), 7) == avg7 and len(avg7) == 4
    out = str(tmp_path / "kp0.5ss")
    logs = []
    assert er.extract(str(tmp_path), out, log=logs.append) == rew
    assert np.array_equal(np.load(out + ".npy"), np.array(rew))
    assert logs[-1].endswith("avg_rews array length is 5")


def test_device_returns_match_the_page_returns(golden, tmp_path):
    pages.write_page(str(tmp_path / "dataset_0.json"), _episodes(golden))
    ds = DeviceDataset(capacity=32, device="cpu")
    ds.load_page(str(tmp_path / "dataset_0.json"))
    np.testing.assert_allclose(er.device_returns(ds).numpy(), er.ExtractReward.get_return(str(tmp_path)), rtol=1e-6)


@pytest.mark.skipif(not os.path.exists(REF_PAGE), reason="reference checkout not present (GPU box)")
def test_the_reference_page_itself(golden, tmp_path):
    shutil.copy(REF_PAGE, tmp_path / "dataset_0.json")   # test-time copy of the fixture data, not committed
    ret, _, rew = _expected(golden, 5)
    assert er.ExtractReward.get_return(str(tmp_path)) == ret
    assert er.ExtractReward.get_avg_reward(str(tmp_path), 5) == rew

"""Dataset pages (reacherdistilation_amd/pages.py) in the reference's on-disk format (gzip'd
JSON written by json_tricks, reference dataset.py:31-35) and the DatasetStore paging
semantics (dataset.py:14-65).

The reference's own page (its test fixture src/distilation/tests/data/dataset.json) is not
copied into this repo: a page in the same layout (keys s, with, rew (scalar), prev, ob, t)
is rebuilt from the committed golden arrays (tests/golden/reacher_fixture.npz, derived from
that fixture by tests/golden/make_golden.py), and where /root/reference exists (this build
container, never the GPU box) the reference file itself is parsed too.
"""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from reacherdistilation_amd import pages
from reacherdistilation_amd.config import MAX_CAPACITY
from reacherdistilation_amd.dataset import DeviceDataset
from tests.conftest import GOLDEN

REF_PAGE = "/root/reference/src/distilation/tests/data/dataset.json"


def _fixture_layout_page(golden, path):
    """A page in the fixture's layout rebuilt from the golden arrays."""
    eps = []
    for e in range(golden["ob"].shape[0]):
        eps.append([{"s": golden["s"][e, k].tolist(), "with": "s" if golden["student"][e, k] else "t",
                     "rew": float(golden["rew"][e, k]), "prev": golden["prev"][e, k].tolist(),
                     "ob": golden["ob"][e, k].tolist(), "t": golden["t"][e, k].tolist()}
                    for k in range(golden["ob"].shape[1])])
    with open(path, "wb") as fh:
        fh.write(gzip.compress(json.dumps(eps).encode()))
    return str(path)


@pytest.fixture
def page(golden, tmp_path):
    return _fixture_layout_page(golden, tmp_path / "fixture_layout.json")


@pytest.mark.skipif(not os.path.exists(REF_PAGE), reason="reference checkout not present (GPU box)")
def test_the_reference_page_itself_parses_to_the_golden_records(golden):
    rec = pages.episodes_to_records(pages.read_page(REF_PAGE))
    np.testing.assert_array_equal(rec[..., pages.F_OB:pages.F_REW], golden["ob"])
    np.testing.assert_array_equal(rec[..., pages.F_REW], golden["rew"])
    np.testing.assert_array_equal(rec[..., pages.F_T:pages.F_S], golden["t"])


def test_reference_layout_page_parses_to_the_golden_records(golden, page):
    eps = pages.read_page(page)
    assert len(eps) == 25 and all(len(e) == 50 for e in eps)
    rec = pages.episodes_to_records(eps)
    np.testing.assert_array_equal(rec[..., pages.F_OB:pages.F_REW], golden["ob"])
    np.testing.assert_array_equal(rec[..., pages.F_REW], golden["rew"])
    np.testing.assert_array_equal(rec[..., pages.F_T:pages.F_S], golden["t"])
    np.testing.assert_array_equal(rec[..., pages.F_S:pages.F_WITH], golden["s"])
    np.testing.assert_array_equal(rec[..., pages.F_WITH] > 0.5, golden["student"])
    # prev as the committed pdflat_at derives it (previous record's teacher pdflat) equals the
    # stored one after teacher-stepped records; after student-stepped records the fixture holds
    # the student's pdflat -- it was written by the variant in pdflat_at's commented-out lines
    # (reference dataset.py:155-159), 196 of its 1225 records
    derived = pages.records_to_episodes(rec)
    n_s = 0
    for e in range(25):
        for k in range(50):
            if k > 0 and eps[e][k - 1]["with"] == "s":
                assert eps[e][k]["prev"] == eps[e][k - 1]["s"]
                n_s += 1
            else:
                assert derived[e][k]["prev"] == eps[e][k]["prev"]
    assert n_s == 196


def test_write_read_roundtrip_is_exact(tmp_path, page):
    rec = pages.episodes_to_records(pages.read_page(page))
    out = tmp_path / "dataset_0.json"
    pages.write_page(str(out), pages.records_to_episodes(rec))
    assert open(out, "rb").read(2) == b"\x1f\x8b"       # gzip, as json_tricks compression=True
    back = pages.episodes_to_records(pages.read_page(str(out)))
    np.testing.assert_array_equal(back, rec)
    st = pages.read_page(str(out))[0][3]
    assert set(st) == {"ob", "rew", "t", "s", "with", "prev", "prew"} and st["rew"] == [rec[0, 3, pages.F_REW]]
    assert st["prew"] == [rec[0, 2, pages.F_REW]]


def test_device_dataset_loads_a_reference_page_and_trains_on_it(page):
    ds = DeviceDataset(capacity=40, device="cpu", seed=3)
    assert ds.load_page(page) == 25 and ds.stored() == 25
    ob, t, prev, prew = next(ds.training_batches())
    rec = torch.as_tensor(pages.episodes_to_records(pages.read_page(page)), dtype=torch.float32)
    # every window column is a contiguous slice of some stored reference episode
    for b in range(ob.shape[1]):
        hits = [(e, s) for e in range(25) for s in range(41) if torch.equal(rec[e, s:s + 10, :11], ob[:, b])]
        assert hits
        e, s = hits[0]
        assert torch.equal(t[:, b], rec[e, s:s + 10, 12:16])


def test_page_store_semantics(tmp_path):
    store = pages.PageStore(str(tmp_path))
    assert store.curr_page.endswith("dataset_0.json") and store.pages == []
    ds = DeviceDataset(capacity=64, device="cpu")
    for e in range(MAX_CAPACITY + 3):
        for k in range(50):
            ds.write(ob=np.full(11, e), reward=k, t_pdflat=np.array([e, k, 0, 0.0]))
        ds.flush()
        if e == 4:
            ds.dump(store)                    # 5 episodes: page 0 rewritten, not yet full
            assert len(pages.read_page(str(tmp_path / "dataset_0.json"))) == 5 and store.pages == []
        if e == MAX_CAPACITY - 1:
            ds.dump(store)                    # full: page 0 closed, new page 1
            assert store.curr_page.endswith("dataset_1.json") and len(store.pages) == 1
    ds.dump(store)
    assert len(pages.read_page(str(tmp_path / "dataset_1.json"))) == 3
    again = pages.PageStore(str(tmp_path))    # reopening collects the pages on disk
    assert sorted(map(os.path.basename, again.sorted_pages())) == ["dataset_0.json", "dataset_1.json"]
    assert again.curr_page.endswith("dataset_2.json")
    open(tmp_path / "dataset_3.json", "wb").close()
    with pytest.raises(FileExistsError):      # never overwrites an existing page
        again.create_new_page()

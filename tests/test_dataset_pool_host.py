"""The reference's training pool (dataset.py:164-194) on pages in the
reference's format built from its own fixture: pool membership at the refresh points
(len(curr_episode) % 25 == 0), windows drawn only from the pool, data_in_memory reset by a
full page, ≤ 10 random stored pages joining it, and the uniform-ring sampler as the option."""
import numpy as np
import pytest
import torch

from reacherdistilation_amd import pages
from reacherdistilation_amd.config import EPISODE_STEPS, MAX_CAPACITY
from reacherdistilation_amd.dataset import DeviceDataset

T = 10


def _episode(golden, e, marker):
    """Fixture episode e (its ob / rew / t / s records) with ob[10] = marker (a tag that
    identifies the episode in a window; the fixture's ob[10] is the constant 0)."""
    recs = []
    for k in range(EPISODE_STEPS):
        ob = golden["ob"][e % 25, k].copy()
        ob[10] = marker
        recs.append(dict(ob=ob, rew=float(golden["rew"][e % 25, k]), t=golden["t"][e % 25, k]))
    return recs


def _write(ds, recs):
    for r in recs:
        ds.write(ob=r["ob"], reward=r["rew"], t_pdflat=r["t"])


def _markers(batches):
    """The episode tags of every window column, checking each column is one tag."""
    out = []
    for ob, t, prev, prew in batches:
        tag = ob[..., 10]
        assert torch.all(tag == tag[0:1])
        out += [int(x) for x in tag[0]]
    return out


def _store_with_pages(tmp_path, golden, npages, base):
    """npages full pages of MAX_CAPACITY fixture episodes tagged base + 100 p + i."""
    store = pages.PageStore(str(tmp_path))
    ds = DeviceDataset(capacity=64, device="cpu", store=store)
    for p in range(npages):
        for i in range(MAX_CAPACITY):
            _write(ds, _episode(golden, p * MAX_CAPACITY + i, base + 100 * p + i))
            ds.flush()
        ds.dump()
    assert len(store.pages) == npages
    return store


def test_pool_refreshes_at_multiples_of_25_records(tmp_path, golden):
    _store_with_pages(tmp_path, golden, 3, 1000)
    page_tags = {1000 + 100 * p + i for p in range(3) for i in range(MAX_CAPACITY)}
    store = pages.PageStore(str(tmp_path))
    ds = DeviceDataset(capacity=64, device="cpu", seed=3, epochs=40, store=store)
    mem_tags = set(range(1, MAX_CAPACITY + 1))
    for e in range(MAX_CAPACITY):                        # data_in_memory: tags 1..10
        _write(ds, _episode(golden, e, 1 + e))
        ds.flush()
    tags = _markers(ds.training_batches())               # curr_len 0: refresh
    assert ds.pool_size() == MAX_CAPACITY + 3 * MAX_CAPACITY   # + all 3 stored pages (< 10)
    pool = mem_tags | page_tags
    assert set(tags) <= pool and len(set(tags)) > 20    # drawn only from the pool, widely
    # mid-episode (7 records) a dump fills the page: data_in_memory empties and a 4th page
    # exists, but the pool is not refreshed (7 % 25 != 0): same pool, same tags
    _write(ds, _episode(golden, 30, 99)[:7])
    ds.dump()
    assert ds._mem_slots == [] and len(store.pages) == 4
    assert set(_markers(ds.training_batches())) <= pool and ds.pool_size() == 4 * MAX_CAPACITY
    # 25 records: refresh -> data_in_memory (empty) + the 4 stored pages (tags 1..10 now
    # come from the new page)
    for r in _episode(golden, 30, 99)[7:25]:
        ds.write(ob=r["ob"], reward=r["rew"], t_pdflat=r["t"])
    assert ds.curr_len == 25
    tags = _markers(ds.training_batches())
    assert ds.pool_size() == 4 * MAX_CAPACITY and set(tags) <= pool and len(ds.pool_pages) == 4
    assert 99 not in tags


def test_newly_flushed_episodes_join_only_at_a_refresh(golden):
    ds = DeviceDataset(capacity=16, device="cpu", seed=5, epochs=30)
    for e in range(3):
        _write(ds, _episode(golden, e, 10 + e))
        ds.flush()
    assert set(_markers(ds.training_batches())) <= {10, 11, 12}
    _write(ds, _episode(golden, 3, 13)[:30])             # 30 records: 30 % 25 != 0, no refresh
    assert set(_markers(ds.training_batches())) <= {10, 11, 12}
    for r in _episode(golden, 3, 13)[30:]:
        ds.write(ob=r["ob"], reward=r["rew"], t_pdflat=r["t"])
    ds.flush()                                           # curr_len 0 -> the refresh includes tag 13
    tags = _markers(ds.training_batches())
    assert set(tags) <= {10, 11, 12, 13} and 13 in tags


def test_at_most_ten_random_pages_and_never_the_current_one(tmp_path, golden):
    _store_with_pages(tmp_path, golden, 12, 1000)
    st = pages.PageStore(str(tmp_path))
    ds = DeviceDataset(capacity=64, device="cpu", seed=1, store=st)
    list(ds.training_batches())
    assert len(ds.pool_pages) == 10 and st.curr_page not in ds.pool_pages
    assert ds.pool_size() == 10 * MAX_CAPACITY          # data_in_memory is empty


def test_ring_sampler_option_draws_from_every_stored_episode(golden):
    ds = DeviceDataset(capacity=8, device="cpu", seed=2, epochs=50, pool="ring")
    for e in range(6):
        _write(ds, _episode(golden, e, 20 + e))
        ds.flush()
    ds._mem_slots = []                                   # the ring sampler ignores data_in_memory
    assert set(_markers(ds.training_batches())) == set(range(20, 26))
    with pytest.raises(ValueError):
        DeviceDataset(device="cpu", pool="other")


def test_incomplete_episode_in_a_page_round_trips_with_its_length(tmp_path, golden):
    store = pages.PageStore(str(tmp_path))
    ds = DeviceDataset(capacity=8, device="cpu", store=store)
    _write(ds, _episode(golden, 0, 1))
    ds.flush()
    _write(ds, _episode(golden, 1, 2)[:13])
    ds.flush()
    ds.dump()
    eps = pages.read_page(store.curr_page)
    assert [len(e) for e in eps] == [50, 13]
    back = DeviceDataset(capacity=8, device="cpu")
    assert back.load_page(store.curr_page) == 2 and back.lens[:2] == [50, 13]
    np.testing.assert_array_equal(back.ring[1, :13, :11].numpy(), ds.ring[1, :13, :11].numpy())


def test_bptt_pool_pages_fixed_until_a_dump_empties_data_in_memory(tmp_path, golden):
    """the BPTT variant's pool aliases data_in_memory (backup/dataset_bbpt.py:164-181),
    so the pages it borrows stay until a dump empties data_in_memory -- not re-drawn per call."""
    store = _store_with_pages(tmp_path, golden, 20, 1000)
    ds = DeviceDataset(capacity=64, device="cpu", seed=5, store=pages.PageStore(str(tmp_path)))
    list(ds.bptt_batches())
    first = list(ds._bptt_pages)
    assert 0 < len(first) <= DeviceDataset.BPTT_POOL_PAGES
    for _ in range(5):                       # data_in_memory empty: the borrowed pages stay
        list(ds.bptt_batches())
        assert ds._bptt_pages == first
    for i in range(MAX_CAPACITY):            # a full page -> the dump empties data_in_memory
        _write(ds, _episode(golden, i, 1 + i))
        ds.flush()
        list(ds.bptt_batches())
        assert ds._bptt_pages == first       # flushed episodes join; the pages do not change
    ds.dump()
    assert not ds._mem_slots
    draws = []
    for _ in range(3):
        list(ds.bptt_batches())
        draws.append(list(ds._bptt_pages))
    assert draws[0] == draws[1] == draws[2]  # one new draw after the emptying dump
    assert len(store.pages) == 20


def test_page_cache_is_bounded(tmp_path, golden):
    """The device page cache keeps the PAGE_CACHE most recently used pages."""
    _store_with_pages(tmp_path, golden, 20, 1000)
    st = pages.PageStore(str(tmp_path))
    ds = DeviceDataset(capacity=64, device="cpu", store=st)
    for page in st.pages:
        ds._page_records(page)
    assert len(ds._page_cache) == DeviceDataset.PAGE_CACHE
    assert list(ds._page_cache) == list(st.pages)[-DeviceDataset.PAGE_CACHE:]
    ds._page_records(list(st.pages)[-DeviceDataset.PAGE_CACHE])     # a hit moves it to the end
    assert list(ds._page_cache)[-1] == list(st.pages)[-DeviceDataset.PAGE_CACHE]

"""Device-resident rollout -> distill buffer: the hand-off the reference's ``Dataset`` provides
(reference dataset.py:72-296), kept in HBM instead of lists of Python dicts.

Mirrored interface (reference dataset.py): ``write(ob, reward, t_pdflat, s_pdflat,
stepped_with)`` appends one step record of the current episode (:118-143, including the
``prev``/``prew`` fields = the previous record's teacher pdflat and reward, zeros at t = 0,
:132-133,152-163); ``flush()`` closes the episode (:146-149); ``num_episodes()``;
``training_batches()`` yields TRAINING_EPOCHS random windows -- LSTM_BATCH_SIZE episodes
drawn with replacement from the TRAINING POOL, one common start in [0, EPISODE_STEPS -
STEPS_UNROLLED] -- as ``(ob [T,B,11], t_pdflat [T,B,4], prev_pdflat [T,B,4], prev_rew
[T,B,1])`` (:179-202).  The pool is the reference's ``training_data`` (:166-182): refreshed
whenever the open episode holds a multiple of 25 records (or the pool is empty) to a copy of
``data_in_memory`` -- the episodes flushed since the last full page -- plus the episodes of
up to 10 random stored pages of the attached ``PageStore`` (not the current one).  Between
refreshes newly flushed episodes are not drawn.  ``pool="ring"`` instead draws uniformly from
every episode in the ring (the sampler of round 1-2);
``test_batch(ob)`` builds the [T,B,11] window ending at the current observation (:205-235);
``dump(store)`` / ``load_page(path)`` move episodes to / from pages in the reference's
on-disk format (``pages.PageStore``, :14-65,72-96).

Storage: one ring of ``capacity`` episodes x EPISODE_STEPS records x 21 floats (ob 11 |
rew 1 | t 4 | s 4 | with 1) plus the open episode, all on ``device``.  ``flush()`` stores the
episode whatever its length (:146-149): an incomplete one keeps its record count, and a
window drawn from it past its end raises IndexError, as the reference's ``episode[i]`` does.
Stored pages the pool draws are read once and kept on the device (full pages never change).
Deviations: ``data_in_memory`` is bounded by the ring (the oldest episodes are overwritten);
``load_page`` ADDS a page's episodes to it (the reference's ``switch`` replaces it); the
draws use a seeded torch generator, not Python's ``random`` (page choice does use
``random.sample`` as PageStore.rand_pages).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from .config import (EPISODE_STEPS, LSTM_BATCH_SIZE, OBSPACE_SHAPE, PDFLAT_SHAPE, STEPS_UNROLLED,
                     TRAINING_EPOCHS)

F_OB, F_REW, F_T, F_S, F_WITH = 0, OBSPACE_SHAPE, OBSPACE_SHAPE + 1, OBSPACE_SHAPE + 1 + PDFLAT_SHAPE, \
    OBSPACE_SHAPE + 1 + 2 * PDFLAT_SHAPE
REC = F_WITH + 1   # 21 floats per step record


class DeviceDataset:
    POOL_REFRESH = 25   # dataset.py:172: len(curr_episode) % 25 == 0
    POOL_PAGES = 10     # dataset.py:166: dstore.rand_pages(10)

    def __init__(self, capacity: int = 5000, device="cuda:0", seed: int = 0, batch_size: int = LSTM_BATCH_SIZE,
                 steps_unrolled: int = STEPS_UNROLLED, epochs: int = TRAINING_EPOCHS, store=None,
                 pool: str = "reference"):
        if pool not in ("reference", "ring"):
            raise ValueError(f"pool must be 'reference' or 'ring', not {pool!r}")
        self.device = torch.device(device)
        self.capacity = int(capacity)
        self.ring = torch.zeros(self.capacity, EPISODE_STEPS, REC, dtype=torch.float32, device=self.device)
        self.curr = torch.zeros(EPISODE_STEPS, REC, dtype=torch.float32, device=self.device)
        self.curr_len = 0
        self.num_total_episodes = 0
        self.B, self.T, self.epochs = int(batch_size), int(steps_unrolled), int(epochs)
        self._gen = torch.Generator().manual_seed(int(seed))   # host RNG: indices only
        self._mem_slots = []   # ring slots flushed since the last full page (reference data_in_memory)
        self.lens = [0] * self.capacity   # records of the episode in each ring slot
        self.store = store                 # pages.PageStore (reference Dataset.dstore) or None
        self.pool_mode = pool
        self._pool = None                  # training pool [P, 50, REC] (reference training_data)
        self._pool_lens = None
        self._page_cache = OrderedDict()   # page path -> (records on the device, lengths); LRU of PAGE_CACHE
        self._bptt_pages = None            # the BPTT pool's borrowed pages (drawn once per emptied data_in_memory)
        self._bptt_stale = True
        self._zeros = torch.zeros(PDFLAT_SHAPE, dtype=torch.float32, device=self.device)
        self._with = torch.tensor([[0.0], [1.0]], dtype=torch.float32, device=self.device)   # stepped with t / s

    # -- reference interface -------------------------------------------------------------
    def num_episodes(self) -> int:
        return self.num_total_episodes

    def write(self, ob, reward=0.0, t_pdflat=None, s_pdflat=None, stepped_with: str = "t"):
        if self.curr_len >= EPISODE_STEPS:
            raise RuntimeError(f"episode already holds {EPISODE_STEPS} steps; flush() first")
        # one concatenation straight into the record (one launch per step; device inputs, as
        # the drivers pass them, are used in place: no host round trip, no sync)
        torch.cat((self._field(ob, OBSPACE_SHAPE), self._field(reward, 1), self._field(t_pdflat, PDFLAT_SHAPE),
                   self._field(s_pdflat, PDFLAT_SHAPE), self._with[1 if stepped_with == "s" else 0]),
                  out=self.curr[self.curr_len])
        self.curr_len += 1

    def write_episodes(self, rec: torch.Tensor, lens=None) -> int:
        """Append a block of whole episodes, rec [E, EPISODE_STEPS, 21] (the ring's record
        layout), as E write() x 50 + flush() calls would (batched collectors,
        teacher.collect_reward); ``lens`` gives incomplete episodes' record counts.  Returns E."""
        if self.curr_len:
            raise RuntimeError("write_episodes: an episode is open; flush() first")
        rec = rec.to(self.device, torch.float32)
        if rec.dim() != 3 or rec.shape[1:] != (EPISODE_STEPS, REC):
            raise ValueError(f"rec must be [E, {EPISODE_STEPS}, {REC}], not {tuple(rec.shape)}")
        E = rec.shape[0]
        lens = [EPISODE_STEPS] * E if lens is None else [int(x) for x in lens]
        if len(lens) != E:
            raise ValueError("lens: one length per episode")
        first = max(0, E - self.capacity)   # the ring keeps the newest `capacity` of them
        self.num_total_episodes += first
        keep, kl = rec[first:], lens[first:]
        s0 = self.num_total_episodes % self.capacity
        k = min(len(kl), self.capacity - s0)   # contiguous slots s0.., then from slot 0
        self.ring[s0:s0 + k].copy_(keep[:k])
        if len(kl) > k:
            self.ring[:len(kl) - k].copy_(keep[k:])
        slots = [(s0 + q) % self.capacity for q in range(len(kl))]
        for slot, ln in zip(slots, kl):
            self.lens[slot] = ln
        new = set(slots)   # data_in_memory: the overwritten episodes leave it
        self._mem_slots = [x for x in self._mem_slots if x not in new] + slots
        self.num_total_episodes += len(kl)
        return E

    def _field(self, x, n):
        if x is None:
            return self._zeros[:n]
        if not (torch.is_tensor(x) and x.device == self.device and x.dtype == torch.float32):
            x = torch.as_tensor(x, dtype=torch.float32).to(self.device)
        return x.reshape(-1)[:n]

    def flush(self):
        """Close the current episode (reference dataset.py:146-149): it enters the ring and
        data_in_memory whatever its length (an incomplete episode keeps its record count)."""
        slot = self.num_total_episodes % self.capacity
        self.ring[slot].copy_(self.curr)
        self.lens[slot] = self.curr_len
        self._remember(slot)
        self.curr.zero_()
        self.curr_len = 0
        self.num_total_episodes += 1

    def _remember(self, slot):
        if slot in self._mem_slots and len(self._mem_slots) >= self.capacity:
            self._mem_slots.remove(slot)   # the ring overwrote that episode
        self._mem_slots.append(slot)

    def dump(self, store=None):
        """Dataset.dump (reference dataset.py:78-83): write data_in_memory (the episodes flushed
        since the last full page) to the store's current page; once a page holds MAX_CAPACITY
        episodes a new page starts and data_in_memory empties."""
        from .pages import records_to_episodes
        store = store if store is not None else self.store
        if store is None:
            raise ValueError("dump: no PageStore attached")
        slots = self._mem_slots
        eps = records_to_episodes(self.ring[slots].double().cpu().numpy(), [self.lens[i] for i in slots]) \
            if slots else []
        if not store.store(eps):
            self._mem_slots = []
            self._bptt_stale = True   # the reference's data_in_memory (and the BPTT pool aliasing it) emptied

    def load_page(self, path: str) -> int:
        """Append a page's episodes (incomplete ones with their length) to the ring and to
        data_in_memory (oldest overwritten); returns how many."""
        from .pages import episodes_to_records, read_page
        rec, lens = episodes_to_records(read_page(path), with_lengths=True)
        rec = torch.as_tensor(rec, dtype=torch.float32)
        for ep, ln in zip(rec, lens):
            slot = self.num_total_episodes % self.capacity
            self.ring[slot].copy_(ep.to(self.device))
            self.lens[slot] = int(ln)
            self._remember(slot)
            self.num_total_episodes += 1
        return rec.shape[0]

    def stored(self) -> int:
        return min(self.num_total_episodes, self.capacity)

    # -- the training pool (reference training_data, dataset.py:164-182) -----------------
    PAGE_CACHE = 15   # pages kept on the device: max(POOL_PAGES, BPTT_POOL_PAGES), least recently used evicted

    def _page_records(self, page):
        if page in self._page_cache:
            self._page_cache.move_to_end(page)
        else:
            from .pages import episodes_to_records
            rec, lens = episodes_to_records(self.store.load(page), with_lengths=True)
            self._page_cache[page] = (torch.as_tensor(rec, dtype=torch.float32).to(self.device), list(map(int, lens)))
            while len(self._page_cache) > self.PAGE_CACHE:
                self._page_cache.popitem(last=False)
        return self._page_cache[page]

    def reset_training_data(self):
        """training_data = data_in_memory[:] + the episodes of up to 10 random stored pages
        other than the current one (reference dataset.py:164-177)."""
        slots = list(self._mem_slots)
        parts = [self.ring[torch.tensor(slots, dtype=torch.long, device=self.device)]] if slots else []
        lens = [self.lens[i] for i in slots]
        self.pool_pages = []
        if self.store is not None and self.store.pages:
            for page in self.store.rand_pages(self.POOL_PAGES):
                if page and page != self.store.curr_page:
                    rec, ln = self._page_records(page)
                    parts.append(rec)
                    lens += ln
                    self.pool_pages.append(page)
        self._pool = torch.cat(parts) if parts else self.ring[:0].clone()
        self._pool_lens = torch.tensor(lens, dtype=torch.long)

    def pool_size(self) -> int:
        return 0 if self._pool is None else int(self._pool.shape[0])

    def _prev(self, rec: torch.Tensor) -> torch.Tensor:
        """prev pdflat / prev reward of each record: the previous record's t and rew."""
        prev = torch.zeros(*rec.shape[:-1], PDFLAT_SHAPE + 1, dtype=rec.dtype, device=rec.device)
        prev[..., 1:, :PDFLAT_SHAPE] = rec[..., :-1, F_T:F_S]
        prev[..., 1:, PDFLAT_SHAPE] = rec[..., :-1, F_REW]
        return prev

    def training_batches(self):
        if self.pool_mode == "ring":
            n = self.stored()
            src, lens = self.ring, torch.tensor(self.lens[:n], dtype=torch.long)
        else:
            if self.curr_len % self.POOL_REFRESH == 0 or not self.pool_size():
                self.reset_training_data()
            n = self.pool_size()
            src, lens = self._pool, self._pool_lens
        if n == 0:
            return
        steps = torch.arange(self.T)
        for _ in range(self.epochs):
            eps = torch.randint(0, n, (self.B,), generator=self._gen)
            start = int(torch.randint(0, EPISODE_STEPS - self.T + 1, (1,), generator=self._gen))
            short = lens[eps] < start + self.T
            if bool(short.any()):   # the reference's episode[i] past an incomplete episode's end
                k = int(eps[short][0])
                raise IndexError(f"training window [{start}, {start + self.T}) past the end of an episode of "
                                 f"{int(lens[k])} records (flushed incomplete)")
            # ONE gather of the window's records and of their predecessors (the prev fields):
            # flat record rows [2, T, B] of the source, built on the host, one copy to the device
            row = (eps * EPISODE_STEPS)[None, :] + (start + steps)[:, None]          # [T, B]
            idx = torch.stack((row, (row - 1).clamp_min(0))).to(self.device)
            g = src.reshape(-1, REC)[idx]                                          # [2, T, B, REC]
            prev_t, prev_r = g[1, ..., F_T:F_S], g[1, ..., F_REW:F_REW + 1]
            if start == 0:   # the first record of an episode has no predecessor: zeros
                prev_t, prev_r = prev_t.clone(), prev_r.clone()
                prev_t[0] = 0.0
                prev_r[0] = 0.0
            yield (g[0, ..., F_OB:F_REW].contiguous(), g[0, ..., F_T:F_S].contiguous(),
                   prev_t.contiguous(), prev_r.contiguous())

    BPTT_POOL_PAGES = 15   # backup/dataset_bbpt.py:173: dstore.rand_pages(15)

    def bptt_batches(self):
        """The truncated-BPTT variant's windows (reference backup/dataset_bbpt.py:179-193):
        LSTM_BATCH_SIZE episodes drawn with replacement once, then every start i in
        [0, EPISODE_STEPS - T) in order -- consecutive windows slide by ONE step, and the
        driver carries the LSTM state from one window to the next (backup/lstm_bbpt.py:
        141-158).  Same tuple layout as training_batches().  Pool (dataset_bbpt.py:164-181):
        training_data IS data_in_memory there (the same list), so episodes flushed since are
        drawn at once; the episodes of up to 15 random stored pages join it on the first call and
        after every dump that emptied data_in_memory, and stay until the next such dump (the
        borrowed episodes are then part of data_in_memory, so it is no longer empty).  (The
        alias also makes its next dump write the borrowed episodes into the current page again;
        that duplication is not reproduced.)"""
        if self.pool_mode == "ring":
            n = self.stored()
            src, lens = self.ring[:n], list(self.lens[:n])
        else:
            if self._bptt_pages is None or (self._bptt_stale and not self._mem_slots):
                self._bptt_stale = False
                self._bptt_pages = []
                if self.store is not None and self.store.pages:
                    self._bptt_pages = [p for p in self.store.rand_pages(self.BPTT_POOL_PAGES)
                                        if p and p != self.store.curr_page]
            slots = list(self._mem_slots)
            parts = [self.ring[torch.tensor(slots, dtype=torch.long, device=self.device)]] if slots else []
            lens = [self.lens[i] for i in slots]
            for page in self._bptt_pages:
                rec, ln = self._page_records(page)
                parts.append(rec)
                lens += ln
            src = torch.cat(parts) if parts else self.ring[:0]
            n = int(src.shape[0])
        if n == 0:
            return
        eps = torch.randint(0, n, (self.B,), generator=self._gen)
        if any(lens[int(e)] < EPISODE_STEPS - 1 for e in eps):
            raise IndexError("BPTT windows run to step 49: an episode flushed incomplete was drawn")
        rec = src[eps.to(self.device)]                                  # [B, 50, REC]
        prev = self._prev(rec)
        for start in range(EPISODE_STEPS - self.T):
            win = rec[:, start:start + self.T].transpose(0, 1)
            p = prev[:, start:start + self.T].transpose(0, 1)
            yield (win[..., F_OB:F_REW].contiguous(), win[..., F_T:F_S].contiguous(),
                   p[..., :PDFLAT_SHAPE].contiguous(), p[..., PDFLAT_SHAPE:].contiguous())

    def current_prev(self):
        """(prev_pdflat [4], prev_rew [1]) of the record about to be written: the open
        episode's last teacher pdflat and reward, zeros at t = 0 (reference dataset.py:
        pdflat_at / rew_at of last_step(), as prev_pdflat_batch_array/prev_rew_batch_array
        put them in the test batch's last row, :250-288)."""
        if self.curr_len == 0:
            return (torch.zeros(PDFLAT_SHAPE, device=self.device), torch.zeros(1, device=self.device))
        r = self.curr[self.curr_len - 1]
        return r[F_T:F_S].clone(), r[F_REW:F_REW + 1].clone()

    def test_windows(self, ob):
        """(ob [T,B,11], prev_pdflat [T,B,4], prev_rew [T,B,1]) for the LSTM student's query:
        column B-1 holds the current episode's last T-1 records and the current step (zero-
        padded at the front), each with its prev fields; other columns are zero.  This is the
        reference's intended test batch (dataset.py:205-288 with the per-step "prev" series its
        commented-out lines build): as committed, prev_pdflat_batch_array holds a single
        element that only broadcasts when the episode has 0 or >= T-1 records."""
        ob_w = self.test_batch(ob)
        prev_w = torch.zeros(self.T, self.B, PDFLAT_SHAPE, device=self.device)
        prew_w = torch.zeros(self.T, self.B, 1, device=self.device)
        n = self.curr_len
        k = min(n, self.T - 1)
        if n > 0:
            rec = self.curr[:n]
            prev_all = self._prev(rec)                               # [n, 5] prev fields of the records
            if k > 0:
                prev_w[self.T - 1 - k:self.T - 1, self.B - 1] = prev_all[n - k:, :PDFLAT_SHAPE]
                prew_w[self.T - 1 - k:self.T - 1, self.B - 1] = prev_all[n - k:, PDFLAT_SHAPE:]
            cp, cr = self.current_prev()
            prev_w[self.T - 1, self.B - 1] = cp
            prew_w[self.T - 1, self.B - 1] = cr
        return ob_w, prev_w, prew_w

    def test_batch(self, ob):
        """[T, B, 11]: batch column B-1 holds the window of the current episode ending at
        `ob` (its last T-1 observations, zero-padded at the front); the other columns are zero,
        as in the reference's ob_batch_test_array (dataset.py:219-240)."""
        ob = torch.as_tensor(ob, dtype=torch.float32).reshape(-1)[:OBSPACE_SHAPE].to(self.device)
        out = torch.zeros(self.T, self.B, OBSPACE_SHAPE, device=self.device)
        k = min(self.curr_len, self.T - 1)
        if k > 0:
            out[self.T - 1 - k:self.T - 1, self.B - 1] = self.curr[self.curr_len - k:self.curr_len, F_OB:F_REW]
        out[self.T - 1, self.B - 1] = ob
        return out

"""Device-resident rollout -> distill buffer: the hand-off the reference's ``Dataset`` provides
(reference dataset.py:72-296), kept in HBM instead of lists of Python dicts.

Mirrored interface (reference dataset.py): ``write(ob, reward, t_pdflat, s_pdflat,
stepped_with)`` appends one step record of the current episode (:118-143, including the
``prev``/``prew`` fields = the previous record's teacher pdflat and reward, zeros at t = 0,
:132-133,152-163); ``flush()`` closes the episode (:146-149); ``num_episodes()``;
``training_batches()`` yields TRAINING_EPOCHS random windows -- LSTM_BATCH_SIZE episodes
drawn with replacement, one common start in [0, EPISODE_STEPS - STEPS_UNROLLED] -- as
``(ob [T,B,11], t_pdflat [T,B,4], prev_pdflat [T,B,4], prev_rew [T,B,1])`` (:179-202);
``test_batch(ob)`` builds the [T,B,11] window ending at the current observation (:205-235);
``dump(store)`` / ``load_page(path)`` move episodes to / from pages in the reference's
on-disk format (``pages.PageStore``, :14-65,72-96).

Storage: one ring of ``capacity`` complete episodes x EPISODE_STEPS records x 21 floats
(ob 11 | rew 1 | t 4 | s 4 | with 1) plus the open episode, all on ``device``.  The
reference's gzip-JSON pages on disk (DatasetStore, :14-65) are out of scope here
(DESIGN.md §7); the ring replaces its paging.
"""
from __future__ import annotations

import torch

from .config import (EPISODE_STEPS, LSTM_BATCH_SIZE, OBSPACE_SHAPE, PDFLAT_SHAPE, STEPS_UNROLLED,
                     TRAINING_EPOCHS)

F_OB, F_REW, F_T, F_S, F_WITH = 0, OBSPACE_SHAPE, OBSPACE_SHAPE + 1, OBSPACE_SHAPE + 1 + PDFLAT_SHAPE, \
    OBSPACE_SHAPE + 1 + 2 * PDFLAT_SHAPE
REC = F_WITH + 1   # 21 floats per step record


class DeviceDataset:
    def __init__(self, capacity: int = 5000, device="cuda:0", seed: int = 0, batch_size: int = LSTM_BATCH_SIZE,
                 steps_unrolled: int = STEPS_UNROLLED, epochs: int = TRAINING_EPOCHS):
        self.device = torch.device(device)
        self.capacity = int(capacity)
        self.ring = torch.zeros(self.capacity, EPISODE_STEPS, REC, dtype=torch.float32, device=self.device)
        self.curr = torch.zeros(EPISODE_STEPS, REC, dtype=torch.float32, device=self.device)
        self.curr_len = 0
        self.num_total_episodes = 0
        self.B, self.T, self.epochs = int(batch_size), int(steps_unrolled), int(epochs)
        self._gen = torch.Generator().manual_seed(int(seed))   # host RNG: indices only
        self._mem_slots = []   # ring slots flushed since the last full page (reference data_in_memory)
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

    def _field(self, x, n):
        if x is None:
            return self._zeros[:n]
        if not (torch.is_tensor(x) and x.device == self.device and x.dtype == torch.float32):
            x = torch.as_tensor(x, dtype=torch.float32).to(self.device)
        return x.reshape(-1)[:n]

    def flush(self):
        """Close the current episode.  Only complete episodes (EPISODE_STEPS records) enter
        the ring: the windows of training_batches() span any start in [0, 40]."""
        if self.curr_len == EPISODE_STEPS:
            self.ring[self.num_total_episodes % self.capacity].copy_(self.curr)
            self._mem_slots.append(self.num_total_episodes % self.capacity)
        self.curr.zero_()
        self.curr_len = 0
        self.num_total_episodes += 1

    def dump(self, store):
        """Dataset.dump (reference dataset.py:78-83): write the episodes flushed since the last
        full page to the store's current page (a new page starts once MAX_CAPACITY are in)."""
        from .pages import records_to_episodes
        eps = records_to_episodes(self.ring[self._mem_slots].double().cpu().numpy()) if self._mem_slots else []
        if not store.store(eps):
            self._mem_slots = []

    def load_page(self, path: str) -> int:
        """Append a page's complete episodes to the ring (oldest overwritten); returns how many."""
        from .pages import episodes_to_records, read_page
        rec = torch.as_tensor(episodes_to_records(read_page(path)), dtype=torch.float32)
        for ep in rec:
            self.ring[self.num_total_episodes % self.capacity].copy_(ep.to(self.device))
            self.num_total_episodes += 1
        return rec.shape[0]

    def stored(self) -> int:
        return min(self.num_total_episodes, self.capacity)

    def _prev(self, rec: torch.Tensor) -> torch.Tensor:
        """prev pdflat / prev reward of each record: the previous record's t and rew."""
        prev = torch.zeros(*rec.shape[:-1], PDFLAT_SHAPE + 1, dtype=rec.dtype, device=rec.device)
        prev[..., 1:, :PDFLAT_SHAPE] = rec[..., :-1, F_T:F_S]
        prev[..., 1:, PDFLAT_SHAPE] = rec[..., :-1, F_REW]
        return prev

    def training_batches(self):
        n = self.stored()
        if n == 0:
            return
        steps = torch.arange(self.T)
        for _ in range(self.epochs):
            eps = torch.randint(0, n, (self.B,), generator=self._gen)
            start = int(torch.randint(0, EPISODE_STEPS - self.T + 1, (1,), generator=self._gen))
            # ONE gather of the window's records and of their predecessors (the prev fields):
            # flat record rows [2, T, B] of the ring, built on the host, one copy to the device
            row = (eps * EPISODE_STEPS)[None, :] + (start + steps)[:, None]          # [T, B]
            idx = torch.stack((row, (row - 1).clamp_min(0))).to(self.device)
            g = self.ring.view(-1, REC)[idx]                                       # [2, T, B, REC]
            prev_t, prev_r = g[1, ..., F_T:F_S], g[1, ..., F_REW:F_REW + 1]
            if start == 0:   # the first record of an episode has no predecessor: zeros
                prev_t, prev_r = prev_t.clone(), prev_r.clone()
                prev_t[0] = 0.0
                prev_r[0] = 0.0
            yield (g[0, ..., F_OB:F_REW].contiguous(), g[0, ..., F_T:F_S].contiguous(),
                   prev_t.contiguous(), prev_r.contiguous())

    def bptt_batches(self):
        """The truncated-BPTT variant's windows (reference backup/dataset_bbpt.py:179-193):
        LSTM_BATCH_SIZE episodes drawn with replacement once, then every start i in
        [0, EPISODE_STEPS - T) in order -- consecutive windows slide by ONE step, and the
        driver carries the LSTM state from one window to the next (backup/lstm_bbpt.py:
        141-158).  Same tuple layout as training_batches()."""
        n = self.stored()
        if n == 0:
            return
        eps = torch.randint(0, n, (self.B,), generator=self._gen)
        rec = self.ring[eps.to(self.device)]                          # [B, 50, REC]
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

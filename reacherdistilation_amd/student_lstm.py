"""Host layer of the reference's LSTM student (include/reacher_student_lstm.h).

``StudentLstmTrainer`` is the 'LSTM' scope of the reference's lstm_train.py (:35-79): the
graph ``student_lstm_graph`` (student_nn.py:21-49: dense prev-pdflat embedding, TF1
LSTMCell(200), a 200-64-128-64-32-4 head per unrolled step), ``kl_loss`` (loss.py:3-13) and TF1 Adam, run by
csrc/student_lstm.hip.  Tensors are the reference's window layout: ob [T, B, 11],
prev_pdflat [T, B, 4], t_pdflat / pdflat [T, B, 4], state [2, B, 200] = (c, m).

Multi-GPU: windows sharded contiguously (row_base = first global window), one
all_reduce(SUM) of the flat gradient (511,880 floats at T = 10: the shared cell and one
head per unrolled step) per optimiser step.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .config import LSTM_BATCH_SIZE, NUM_UNITS, OBSPACE_SHAPE, PDFLAT_SHAPE, STEPS_UNROLLED
from .dist import allreduce_sum_

P = nat.P
I32, I64, U64, F32, INT = nat.I32, nat.I64, nat.U64, nat.F32, nat.INT

HEAD = (NUM_UNITS, 64, 128, 64, 32, 4)
CELL_SHAPES = [("Wp", (4, 32)), ("bp", (32,)), ("Wl", (OBSPACE_SHAPE + 32 + NUM_UNITS, 4 * NUM_UNITS)),
               ("bl", (4 * NUM_UNITS,))]
HEAD_SHAPES = [x for k, (a, b) in enumerate(zip(HEAD[:-1], HEAD[1:]))
               for x in ((f"W{k + 1}", (a, b)), (f"b{k + 1}", (b,)))]


def shapes(T: int = STEPS_UNROLLED):
    """The flat layout in variable-creation order: the shared prev-pdflat dense and LSTMCell, then
    one head per unrolled step (the reference's tf.layers.dense calls inside its loop over the T
    steps create new variables at every step, student_nn.py:40-47; TF names dense_1..dense_5T)."""
    return CELL_SHAPES + [(f"h{t}/{n}", s) for t in range(T) for n, s in HEAD_SHAPES]


def n_params(T: int = STEPS_UNROLLED) -> int:
    return sum(int(np.prod(s)) for _, s in shapes(T))


N_PARAMS = n_params(STEPS_UNROLLED)   # 511,880 at the reference's T = 10
LOSSES = {"mse": 0, "kl": 1}


class RdlConfig(ctypes.Structure):
    _fields_ = [("loss", I32), ("lr", F32), ("beta1", F32), ("beta2", F32), ("eps", F32), ("steps", I32),
                ("max_windows", I32), ("metrics_len", I32), ("keep_prob", F32), ("seed", U64), ("row_base", I64),
                ("kernels", I32)]


nat.register({
    "rdl_param_count": (I64, [I32]),
    "rdl_create": (INT, [ctypes.POINTER(P), ctypes.POINTER(RdlConfig), INT, P]),
    "rdl_destroy": (INT, [P]),
    "rdl_set_stream": (INT, [P, P]),
    "rdl_set_params": (INT, [P, P]),
    "rdl_get_params": (INT, [P, P]),
    "rdl_reset": (INT, [P]),
    "rdl_forward": (INT, [P, P, P, P, I64, P, P]),
    "rdl_rollout": (INT, [P, P, P, P, P, I64, I64]),
    "rdl_apply": (INT, [P]),
    "rdl_step": (INT, [P, P, P, P, P, I64]),
    "rdl_grad_buffer": (P, [P]),
    "rdl_bind_grad_buffer": (INT, [P, P]),
    "rdl_get_counter": (INT, [P, ctypes.POINTER(I64)]),
    "rdl_read_metrics": (INT, [P, I64, P]),
    "rdl_final_state": (INT, [P, I64, P]),
    "rdl_get_slots": (INT, [P, P, P]),
    "rdl_set_slots": (INT, [P, P, P]),
    "rdl_head_path": (INT, [P]),
})


def glorot_init(seed: int = 3, T: int = STEPS_UNROLLED) -> np.ndarray:
    """glorot_uniform kernels (tf.layers.dense and LSTMCell defaults), zero biases."""
    rng = np.random.RandomState(seed)
    out = []
    for _, s in shapes(T):
        if len(s) == 2:
            lim = math.sqrt(6.0 / (s[0] + s[1]))
            out.append(rng.uniform(-lim, lim, s[0] * s[1]).astype(np.float32))
        else:
            out.append(np.zeros(s, np.float32))
    return np.concatenate(out)


@dataclass
class StudentLstmConfig:
    loss: str = "kl"                  # lstm_train.py:71
    lr: float = 1e-3                  # lstm_train.py:74
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    steps: int = STEPS_UNROLLED       # T
    max_windows: int = LSTM_BATCH_SIZE
    keep_prob: float = 1.0            # reference trains with KEEP_PROB = 0.5
    seed: int = 0
    init_seed: int = 3
    metrics_len: int = 4096
    step_recurrence: bool = False     # force the per-step recurrence launches (else: persistent at <= 32 windows)
    layer_head: bool = False          # force the per-layer head GEMMs (else: one launch at <= 16,384 rows)


class StudentLstmTrainer:
    def __init__(self, cfg: StudentLstmConfig | None = None, device="cuda:0", rank: int = 0, world_size: int = 1,
                 process_group=None, params=None, row_base: int = 0):
        self.cfg = cfg or StudentLstmConfig()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("StudentLstmTrainer runs on a GPU (HIP) device only; there is no CPU path")
        self.rank, self.world, self.pg = rank, world_size, process_group
        self.T = int(self.cfg.steps)
        self._lib = nat.load()
        self.n_params = n_params(self.T)
        assert self._lib.rdl_param_count(self.T) == self.n_params
        c = RdlConfig(loss=LOSSES[self.cfg.loss], lr=self.cfg.lr, beta1=self.cfg.beta1, beta2=self.cfg.beta2,
                      eps=self.cfg.eps, steps=self.T, max_windows=int(self.cfg.max_windows),
                      metrics_len=self.cfg.metrics_len, keep_prob=self.cfg.keep_prob,
                      seed=self.cfg.seed % 2 ** 64, row_base=int(row_base),
                      kernels=int(bool(self.cfg.step_recurrence)) | 2 * int(bool(self.cfg.layer_head)))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self._lib.rdl_create(ctypes.byref(h), ctypes.byref(c), self.device.index or 0,
                                           nat.stream_handle(self.device)), "rdl_create")
        self._h = h
        self._grad = torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        nat.check(self._lib.rdl_bind_grad_buffer(self._h, nat.ptr(self._grad)), "rdl_bind_grad_buffer")
        self.set_params(glorot_init(self.cfg.init_seed, self.T) if params is None else params)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rdl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync_stream(self):
        nat.check(self._lib.rdl_set_stream(self._h, nat.stream_handle(self.device)), "rdl_set_stream")

    # -- parameters ------------------------------------------------------------------
    def set_params(self, params):
        p = (params if torch.is_tensor(params) else torch.from_numpy(np.asarray(params, np.float32)))
        p = p.to(self.device, torch.float32).reshape(-1).contiguous()
        if p.numel() != self.n_params:
            raise ValueError(f"expected {self.n_params} parameters, got {p.numel()}")
        self._sync_stream()
        nat.check(self._lib.rdl_set_params(self._h, nat.ptr(p)), "rdl_set_params")
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def fused_head(self) -> bool:
        """True if batches of at most 16,384 rows run the fused head kernels (rdl_head_path)."""
        r = self._lib.rdl_head_path(self._h)
        if r < 0:
            nat.check(r, "rdl_head_path")
        return r == 1

    def params(self) -> torch.Tensor:
        out = torch.empty(self.n_params, dtype=torch.float32, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdl_get_params(self._h, nat.ptr(out)), "rdl_get_params")
        return out

    def _slots(self):
        m = torch.empty(self.n_params, dtype=torch.float32, device=self.device)
        v = torch.empty_like(m)
        self._sync_stream()
        nat.check(self._lib.rdl_get_slots(self._h, nat.ptr(m), nat.ptr(v)), "rdl_get_slots")
        torch.cuda.current_stream(self.device).synchronize()
        return m, v

    def save(self, path: str):
        """tf.train.Saver(var_list=LSTM/*).save (reference lstm_train.py:86-87,199): the
        parameters and the Adam slots m, v.  A path ending in '.safetensors' is written as one
        safetensors file; any other path is a TF checkpoint prefix (``path.index`` +
        ``path.data-00000-of-00001``, the reference's own format and variable names,
        tf_checkpoint.save_lstm).  Nothing executable either way."""
        m, v = self._slots()
        p = self.params()
        if path.endswith(".safetensors"):
            from safetensors.torch import save_file
            save_file({"params": p.cpu(), "adam_m": m.cpu(), "adam_v": v.cpu()}, path)
        else:
            from . import tf_checkpoint
            tf_checkpoint.save_lstm(path, p.cpu().numpy(), m.cpu().numpy(), v.cpu().numpy(), self.T)

    @staticmethod
    def checkpoint_exists(path: str) -> bool:
        from . import tf_checkpoint
        return os.path.exists(path) if path.endswith(".safetensors") else tf_checkpoint.exists(path)

    def load(self, path: str):
        """saver.restore (reference lstm_train.py:102-107): parameters and Adam slots from
        `path` (format by suffix, as save); the beta powers and step counter start afresh, as
        the reference initialises the Adam variables before restoring the 'LSTM' scope
        (:99-105).  A TF checkpoint without Adam slots restores the parameters and zero slots."""
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file
            d = load_file(path)
            p, m, v = d["params"], d["adam_m"], d["adam_v"]
        else:
            from . import tf_checkpoint
            p, m, v = tf_checkpoint.load_lstm(path, self.T)
            p = torch.from_numpy(p)
            m = torch.zeros_like(p) if m is None else torch.from_numpy(m)
            v = torch.zeros_like(p) if v is None else torch.from_numpy(v)
        if p.numel() != self.n_params:
            raise ValueError(f"{path}: {p.numel()} parameters, expected {self.n_params}")
        self.reset_optimizer()
        self.set_params(p)
        m = m.to(self.device, torch.float32).contiguous()
        v = v.to(self.device, torch.float32).contiguous()
        self._sync_stream()
        nat.check(self._lib.rdl_set_slots(self._h, nat.ptr(m), nat.ptr(v)), "rdl_set_slots")
        torch.cuda.current_stream(self.device).synchronize()

    def reset_optimizer(self):
        self._sync_stream()
        nat.check(self._lib.rdl_reset(self._h), "rdl_reset")

    # -- compute -----------------------------------------------------------------------
    def _t(self, x, last):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.device).contiguous()
        if x.dim() != 3 or x.shape[0] != self.T or x.shape[2] != last:
            raise ValueError(f"expected [T={self.T}, B, {last}], got {tuple(x.shape)}")
        return x

    def _windows(self, ob, prev, tgt=None, state0=None):
        ob, prev = self._t(ob, OBSPACE_SHAPE), self._t(prev, PDFLAT_SHAPE)
        B = ob.shape[1]
        if B == 0 or prev.shape[1] != B or B > self.cfg.max_windows:
            raise ValueError(f"bad window count {B} (max_windows {self.cfg.max_windows})")
        if tgt is not None:
            tgt = self._t(tgt, PDFLAT_SHAPE)
            if tgt.shape[1] != B:
                raise ValueError("t_pdflat window count differs")
        if state0 is not None:
            state0 = torch.as_tensor(state0, dtype=torch.float32, device=self.device).contiguous()
            if tuple(state0.shape) != (2, B, NUM_UNITS):
                raise ValueError(f"state must be [2, {B}, {NUM_UNITS}]")
        return ob, prev, tgt, state0, B

    def forward(self, ob, prev_pdflat, state0=None):
        """(pdflat [T, B, 4], final state [2, B, 200]) with dropout off (lstm_train.py:171-183)."""
        ob, prev, _, st, B = self._windows(ob, prev_pdflat, None, state0)
        out = torch.empty(self.T, B, PDFLAT_SHAPE, dtype=torch.float32, device=self.device)
        fin = torch.empty(2, B, NUM_UNITS, dtype=torch.float32, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdl_forward(self._h, nat.ptr(ob), nat.ptr(prev), nat.ptr(st) if st is not None else None,
                                        B, nat.ptr(out), nat.ptr(fin)), "rdl_forward")
        return out, fin

    def rollout(self, ob, prev_pdflat, t_pdflat, state0=None, windows_global: int | None = None):
        ob, prev, tgt, st, B = self._windows(ob, prev_pdflat, t_pdflat, state0)
        self._sync_stream()
        nat.check(self._lib.rdl_rollout(self._h, nat.ptr(ob), nat.ptr(prev), nat.ptr(tgt),
                                        nat.ptr(st) if st is not None else None, B, int(windows_global or B)),
                  "rdl_rollout")
        self._keep = (ob, prev, tgt, st)
        return self._grad

    def apply(self):
        self._sync_stream()
        nat.check(self._lib.rdl_apply(self._h), "rdl_apply")

    def step(self, ob, prev_pdflat, t_pdflat, state0=None, windows_global: int | None = None):
        """sess.run([loss, minimize_adam]) (lstm_train.py:145-160)."""
        if self.world == 1:
            ob, prev, tgt, st, B = self._windows(ob, prev_pdflat, t_pdflat, state0)
            self._sync_stream()
            nat.check(self._lib.rdl_step(self._h, nat.ptr(ob), nat.ptr(prev), nat.ptr(tgt),
                                         nat.ptr(st) if st is not None else None, B), "rdl_step")
            self._keep = (ob, prev, tgt, st)
            return
        self.rollout(ob, prev_pdflat, t_pdflat, state0, windows_global)
        allreduce_sum_(self._grad, self.pg)
        self.apply()

    def graph_step(self, windows: int):
        """One training step (rdl_step, zero initial state) for `windows` windows captured
        into a HIP graph: returns step(ob, prev_pdflat, t_pdflat), which copies the inputs
        into the graph's static buffers and replays (no host launches; the reference's
        20-window step is launch-bound).  Replays are the same computation as step()."""
        if self.world != 1:
            raise RuntimeError("graph capture is for the single-rank step")
        T, B = self.T, int(windows)
        if not 0 < B <= self.cfg.max_windows:
            raise ValueError(f"bad window count {B}")
        ob = torch.zeros(T, B, OBSPACE_SHAPE, device=self.device)
        prev = torch.zeros(T, B, PDFLAT_SHAPE, device=self.device)
        tgt = torch.zeros(T, B, PDFLAT_SHAPE, device=self.device)
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        with torch.cuda.graph(g):
            self._sync_stream()
            nat.check(self._lib.rdl_step(self._h, nat.ptr(ob), nat.ptr(prev), nat.ptr(tgt), None, B), "rdl_step")
        self._sync_stream()

        def step(o, p, t):
            ob.copy_(torch.as_tensor(o, dtype=torch.float32).reshape(ob.shape))
            prev.copy_(torch.as_tensor(p, dtype=torch.float32).reshape(prev.shape))
            tgt.copy_(torch.as_tensor(t, dtype=torch.float32).reshape(tgt.shape))
            g.replay()

        step.graph, step.inputs = g, (ob, prev, tgt)
        return step

    def final_state(self, windows: int) -> torch.Tensor:
        """final_state_batch [2, B, 200] = (c, h) of the last forward pass over `windows`
        windows (rollout/step: computed with the parameters before that step's update, as
        the reference's sess.run([loss, final_state_batch, minimize_adam]) returns it,
        backup/lstm_bbpt.py:147-155)."""
        out = torch.empty(2, int(windows), NUM_UNITS, dtype=torch.float32, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdl_final_state(self._h, int(windows), nat.ptr(out)), "rdl_final_state")
        return out

    def grad(self) -> torch.Tensor:
        return self._grad

    def counter(self) -> int:
        v = ctypes.c_int64()
        nat.check(self._lib.rdl_get_counter(self._h, ctypes.byref(v)), "rdl_get_counter")
        return v.value

    def metrics(self, count: int = 1) -> np.ndarray:
        """[count, 4]: loss, sum |mu_s - mu_t|^2, rows (T x B), 0."""
        out = np.zeros((count, 4), np.float64)
        nat.check(self._lib.rdl_read_metrics(self._h, count, out.ctypes.data_as(ctypes.c_void_p)),
                  "rdl_read_metrics")
        return out

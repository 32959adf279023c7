"""Host layer of the reference's own MLP student (include/reacher_student_mlp.h).

``StudentMlpTrainer`` is the 'MLP' scope of the reference's mlp_train.py (:35-80): the
graph ``student_mlp_graph`` (student_nn.py:51-57, 16 -> 24 -> 128 -> 128 -> 32 -> 4 with a
state-dependent log-std), ``kl_loss`` (loss.py:3-13) or action-MSE, and TF1 Adam, run by the
HIP kernels in csrc/student_mlp.hip.  ``rows()`` is the input concat of mlp_train.py:50-52
(dropout(ob) | prev_pdflat | prev_rew; the dropout itself runs inside the kernel).

Multi-GPU: rows sharded contiguously (dist.shard); one all_reduce(SUM) of the flat
24,380-float gradient per optimiser step.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .config import OBSPACE_SHAPE, PDFLAT_SHAPE
from .dist import allreduce_sum_

P = nat.P
I32, I64, U64, F32, INT = nat.I32, nat.I64, nat.U64, nat.F32, nat.INT

DIMS = (16, 24, 128, 128, 32, 4)          # student_nn.py:51-57
N_PARAMS = sum(a * b + b for a, b in zip(DIMS[:-1], DIMS[1:]))   # 24,380
IN_DIM = OBSPACE_SHAPE + PDFLAT_SHAPE + 1
LOSSES = {"mse": 0, "kl": 1}


class RdmConfig(ctypes.Structure):
    _fields_ = [("loss", I32), ("lr", F32), ("beta1", F32), ("beta2", F32), ("eps", F32), ("grid", I32),
                ("metrics_len", I32), ("keep_prob", F32), ("seed", U64), ("row_base", I64)]


nat.register({
    "rdm_param_count": (INT, []),
    "rdm_create": (INT, [ctypes.POINTER(P), ctypes.POINTER(RdmConfig), INT, P]),
    "rdm_destroy": (INT, [P]),
    "rdm_set_stream": (INT, [P, P]),
    "rdm_set_params": (INT, [P, P]),
    "rdm_get_params": (INT, [P, P]),
    "rdm_reset": (INT, [P]),
    "rdm_forward": (INT, [P, P, I64, P]),
    "rdm_rollout": (INT, [P, P, P, I64, I64]),
    "rdm_apply": (INT, [P]),
    "rdm_step": (INT, [P, P, P, I64]),
    "rdm_grad_buffer": (P, [P]),
    "rdm_bind_grad_buffer": (INT, [P, P]),
    "rdm_get_counter": (INT, [P, ctypes.POINTER(I64)]),
    "rdm_read_metrics": (INT, [P, I64, P]),
})


def glorot_init(seed: int = 2) -> np.ndarray:
    """tf.layers.dense defaults: glorot_uniform kernels, zero biases (flat f32 [24,380])."""
    rng = np.random.RandomState(seed)
    out = []
    for a, b in zip(DIMS[:-1], DIMS[1:]):
        lim = math.sqrt(6.0 / (a + b))
        out.append(rng.uniform(-lim, lim, a * b).astype(np.float32))
        out.append(np.zeros(b, np.float32))
    return np.concatenate(out)


def rows(ob, prev_pdflat, prev_rew) -> torch.Tensor:
    """[..., 11] | [..., 4] | [..., 1] -> contiguous [n, 16] rows (mlp_train.py:52)."""
    x = torch.cat([ob, prev_pdflat, prev_rew], dim=-1).to(torch.float32)
    return x.reshape(-1, IN_DIM).contiguous()


@dataclass
class StudentMlpConfig:
    loss: str = "kl"            # mlp_train.py:71 (kl_loss); "mse" = action-MSE
    lr: float = 1e-4            # mlp_train.py:75-78
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    keep_prob: float = 1.0      # reference trains with KEEP_PROB = 0.5 (config.py:30)
    seed: int = 0               # dropout key
    init_seed: int = 2
    grid: int = 0
    metrics_len: int = 4096


class StudentMlpTrainer:
    def __init__(self, cfg: StudentMlpConfig | None = None, device="cuda:0", rank: int = 0, world_size: int = 1,
                 process_group=None, params=None, row_base: int = 0):
        self.cfg = cfg or StudentMlpConfig()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("StudentMlpTrainer runs on a GPU (HIP) device only; there is no CPU path")
        self.rank, self.world, self.pg = rank, world_size, process_group
        self._lib = nat.load()
        assert self._lib.rdm_param_count() == N_PARAMS
        c = RdmConfig(loss=LOSSES[self.cfg.loss], lr=self.cfg.lr, beta1=self.cfg.beta1, beta2=self.cfg.beta2,
                      eps=self.cfg.eps, grid=self.cfg.grid, metrics_len=self.cfg.metrics_len,
                      keep_prob=self.cfg.keep_prob, seed=self.cfg.seed % 2 ** 64, row_base=int(row_base))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self._lib.rdm_create(ctypes.byref(h), ctypes.byref(c), self.device.index or 0,
                                           nat.stream_handle(self.device)), "rdm_create")
        self._h = h
        self._grad = torch.zeros(N_PARAMS, dtype=torch.float32, device=self.device)
        nat.check(self._lib.rdm_bind_grad_buffer(self._h, nat.ptr(self._grad)), "rdm_bind_grad_buffer")
        self.set_params(glorot_init(self.cfg.init_seed) if params is None else params)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rdm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return nat.stream_handle(self.device)

    def _sync_stream(self):
        nat.check(self._lib.rdm_set_stream(self._h, self._stream()), "rdm_set_stream")

    # -- parameters ------------------------------------------------------------------
    def set_params(self, params):
        p = torch.as_tensor(np.asarray(params, np.float32) if not torch.is_tensor(params) else params,
                            dtype=torch.float32).reshape(-1).to(self.device).contiguous()
        if p.numel() != N_PARAMS:
            raise ValueError(f"expected {N_PARAMS} parameters, got {p.numel()}")
        self._sync_stream()
        nat.check(self._lib.rdm_set_params(self._h, nat.ptr(p)), "rdm_set_params")
        torch.cuda.current_stream(self.device).synchronize()

    def params(self) -> torch.Tensor:
        out = torch.empty(N_PARAMS, dtype=torch.float32, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdm_get_params(self._h, nat.ptr(out)), "rdm_get_params")
        return out

    def reset_optimizer(self):
        self._sync_stream()
        nat.check(self._lib.rdm_reset(self._h), "rdm_reset")

    # -- compute -----------------------------------------------------------------------
    def _rows(self, x):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.device).reshape(-1, IN_DIM).contiguous()
        if x.shape[0] == 0:
            raise ValueError("empty batch")
        return x

    def forward(self, x) -> torch.Tensor:
        """s_pdflat [n, 4] of rows x [n, 16] (dropout off, as the reference's queries)."""
        x = self._rows(x)
        out = torch.empty(x.shape[0], PDFLAT_SHAPE, dtype=torch.float32, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdm_forward(self._h, nat.ptr(x), x.shape[0], nat.ptr(out)), "rdm_forward")
        return out

    def rollout(self, x, t_pdflat, n_global: int | None = None) -> torch.Tensor:
        """Gradient of this rank's rows into grad(); returns the gradient tensor."""
        x = self._rows(x)
        t = torch.as_tensor(t_pdflat, dtype=torch.float32, device=self.device).reshape(-1, PDFLAT_SHAPE).contiguous()
        if t.shape[0] != x.shape[0]:
            raise ValueError("x and t_pdflat row counts differ")
        self._sync_stream()
        nat.check(self._lib.rdm_rollout(self._h, nat.ptr(x), nat.ptr(t), x.shape[0],
                                        int(n_global or x.shape[0])), "rdm_rollout")
        self._keep = (x, t)   # kernels are asynchronous: keep the inputs alive
        return self._grad

    def apply(self):
        self._sync_stream()
        nat.check(self._lib.rdm_apply(self._h), "rdm_apply")

    def step(self, x, t_pdflat, n_global: int | None = None):
        """sess.run([loss, minimize_adam]) (mlp_train.py:145-160): one optimiser step."""
        if self.world == 1:
            x = self._rows(x)
            t = torch.as_tensor(t_pdflat, dtype=torch.float32,
                                device=self.device).reshape(-1, PDFLAT_SHAPE).contiguous()
            if t.shape[0] != x.shape[0]:
                raise ValueError("x and t_pdflat row counts differ")
            self._sync_stream()
            nat.check(self._lib.rdm_step(self._h, nat.ptr(x), nat.ptr(t), x.shape[0]), "rdm_step")
            self._keep = (x, t)
            return
        self.rollout(x, t_pdflat, n_global)
        allreduce_sum_(self._grad, self.pg)
        self.apply()

    def graph_step(self, n: int):
        """One training step (rdm_step) on n rows captured into a HIP graph: returns
        step(x, t_pdflat), which copies into the graph's static buffers and replays."""
        if self.world != 1:
            raise RuntimeError("graph capture is for the single-rank step")
        x = torch.zeros(int(n), IN_DIM, device=self.device)
        t = torch.zeros(int(n), PDFLAT_SHAPE, device=self.device)
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        with torch.cuda.graph(g):
            self._sync_stream()
            nat.check(self._lib.rdm_step(self._h, nat.ptr(x), nat.ptr(t), int(n)), "rdm_step")
        self._sync_stream()

        def step(xv, tv):
            x.copy_(torch.as_tensor(xv, dtype=torch.float32).reshape(x.shape))
            t.copy_(torch.as_tensor(tv, dtype=torch.float32).reshape(t.shape))
            g.replay()

        step.graph, step.inputs = g, (x, t)
        return step

    def grad(self) -> torch.Tensor:
        return self._grad

    def counter(self) -> int:
        v = ctypes.c_int64()
        nat.check(self._lib.rdm_get_counter(self._h, ctypes.byref(v)), "rdm_get_counter")
        return v.value

    def metrics(self, count: int = 1) -> np.ndarray:
        """[count, 4]: loss, sum |mu_s - mu_t|^2, rows, 0 of the last optimiser steps."""
        out = np.zeros((count, 4), np.float64)
        nat.check(self._lib.rdm_read_metrics(self._h, count, out.ctypes.data_as(ctypes.c_void_p)),
                  "rdm_read_metrics")
        return out

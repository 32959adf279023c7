"""Host driver of the fused rollout + distillation step (include/reacher_distill.h).

``DistillTrainer`` is the batched, device-resident form of the reference's MLP DAgger loop
(reference mlp_train.py:18-204): per step it queries the teacher, runs the student
forward/backward against the distillation loss (kl_loss, reference loss.py:3-13, or
action-MSE), takes one TF1 Adam step (mlp_train.py:73-80) and steps N Reacher-v2 envs
with the teacher mean (configs 2-4) or the student mean (DAgger, config 5).

Multi-GPU: one process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm), envs
sharded contiguously; the only exchange is one all_reduce(SUM) of the flat 5060-float
student gradient per optimiser step.  Student weights start identical on every rank
(same seed) and stay identical because every rank applies the same reduced gradient.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .dist import allreduce_sum_, replicas_identical, shard
from .policy import P_TOT, MlpPolicyParams, student_init, synthetic_teacher

P = nat.P
I32, I64, U64, F32, INT = nat.I32, nat.I64, nat.U64, nat.F32, nat.INT

LOSSES = {"mse": 0, "kl": 1}
ACTORS = {"teacher": 0, "student": 1}
DTYPES = {"f32": 0, "bf16": 1}


class RddConfig(ctypes.Structure):
    _fields_ = [("n_envs", I64), ("n_envs_global", I64), ("env_base", I64), ("seed", U64),
                ("loss", I32), ("act_with", I32), ("lr", F32), ("beta1", F32), ("beta2", F32),
                ("eps", F32), ("grid", I32), ("metrics_len", I32), ("stagger", I32),
                ("student_dtype", I32), ("accum_steps", I32), ("f32_split", I32), ("group_envs", I32)]


nat.register({
    "rdd_create": (INT, [ctypes.POINTER(P), ctypes.POINTER(RddConfig), INT, P]),
    "rdd_destroy": (INT, [P]),
    "rdd_param_count": (INT, []),
    "rdd_set_stream": (INT, [P, P]),
    "rdd_set_teacher": (INT, [P, P, P, P]),
    "rdd_set_student": (INT, [P, P, P, P]),
    "rdd_get_student": (INT, [P, P]),
    "rdd_reset": (INT, [P]),
    "rdd_rollout": (INT, [P]),
    "rdd_apply": (INT, [P]),
    "rdd_step": (INT, [P]),
    "rdd_rollout_accum": (INT, [P]),
    "rdd_step_accum": (INT, [P]),
    "rdd_launch_stage": (INT, [P, INT]),
    "rdd_grad_buffer": (P, [P]),
    "rdd_bind_grad_buffer": (INT, [P, P]),
    "rdd_forward": (INT, [P, P, I64, P, P]),
    "rdd_get_env_state": (INT, [P, P]),
    "rdd_set_env_state": (INT, [P, P]),
    "rdd_get_counter": (INT, [P, ctypes.POINTER(I64)]),
    "rdd_get_counters": (INT, [P, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
    "rdd_rollout_obs": (INT, [P, P, I64, I64]),
    "rdd_step_obs": (INT, [P, P, I64]),
    "rdd_rollout_rows": (INT, [P, P, P, I64, I64]),
    "rdd_step_rows": (INT, [P, P, P, I64]),
    "rdd_read_metrics": (INT, [P, I64, P]),
    "rdd_bind_comm": (INT, [P, P]),
    "rdd_allreduce_grad": (INT, [P]),
})


@dataclass
class DistillConfig:
    n_envs: int = 4096                 # envs on this rank (weak scaling: fixed per rank)
    n_envs_global: int = 0             # if > 0: total envs, sharded over ranks (strong scaling)
    seed: int = 0                      # Philox reset seed
    loss: str = "mse"                  # "mse" (configs 2,5) | "kl" (config 3, reference loss.py)
    act_with: str = "teacher"          # "teacher" (configs 2-4) | "student" (DAgger, config 5)
    lr: float = 1e-4                   # reference mlp_train.py:75
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    teacher_seed: int = 1
    student_seed: int = 2
    grid: int = 0
    metrics_len: int = 4096
    stagger: bool = True               # spread episode phases over the batch (reacher_distill.h)
    student_dtype: str = "f32"         # "f32" | "bf16" (BASELINE config 5: bf16 student MLP)
    accum_steps: int = 1               # env steps per optimiser step (1 = the reference)
    f32_split: bool = True             # f32 hidden layers on bf16 MFMAs via exact 3-piece splits (reacher_distill.h);
    #                                    False: every product on the f32 MFMA (same tolerances, ~20 % slower)
    group_envs: int = 0                # envs per rollout group: 0 = auto, 16 | 32 | 64 fixed (summation order only)


class DistillTrainer:
    def __init__(self, cfg: DistillConfig, device="cuda:0", rank: int = 0, world_size: int = 1,
                 process_group=None, teacher: MlpPolicyParams | None = None,
                 student: MlpPolicyParams | None = None, comm=None):
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DistillTrainer runs on a GPU (HIP) device only; there is no CPU path")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.rank, self.world = rank, world_size
        self.pg = process_group
        self._lib = nat.load()
        assert self._lib.rdd_param_count() == P_TOT
        if cfg.n_envs_global > 0:
            self.n_local, self.env_base = shard(cfg.n_envs_global, rank, world_size)
            self.n_global = cfg.n_envs_global
        else:
            self.n_local, self.env_base = cfg.n_envs, cfg.n_envs * rank
            self.n_global = cfg.n_envs * world_size
        c = RddConfig(n_envs=self.n_local, n_envs_global=self.n_global, env_base=self.env_base,
                      seed=cfg.seed % 2 ** 64, loss=LOSSES[cfg.loss], act_with=ACTORS[cfg.act_with], lr=cfg.lr,
                      beta1=cfg.beta1, beta2=cfg.beta2, eps=cfg.eps, grid=cfg.grid, metrics_len=cfg.metrics_len,
                      stagger=int(bool(cfg.stagger)), student_dtype=DTYPES[cfg.student_dtype],
                      accum_steps=max(1, int(cfg.accum_steps)), f32_split=int(bool(cfg.f32_split)),
                      group_envs=int(cfg.group_envs))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self._lib.rdd_create(ctypes.byref(h), ctypes.byref(c), self.device.index or 0,
                                           nat.stream_handle(self.device)), "rdd_create")
        self._h = h
        self.teacher = teacher or synthetic_teacher(cfg.teacher_seed)
        self.student = student or student_init(cfg.student_seed)
        self.set_teacher(self.teacher)
        self.set_student(self.student)
        self.reset()
        # the flat gradient lives in a torch tensor bound into the trainer, so the host
        # all-reduces it in place (RCCL) between rdd_rollout and rdd_apply
        self._grad = torch.zeros(P_TOT, dtype=torch.float32, device=self.device)
        nat.check(self._lib.rdd_bind_grad_buffer(self._h, nat.ptr(self._grad)), "rdd_bind_grad_buffer")
        self.steps = 0
        self._k = 0   # rollouts accumulated into the current optimiser step (accum_steps > 1)
        # an RcclComm (dist.py) makes the exchange part of the native step, on this stream
        self.comm = None
        if comm is not None:
            self.bind_comm(comm)

    def bind_comm(self, comm):
        if comm is not None:
            if comm.world != self.world or comm.rank != self.rank:
                raise ValueError(f"communicator rank {comm.rank} of {comm.world} for a trainer at rank "
                                 f"{self.rank} of {self.world}")
            if comm.device != self.device:   # RCCL would run on the wrong device's context
                raise ValueError(f"communicator on {comm.device} for a trainer on {self.device}")
        nat.check(self._lib.rdd_bind_comm(self._h, comm.handle if comm is not None else None), "rdd_bind_comm")
        self.comm = comm

    # -- parameters ------------------------------------------------------------------
    def set_teacher(self, p: MlpPolicyParams):
        f, mu, sd = p.device_tensors(self.device)
        nat.check(self._lib.rdd_set_teacher(self._h, nat.ptr(f), nat.ptr(mu), nat.ptr(sd)), "rdd_set_teacher")
        torch.cuda.current_stream(self.device).synchronize()

    def set_student(self, p: MlpPolicyParams):
        f, mu, sd = p.device_tensors(self.device)
        nat.check(self._lib.rdd_set_student(self._h, nat.ptr(f), nat.ptr(mu), nat.ptr(sd)), "rdd_set_student")
        torch.cuda.current_stream(self.device).synchronize()

    def student_params(self) -> torch.Tensor:
        out = torch.empty(P_TOT, dtype=torch.float32, device=self.device)
        nat.check(self._lib.rdd_get_student(self._h, nat.ptr(out)), "rdd_get_student")
        return out

    def reset(self):
        nat.check(self._lib.rdd_reset(self._h), "rdd_reset")
        self.steps = 0

    # -- the step ----------------------------------------------------------------------
    def step(self):
        """One env step of this rank's envs: rollout + distill.  With accum_steps = K the
        gradients of K consecutive env steps are summed and one (all-reduce +) Adam step is
        taken every K-th call."""
        K = max(1, int(self.cfg.accum_steps))
        if K == 1:
            if self.world == 1 or self.comm is not None:   # one host call (+ RCCL on our stream)
                nat.check(self._lib.rdd_step(self._h), "rdd_step")
            else:
                nat.check(self._lib.rdd_rollout(self._h), "rdd_rollout")
                self.allreduce_grad()
                nat.check(self._lib.rdd_apply(self._h), "rdd_apply")
        else:
            k = self._k
            last = k == K - 1
            self.launch(self.STAGE_ROLLOUT)
            if last and self.world == 1 and self.comm is None:
                self.launch(self.STAGE_REDUCE_ACCUM_APPLY if k else self.STAGE_REDUCE_APPLY)
            else:
                self.launch(self.STAGE_REDUCE_ACCUM if k else self.STAGE_REDUCE)
                if last:
                    self.allreduce_grad()
                    self.launch(self.STAGE_APPLY)
            self._k = 0 if last else k + 1
        self.steps += 1

    def step_accum(self):
        """One optimiser step of K = accum_steps env steps in ONE rollout launch
        (rdd_step_accum): the weight images stay in LDS and the gradient partials in registers
        over the K env steps, then one reduction, (all-reduce,) TF1 Adam.  Same result as K
        step() calls up to f32 reordering of the gradient sums; the envs step bitwise alike."""
        K = max(1, int(self.cfg.accum_steps))
        if self._k:
            raise RuntimeError("step_accum inside a staged accumulation (step() was called "
                               f"{self._k} of {K} times)")
        if self.world == 1 or self.comm is not None:
            nat.check(self._lib.rdd_step_accum(self._h), "rdd_step_accum")
        else:
            nat.check(self._lib.rdd_rollout_accum(self._h), "rdd_rollout_accum")
            self.allreduce_grad()
            nat.check(self._lib.rdd_apply(self._h), "rdd_apply")
        self.steps += K

    def rollout_accum(self):
        """The K env steps of step_accum and their gradient sum in grad() (no Adam)."""
        nat.check(self._lib.rdd_rollout_accum(self._h), "rdd_rollout_accum")

    # -- observation-batch mode (the reference's dataset-window training) ---------------
    def step_obs(self, obs: torch.Tensor):
        """One distillation step on given observation rows [n, 11] (no env step): teacher
        relabel, student forward/backward, loss, (all-reduce), TF1 Adam."""
        obs = self._obs_arg(obs)
        n = obs.shape[0]
        if self.world == 1:
            nat.check(self._lib.rdd_step_obs(self._h, nat.ptr(obs), n), "rdd_step_obs")
        else:
            nat.check(self._lib.rdd_rollout_obs(self._h, nat.ptr(obs), n, n * self.world), "rdd_rollout_obs")
            self.allreduce_grad()
            nat.check(self._lib.rdd_apply(self._h), "rdd_apply")
        self._keep = obs   # the launch reads it asynchronously

    def rollout_obs(self, obs: torch.Tensor, n_global: int | None = None):
        obs = self._obs_arg(obs)
        nat.check(self._lib.rdd_rollout_obs(self._h, nat.ptr(obs), obs.shape[0], n_global or obs.shape[0]),
                  "rdd_rollout_obs")
        self._keep = obs

    # -- rows mode: observations with their recorded teacher pdflat (the reference's dataset) --
    def step_rows(self, obs: torch.Tensor, t_pdflat: torch.Tensor):
        """One distillation step on dataset rows: observations [n, 11] and the teacher's recorded
        pdflat [n, 4] (mean | logstd), the reference's sess.run([loss, minimize_adam],
        {..., t_pdflat_batch_ph: t_pdflat_batch_array}) (mlp_train.py:146-161).  No teacher
        network runs; student forward/backward, loss, (all-reduce), TF1 Adam."""
        obs, tp = self._obs_arg(obs), self._tflat_arg(t_pdflat, obs.shape[0])
        n = obs.shape[0]
        if self.world == 1:
            nat.check(self._lib.rdd_step_rows(self._h, nat.ptr(obs), nat.ptr(tp), n), "rdd_step_rows")
        else:
            nat.check(self._lib.rdd_rollout_rows(self._h, nat.ptr(obs), nat.ptr(tp), n, n * self.world),
                      "rdd_rollout_rows")
            self.allreduce_grad()
            nat.check(self._lib.rdd_apply(self._h), "rdd_apply")
        self._keep = (obs, tp)
        self.steps += 1   # one optimiser step, as step() (fit_records' eager tail)

    def rollout_rows(self, obs: torch.Tensor, t_pdflat: torch.Tensor, n_global: int | None = None):
        obs, tp = self._obs_arg(obs), self._tflat_arg(t_pdflat, obs.shape[0])
        nat.check(self._lib.rdd_rollout_rows(self._h, nat.ptr(obs), nat.ptr(tp), obs.shape[0],
                                             n_global or obs.shape[0]), "rdd_rollout_rows")
        self._keep = (obs, tp)

    def _tflat_arg(self, t, n):
        t = torch.as_tensor(t).to(self.device, torch.float32).contiguous()
        if t.dim() != 2 or t.shape != (n, 4):
            raise ValueError("t_pdflat must be [n, 4] (teacher mean | logstd per row)")
        return t

    def _obs_arg(self, obs):
        obs = torch.as_tensor(obs).to(self.device, torch.float32).contiguous()
        if obs.dim() != 2 or obs.shape[1] != 11 or obs.shape[0] == 0:
            raise ValueError("obs must be [n, 11]")
        return obs

    def counters(self):
        """(env steps, optimiser steps)."""
        e, o = ctypes.c_int64(), ctypes.c_int64()
        nat.check(self._lib.rdd_get_counters(self._h, ctypes.byref(e), ctypes.byref(o)), "rdd_get_counters")
        return e.value, o.value

    def set_stream(self, stream: torch.cuda.Stream):
        nat.check(self._lib.rdd_set_stream(self._h, ctypes.c_void_p(stream.cuda_stream)), "rdd_set_stream")

    def capture(self, steps: int = 1, fused: bool = False) -> torch.cuda.CUDAGraph:
        """Capture `steps` single-rank steps into a HIP graph (replay = `steps` steps, no
        host launches).  fused: `steps` step_accum() calls (K env steps each).  The trainer's
        stream is restored afterwards."""
        if self.world != 1:
            raise RuntimeError("graph capture is for the single-rank step")
        g = torch.cuda.CUDAGraph()
        prev = torch.cuda.current_stream(self.device)
        torch.cuda.synchronize(self.device)
        if not fused and max(1, int(self.cfg.accum_steps)) > 1 and steps % self.cfg.accum_steps:
            raise ValueError("capture whole optimiser steps: steps must be a multiple of accum_steps")
        s0 = self.steps
        with torch.cuda.graph(g):
            self.set_stream(torch.cuda.current_stream(self.device))
            for _ in range(steps):
                self.step_accum() if fused else self.step()
        self.steps = s0   # capture only records launches
        self.set_stream(prev)
        return g

    STAGE_ROLLOUT, STAGE_REDUCE, STAGE_APPLY, STAGE_REDUCE_APPLY = 1, 2, 3, 4
    STAGE_REDUCE_ACCUM, STAGE_REDUCE_ACCUM_APPLY = 5, 6

    def launch(self, stage: int):
        nat.check(self._lib.rdd_launch_stage(self._h, stage), "rdd_launch_stage")

    def rollout(self):
        nat.check(self._lib.rdd_rollout(self._h), "rdd_rollout")

    def apply(self):
        nat.check(self._lib.rdd_apply(self._h), "rdd_apply")
        self.steps += 1

    def grad(self) -> torch.Tensor:
        """The gradient of the last rollout (rank-local until all-reduced)."""
        return self._grad

    def allreduce_grad(self):
        if self.comm is not None:
            nat.check(self._lib.rdd_allreduce_grad(self._h), "rdd_allreduce_grad")
        else:
            allreduce_sum_(self._grad, self.pg)

    def replicas_identical(self) -> bool:
        """student weights stay bit-identical across ranks (same init, same
        all-reduced gradient); checked with an exact integer checksum (all ranks agree)."""
        return replicas_identical(self.student_params(), self.pg)

    # -- queries -----------------------------------------------------------------------
    def forward(self, obs: torch.Tensor, teacher=True, student=True):
        obs = obs.to(self.device, torch.float32).contiguous()
        n = obs.shape[0]
        t = torch.empty(n, 4, device=self.device) if teacher else None
        s = torch.empty(n, 4, device=self.device) if student else None
        nat.check(self._lib.rdd_forward(self._h, nat.ptr(obs), n, nat.ptr(t) if t is not None else None,
                                        nat.ptr(s) if s is not None else None), "rdd_forward")
        return t, s

    def env_state(self) -> torch.Tensor:
        st = torch.empty(8, self.n_local, dtype=torch.float32, device=self.device)
        nat.check(self._lib.rdd_get_env_state(self._h, nat.ptr(st)), "rdd_get_env_state")
        return st

    def set_env_state(self, st: torch.Tensor):
        """Replace the envs' state ([8, n] SoA).  Raises NativeError for joint angles outside the
        fused rollout's range (|q0| < 8192, |q1| <= 4 rad, finite; include/reacher_distill.h)."""
        st = st.to(self.device, torch.float32).contiguous()
        nat.check(self._lib.rdd_set_env_state(self._h, nat.ptr(st)), "rdd_set_env_state")
        torch.cuda.current_stream(self.device).synchronize()

    def counter(self) -> int:
        c = ctypes.c_int64()
        nat.check(self._lib.rdd_get_counter(self._h, ctypes.byref(c)), "rdd_get_counter")
        return c.value

    def metrics(self, count: int) -> np.ndarray:
        """[count, 4] per step: sum reward, loss, sum (mu_s-mu_t)^2, envs (this rank)."""
        out = np.zeros((count, 4), np.float64)
        nat.check(self._lib.rdd_read_metrics(self._h, count, out.ctypes.data_as(ctypes.c_void_p)),
                  "rdd_read_metrics")
        return out

    def close(self):
        if getattr(self, "_h", None):
            nat.load().rdd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

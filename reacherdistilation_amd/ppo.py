"""Teacher training by PPO on batched Reacher-v2 (include/reacher_ppo.h): the reference's
``teacher.train(env_id, num_timesteps, seed)`` (teacher.py:23-37, baselines ppo1
``pposgd_simple.learn``) over ``n_envs`` parallel envs on one GPU.

``PPOTrainer.iterate()`` is one learn-loop iteration: collect the actor batch with the
stochastic policy, GAE(lambda), advantage standardization, observation-filter update,
old-policy freeze, ``optim_epochs`` epochs of shuffled minibatch Adam steps.  The trained
policy is a 2x64 MlpPolicy in the distillation layout (``teacher()`` returns it with its
filter), so it drops into ``DistillTrainer`` / ``TeacherAgent`` as the teacher.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .policy import HID, OBD, MlpPolicyParams, normc

P = nat.P
I32, I64, U64, F32, INT = nat.I32, nat.I64, nat.U64, nat.F32, nat.INT
P_POL, P_VF = 5060, 4993
METRICS = ("ep_ret_mean", "episodes", "pol_surr", "vf_loss", "entropy", "clipfrac", "lrmult", "timesteps")


class RdpConfig(ctypes.Structure):
    _fields_ = [("n_envs", I64), ("horizon", I32), ("seed", U64), ("env_base", I64), ("clip_param", F32),
                ("entcoeff", F32), ("optim_epochs", I32), ("optim_stepsize", F32), ("optim_batchsize", I32),
                ("gamma", F32), ("lam", F32), ("schedule_linear", I32), ("max_timesteps", I64),
                ("metrics_len", I32)]


nat.register({
    "rdp_param_counts": (INT, [ctypes.POINTER(I32), ctypes.POINTER(I32)]),
    "rdp_create": (INT, [ctypes.POINTER(P), ctypes.POINTER(RdpConfig), INT, P]),
    "rdp_destroy": (INT, [P]),
    "rdp_set_stream": (INT, [P, P]),
    "rdp_set_policy": (INT, [P, P]),
    "rdp_get_policy": (INT, [P, P]),
    "rdp_set_value": (INT, [P, P]),
    "rdp_get_value": (INT, [P, P]),
    "rdp_get_obfilter": (INT, [P, P, P]),
    "rdp_reset": (INT, [P]),
    "rdp_iterate": (INT, [P]),
    "rdp_rollout": (INT, [P]),
    "rdp_optimize": (INT, [P]),
    "rdp_get_batch": (INT, [P, P, P, P, P, P, P, P, P]),
    "rdp_grad_buffer": (P, [P]),
    "rdp_bind_grad_buffer": (INT, [P, P]),
    "rdp_get_counter": (INT, [P, ctypes.POINTER(I64)]),
    "rdp_read_metrics": (INT, [P, I64, P]),
})


def value_init(seed: int = 4) -> np.ndarray:
    """baselines MlpPolicy 'vf': normc(1.0) kernels (fc1, fc2, final), zero biases."""
    rng = np.random.RandomState(seed)
    return np.concatenate([normc(rng, (OBD, HID), 1.0).ravel(), np.zeros(HID, np.float32),
                           normc(rng, (HID, HID), 1.0).ravel(), np.zeros(HID, np.float32),
                           normc(rng, (HID, 1), 1.0).ravel(), np.zeros(1, np.float32)]).astype(np.float32)


@dataclass
class PPOConfig:
    n_envs: int = 2048
    horizon: int = 32                  # actor batch = n_envs x horizon (reference: 2048 x 1 env)
    seed: int = 0
    clip_param: float = 0.2            # teacher.py:31-35
    entcoeff: float = 0.0
    optim_epochs: int = 10
    optim_stepsize: float = 3e-4
    optim_batchsize: int = 4096        # reference 64 (one env); 0 = the whole actor batch
    gamma: float = 0.99
    lam: float = 0.95
    schedule: str = "linear"
    max_timesteps: int = 1_000_000
    policy_seed: int = 1
    value_seed: int = 4
    metrics_len: int = 1024


class PPOTrainer:
    def __init__(self, cfg: PPOConfig | None = None, device="cuda:0", policy: MlpPolicyParams | None = None,
                 value=None, env_base: int = 0):
        self.cfg = cfg or PPOConfig()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("PPOTrainer runs on a GPU (HIP) device only; there is no CPU path")
        self._lib = nat.load()
        c = self.cfg
        rc = RdpConfig(n_envs=c.n_envs, horizon=c.horizon, seed=c.seed % 2 ** 64, env_base=env_base,
                       clip_param=c.clip_param, entcoeff=c.entcoeff, optim_epochs=c.optim_epochs,
                       optim_stepsize=c.optim_stepsize, optim_batchsize=c.optim_batchsize, gamma=c.gamma, lam=c.lam,
                       schedule_linear=1 if c.schedule == "linear" else 0, max_timesteps=int(c.max_timesteps),
                       metrics_len=c.metrics_len)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self._lib.rdp_create(ctypes.byref(h), ctypes.byref(rc), self.device.index or 0,
                                           nat.stream_handle(self.device)), "rdp_create")
        self._h = h
        self.S = c.n_envs * c.horizon
        pol = policy.flat if policy is not None else MlpPolicyParams.init(c.policy_seed).flat
        self.set_policy(pol)
        self.set_value(value_init(c.value_seed) if value is None else value)
        self._grad = torch.zeros(P_POL + P_VF, device=self.device)
        nat.check(self._lib.rdp_bind_grad_buffer(self._h, nat.ptr(self._grad)), "rdp_bind_grad_buffer")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rdp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync_stream(self):
        nat.check(self._lib.rdp_set_stream(self._h, nat.stream_handle(self.device)), "rdp_set_stream")

    def _dev(self, x, n):
        x = (x if torch.is_tensor(x) else torch.from_numpy(np.asarray(x, np.float32)))
        x = x.to(self.device, torch.float32).reshape(-1).contiguous()
        if x.numel() != n:
            raise ValueError(f"expected {n} parameters, got {x.numel()}")
        return x

    def set_policy(self, p):
        x = self._dev(p, P_POL)
        self._sync_stream()
        nat.check(self._lib.rdp_set_policy(self._h, nat.ptr(x)), "rdp_set_policy")
        torch.cuda.current_stream(self.device).synchronize()

    def set_value(self, p):
        x = self._dev(p, P_VF)
        self._sync_stream()
        nat.check(self._lib.rdp_set_value(self._h, nat.ptr(x)), "rdp_set_value")
        torch.cuda.current_stream(self.device).synchronize()

    def policy(self) -> torch.Tensor:
        out = torch.empty(P_POL, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdp_get_policy(self._h, nat.ptr(out)), "rdp_get_policy")
        return out

    def value(self) -> torch.Tensor:
        out = torch.empty(P_VF, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdp_get_value(self._h, nat.ptr(out)), "rdp_get_value")
        return out

    def obfilter(self):
        mean = torch.empty(OBD, device=self.device)
        std = torch.empty(OBD, device=self.device)
        self._sync_stream()
        nat.check(self._lib.rdp_get_obfilter(self._h, nat.ptr(mean), nat.ptr(std)), "rdp_get_obfilter")
        return mean, std

    def teacher(self) -> MlpPolicyParams:
        """The current policy with its observation filter, in the distillation layout."""
        mean, std = self.obfilter()
        return MlpPolicyParams(self.policy().cpu().numpy(), mean.cpu().numpy(), std.cpu().numpy())

    # -- training ----------------------------------------------------------------------
    def iterate(self):
        self._sync_stream()
        nat.check(self._lib.rdp_iterate(self._h), "rdp_iterate")

    def rollout(self):
        self._sync_stream()
        nat.check(self._lib.rdp_rollout(self._h), "rdp_rollout")

    def optimize(self):
        self._sync_stream()
        nat.check(self._lib.rdp_optimize(self._h), "rdp_optimize")

    def batch(self) -> dict:
        S, n = self.S, self.cfg.n_envs
        T = self.cfg.horizon
        out = dict(ob=torch.empty(T, n, OBD), ac=torch.empty(T, n, 2), vpred=torch.empty(T, n), rew=torch.empty(T, n),
                   new=torch.empty(T, n), nextvpred=torch.empty(n), adv=torch.empty(T, n), ret=torch.empty(T, n))
        out = {k: v.to(self.device) for k, v in out.items()}
        self._sync_stream()
        nat.check(self._lib.rdp_get_batch(self._h, *[nat.ptr(out[k]) for k in
                                                     ("ob", "ac", "vpred", "rew", "new", "nextvpred", "adv", "ret")]),
                  "rdp_get_batch")
        assert out["vpred"].numel() == S
        return out

    def grad(self) -> torch.Tensor:
        """Gradient of the last minibatch, [pol | vf] (the trainer's bound buffer)."""
        return self._grad

    def iterations(self) -> int:
        v = ctypes.c_int64()
        nat.check(self._lib.rdp_get_counter(self._h, ctypes.byref(v)), "rdp_get_counter")
        return v.value

    def metrics(self, count: int = 1) -> np.ndarray:
        out = np.zeros((count, len(METRICS)), np.float64)
        nat.check(self._lib.rdp_read_metrics(self._h, count, out.ctypes.data_as(ctypes.c_void_p)),
                  "rdp_read_metrics")
        return out


def train(env_id: str = "Reacher-v2", num_timesteps: int = 1_000_000, seed: int = 0, device="cuda:0", log=print,
          **kw) -> PPOTrainer:
    """teacher.train (reference teacher.py:23-37): PPO until num_timesteps env steps."""
    if env_id != "Reacher-v2":
        raise ValueError("only Reacher-v2 is built")
    tr = PPOTrainer(PPOConfig(seed=seed, max_timesteps=num_timesteps, **kw), device=device)
    while tr.iterations() * tr.S < num_timesteps:
        tr.iterate()
        m = tr.metrics(1)[0]
        log(" ".join(f"{k}={v:.4g}" for k, v in zip(METRICS, m)))
    return tr

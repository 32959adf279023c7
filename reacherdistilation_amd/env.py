"""Gym-shaped host API over the HIP Reacher-v2 kernels (libreacher.so, include/reacher.h).

Two entry points mirror what the reference drivers hold:

* ``BatchedReacher(n, seed, device)`` -- N Reacher-v2 envs in lockstep on one GPU,
  torch tensors in/out, no host sync per step.  Replaces the single gym env object of
  reference mlp_train.py:21 for the batched rollout.
* ``make_mujoco_env("Reacher-v2", seed)`` -- the single-env, numpy-float64 drop-in for
  baselines.common.cmd_util.make_mujoco_env as the reference drivers call it
  (reference mlp_train.py:21, lstm_train.py:21): ``env.reset() -> ob[11]``,
  ``env.step(a) -> (ob, reward, done, info)``; gym seeding (seed 0 reproduces the
  reference fixture's resets bit for bit).  It runs the same HIP kernel with N = 1.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as nat
from .config import ACSPACE_SHAPE, EPISODE_STEPS, OBSPACE_SHAPE

STATE_DIM = 8  # q0 q1 v0 v1 tx ty dx dy


def gym_reset_draws(seed: int, n_episodes: int) -> np.ndarray:
    """Native gym seeding + reset_model draws for one env: [n_episodes, 6] f64."""
    out = np.zeros((n_episodes, 6), np.float64)
    nat.check(nat.load().rd_gym_reset_draws(int(seed) % 2 ** 64, int(n_episodes),
                                            out.ctypes.data_as(ctypes.c_void_p)), "rd_gym_reset_draws")
    return out


class BatchedReacher:
    """N lockstep Reacher-v2 environments on one GPU.

    reset: "philox" -> synthetic targets/resets from Philox(seed, env_base+i, episode);
           "gym"    -> env i seeded like gym/baselines with seed + env_base + i (MT19937),
                       reproducing the reference env's reset sequence exactly.
    Returned tensors are persistent device buffers reused by the next call (clone to keep).
    """

    def __init__(self, n: int, seed: int = 0, device="cuda:0", env_base: int = 0, reset: str = "philox",
                 gym_episodes: int = 64):
        self.n = int(n)
        self.seed = int(seed)
        self.env_base = int(env_base)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchedReacher runs on a GPU (HIP) device only; there is no CPU path")
        self.mode = reset
        self._lib = nat.load()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(self._lib.rd_create(ctypes.byref(h), self.n, self.env_base, self.seed % 2 ** 64,
                                          self.device.index or 0, nat.stream_handle(self.device)),
                      "rd_create")
        self._h = h
        kw = dict(device=self.device)
        self.obs = torch.empty(self.n, OBSPACE_SHAPE, dtype=torch.float32, **kw)
        self.rew = torch.empty(self.n, dtype=torch.float32, **kw)
        self.done = torch.empty(self.n, dtype=torch.uint8, **kw)
        self._table = None
        self._table_eps = 0
        self._episode = -1
        self._step = 0
        if reset == "gym":
            self._grow_table(gym_episodes)
        elif reset != "philox":
            raise ValueError(f"unknown reset mode {reset!r}")

    # -- gym-seeded reset table ------------------------------------------------------
    def _grow_table(self, n_eps: int):
        draws = np.stack([gym_reset_draws(self.seed + self.env_base + i, n_eps) for i in range(self.n)],
                         axis=1)                                   # [E, N, 6] f64
        self._table = torch.from_numpy(draws.astype(np.float32)).to(self.device)
        self._table_eps = n_eps
        nat.check(self._lib.rd_set_reset_mode(self._h, nat.RD_RESET_TABLE, nat.ptr(self._table), n_eps),
                  "rd_set_reset_mode")

    def _ensure_table(self, episode: int):
        if self.mode == "gym" and episode >= self._table_eps:
            self._grow_table(max(2 * self._table_eps, episode + 1))

    def set_reset_table(self, draws):
        """Explicit reset draws [E, N, 6] (q0, q1, v0, v1, tx, ty) for episodes 0..E-1."""
        t = torch.as_tensor(np.asarray(draws, np.float32)).to(self.device).contiguous()
        if t.dim() != 3 or t.shape[1:] != (self.n, 6):
            raise ValueError(f"draws must be [E, {self.n}, 6]")
        self._table, self._table_eps, self.mode = t, t.shape[0], "table"
        nat.check(self._lib.rd_set_reset_mode(self._h, nat.RD_RESET_TABLE, nat.ptr(t), t.shape[0]),
                  "rd_set_reset_mode")

    # -- gym API -------------------------------------------------------------------
    def reset(self) -> torch.Tensor:
        self._ensure_table(self._episode + 1)
        with torch.cuda.device(self.device):
            nat.check(self._lib.rd_reset(self._h, nat.ptr(self.obs)), "rd_reset")
        self._episode += 1
        self._step = 0
        return self.obs

    def step(self, act: torch.Tensor):
        if act.shape != (self.n, ACSPACE_SHAPE) or act.dtype != torch.float32 or act.device != self.device:
            raise ValueError(f"act must be float32 [{self.n},{ACSPACE_SHAPE}] on {self.device}")
        act = act.contiguous()
        if self._step + 1 >= EPISODE_STEPS:
            self._ensure_table(self._episode + 1)
        with torch.cuda.device(self.device):
            nat.check(self._lib.rd_step(self._h, nat.ptr(act), nat.ptr(self.obs), nat.ptr(self.rew),
                                        nat.ptr(self.done)), "rd_step")
        if self._step + 1 >= EPISODE_STEPS:
            self._episode += 1
            self._step = 0
        else:
            self._step += 1
        return self.obs, self.rew, self.done, {}

    # -- state hooks ---------------------------------------------------------------
    def get_state(self):
        st = torch.empty(STATE_DIM, self.n, dtype=torch.float32, device=self.device)
        s, e = ctypes.c_int32(), ctypes.c_int32()
        nat.check(self._lib.rd_get_state(self._h, nat.ptr(st), ctypes.byref(s), ctypes.byref(e)),
                  "rd_get_state")
        return st, s.value, e.value

    def set_state(self, state: torch.Tensor, step: int = 0, episode: int = 0):
        state = state.to(self.device, torch.float32).contiguous()
        assert state.shape == (STATE_DIM, self.n)
        nat.check(self._lib.rd_set_state(self._h, nat.ptr(state), int(step), int(episode)), "rd_set_state")
        torch.cuda.current_stream(self.device).synchronize()  # state is copied before it is freed
        self._step, self._episode = int(step), int(episode)

    def close(self):
        if getattr(self, "_h", None):
            nat.load().rd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ReacherEnv:
    """Single Reacher-v2 env with the gym 0.10.5 API (numpy float64 out), on the GPU kernel.

    step() returns the TERMINAL observation on the step that ends the episode (done=True),
    as gym's TimeLimit does; the following reset() returns the next episode's first
    observation.  The kernel auto-resets at that step, so the terminal observation comes from
    a one-env shadow handle stepped from the same state with the episode clock at 0 (the same
    kernel and arithmetic, no reset)."""

    class _Box:
        def __init__(self, shape, low, high):
            self.shape, self.low, self.high = shape, low, high

    def __init__(self, seed: int = 0, device="cuda:0"):
        self._env = BatchedReacher(1, seed=seed, device=device, reset="gym")
        self.observation_space = self._Box((OBSPACE_SHAPE,), -np.inf, np.inf)
        self.action_space = self._Box((ACSPACE_SHAPE,), -1.0, 1.0)
        self._needs_reset = True
        self._pending = None
        self._shadow = None

    def seed(self, seed=None):
        dev = self._env.device
        self._env.close()
        self._env = BatchedReacher(1, seed=int(seed or 0), device=dev, reset="gym")
        self._needs_reset = True
        self._pending = None
        return [seed]

    def reset(self):
        self._needs_reset = False
        if self._pending is not None:          # the episode ended: the kernel already reset
            ob, self._pending = self._pending, None
            return ob
        return self._env.reset()[0].double().cpu().numpy()

    def step(self, a):
        if self._needs_reset:
            # baselines Monitor: "Tried to step environment that needs reset"
            raise RuntimeError("Tried to step environment that needs reset")
        a32 = np.asarray(a, dtype=np.float32).reshape(ACSPACE_SHAPE)
        act = torch.from_numpy(a32).view(1, ACSPACE_SHAPE).to(self._env.device)
        if self._env._episode < 0:
            self._env.reset()
        terminal = None
        if self._env._step + 1 >= EPISODE_STEPS:   # this step ends the episode
            if self._shadow is None:
                self._shadow = BatchedReacher(1, seed=0, device=self._env.device)
            st, _, _ = self._env.get_state()
            self._shadow.set_state(st, step=0, episode=0)
            terminal = self._shadow.step(act)[0][0].double().cpu().numpy()
        ob, r, d, _ = self._env.step(act)
        done = bool(d[0].item())
        ob = ob[0].double().cpu().numpy()
        if done:
            self._needs_reset = True
            # the kernel already auto-reset; the reference calls env.reset() next, which
            # must hand out that same reset observation (not draw another one)
            self._pending = ob
            ob = terminal
        reward_ctrl = -float(np.square(a32).sum())
        rew = float(r[0].item())
        info = dict(reward_dist=rew - reward_ctrl, reward_ctrl=reward_ctrl)
        return ob, rew, done, info


def make_mujoco_env(env_id: str, seed: int, device="cuda:0"):
    """baselines.common.cmd_util.make_mujoco_env for "Reacher-v2" on the HIP env."""
    if env_id != "Reacher-v2":
        raise ValueError(f"only Reacher-v2 is provided, got {env_id!r}")
    return ReacherEnv(seed=seed, device=device)

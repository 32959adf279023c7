"""The single Reacher-v2 env of the reference-shaped drivers (mlp_train.train, lstm_train.train,
lstm_train.train_bptt; reference mlp_train.py:21,112,135-139,196-202 and lstm_train.py:21,
111-136,192-196), with the env I/O kept on the device.

The reference loop makes host round trips every env step: the action goes to the env as
numpy, and the observation, reward and done come back.  Here the observation and reward stay
device tensors from the env kernel to the dataset and the policy queries, and the action goes
from the student's output straight into the env kernel.  `done` is the TimeLimit(50) count
the host already keeps: Reacher has no other termination, and the kernel auto-resets, so
after `done` the observation it returned is the one the reference's env.reset() hands back.
Nothing waits on the GPU inside an episode.

``gym_api=True`` runs the same interface through the gym-API env (make_mujoco_env: numpy
float64 every step, as the reference does); the drivers produce the same records bit for bit
either way (tests/test_c1_gpu.py).
"""
from __future__ import annotations

import numpy as np
import torch

from .config import ACSPACE_SHAPE, OBSPACE_SHAPE
from .env import BatchedReacher, make_mujoco_env


class DriverEnv:
    def __init__(self, seed: int = 0, device="cuda:0", gym_api: bool = False):
        self.device = torch.device(device)
        self.gym_api = bool(gym_api)
        if self.gym_api:
            self._gym = make_mujoco_env("Reacher-v2", seed, device=device)
        else:
            self._env = BatchedReacher(1, seed=seed, device=device, reset="gym")   # make_mujoco_env's env

    def _dev(self, ob) -> torch.Tensor:
        return torch.from_numpy(np.asarray(ob, np.float32)).view(1, OBSPACE_SHAPE).to(self.device)

    def reset(self) -> torch.Tensor:
        """The first observation, [1, 11] f32 on the device."""
        if self.gym_api:
            return self._dev(self._gym.reset())
        return self._env.reset()

    def step(self, a: torch.Tensor):
        """env.step with the first two entries of the pdflat `a` (its mean): (observation
        [1, 11], reward [1], done).  After done the observation is the next episode's first
        (the reference's env.reset() is folded in).  Returned device tensors are the env's
        persistent buffers: consumed by later launches on the same stream before the next step
        overwrites them."""
        if self.gym_api:
            ob, r, done, _ = self._gym.step(a[:ACSPACE_SHAPE].detach().cpu().numpy())
            if done:
                ob = self._gym.reset()
            return self._dev(ob), torch.tensor([r], dtype=torch.float32, device=self.device), bool(done)
        ob, r, _, _ = self._env.step(a[:ACSPACE_SHAPE].reshape(1, ACSPACE_SHAPE).contiguous())
        return ob, r, self._env._step == 0


def episode_loss(values) -> float:
    """The reference's per-episode running float sum of the step losses, in step order."""
    total = 0.0
    for v in values:
        total += float(v)
    return total

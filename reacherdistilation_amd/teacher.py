"""The reference's teacher module (src/distilation/teacher.py) on the MI355X path.

  TeacherAgent (teacher.py:12-20)  -> policy.TeacherAgent (TF checkpoint or safetensors restore)
  train (:23-37, ppo1 learn)       -> ppo.train
  collect_reward (:39-62)          -> collect_reward below, batched over ``n_envs`` envs

``collect_reward`` as committed cannot run (``TeaherAgent``, ``ob_ph``, ``t_pdflat``,
``reward`` and ``Dataset`` are undefined there).  Its evident intent -- the teacher's mean
action steps the env, every step is recorded with the teacher's pdflat, a zero student pdflat
and stepped_with 't', and an episode end resets the env and flushes the dataset -- is the
warm-up phase of lstm_train.py:113-135, which does run; the records follow that loop: the
reward of a record is the one the previous env.step returned (0 before the first step, carried
over a reset, :113,133).  Batched: the envs step in lockstep and env i is seeded as
make_mujoco_env(env_id, seed + i) (``reset="gym"``), so ``n_envs = 1`` gives lstm_train's
warm-up records bit for bit and env i's episodes are those of a one-env collection with seed
+ i.  Each round of 50 steps adds one episode per env to the dataset (env order); with a page
store attached, full pages of MAX_CAPACITY episodes are written as the drivers do
(lstm_train.py:200).
"""
from __future__ import annotations

import torch

from .config import ACSPACE_SHAPE, EPISODE_STEPS, MAX_CAPACITY
from .dataset import F_OB, F_REW, F_S, F_T, REC, DeviceDataset
from .distill import DistillConfig, DistillTrainer
from .env import BatchedReacher
from .pages import PageStore
from .policy import MlpPolicyParams, TeacherAgent
from .ppo import train  # noqa: F401  (teacher.train: PPO on the batched env)

__all__ = ["TeacherAgent", "train", "collect_reward"]


def collect_reward(episodes: int, n_envs: int = 1, *, seed: int = 0, teacher: MlpPolicyParams | None = None,
                   teacher_path: str | None = None, dataset: DeviceDataset | None = None,
                   store_dir: str | None = None, device="cuda:0", reset: str = "gym") -> DeviceDataset:
    """Record ``episodes`` teacher-stepped episodes (rounded up to whole rounds of ``n_envs``;
    the last round's surplus is dropped) into ``dataset`` (a new DeviceDataset when None, its
    pages in ``store_dir``).  The teacher is ``teacher``, else restored from ``teacher_path``
    (TeacherAgent), else the synthetic one.  Returns the dataset."""
    if episodes < 0 or n_envs < 1:
        raise ValueError("episodes >= 0 and n_envs >= 1")
    dev = torch.device(device)
    pi = teacher if teacher is not None else TeacherAgent(restore=teacher_path is not None, path=teacher_path).pi
    if dataset is None:
        dataset = DeviceDataset(capacity=max(5000, int(episodes)), device=dev, seed=seed,
                                store=PageStore(store_dir) if store_dir else None)
    env = BatchedReacher(n_envs, seed=seed, device=dev, reset=reset)
    tq = DistillTrainer(DistillConfig(n_envs=64, seed=seed), device=dev, teacher=pi)
    block = torch.zeros(EPISODE_STEPS, n_envs, REC, dtype=torch.float32, device=dev)
    reward = torch.zeros(n_envs, dtype=torch.float32, device=dev)
    ob = env.reset()
    done = 0
    while done < episodes:
        for s in range(EPISODE_STEPS):
            t, _ = tq.forward(ob, student=False)
            rec = block[s]
            rec[:, F_OB:F_REW] = ob
            rec[:, F_REW] = reward
            rec[:, F_T:F_S] = t   # s_pdflat and stepped_with ('t' = 0) stay zero
            ob, rew, _, _ = env.step(t[:, :ACSPACE_SHAPE].contiguous())
            reward = rew.clone()
        take = min(n_envs, episodes - done)
        eps = block.transpose(0, 1)[:take]
        if dataset.store is None:
            dataset.write_episodes(eps)
        else:   # page by page: dump whenever the episode count reaches a multiple of MAX_CAPACITY
            e = 0
            while e < take:
                k = min(take - e, MAX_CAPACITY - dataset.num_episodes() % MAX_CAPACITY)
                dataset.write_episodes(eps[e:e + k])
                e += k
                if dataset.num_episodes() % MAX_CAPACITY == 0:
                    dataset.dump()
        done += take
    env.close()
    tq.close()
    return dataset

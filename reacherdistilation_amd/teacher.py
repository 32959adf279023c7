"""The reference's teacher module (src/distilation/teacher.py) on the MI355X path.

  TeacherAgent (teacher.py:12-20)  -> policy.TeacherAgent (TF checkpoint or safetensors restore)
  train (:23-37, ppo1 learn)       -> ppo.train
  collect_reward (:39-62)          -> collect_reward below, batched over ``n_envs`` envs
  (the restored teacher.ckpt)      -> ppo_teacher below: the checkpoint ppo.train writes with the
                                      reference's hyperparameters (teachers/ppo_teacher.ckpt), or
                                      fit_teacher: the teacher's structure fitted to the teacher
                                      records the reference ships (its checkpoint does not)

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

import os

import numpy as np
import torch

from .config import ACSPACE_SHAPE, EPISODE_STEPS, MAX_CAPACITY, OBSPACE_SHAPE
from .dataset import F_OB, F_REW, F_S, F_T, REC, DeviceDataset
from .distill import DistillConfig, DistillTrainer
from .env import BatchedReacher
from .pages import PageStore
from .policy import MlpPolicyParams, TeacherAgent
from .ppo import train  # noqa: F401  (teacher.train: PPO on the batched env)

__all__ = ["TeacherAgent", "train", "collect_reward", "fit_teacher", "episode_returns", "ppo_teacher", "PPO_TEACHER"]

# The teacher trained by PPO here (scripts/train_ppo_teacher.py): the reference's
# teacher.train with its own hyperparameters (teacher.py:30-36; one env, 2,048-step actor batches,
# 1e6 steps, 9.8 s on one MI355X), saved as the reference Saver's scope-'pi' checkpoint; mean
# 50-step return of its mean action -4.61 over 4,096 fresh episodes against the reference
# teacher's -7.53 on the fixture (profiles/r06_ppo_teacher.json)
PPO_TEACHER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "teachers", "ppo_teacher.ckpt")


def ppo_teacher(path: str = PPO_TEACHER) -> MlpPolicyParams:
    """The committed PPO-trained teacher (TeacherAgent(restore=True, path=...).pi)."""
    return TeacherAgent(restore=True, path=path).pi


def episode_returns(teacher: MlpPolicyParams, episodes: int, seed: int = 0, device="cuda:0") -> np.ndarray:
    """50-step returns (gym's episode reward: the 50 step rewards summed) of ``episodes`` fresh
    gym-seeded envs (env i seeded seed + i) stepped with ``teacher``'s mean action, as the
    reference's collect_reward steps the teacher (teacher.py:39-62).  The fixture's -7.53 sums each
    episode's 50 recorded rewards, whose first is the previous episode's last: the
    same quantity in expectation."""
    dev = torch.device(device)
    env = BatchedReacher(episodes, seed=seed, device=dev, reset="gym")
    tq = DistillTrainer(DistillConfig(n_envs=64, seed=seed), device=dev, teacher=teacher)
    ob = env.reset()
    ret = torch.zeros(episodes, dtype=torch.float64, device=dev)
    for _ in range(EPISODE_STEPS):
        t, _ = tq.forward(ob, student=False)
        ob, rew, _, _ = env.step(t[:, :ACSPACE_SHAPE].contiguous())
        ret += rew.double()
    env.close()
    tq.close()
    return ret.cpu().numpy()


def fit_teacher(ob, t_pdflat, *, phases=((30_000, 1e-3), (20_000, 1e-4)), seed: int = 0, device="cuda:0",
                log_every: int = 0):
    """A teacher of the reference's structure (teacher.py:14-16: baselines MlpPolicy, observation
    filter -> 2 x 64 tanh -> linear mean, state-independent logstd) fitted to recorded teacher
    data: episodes ob [E, 50, 11] with the teacher's pdflat t_pdflat [E, 50, 4] -- the
    reference's own fixture (tests/golden/reacher_fixture.npz, its 21 teacher-stepped episodes =
    1,050 records).  The reference restores a trained teacher.ckpt that it does not ship
    (teacher.py:17-20); this stands in for it where a teacher "shaped like the reference's"
    matters (the student-MSE north star).
      filter  baselines RunningMeanStd over the records' observations, as the reference graph's
              pi/obfilter ops compute it (tf_checkpoint.obfilter: std floored at 0.1);
      logstd  the records' (constant) teacher logstd;
      weights the rows-mode trainer (rdd_step_rows: the recorded pdflat as the MSE target,
              200-row windows drawn as dataset.py:179-194, TF1 Adam) for each (steps, lr) phase,
              from normc(1.0) / normc(0.01) init (seed).
    Returns (MlpPolicyParams, history [(phase, step, mean training MSE)])."""
    from .distill import DistillConfig, DistillTrainer
    from .mlp_train import fit_records
    from .tf_checkpoint import obfilter
    ob = np.asarray(ob, np.float32).reshape(-1, EPISODE_STEPS, OBSPACE_SHAPE)
    tp = np.asarray(t_pdflat, np.float32).reshape(-1, EPISODE_STEPS, 4)
    flat = ob.reshape(-1, OBSPACE_SHAPE).astype(np.float64)
    mean, std = obfilter(flat.sum(0), np.square(flat).sum(0), flat.shape[0])
    logstd = tuple(float(x) for x in tp.reshape(-1, 4)[:, 2:].astype(np.float64).mean(0))   # (f64: exact when constant)
    p = MlpPolicyParams.init(seed, logstd=logstd, out_std=0.01)
    p.ob_mean, p.ob_std = mean, std
    hist = []
    for k, (steps, lr) in enumerate(phases):
        tr = DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss="mse", lr=lr, metrics_len=100), device=device,
                            student=p)
        tr, h = fit_records(ob, tp, steps=int(steps), loss="mse", lr=lr, seed=seed + k, device=device,
                            log_every=log_every, trainer=tr)
        hist += [(k, s, m) for s, m in h]
        p = MlpPolicyParams(tr.student_params().cpu().numpy(), mean, std)
        tr.close()
    p.flat[p.flat.size - 2:] = np.asarray(logstd, np.float32)   # (MSE leaves logstd untouched)
    return p, hist


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

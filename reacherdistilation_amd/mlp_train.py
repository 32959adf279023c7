"""The reference's MLP distillation driver, ``mlp_train.train(train, restore)`` (reference
src/distilation/mlp_train.py:18-204), re-expressed over the MI355X path: the env is the HIP
Reacher-v2 (``make_mujoco_env``), teacher queries and the student's training step are the
fused kernels behind ``DistillTrainer`` (``rdd_forward`` / ``rdd_step_obs``), and the
rollout -> distill buffer is the device-resident ``DeviceDataset``.

Phases as in the reference:
  1. (:120-139) the teacher steps the env until ``num_episodes() > 2 * MLP_BATCH_SIZE``,
     every step recorded (ob, reward of the previous step, teacher pdflat, 't');
  2. (:143-204) per env step: one optimiser step on each window from
     ``dataset.training_batches()``, teacher relabel of the current observation, the student's
     (deterministic mean) action, record with 's', env.step with the student action; episode
     boundaries reset the env and flush the dataset; stop after ``episodes`` episodes.

Students: ``student="policy"`` (default) is the 2x64 MlpPolicy taking the observation (the
fused DistillTrainer path); ``student="mlp"`` is the reference's own ``student_mlp_graph``
(student_nn.py:51-57) on rows ob | prev_pdflat | prev_rew (StudentMlpTrainer), trained on the
recorded teacher pdflat with input dropout ``keep_prob`` (reference KEEP_PROB = 0.5).

Fixes of the reference as committed: the committed
graph's (10,20,.) vs (1,20,.) placeholder mismatch is not reproduced -- every row of a [T, B]
window is a training row; prev_pdflat / prev_rew are the dataset's recorded fields, not the
committed np.random.rand "TODO revert" stand-ins (mlp_train.py:151-158).
"""
from __future__ import annotations

import numpy as np
import torch

from .config import MLP_BATCH_SIZE, MLP_EPISODE_BUDGET, OBSPACE_SHAPE
from .dataset import DeviceDataset
from .distill import DistillConfig, DistillTrainer
from .env import make_mujoco_env
from .policy import TeacherAgent
from .student_mlp import StudentMlpConfig, StudentMlpTrainer, rows


def train(train: bool = True, restore: bool = False, *, episodes: int = MLP_EPISODE_BUDGET,
          loss: str = "kl", lr: float = 1e-4, seed: int = 0, device="cuda:0", teacher_path: str | None = None,
          warmup_episodes: int = 2 * MLP_BATCH_SIZE, student: str = "policy", keep_prob: float = 1.0,
          log=print, gym_env: bool = False):
    """Returns (trainer, dataset, per-episode summed training loss); the trainer is the
    DistillTrainer (student="policy") or the StudentMlpTrainer (student="mlp").

    By default the loop never waits on the GPU inside an episode: observations, rewards and
    actions stay device tensors from the env kernel to the dataset and the policy queries,
    `done` is the TimeLimit count the host already keeps, and the per-window losses are read
    from the trainer's metrics ring once per episode.  gym_env=True runs the same loop through
    the gym-API env (numpy round trips every step, as the reference does); both give the
    same records bit for bit (tests/test_c1_gpu.py)."""
    if student not in ("policy", "mlp"):
        raise ValueError(f"unknown student {student!r}")
    if not gym_env:
        return _train_device(train, restore, episodes=episodes, loss=loss, lr=lr, seed=seed, device=device,
                             teacher_path=teacher_path, warmup_episodes=warmup_episodes, student=student,
                             keep_prob=keep_prob, log=log)
    env = make_mujoco_env("Reacher-v2", seed, device=device)
    teacher = TeacherAgent(restore=restore, path=teacher_path)
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss=loss, lr=lr), device=device, teacher=teacher.pi)
    sm = StudentMlpTrainer(StudentMlpConfig(loss=loss, lr=lr, keep_prob=keep_prob, seed=seed),
                           device=device) if student == "mlp" else None
    dataset = DeviceDataset(device=device, seed=seed)
    ob = env.reset()
    reward = 0.0
    losses = []
    if not train:
        return (sm or tr), dataset, losses

    def query(o):
        t, s = tr.forward(torch.as_tensor(np.asarray(o, np.float32)).view(1, OBSPACE_SHAPE))
        if sm is not None:   # the reference student: row = ob | prev_pdflat | prev_rew
            prev, prew = dataset.current_prev()
            ob_t = torch.as_tensor(np.asarray(o, np.float32), device=prev.device).view(OBSPACE_SHAPE)
            s = sm.forward(rows(ob_t, prev, prew))
        return t[0].cpu().numpy(), s[0].cpu().numpy()

    log("Begin Training! First Accumulate observation with teacher")
    while dataset.num_episodes() <= warmup_episodes:
        t_pdflat, _ = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, stepped_with="t")
        ob, reward, new, _ = env.step(t_pdflat[:2])
        if new:
            ob = env.reset()
            dataset.flush()
    log("Accumulated sufficient data points from teacher. now train")

    total_loss = 0.0
    while True:
        for ob_batch, t_batch, prev_batch, prew_batch in dataset.training_batches():
            if sm is not None:   # mlp_train.py:145-160 on the reference graph
                sm.step(rows(ob_batch, prev_batch, prew_batch), t_batch.reshape(-1, 4))
                total_loss += float(sm.metrics(1)[0, 0])
            else:
                tr.step_obs(ob_batch.reshape(-1, OBSPACE_SHAPE))
                total_loss += float(tr.metrics(1)[0, 1])
        t_pdflat, s_pdflat = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, s_pdflat=s_pdflat, stepped_with="s")
        ob, reward, new, _ = env.step(s_pdflat[:2])
        if new:
            log("************** Episode {0} ****************".format(dataset.num_episodes()))
            ob = env.reset()
            log("recent loss: %f " % total_loss)
            losses.append(total_loss)
            total_loss = 0.0
            dataset.flush()
            if dataset.num_episodes() >= episodes:
                break
    return (sm or tr), dataset, losses


def _train_device(train, restore, *, episodes, loss, lr, seed, device, teacher_path, warmup_episodes, student,
                  keep_prob, log):
    """train() with device-resident env I/O (see train's docstring)."""
    from .env import BatchedReacher
    env = BatchedReacher(1, seed=seed, device=device, reset="gym")   # = make_mujoco_env's env
    teacher = TeacherAgent(restore=restore, path=teacher_path)
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss=loss, lr=lr), device=device, teacher=teacher.pi)
    sm = StudentMlpTrainer(StudentMlpConfig(loss=loss, lr=lr, keep_prob=keep_prob, seed=seed),
                           device=device) if student == "mlp" else None
    dataset = DeviceDataset(device=device, seed=seed)
    ob = env.reset()                                  # [1, 11], the env's persistent buffer
    reward = torch.zeros(1, device=env.device)
    losses = []
    if not train:
        return (sm or tr), dataset, losses

    def query(o):
        t, s = tr.forward(o)
        if sm is not None:   # the reference student: row = ob | prev_pdflat | prev_rew
            prev, prew = dataset.current_prev()
            s = sm.forward(rows(o.view(OBSPACE_SHAPE), prev, prew))
        return t[0], s[0]

    def env_step(a):
        """env.step on the device: the kernel auto-resets at the TimeLimit, so after `done`
        the returned observation is already the reset one (what the reference's env.reset()
        hands back next)."""
        o, r, _, _ = env.step(a[:2].reshape(1, 2).contiguous())
        return o, r, env._step == 0

    log("Begin Training! First Accumulate observation with teacher")
    while dataset.num_episodes() <= warmup_episodes:
        t_pdflat, _ = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, stepped_with="t")
        ob, reward, new = env_step(t_pdflat)
        if new:
            dataset.flush()
    log("Accumulated sufficient data points from teacher. now train")

    opt_steps = 0   # optimiser steps of the open episode (their losses are read at its end)
    while True:
        for ob_batch, t_batch, prev_batch, prew_batch in dataset.training_batches():
            if sm is not None:
                sm.step(rows(ob_batch, prev_batch, prew_batch), t_batch.reshape(-1, 4))
            else:
                tr.step_obs(ob_batch.reshape(-1, OBSPACE_SHAPE))
            opt_steps += 1
        t_pdflat, s_pdflat = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, s_pdflat=s_pdflat, stepped_with="s")
        ob, reward, new = env_step(s_pdflat)
        if new:
            log("************** Episode {0} ****************".format(dataset.num_episodes()))
            m = (sm.metrics(opt_steps)[:, 0] if sm is not None else tr.metrics(opt_steps)[:, 1]) if opt_steps else []
            total_loss = 0.0
            for v in m:   # the reference's running float sum, in step order
                total_loss += float(v)
            log("recent loss: %f " % total_loss)
            losses.append(total_loss)
            opt_steps = 0
            dataset.flush()
            if dataset.num_episodes() >= episodes:
                break
    return (sm or tr), dataset, losses

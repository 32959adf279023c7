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

import torch

from .config import MLP_BATCH_SIZE, MLP_EPISODE_BUDGET, OBSPACE_SHAPE
from .dataset import DeviceDataset
from .pages import PageStore
from .distill import DistillConfig, DistillTrainer
from .driver_env import DriverEnv, episode_loss
from .policy import TeacherAgent
from .student_mlp import StudentMlpConfig, StudentMlpTrainer, rows


def train(train: bool = True, restore: bool = False, *, episodes: int = MLP_EPISODE_BUDGET,
          loss: str = "kl", lr: float = 1e-4, seed: int = 0, device="cuda:0", teacher_path: str | None = None,
          warmup_episodes: int = 2 * MLP_BATCH_SIZE, student: str = "policy", keep_prob: float = 1.0,
          log=print, gym_env: bool = False, store_dir: str | None = None, pool: str = "reference",
          stop_loss: float | None = None):
    """Returns (trainer, dataset, per-episode summed training loss); the trainer is the
    DistillTrainer (student="policy") or the StudentMlpTrainer (student="mlp").  The env I/O
    stays on the device (driver_env.DriverEnv; gym_env=True: through the gym-API env, numpy
    every step) and the window losses are read from the trainer's metrics ring once per
    episode, so nothing waits on the GPU inside an episode.  ``store_dir``: the dataset's page
    directory (mlp_train.py:105-110); episodes are dumped to it every 5 episodes (:203) and its
    stored pages join the training pool (dataset.py:164-177); ``pool="ring"`` draws windows
    uniformly from the device ring instead.  ``stop_loss``: also stop after the first DAgger
    episode whose mean window loss falls below it (convergence measurements)."""
    if student not in ("policy", "mlp"):
        raise ValueError(f"unknown student {student!r}")
    env = DriverEnv(seed, device, gym_api=gym_env)
    teacher = TeacherAgent(restore=restore, path=teacher_path)
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss=loss, lr=lr), device=device, teacher=teacher.pi)
    sm = StudentMlpTrainer(StudentMlpConfig(loss=loss, lr=lr, keep_prob=keep_prob, seed=seed),
                           device=device) if student == "mlp" else None
    dataset = DeviceDataset(device=device, seed=seed, store=PageStore(store_dir) if store_dir else None, pool=pool)
    ob = env.reset()                                  # [1, 11] on the device
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

    log("Begin Training! First Accumulate observation with teacher")
    while dataset.num_episodes() <= warmup_episodes:
        t_pdflat, _ = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, stepped_with="t")
        ob, reward, new = env.step(t_pdflat)
        if new:
            dataset.flush()
    log("Accumulated sufficient data points from teacher. now train")

    opt_steps = 0   # optimiser steps of the open episode (their losses are read at its end)
    while True:
        for ob_batch, t_batch, prev_batch, prew_batch in dataset.training_batches():
            if sm is not None:   # mlp_train.py:145-160 on the reference graph
                sm.step(rows(ob_batch, prev_batch, prew_batch), t_batch.reshape(-1, 4))
            else:
                tr.step_obs(ob_batch.reshape(-1, OBSPACE_SHAPE))
            opt_steps += 1
        t_pdflat, s_pdflat = query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, s_pdflat=s_pdflat, stepped_with="s")
        ob, reward, new = env.step(s_pdflat)
        if new:
            log("************** Episode {0} ****************".format(dataset.num_episodes()))
            m = (sm.metrics(opt_steps)[:, 0] if sm is not None else tr.metrics(opt_steps)[:, 1]) if opt_steps else []
            total_loss = episode_loss(m)
            log("recent loss: %f " % total_loss)
            losses.append(total_loss)
            done = stop_loss is not None and opt_steps and total_loss / opt_steps < stop_loss
            opt_steps = 0
            dataset.flush()
            if dataset.store is not None and dataset.num_episodes() % 5 == 0:
                dataset.dump()          # mlp_train.py:203
            if dataset.num_episodes() >= episodes or done:
                break
    return (sm or tr), dataset, losses

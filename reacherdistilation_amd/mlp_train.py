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

from . import _native as nat
from .config import EPISODE_STEPS, LSTM_BATCH_SIZE, MLP_BATCH_SIZE, MLP_EPISODE_BUDGET, OBSPACE_SHAPE, STEPS_UNROLLED
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
          stop_loss: float | None = None, teacher=None):
    """Returns (trainer, dataset, per-episode summed training loss); the trainer is the
    DistillTrainer (student="policy") or the StudentMlpTrainer (student="mlp").  The env I/O
    stays on the device (driver_env.DriverEnv; gym_env=True: through the gym-API env, numpy
    every step) and the window losses are read from the trainer's metrics ring once per
    episode, so nothing waits on the GPU inside an episode.  ``store_dir``: the dataset's page
    directory (mlp_train.py:105-110); episodes are dumped to it every 5 episodes (:203) and its
    stored pages join the training pool (dataset.py:164-177); ``pool="ring"`` draws windows
    uniformly from the device ring instead.  ``stop_loss``: also stop after the first DAgger
    episode whose mean window loss falls below it (convergence measurements).  ``teacher``: an
    MlpPolicyParams used instead of the restored / synthetic one (e.g. teacher.fit_teacher)."""
    if student not in ("policy", "mlp"):
        raise ValueError(f"unknown student {student!r}")
    env = DriverEnv(seed, device, gym_api=gym_env)
    pi = teacher if teacher is not None else \
        TeacherAgent(restore=teacher_path is not None, path=teacher_path).pi   # always restored (ref. :29)
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss=loss, lr=lr), device=device, teacher=pi)
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
            else:           # the same feed: the window's recorded teacher pdflat (rows mode)
                tr.step_rows(ob_batch.reshape(-1, OBSPACE_SHAPE), t_batch.reshape(-1, 4))
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


# -- phase 2 on recorded teacher data (no env) ------------------------------------------------
def _windows(gen, n_eps, lens_ok, count, B=LSTM_BATCH_SIZE, T=STEPS_UNROLLED, device="cuda:0"):
    """[count, T * B] flat record indices of `count` training batches drawn as the reference's
    training_batches (dataset.py:179-194): B episodes with replacement and ONE start per batch,
    T consecutive steps from it."""
    out = torch.empty(count, T, B, dtype=torch.long)
    for k in range(count):   # batch by batch, so the sequence does not depend on how it is chunked
        eps = torch.randint(0, n_eps, (B,), generator=gen)
        start = int(torch.randint(0, EPISODE_STEPS - T + 1, (1,), generator=gen))
        out[k] = eps[None, :] * EPISODE_STEPS + start + torch.arange(T)[:, None]
    return out.reshape(count, T * B).to(device)


def fit_records(ob, t_pdflat, rew=None, *, student: str = "policy", steps: int = 250_000, loss: str = "mse",
                lr: float = 1e-4, seed: int = 0, device="cuda:0", graph_steps: int = 100, log_every: int = 0,
                trainer=None):
    """The reference's phase-2 optimiser steps (mlp_train.py:143-161) on RECORDED teacher data:
    episodes ob [E, 50, 11] with the teacher's pdflat t_pdflat [E, 50, 4] (and rewards [E, 50]
    for the reference student's prev_rew), e.g. the fixture's teacher-stepped episodes.  Each
    step is one Adam step on one training batch of 20 windows x 10 steps (200 rows, drawn as
    dataset.py:179-194 draws them, from a seeded host generator), with the recorded t_pdflat
    as the target (rows mode: no teacher network runs).  student="policy": the 2x64 MlpPolicy
    (DistillTrainer.step_rows), captured `graph_steps` steps per HIP graph with the batch
    indices drawn ahead into a device buffer; student="mlp": the reference graph
    (StudentMlpTrainer.step on rows ob | prev_pdflat | prev_rew).  Returns (trainer, history)
    with history = [(step, mean training action-MSE of the last steps)] every `log_every`."""
    ob = torch.as_tensor(ob, dtype=torch.float32)
    tp = torch.as_tensor(t_pdflat, dtype=torch.float32)
    E = ob.shape[0]
    dev = torch.device(device)
    ob_all = ob.reshape(-1, OBSPACE_SHAPE).to(dev).contiguous()
    t_all = tp.reshape(-1, 4).to(dev).contiguous()
    gen = torch.Generator().manual_seed(int(seed))
    history = []
    if student == "policy":
        tr = trainer or DistillTrainer(DistillConfig(n_envs=64, seed=seed, loss=loss, lr=lr, metrics_len=graph_steps),
                                       device=device)
        rows_per = LSTM_BATCH_SIZE * STEPS_UNROLLED
        idx_buf = torch.zeros(graph_steps, rows_per, dtype=torch.long, device=dev)
        ob_buf = torch.zeros(graph_steps, rows_per, OBSPACE_SHAPE, device=dev)
        t_buf = torch.zeros(graph_steps, rows_per, 4, device=dev)
        g = torch.cuda.CUDAGraph()
        prev = torch.cuda.current_stream(dev)
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(g):
            tr.set_stream(torch.cuda.current_stream(dev))
            torch.index_select(ob_all, 0, idx_buf.reshape(-1), out=ob_buf.reshape(-1, OBSPACE_SHAPE))
            torch.index_select(t_all, 0, idx_buf.reshape(-1), out=t_buf.reshape(-1, 4))
            for k in range(graph_steps):
                nat.check(tr._lib.rdd_step_rows(tr._h, nat.ptr(ob_buf[k]), nat.ptr(t_buf[k]), rows_per),
                          "rdd_step_rows")
        tr.set_stream(prev)
        done = 0
        while done + graph_steps <= steps:
            idx_buf.copy_(_windows(gen, E, None, graph_steps, device=dev))
            g.replay()
            done += graph_steps
            tr.steps += graph_steps
            if log_every and done % log_every < graph_steps:
                m = tr.metrics(graph_steps)
                history.append((done, float((m[:, 2] / (2 * m[:, 3])).mean())))
        if done < steps:   # the last steps % graph_steps steps eagerly: exactly `steps` Adam steps
            for i in _windows(gen, E, None, steps - done, device=dev):
                tr.step_rows(ob_all[i], t_all[i])
            done = steps
        torch.cuda.synchronize(dev)
        return tr, history
    if student != "mlp":
        raise ValueError(f"unknown student {student!r}")
    r = torch.zeros(E, EPISODE_STEPS) if rew is None else torch.as_tensor(rew, dtype=torch.float32)
    prev_t = torch.zeros_like(tp)
    prev_t[:, 1:] = tp[:, :-1]
    prev_r = torch.zeros(E, EPISODE_STEPS, 1)
    prev_r[:, 1:, 0] = r[:, :-1]
    x_all = rows(ob, prev_t, prev_r).to(dev)
    sm = trainer or StudentMlpTrainer(StudentMlpConfig(loss=loss, lr=lr, seed=seed), device=device)
    done = 0
    while done < steps:
        for i in _windows(gen, E, None, min(graph_steps, steps - done), device=dev):
            sm.step(x_all[i], t_all[i])
        done += min(graph_steps, steps - done)
        if log_every and done % log_every < graph_steps:
            m = sm.metrics(min(graph_steps, done))
            history.append((done, float((m[:, 1] / (2 * m[:, 2])).mean())))
    torch.cuda.synchronize(dev)
    return sm, history


def action_mse(trainer, ob, t_pdflat, rew=None) -> float:
    """mean over records and both action dims of (mu_student - mu_teacher)^2 on recorded
    episodes ob [E, 50, 11] / t_pdflat [E, 50, 4] (the reference LSTM student's
    0.0212 on the fixture's episodes 21-24 is this quantity)."""
    ob = torch.as_tensor(ob, dtype=torch.float32)
    tp = torch.as_tensor(t_pdflat, dtype=torch.float32)
    dev = trainer.device
    if isinstance(trainer, DistillTrainer):
        _, s = trainer.forward(ob.reshape(-1, OBSPACE_SHAPE).to(dev), teacher=False)
    else:
        E = ob.shape[0]
        r = torch.zeros(E, EPISODE_STEPS) if rew is None else torch.as_tensor(rew, dtype=torch.float32)
        prev_t = torch.zeros_like(tp)
        prev_t[:, 1:] = tp[:, :-1]
        prev_r = torch.zeros(E, EPISODE_STEPS, 1)
        prev_r[:, 1:, 0] = r[:, :-1]
        s = trainer.forward(rows(ob, prev_t, prev_r).to(dev))
    d = s[:, :2].double().cpu() - tp.reshape(-1, 4)[:, :2].double()
    return float((d ** 2).mean())

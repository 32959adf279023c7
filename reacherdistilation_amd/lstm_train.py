"""The reference's LSTM distillation driver, ``lstm_train.train(train, restore)`` (reference
src/distilation/lstm_train.py:18-201), re-expressed over the MI355X path: the env is the HIP
Reacher-v2 (``make_mujoco_env``), the teacher query is ``rdd_forward``, and the student is
the reference's ``student_lstm_graph`` trained by the kernels behind ``StudentLstmTrainer``
on windows from the device-resident ``DeviceDataset``.

Phases as in the reference:
  1. (:114-135) the teacher steps the env until ``num_episodes() > 2 * LSTM_BATCH_SIZE``;
  2. (:139-201) per env step: one optimiser step on each [T, B] window from
     ``training_batches()`` (zero initial LSTM state, :159), teacher relabel of the current
     observation, the student's mean action from the test window's last output with the
     previous query's final state as initial state (:166-183), record with 's', env.step
     with the student action; episode boundaries reset the env and flush the dataset.

Fixes of the reference as committed: the test window's prev_pdflat column is
the per-step series (``DeviceDataset.test_windows``), not the single element that only
broadcasts at 0 or >= T-1 records.
"""
from __future__ import annotations


import torch

from .config import LSTM_BATCH_SIZE, MAX_CAPACITY, STEPS_UNROLLED, TOTAL_EPISODES
from .dataset import DeviceDataset
from .distill import DistillConfig, DistillTrainer
from .driver_env import DriverEnv, episode_loss
from .pages import PageStore
from .policy import TeacherAgent
from .student_lstm import StudentLstmConfig, StudentLstmTrainer


def _restore(st, restore: bool, path: str | None, log):
    """lstm_train.py:102-107: fresh variables unless restoring; a missing checkpoint only
    prints, as the reference does."""
    if not restore:
        return
    if path and st.checkpoint_exists(path):
        st.load(path)
    else:
        log("attempt to restore trained data but {0} does not exist".format(path))


def train(train: bool = True, restore: bool = False, *, episodes: int = TOTAL_EPISODES, loss: str = "kl",
          lr: float = 1e-3, keep_prob: float = 1.0, seed: int = 0, device="cuda:0", teacher_path: str | None = None,
          warmup_episodes: int = 2 * LSTM_BATCH_SIZE, student_path: str | None = None, log=print,
          gym_env: bool = False, store_dir: str | None = None, pool: str = "reference"):
    """Returns (student trainer, dataset, per-episode summed training loss).  ``store_dir``:
    the dataset's page directory (lstm_train.py:104-109); episodes are dumped to it every
    MAX_CAPACITY episodes (:200) and its stored pages join the training pool (dataset.py:
    164-177); ``pool="ring"`` draws windows uniformly from the device ring instead.  With
    ``student_path`` the student (params + Adam slots) is restored from it when ``restore``
    (lstm_train.py:102-107) and saved to it after every episode (:199).  Env I/O on the device
    (driver_env.DriverEnv; gym_env=True through the gym-API env), window losses read once per
    episode."""
    env = DriverEnv(seed, device, gym_api=gym_env)
    teacher = TeacherAgent(restore=teacher_path is not None, path=teacher_path)   # always restored (ref. :29)
    tq = DistillTrainer(DistillConfig(n_envs=64, seed=seed), device=device, teacher=teacher.pi)
    st = StudentLstmTrainer(StudentLstmConfig(loss=loss, lr=lr, keep_prob=keep_prob, seed=seed,
                                              steps=STEPS_UNROLLED, max_windows=LSTM_BATCH_SIZE), device=device)
    dataset = DeviceDataset(device=device, seed=seed, batch_size=LSTM_BATCH_SIZE, steps_unrolled=STEPS_UNROLLED,
                            store=PageStore(store_dir) if store_dir else None, pool=pool)
    _restore(st, restore, student_path, log)
    losses = []
    if not train:
        return st, dataset, losses
    ob = env.reset()
    reward = torch.zeros(1, device=env.device)

    def teacher_query(o):
        t, _ = tq.forward(o, student=False)
        return t[0]

    log("Begin Training! First Accumulate observation with teacher")
    while dataset.num_episodes() <= warmup_episodes:
        t_pdflat = teacher_query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, stepped_with="t")
        ob, reward, new = env.step(t_pdflat)
        if new:
            dataset.flush()
    log("Accumulated sufficient data points from teacher. now train")

    state = None   # curr_state_batch: zero at the start (lstm_train.py:88-89)
    opt_steps = 0
    while True:
        for ob_b, t_b, prev_b, _prew_b in dataset.training_batches():
            st.step(ob_b, prev_b, t_b)          # zero initial state (lstm_train.py:159)
            opt_steps += 1
        t_pdflat = teacher_query(ob)
        ob_w, prev_w, _ = dataset.test_windows(ob)
        out, state = st.forward(ob_w, prev_w, state)
        s_pdflat = out[STEPS_UNROLLED - 1, LSTM_BATCH_SIZE - 1].clone()
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, s_pdflat=s_pdflat, stepped_with="s")
        ob, reward, new = env.step(s_pdflat)
        if new:
            log("************** Episode {0} ****************".format(dataset.num_episodes()))
            total_loss = episode_loss(st.metrics(opt_steps)[:, 0] if opt_steps else [])
            log("recent loss: %f " % total_loss)
            losses.append(total_loss)
            opt_steps = 0
            dataset.flush()
            if dataset.store is not None and dataset.num_episodes() % MAX_CAPACITY == 0:
                dataset.dump()          # lstm_train.py:200
            if student_path:
                st.save(student_path)   # saver.save every episode (lstm_train.py:199)
            if dataset.num_episodes() >= episodes:
                break
    return st, dataset, losses


def train_bptt(train: bool = True, restore: bool = False, *, episodes: int = TOTAL_EPISODES, loss: str = "kl",
               lr: float = 1e-3, keep_prob: float = 1.0, seed: int = 0, device="cuda:0", teacher_path: str | None = None,
               warmup_episodes: int = 2 * LSTM_BATCH_SIZE, student_path: str | None = None, log=print,
               gym_env: bool = False, store_dir: str | None = None, pool: str = "reference"):
    """The truncated-BPTT variant of the driver (reference backup/lstm_bbpt.py:18-208), same
    graph, loss and Adam.  After the teacher warm-up (:115-139) each round is
      * one BPTT pass (:141-158): ``dataset.bptt_batches()`` -- LSTM_BATCH_SIZE episodes, the
        40 windows that slide by one step -- one Adam step per window, the LSTM state carried
        from window to window (the step's final_state_batch becomes the next window's
        initial_state_batch; zero at the start of the pass);
      * then one whole episode stepped by the student (:160-205): teacher relabel, the test
        window's query with the carried query state, record with 's', env.step(student mean).
    Returns (student trainer, dataset, per-episode summed training loss).  Env I/O as in
    train()."""
    env = DriverEnv(seed, device, gym_api=gym_env)
    teacher = TeacherAgent(restore=teacher_path is not None, path=teacher_path)   # always restored (ref. :29)
    tq = DistillTrainer(DistillConfig(n_envs=64, seed=seed), device=device, teacher=teacher.pi)
    st = StudentLstmTrainer(StudentLstmConfig(loss=loss, lr=lr, keep_prob=keep_prob, seed=seed,
                                              steps=STEPS_UNROLLED, max_windows=LSTM_BATCH_SIZE), device=device)
    dataset = DeviceDataset(device=device, seed=seed, batch_size=LSTM_BATCH_SIZE, steps_unrolled=STEPS_UNROLLED,
                            store=PageStore(store_dir) if store_dir else None, pool=pool)
    _restore(st, restore, student_path, log)
    losses = []
    if not train:
        return st, dataset, losses
    ob = env.reset()
    reward = torch.zeros(1, device=env.device)

    def teacher_query(o):
        t, _ = tq.forward(o, student=False)
        return t[0]

    log("Begin Training! First Accumulate observation with teacher")
    while dataset.num_episodes() <= warmup_episodes:
        t_pdflat = teacher_query(ob)
        dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, stepped_with="t")
        ob, reward, new = env.step(t_pdflat)
        if new:
            dataset.flush()
    log("Accumulated sufficient data points from teacher. now train")

    query_state = None   # curr_state_batch (lstm_bbpt.py:94)
    while True:
        s = None         # zero_state_batch at the start of each pass (:142)
        opt_steps = 0
        for ob_b, t_b, prev_b, _prew_b in dataset.bptt_batches():
            st.step(ob_b, prev_b, t_b, state0=s)
            s = st.final_state(LSTM_BATCH_SIZE)
            opt_steps += 1
        total_loss = episode_loss(st.metrics(opt_steps)[:, 0] if opt_steps else [])
        new = False
        while not new:
            t_pdflat = teacher_query(ob)
            ob_w, prev_w, _ = dataset.test_windows(ob)
            out, query_state = st.forward(ob_w, prev_w, query_state)
            s_pdflat = out[STEPS_UNROLLED - 1, LSTM_BATCH_SIZE - 1].clone()
            dataset.write(ob=ob, reward=reward, t_pdflat=t_pdflat, s_pdflat=s_pdflat, stepped_with="s")
            ob, reward, new = env.step(s_pdflat)
        log("************** Episode {0} ****************".format(dataset.num_episodes()))
        log("recent loss: %f " % total_loss)
        losses.append(total_loss)
        dataset.flush()
        if dataset.store is not None and dataset.num_episodes() % MAX_CAPACITY == 0:
            dataset.dump()              # backup/lstm_bbpt.py:207
        if student_path:
            st.save(student_path)
        if dataset.num_episodes() >= episodes:
            break
    return st, dataset, losses

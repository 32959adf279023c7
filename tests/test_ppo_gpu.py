"""GPU parity of the PPO teacher trainer (csrc/ppo.hip) against oracle/ppo_np.py.

The actor batch is checked record by record: value predictions (f32 MLP vs f64: 2e-5 +
1e-4 rel), actions = mean + exp(logstd) * the Box-Muller normal of the documented Philox
words (1e-5 + 1e-4 rel), rewards from the record's own observation (the stale-fingertip
reward -|tip - target| - |a|^2, 1e-5), episode-start flags, GAE (1e-4 rel of max|adv|); the
observation filter's moments; the full-batch minibatch gradient (relative L2 < 1e-3; ratios
straddle the clip range after one update) and learning.
"""
import numpy as np
import pytest
import torch

from oracle import ppo_np as pp
from oracle.refnet_np import M32, philox4x32_10

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainer(**kw):
    from reacherdistilation_amd.ppo import PPOConfig, PPOTrainer
    cfg = dict(n_envs=256, horizon=64, seed=11, optim_batchsize=0, optim_epochs=1, max_timesteps=10 ** 6)
    cfg.update(kw)
    return PPOTrainer(PPOConfig(**cfg), device=DEV)


def _normals(seed, n, it, T):
    gid = np.arange(n, dtype=np.uint64)
    out = np.zeros((T, n, 2))
    for t in range(T):
        w = philox4x32_10([gid & M32, gid >> np.uint64(32), np.full(n, it, np.uint64), np.full(n, t, np.uint64)],
                          seed & 0xFFFFFFFF, (seed >> 32) ^ 0xA5A5A5A5)
        u1 = ((w[0] >> np.uint32(8)).astype(np.float64) + 1) / 16777216.0
        u2 = (w[1] >> np.uint32(8)).astype(np.float64) / 16777216.0
        rad = np.sqrt(-2 * np.log(u1))
        out[t, :, 0] = rad * np.cos(2 * np.pi * u2)
        out[t, :, 1] = rad * np.sin(2 * np.pi * u2)
    return out


def test_actor_batch_matches_oracle():
    tr = _trainer()
    n, T = 256, 64
    pol, vf = tr.policy().cpu().numpy(), tr.value().cpu().numpy()
    tr.rollout()
    b = {k: v.cpu().numpy().astype(np.float64) for k, v in tr.batch().items()}
    ob = b["ob"].reshape(T * n, 11)
    z = pp.obz(ob, np.zeros(11), np.ones(11))          # initial filter: mean 0, std 1
    fv = pp.vf_forward(vf, z)
    np.testing.assert_allclose(b["vpred"].reshape(-1), fv["v"], atol=2e-5, rtol=1e-4)
    fp = pp.pol_forward(pol, z)
    want_ac = fp["mean"] + np.exp(fp["logstd"]) * _normals(11, n, 0, T).reshape(T * n, 2)
    np.testing.assert_allclose(b["ac"].reshape(T * n, 2), want_ac, atol=1e-5, rtol=1e-4)
    rew = -np.sqrt(ob[:, 8] ** 2 + ob[:, 9] ** 2) - (b["ac"].reshape(-1, 2) ** 2).sum(1)
    np.testing.assert_allclose(b["rew"].reshape(-1), rew, atol=1e-5)
    new = np.zeros((T, n))
    new[0] = 1
    new[50] = 1                                          # every env's first episode ends at step 50
    np.testing.assert_array_equal(b["new"], new)
    adv, ret = pp.gae(b["rew"], b["vpred"], b["new"], b["nextvpred"], 0.99, 0.95)
    np.testing.assert_allclose(b["adv"], adv, atol=1e-4 * np.abs(adv).max())
    np.testing.assert_allclose(b["ret"], ret, atol=1e-4 * np.abs(ret).max())
    # the filter now holds the batch's moments (RunningMeanStd from count 1e-2)
    rms = pp.RunningMeanStd()
    rms.update(ob)
    mean, std = (x.cpu().numpy() for x in tr.obfilter())
    np.testing.assert_allclose(mean, rms.mean, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(std, rms.std, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("n,T", [(256, 64), (255, 63), (1, 50), (3, 7)])
def test_full_batch_gradient_matches_oracle(n, T):
    """One minibatch over the whole actor batch: 512 / 503 32-row tiles (more than the 256
    workgroups of minibatch_kernel, so workgroups carry sums over several tiles; 255 x 63 ends
    in a ragged tile), and 2 / 1 tiles (50 and 21 rows: padded rows must add nothing)."""
    tr = _trainer(n_envs=n, horizon=T, optim_epochs=1, optim_batchsize=0)
    tr.iterate()                                         # one update: the policy moves off the rollout policy
    pol, vf = tr.policy().cpu().numpy(), tr.value().cpu().numpy()
    mean0, std0 = (x.cpu().numpy().astype(np.float64) for x in tr.obfilter())
    tr.rollout()
    b = {k: v.cpu().numpy().astype(np.float64) for k, v in tr.batch().items()}
    mean1, std1 = (x.cpu().numpy().astype(np.float64) for x in tr.obfilter())
    assert not np.allclose(mean0, mean1)
    ob = b["ob"].reshape(-1, 11)
    z = pp.obz(ob, mean1, std1)
    a = b["ac"].reshape(-1, 2)
    fp = pp.pol_forward(pol, z)
    lpo = pp.logp(fp["mean"], fp["logstd"], a)
    atarg = pp.standardize(b["adv"].reshape(-1))
    lrmult = 1.0 - tr.S / 10 ** 6
    tr.optimize()
    g = tr.grad().cpu().numpy().astype(np.float64)
    # first minibatch of the epoch: old == current parameters, ratio = 1 (inside the clip)
    r = pp.loss_and_grads(pol, vf, z, a, lpo, atarg, b["ret"].reshape(-1), 0.2 * lrmult)
    want = np.concatenate([r["gpol"], r["gvf"]])
    rel = np.linalg.norm(g - want) / np.linalg.norm(want)
    assert rel < 1e-3, rel
    m = tr.metrics(1)[0]
    assert abs(m[2] - r["pol_surr"]) < 1e-4 and abs(m[3] - r["vf_loss"]) <= 1e-4 * r["vf_loss"] + 1e-5
    assert m[6] == pytest.approx(lrmult, rel=1e-6)


def test_clipped_branch_gradient_matches_oracle():
    """Two minibatch steps on the same full batch: the second sees ratios != 1, some outside
    the clip range; its gradient must follow TF's min/clip conventions."""
    tr = _trainer(optim_epochs=2, optim_batchsize=0, optim_stepsize=3e-3)
    tr.rollout()
    pol0 = tr.policy().cpu().numpy()
    b = {k: v.cpu().numpy().astype(np.float64) for k, v in tr.batch().items()}
    mean1, std1 = (x.cpu().numpy().astype(np.float64) for x in tr.obfilter())
    z = pp.obz(b["ob"].reshape(-1, 11), mean1, std1)
    a = b["ac"].reshape(-1, 2)
    fp0 = pp.pol_forward(pol0, z)
    lpo = pp.logp(fp0["mean"], fp0["logstd"], a)
    atarg = pp.standardize(b["adv"].reshape(-1))
    # run epoch 1 through a separate trainer copy is not possible; emulate: optimize with 2
    # epochs, then rebuild epoch 2's gradient from the parameters after epoch 1 (the Adam
    # step of epoch 1 is reproduced on device: read params after a 1-epoch optimize)
    tr1 = _trainer(optim_epochs=1, optim_batchsize=0, optim_stepsize=3e-3)
    tr1.rollout()
    tr1.optimize()
    pol1, vf1 = tr1.policy().cpu().numpy(), tr1.value().cpu().numpy()
    tr.optimize()
    g = tr.grad().cpu().numpy().astype(np.float64)
    r = pp.loss_and_grads(pol1, vf1, z, a, lpo, atarg, b["ret"].reshape(-1), 0.2 * (1.0 - tr.S / 10 ** 6))
    clipped = np.abs(r["ratio"] - 1) > 0.2 * (1.0 - tr.S / 10 ** 6)
    assert clipped.any()
    want = np.concatenate([r["gpol"], r["gvf"]])
    rel = np.linalg.norm(g - want) / np.linalg.norm(want)
    assert rel < 2e-3, rel


def test_ppo_improves_the_return():
    tr = _trainer(n_envs=1024, horizon=50, optim_batchsize=4096, optim_epochs=10, max_timesteps=3 * 10 ** 6)
    for _ in range(25):
        tr.iterate()
    m = tr.metrics(25)
    assert np.all(np.isfinite(m))
    first, last = m[:3, 0].mean(), m[-3:, 0].mean()
    assert last > first + 3.0, (first, last)
    assert np.all(np.diff(m[:, 7]) == 1024 * 50)         # timesteps advance by the actor batch
    teacher = tr.teacher()
    assert teacher.flat.shape == (5060,) and np.all(teacher.ob_std > 0)


def test_trained_teacher_plugs_into_distillation():
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    tr = _trainer(n_envs=128, horizon=50)
    tr.iterate()
    d = DistillTrainer(DistillConfig(n_envs=1024), device=DEV, teacher=tr.teacher())
    d.step()
    assert np.isfinite(d.metrics(1)).all()


def test_two_trainers_are_bitwise_equal():
    """Same config and seed: the actor batch, the parameters after two iterations (ragged
    minibatch tiles: 1,000 rows) and the metrics are bitwise equal (fixed-order sums only)."""
    runs = []
    for _ in range(2):
        tr = _trainer(n_envs=500, horizon=50, optim_batchsize=1000, optim_epochs=2)
        for _ in range(2):
            tr.iterate()
        runs.append((tr.policy().cpu(), tr.value().cpu(), tr.batch()["vpred"].cpu(), tr.metrics(2)))
    (p0, v0, b0, m0), (p1, v1, b1, m1) = runs
    assert torch.equal(p0, p1) and torch.equal(v0, v1) and torch.equal(b0, b1)
    np.testing.assert_array_equal(m0, m1)


def test_committed_ppo_teacher_reaches_the_reference_teachers_return():
    """the teacher PPO-trained with the reference's hyperparameters
    (scripts/train_ppo_teacher.py, profiles/r06_ppo_teacher.json) and committed as the reference
    Saver's scope-'pi' checkpoint restores through TeacherAgent, and its mean action's 50-step
    return on 512 fresh gym-seeded episodes is at least the reference teacher's -7.53 (fixture)."""
    from reacherdistilation_amd.policy import TeacherAgent
    from reacherdistilation_amd.teacher import PPO_TEACHER, episode_returns, ppo_teacher
    p = ppo_teacher()
    q = TeacherAgent(restore=True, path=PPO_TEACHER).pi
    assert np.array_equal(p.flat, q.flat) and p.flat.shape == (5060,)
    r = episode_returns(p, 512, seed=31, device=DEV)
    assert r.mean() >= -7.53, r.mean()

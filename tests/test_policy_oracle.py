"""The policy/loss/Adam oracles checked against each other and against finite differences.

Parity of this part is UNPINNED by the reference (TF/baselines absent, no reference test
covers it): these tests pin the restatement to the formulas of
reference loss.py:3-13 (KL(s||t) summed), baselines' MlpPolicy/DiagGaussianPd, and TF1's
ApplyAdam functor.
"""
import numpy as np
import pytest

from oracle import policy_np as pn
from oracle import reacher_np as rn


def _params(seed, out_std=1.0, ls=(0.0, 0.0)):
    rng = np.random.RandomState(seed)
    W1 = pn.normc(rng, (11, 64), 1.0); W2 = pn.normc(rng, (64, 64), 1.0); W3 = pn.normc(rng, (64, 2), out_std)
    b1 = rng.uniform(-.1, .1, 64); b2 = rng.uniform(-.1, .1, 64); b3 = rng.uniform(-.1, .1, 2)
    return pn.pack(W1, b1, W2, b2, W3, b3, np.asarray(ls)).astype(np.float64)


def _obs(n, seed=0):
    rs = np.random.RandomState(seed)
    q = rs.uniform(-3, 3, (n, 2)); v = rs.uniform(-5, 5, (n, 2)); t = rs.uniform(-.2, .2, (n, 2))
    fx, fy = rn.fingertip(q[:, 0], q[:, 1])
    return rn.observe(q[:, 0], q[:, 1], v[:, 0], v[:, 1], t[:, 0], t[:, 1], q[:, 0], q[:, 1])


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_gradient_matches_finite_differences(loss):
    sp = _params(2, 0.01, (-0.5, -0.7))
    tp = _params(1, 1.0, (-3.29, -3.36))
    mu, sd = np.zeros(11), np.ones(11)
    ob = _obs(64)
    fs, ft = pn.forward(sp, mu, sd, ob), pn.forward(tp, mu, sd, ob)
    _, dmean, dls, _ = pn.loss_and_dmean(fs, ft, loss, 64)
    g = pn.backward(sp, fs, dmean, dls)
    rs = np.random.RandomState(0)
    idx = np.concatenate([rs.choice(pn.P_TOT - 4, 60, replace=False), np.arange(pn.P_TOT - 4, pn.P_TOT)])
    for i in idx:
        e = np.zeros(pn.P_TOT); e[i] = 1e-6
        num = (pn.loss_fn(sp + e, mu, sd, tp, mu, sd, ob, loss, 64) -
               pn.loss_fn(sp - e, mu, sd, tp, mu, sd, ob, loss, 64)) / 2e-6
        assert abs(num - g[i]) <= 1e-6 + 1e-4 * abs(g[i]), (i, num, g[i])


def test_kl_matches_reference_formula():
    """loss.py:11-13: sum over [T,B,2] of t.logstd - s.logstd + (s.std^2 + (s.mean-t.mean)^2)
    / (2 t.std^2) - 0.5, with DiagGaussianPd std = exp(logstd)."""
    rs = np.random.RandomState(1)
    ms, mt = rs.randn(7, 2), rs.randn(7, 2)
    ls, lt = rs.randn(2) * .3, rs.randn(2) * .3
    ref = (lt - ls + (np.exp(ls) ** 2 + (ms - mt) ** 2) / (2 * np.exp(lt) ** 2) - 0.5).sum()
    kl, _, _, _ = pn.loss_and_dmean(dict(mean=ms, logstd=ls), dict(mean=mt, logstd=lt), "kl", 7)
    assert abs(kl - ref) < 1e-12


def test_adam_tf1_first_steps():
    """TF1 Adam: the first update is lr*sqrt(1-b2)/(1-b1) * g/(sqrt((1-b2) g^2)+eps) ~ lr*sign(g)."""
    opt = pn.AdamTF1(3, lr=1e-3, dtype=np.float64)
    x = np.zeros(3)
    g = np.array([2.0, -0.5, 0.0])
    opt.step(x, g)
    assert np.allclose(x, [-1e-3, 1e-3, 0.0], atol=1e-9)
    assert opt.b1p == pytest.approx(0.81) and opt.b2p == pytest.approx(0.998001)


def test_adam_c_matches_numpy(oracle_c):
    rs = np.random.RandomState(2)
    th = rs.randn(100).astype(np.float32)
    th_c = th.copy(); m = np.zeros(100, np.float32); v = np.zeros(100, np.float32)
    opt = pn.AdamTF1(100)
    for k in range(5):
        g = rs.randn(100).astype(np.float32)
        oracle_c.adam_tf1(th_c, m, v, g, float(opt.b1p), float(opt.b2p))
        opt.step(th, g)
    assert np.allclose(th, th_c, atol=1e-7, rtol=0)


@pytest.mark.parametrize("loss,act", [("mse", False), ("kl", False), ("mse", True)])
def test_c_distill_step_matches_numpy(oracle_c, loss, act):
    """The C f32 distill step (grad + env transition) vs the f64 numpy oracle."""
    n, seed = 300, 4
    tp = _params(1, 1.0, (-3.29, -3.36)).astype(np.float32)
    sp = _params(2, 0.01, (-0.2, 0.1)).astype(np.float32)
    mu, sd = np.zeros(11, np.float32), np.ones(11, np.float32)
    st = oracle_c.philox_reset(n, 0, seed, 0)
    st64 = st.astype(np.float64)
    ob = rn.observe(st64[0], st64[1], st64[2], st64[3], st64[4], st64[5], 0 * st64[0], 0 * st64[0])
    ob[:, 8], ob[:, 9] = st64[6], st64[7]
    g, met = oracle_c.distill_step(st, 7, (tp, mu, sd), (sp, mu, sd), seed=seed, loss=loss, act_student=act,
                                   nthreads=2)
    fs, ft = pn.forward(sp.astype(np.float64), mu, sd, ob), pn.forward(tp.astype(np.float64), mu, sd, ob)
    L, dmean, dls, sq = pn.loss_and_dmean(fs, ft, loss, n)
    g64 = pn.backward(sp.astype(np.float64), fs, dmean, dls)
    assert np.abs(g - g64).max() <= 1e-5 * np.abs(g64).max() + 1e-7
    assert met[1] == pytest.approx(L, rel=1e-4)
    assert met[2] == pytest.approx(sq, rel=1e-4)
    # env transition with the chosen action
    a = (fs if act else ft)["mean"].astype(np.float32)
    ref = np.ascontiguousarray(st64.copy())
    oracle_c.step(ref, a, np.float64)
    assert np.abs(st - ref).max() < 5e-4

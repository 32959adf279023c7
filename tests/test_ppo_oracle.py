"""CPU checks of the PPO oracle (oracle/ppo_np.py): the clipped-surrogate + value loss
gradient by finite differences (ratios inside and outside the clip range), GAE against its
definition, RunningMeanStd's moments.  Parity of PPO itself is UNPINNED by the reference
(baselines/TF absent, no reference test): these pin the restatement to the formulas."""
import numpy as np
import pytest

from oracle import policy_np as pn
from oracle import ppo_np as pp


def _nets(seed=0):
    rs = np.random.RandomState(seed)
    pol = np.concatenate([pn.normc(rs, (11, 64), 1.0).ravel(), rs.uniform(-.1, .1, 64),
                          pn.normc(rs, (64, 64), 1.0).ravel(), rs.uniform(-.1, .1, 64),
                          pn.normc(rs, (64, 2), 0.5).ravel(), rs.uniform(-.1, .1, 2), [-0.3, 0.2]])
    vf = np.concatenate([pn.normc(rs, (11, 64), 1.0).ravel(), rs.uniform(-.1, .1, 64),
                         pn.normc(rs, (64, 64), 1.0).ravel(), rs.uniform(-.1, .1, 64),
                         pn.normc(rs, (64, 1), 1.0).ravel(), [0.05]])
    assert pol.size == pp.P_POL and vf.size == pp.P_VF
    return pol, vf


def _batch(n, pol, seed=1, spread=0.6):
    rs = np.random.RandomState(seed)
    z = rs.uniform(-2, 2, (n, 11))
    fp = pp.pol_forward(pol, z)
    a = fp["mean"] + np.exp(fp["logstd"]) * rs.randn(n, 2)
    # old log-probs spread so that ratios fall inside and outside [1 - e, 1 + e]
    logp_old = pp.logp(fp["mean"], fp["logstd"], a) + rs.uniform(-spread, spread, n)
    return z, a, logp_old, rs.randn(n), rs.randn(n)


@pytest.mark.parametrize("seed", [0, 1])
def test_gradient_matches_finite_differences(seed):
    pol, vf = _nets(seed)
    z, a, lpo, atarg, ret = _batch(40, pol, seed + 5)
    r = pp.loss_and_grads(pol, vf, z, a, lpo, atarg, ret, 0.2)
    inside = (r["ratio"] > 0.8) & (r["ratio"] < 1.2)
    assert 0 < inside.sum() < 40        # both branches exercised
    g = np.concatenate([r["gpol"], r["gvf"]])
    x = np.concatenate([pol, vf])
    rs = np.random.RandomState(3)
    idx = list(rs.choice(x.size, 40, replace=False)) + [pp.P_POL - 1, pp.P_POL - 2, pp.P_POL - 3, x.size - 1]
    h = 1e-6
    for k in idx:
        xp, xm = x.copy(), x.copy()
        xp[k] += h
        xm[k] -= h
        fp_ = pp.total_loss(xp[:pp.P_POL], xp[pp.P_POL:], z, a, lpo, atarg, ret, 0.2)
        fm_ = pp.total_loss(xm[:pp.P_POL], xm[pp.P_POL:], z, a, lpo, atarg, ret, 0.2)
        num = (fp_ - fm_) / (2 * h)
        assert abs(num - g[k]) <= 1e-6 + 1e-5 * abs(num), (k, num, g[k])


def test_gae_matches_definition():
    rs = np.random.RandomState(2)
    T, N = 7, 3
    rew, v = rs.randn(T, N), rs.randn(T, N)
    new = np.zeros((T, N))
    new[3, 0] = 1
    new[0, :] = 1
    nv = rs.randn(N)
    adv, ret = pp.gae(rew, v, new, nv, 0.9, 0.8)
    for n in range(N):
        for t in range(T):
            # sum over l of (gamma lam)^l delta_{t+l} until the episode ends
            acc, coef = 0.0, 1.0
            for u in range(t, T):
                nxt_new = new[u + 1, n] if u + 1 < T else 0.0
                vnext = v[u + 1, n] if u + 1 < T else nv[n]
                delta = rew[u, n] + 0.9 * vnext * (1 - nxt_new) - v[u, n]
                acc += coef * delta
                if nxt_new:
                    break
                coef *= 0.9 * 0.8
            assert abs(adv[t, n] - acc) < 1e-12
    np.testing.assert_allclose(ret, adv + v)


def test_running_mean_std():
    rms = pp.RunningMeanStd()
    rs = np.random.RandomState(0)
    x = rs.randn(1000, 11) * 3 + 1
    rms.update(x[:400])
    rms.update(x[400:])
    c = 1000 + 1e-2
    np.testing.assert_allclose(rms.mean, x.sum(0) / c)
    np.testing.assert_allclose(rms.std, np.sqrt((1e-2 + (x ** 2).sum(0)) / c - (x.sum(0) / c) ** 2))

"""CPU mutation test of the round-4 parity checks: each tightened check
rejects ONE wrong env in lanes 48-63, and the round-3 check it replaces did not.

The "kernel result" is the oracle's own gradient carried through f32 (a faithful stand-in for
a correct kernel at f32 rounding); the mutations are the failure class the suite missed in
r03w -- a value lost for the lanes 48-63 of a wave:
  * env: one env of lanes 48-63 of its 64-env group loses its whole contribution
    (a lost per-lane load in the producer: its observation, action or loss);
  * lane group: one 16-env tile loses its contribution to the output rows 12-15 of every
    16x16 block of dW3 (a lost SrcC load in an MFMA's last row group);
  * state: one env of lanes 48-63 ends its step with one velocity off by 1e-4 (a lost
    register in the physics).
"""
import numpy as np
import pytest

from oracle import policy_np as pn
from tests import parity


def _batch(n, seed=0):
    from reacherdistilation_amd.policy import student_init, synthetic_teacher
    t, s = synthetic_teacher(1), student_init(2)
    rs = np.random.RandomState(seed)
    q0, q1 = rs.uniform(-3, 3, n), rs.uniform(-2.5, 2.5, n)
    ob = np.stack([np.cos(q0), np.cos(q1), np.sin(q0), np.sin(q1), rs.uniform(-.2, .2, n), rs.uniform(-.2, .2, n),
                   rs.uniform(-5, 5, n), rs.uniform(-5, 5, n), rs.uniform(-.3, .3, n), rs.uniform(-.3, .3, n),
                   np.zeros(n)], 1)
    return t, s, ob


def _old_check(g, g64):
    return np.abs(g - g64).max() / np.abs(g64).max() < 2e-4


def _contrib(s, fs, dmean, rows):
    sp = s.flat.astype(np.float64)
    f = {k: (v[rows] if getattr(v, "ndim", 0) == 2 else v) for k, v in fs.items()}
    return pn.backward(sp, f, dmean[rows], np.zeros(2))


@pytest.mark.parametrize("n", [64, 128, 4096, 65536])
@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_gradient_checks_reject_one_wrong_env_or_lane_group(n, loss):
    t, s, ob = _batch(n)
    g64, M, (fs, ft, L, sq) = parity.oracle_grad(s.flat, t, s, ob, loss, n)
    g32 = g64.astype(np.float32)
    ok, rep = parity.grad_ok(g32, g64, M)
    assert ok, rep                                  # a correct f32 result passes
    _, dmean, _, _ = pn.loss_and_dmean(fs, ft, loss, n)
    # one env in lanes 48-63 of a group loses its contribution: rejected by the per-entry check
    # at every size here (at 65,536 envs one env is ~2.5e-5 of its entries' scale)
    for e in (48, 55, 63):
        bad = (g64 - _contrib(s, fs, dmean, [e])).astype(np.float32)
        assert not parity.grad_ok(bad, g64, M)[0], (n, e)
    # one tile's lanes 48-63 (output rows 12-15 of every 16x16 block of dW3) lose its contribution
    ct = _contrib(s, fs, dmean, list(range(min(n, 64) - 16, min(n, 64))))
    f = np.arange(64)[np.arange(64) % 16 >= 12]
    mask = np.zeros(pn.P_TOT, bool)
    mask[pn.P_W3 + 2 * f] = mask[pn.P_W3 + 2 * f + 1] = True
    bad = (g64 - np.where(mask, ct, 0.0)).astype(np.float32)
    assert not parity.grad_ok(bad, g64, M)[0]
    if n >= 65536:   # the round-3 bound saw neither at the c3 size
        assert _old_check((g64 - _contrib(s, fs, dmean, [50])).astype(np.float32), g64)
        if loss == "kl":
            assert _old_check(bad, g64)


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_env_isolation_rejects_a_wrong_lane(loss):
    """The per-env isolation of tests/test_distill_gpu.py at 64 envs: env e's contribution
    c(x_e) - c(z) recovered from two f32 batch gradients passes its bound when correct and fails
    when env e's output rows 12-15 of dW3 and dW2 (its lanes 48-63) are lost."""
    n = 64
    t, s, ob = _batch(n, 3)
    z = ob[0].copy()
    z[:4] = np.cos(0.3), np.cos(-0.2), np.sin(0.3), np.sin(-0.2)
    g_all, M_all, (fs, ft, _, _) = parity.oracle_grad(s.flat, t, s, ob, loss, n)
    _, Mz, _ = parity.oracle_grad(s.flat, t, s, z[None], loss, n)
    _, dmean, _, _ = pn.loss_and_dmean(fs, ft, loss, n)
    f = np.arange(64)[np.arange(64) % 16 >= 12]
    lanes = np.zeros(pn.P_TOT, bool)
    lanes[pn.P_W3 + 2 * f] = lanes[pn.P_W3 + 2 * f + 1] = True
    for k in f:
        lanes[pn.P_W2 + np.arange(64) * 64 + k] = True
    for e in range(48, 64):
        obe = ob.copy()
        obe[e] = z
        g_e, M_e, _ = parity.oracle_grad(s.flat, t, s, obe, loss, n)
        _, Mx, _ = parity.oracle_grad(s.flat, t, s, ob[e:e + 1], loss, n)
        bound = 1e-5 * (Mx + Mz) + 5e-6 * np.maximum(M_all, M_e)
        d64 = g_all - g_e
        d_f32 = g_all.astype(np.float32).astype(np.float64) - g_e.astype(np.float32).astype(np.float64)
        assert (np.abs(d_f32 - d64) <= bound).all()
        ce = _contrib(s, fs, dmean, [e])
        d_bad = d_f32 - np.where(lanes, ce, 0.0)
        assert (np.abs(d_bad - d64) > bound).any(), e


def test_state_check_rejects_one_wrong_velocity():
    """Per-component env-state bounds: a 1e-4 error in one velocity of one env in lanes 48-63
    fails them; the round-3 bound (3e-4 + 1e-4 rel) let it pass."""
    rs = np.random.RandomState(1)
    n = 4096
    ref = np.stack([rs.uniform(-3, 3, n), rs.uniform(-2.5, 2.5, n), rs.uniform(-5, 5, n), rs.uniform(-5, 5, n),
                    rs.uniform(-.2, .2, n), rs.uniform(-.2, .2, n), rs.uniform(-.3, .3, n), rs.uniform(-.3, .3, n)])
    ref[4:6] = ref[4:6].astype(np.float32)     # targets: f32 values the step keeps
    st = ref.astype(np.float32).astype(np.float64)
    active = np.zeros(n, bool)
    assert parity.state_ok(st, ref, active)[0]
    for e in (48, 63, 64 * 7 + 50):
        bad = st.copy()
        bad[3, e] += 1e-4
        assert not parity.state_ok(bad, ref, active)[0]
        assert np.isclose(bad, ref, atol=3e-4, rtol=1e-4).all()

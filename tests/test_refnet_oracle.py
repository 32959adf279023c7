"""CPU checks of the reference-student oracle (oracle/refnet_np.py): layout, backward vs
finite differences for both losses, and the numpy Philox restatement vs the C oracle's
(the same Philox4x32-10 the env resets use, pinned there by the reset tests).

Parity of the reference student's math is UNPINNED by the reference itself (TensorFlow is
absent and no reference test covers student_mlp_graph): the formulas of student_nn.py:51-57
and loss.py:3-13 are checked here by finite differences.
"""
import numpy as np
import pytest

from oracle import refnet_np as rn


def _batch(n, seed=0):
    rs = np.random.RandomState(seed)
    x = rs.uniform(-1, 1, (n, 16)).astype(np.float32)
    t = np.concatenate([rs.uniform(-.5, .5, (n, 2)), rs.uniform(-1.0, -0.2, (n, 2))], 1).astype(np.float32)
    return x, t


def test_layout_matches_reference_graph():
    assert rn.P_REF == 24380
    dims = [(a, b) for (_, _, a, b) in rn.LAYOUT]
    assert dims == [(16, 24), (24, 128), (128, 128), (128, 32), (32, 4)]
    p = rn.init(3)
    for (w, bo, a, b) in rn.LAYOUT:
        lim = np.sqrt(6.0 / (a + b))
        assert np.abs(p[w:bo]).max() <= lim and np.all(p[bo:bo + b] == 0)


def test_student_logstd_is_state_dependent():
    p = rn.init(1)
    x, _ = _batch(4)
    out = rn.forward(p, x)["pdflat"]
    assert out.shape == (4, 4) and np.ptp(out[:, 2]) > 0


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_backward_matches_finite_differences(loss):
    p = rn.init(5).astype(np.float64)
    rs = np.random.RandomState(1)
    for (w, bo, a, b) in rn.LAYOUT:   # non-zero biases so their gradients are exercised
        p[bo:bo + b] = rs.uniform(-.1, .1, b)
    x, t = _batch(7, 2)
    fw = rn.forward(p, x)
    _, d, _ = rn.loss_and_dout(fw["pdflat"], t, loss, 7)
    g = rn.backward(p, fw, d)
    idx = np.concatenate([rs.choice(rn.P_REF, 40, replace=False),
                          [bo for (_, bo, _, _) in rn.LAYOUT], [rn.P_REF - 1]])
    h = 1e-6
    for k in idx:
        pp, pm = p.copy(), p.copy()
        pp[k] += h
        pm[k] -= h
        num = (rn.loss_fn(pp, x, t, loss, 7) - rn.loss_fn(pm, x, t, loss, 7)) / (2 * h)
        assert abs(num - g[k]) <= 1e-6 + 1e-5 * abs(num), (k, num, g[k])


def test_kl_is_zero_at_the_target_and_positive_elsewhere():
    t = np.array([[0.1, -0.2, -1.0, -0.5]])
    kl, d, _ = rn.loss_and_dout(t.copy(), t, "kl", 1)
    assert abs(kl) < 1e-12 and np.abs(d).max() < 1e-12
    kl2, _, _ = rn.loss_and_dout(t + 0.1, t, "kl", 1)
    assert kl2 > 0


def test_numpy_philox_matches_the_c_oracle(oracle_c):
    """Philox4x32-10 restated in numpy == the C oracle's (whose draws pin the env resets)."""
    seed, ids, episode = 0x123456789ABCDEF, np.arange(5, dtype=np.uint64) * 977 + 3, 7
    want = oracle_c.philox_draws(seed, ids, episode)
    for q, lo, scale in ((0, (0, 4), (0.2, 0.2, 0.01, 0.01)), (1, (4, 6), (0.4, 0.4))):
        w = rn.philox4x32_10([ids & rn.M32, ids >> np.uint64(32), np.full(5, episode, np.uint64),
                              np.full(5, q, np.uint64)], seed & 0xFFFFFFFF, seed >> 32)
        u = (w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        for k, s in enumerate(scale):
            got = np.float32(s) * u[k] - np.float32(s / 2)
            np.testing.assert_allclose(got, want[:, lo[0] + k], atol=1e-7)


def test_dropout_mask_statistics_and_scaling():
    x = np.ones((4000, 16), np.float32)
    y = rn.dropout(x, 0.5, seed=11, step=3)
    kept = y[:, :11] != 0
    assert abs(kept.mean() - 0.5) < 0.02
    assert np.all(y[:, :11][kept] == 2.0) and np.all(y[:, 11:] == 1.0)
    assert not np.array_equal(y, rn.dropout(x, 0.5, seed=11, step=4))
    assert np.array_equal(rn.dropout(x, 1.0, 11, 3), x)
    # row_base shifts the key: rows [10, 20) of a batch == a batch starting at row 10
    np.testing.assert_array_equal(rn.dropout(x[:20], 0.5, 11, 3)[10:20], rn.dropout(x[:10], 0.5, 11, 3, row_base=10))

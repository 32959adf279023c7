"""CPU checks of the LSTM-student oracle (oracle/lstm_np.py): layout, TF1 LSTMCell gate
algebra, BPTT backward vs finite differences (both losses), dropout keying.

Parity of the LSTM math is UNPINNED by the reference (TensorFlow is absent and no reference
test covers student_lstm_graph); the formulas of student_nn.py:21-49 / TF1 LSTMCell
(i, j, f, o split, forget_bias 1) are pinned here by finite differences.
"""
import numpy as np
import pytest

from oracle import lstm_np as ln


def _batch(T, B, seed=0):
    rs = np.random.RandomState(seed)
    ob = rs.uniform(-1, 1, (T, B, 11))
    prev = rs.uniform(-1, 1, (T, B, 4))
    t = np.concatenate([rs.uniform(-.5, .5, (T, B, 2)), rs.uniform(-1.0, -0.2, (T, B, 2))], 2)
    return ob, prev, t


def test_layout():
    """One head per unrolled step (the reference's tf.layers.dense calls inside its loop over
    the T steps create new variables each time, student_nn.py:40-47): 195,360 shared + 31,652
    per step, 511,880 at the reference's T = 10; the ABI's RDL_PARAMS_T agrees."""
    assert ln.P_LSTM == 511880 and ln.CELL_PARAMS == 195360 and ln.HEAD_PARAMS == 31652
    o, s = ln.LAYOUT["Wl"]
    assert s == (243, 800) and o == 4 * 32 + 32
    lay, n = ln.layout(3)
    assert n == 195360 + 3 * 31652 and lay["h0/W1"][0] == 195360 and lay["h2/b5"][0] == n - 4
    import re as _re
    from tests.conftest import ROOT
    import os
    hdr = open(os.path.join(ROOT, "include", "reacher_student_lstm.h")).read()
    assert int(_re.search(r"#define RDL_CELL_PARAMS (\d+)", hdr).group(1)) == ln.CELL_PARAMS
    assert int(_re.search(r"#define RDL_HEAD_PARAMS (\d+)", hdr).group(1)) == ln.HEAD_PARAMS


def test_each_step_has_its_own_head():
    """Changing step 1's head changes only step 1's output (the reference's per-step dense
    variables), while the cell is shared by every step."""
    T, B = 3, 2
    p = ln.init(2, T)
    ob, prev, _ = _batch(T, B, 1)
    y0 = ln.forward(p, ob, prev)["pdflat"]
    lay, _ = ln.layout(T)
    q = p.copy()
    o, s = lay["h1/W5"]
    q[o:o + s[0] * s[1]] += 0.5
    y1 = ln.forward(q, ob, prev)["pdflat"]
    assert np.array_equal(y0[0], y1[0]) and np.array_equal(y0[2], y1[2]) and not np.allclose(y0[1], y1[1])


def test_cell_matches_hand_computation():
    p = ln.init(1)
    W = ln.unpack(p)
    ob, prev, _ = _batch(1, 2)
    fw = ln.forward(p, ob, prev)
    x = np.concatenate([ob[0], prev[0] @ W["Wp"] + W["bp"]], 1)
    z = np.concatenate([x, np.zeros((2, 200))], 1) @ W["Wl"] + W["bl"]
    i, j, f, o = z[:, :200], z[:, 200:400], z[:, 400:600], z[:, 600:]
    c = ln.sig(i) * np.tanh(j)          # c_prev = 0
    h = ln.sig(o) * np.tanh(c)
    np.testing.assert_allclose(fw["state"][0], c, rtol=1e-12)
    np.testing.assert_allclose(fw["state"][1], h, rtol=1e-12)


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_bptt_matches_finite_differences(loss):
    rs = np.random.RandomState(4)
    T, B = 4, 3
    lay, n = ln.layout(T)
    p = ln.init(5, T).astype(np.float64)
    for k, (o, s) in lay.items():
        if len(s) == 1:
            p[o:o + s[0]] = rs.uniform(-.2, .2, s[0])
    ob, prev, t = _batch(T, B, 2)
    fw = ln.forward(p, ob, prev)
    _, d, _ = ln.loss_and_dout(fw["pdflat"], t, loss, T * B)
    g = ln.backward(p, fw, d)
    idx = list(rs.choice(n, 40, replace=False))
    for name in ("Wp", "bp", "bl", "h0/b1", "h0/b5", "h3/W1", "h2/b5"):
        idx.append(lay[name][0])
    o = lay["Wl"][0]
    idx += [o + 5 * 800 + 3, o + 100 * 800 + 250, o + 242 * 800 + 799, o + 42 * 800 + 420]   # x and h rows, all gates
    h = 1e-6
    for k in idx:
        pp, pm = p.copy(), p.copy()
        pp[k] += h
        pm[k] -= h
        num = (ln.loss_fn(pp, ob, prev, t, loss, T * B) - ln.loss_fn(pm, ob, prev, t, loss, T * B)) / (2 * h)
        assert abs(num - g[k]) <= 1e-6 + 1e-5 * abs(num), (k, num, g[k])


def test_dropout_keys_each_step_and_row():
    ob = np.ones((3, 50, 11), np.float32)
    y = ln.dropout(ob, 0.5, 9, 2)
    assert not np.array_equal(y[0], y[1])
    assert abs((y != 0).mean() - 0.5) < 0.05
    np.testing.assert_array_equal(ln.dropout(ob[:, :20], 0.5, 9, 2)[:, 10:20], ln.dropout(ob[:, :10], 0.5, 9, 2, 10))

"""ORACLE (test infrastructure only) -- numpy f64 restatement of the reference's LSTM student
and its truncated-BPTT training step.

  student_lstm_graph (reference student_nn.py:21-49), unrolled over T = STEPS_UNROLLED:
      p_t = prev_pdflat_t . Wp + bp                              (dense 4 -> 32, linear)
      x_t = [dropout(ob_t) (11), p_t (32)]                       (43)
      z_t = [x_t, h_{t-1}] . Wl + bl  -> i, j, f, o              (TF1 LSTMCell, 200 units,
      c_t = sig(f + 1) c_{t-1} + sig(i) tanh(j)                   forget_bias 1, no peepholes,
      h_t = sig(o) tanh(c_t)                                      no projection)
      y_t = dense(tanh dense 32 (tanh dense 64 (tanh dense 128 (tanh dense 64 (h_t))))) (4)
            with step t's OWN head: the reference calls tf.layers.dense inside its Python loop
            over the T steps without reuse (student_nn.py:40-47), so every call creates new
            variables (dense_1 .. dense_5T); the LSTMCell object and the prev dense are shared
  loss: kl_loss (loss.py:3-13, summed over T and B) or MSE; Adam lr 1e-3 (lstm_train.py:75-80).
  Flat parameters in the variables' creation order (lstm_train.py:53 builds the graph):
      Wp[4][32] bp[32] | Wl[243][800] bl[800] | head_0 | ... | head_{T-1},
      head_t = W1[200][64] b1 | W2[64][128] b2 | W3[128][64] b3 | W4[64][32] b4 | W5[32][4] b5
      = 195,360 + 31,652 T floats (511,880 at the reference's T = 10)
  Dropout mask on ob (tf.nn.dropout, keep_prob): Philox4x32-10 keyed like the MLP student's
  (refnet_np.dropout) with counter word 3 = 4 t + q, so the oracle reproduces it exactly.

Parity status: the cell (forward), its constants and the kl loss gradient are pinned to the
reference's logged GraphDef; the backward's building blocks -- bptt / cell_backward (the
cell's generated BPTT over T = 2 steps), refnet_np.dense_backward, tanh_grad -- are pinned to
the graph's own TF-generated gradients of all 30 ApplyAdam inputs (tests/test_graph_pins.py);
this 200-unit composition is checked by finite differences in tests/test_lstm_oracle.py.
"""
from __future__ import annotations

import numpy as np

from oracle.refnet_np import M32, dense_backward, philox4x32_10, tanh_grad

UNITS = 200
IN_X = 11 + 32
HEAD = (UNITS, 64, 128, 64, 32, 4)


CELL_PARAMS = 4 * 32 + 32 + (IN_X + UNITS) * 4 * UNITS + 4 * UNITS          # 195,360
HEAD_PARAMS = sum(a * b + b for a, b in zip(HEAD[:-1], HEAD[1:]))            # 31,652


def layout(T=10):
    """name -> (offset, shape) in the flat vector; head t's layers are "h{t}/W1" .. "h{t}/b5"."""
    shapes = [("Wp", (4, 32)), ("bp", (32,)), ("Wl", (IN_X + UNITS, 4 * UNITS)), ("bl", (4 * UNITS,))]
    for t in range(T):
        for k, (a, b) in enumerate(zip(HEAD[:-1], HEAD[1:])):
            shapes += [(f"h{t}/W{k + 1}", (a, b)), (f"h{t}/b{k + 1}", (b,))]
    out, off = {}, 0
    for name, shp in shapes:
        out[name] = (off, shp)
        off += int(np.prod(shp))
    return out, off


LAYOUT, P_LSTM = layout()   # 511,880 at T = 10


def steps_of(p):
    """T of a flat parameter vector (its number of heads)."""
    t, r = divmod(np.asarray(p).size - CELL_PARAMS, HEAD_PARAMS)
    assert r == 0 and t > 0, "not an LSTM student parameter vector"
    return t


def unpack(p):
    p = np.asarray(p, np.float64)
    lay, _ = layout(steps_of(p))
    return {k: p[o:o + int(np.prod(s))].reshape(s) for k, (o, s) in lay.items()}


def init(seed=3, T=10):
    """glorot_uniform kernels (tf.layers.dense / LSTMCell defaults), zero biases."""
    rng = np.random.RandomState(seed)
    lay, n = layout(T)
    p = np.zeros(n, np.float32)
    for k, (o, s) in lay.items():
        if len(s) == 2:
            lim = np.sqrt(6.0 / (s[0] + s[1]))
            p[o:o + s[0] * s[1]] = rng.uniform(-lim, lim, s[0] * s[1]).astype(np.float32)
    return p


def dropout(ob, keep_prob, seed, step, row_base=0):
    """ob [T, B, 11] f32 -> dropped f32 (mask word k%4 of Philox(ctr = {b lo, b hi, step,
    4 t + k/4}, key = seed), keep iff u < keep_prob, kept values / keep_prob)."""
    ob = np.array(ob, np.float32)
    if keep_prob >= 1.0:
        return ob
    T, B, _ = ob.shape
    rows = np.arange(B, dtype=np.uint64) + np.uint64(row_base)
    kp = np.float32(keep_prob)
    for t in range(T):
        for q in range(3):
            w = philox4x32_10([rows & M32, rows >> np.uint64(32), np.full(B, step, np.uint64),
                               np.full(B, 4 * t + q, np.uint64)], seed & 0xFFFFFFFF, seed >> 32)
            u = (w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            for k in range(4):
                col = 4 * q + k
                if col < 11:
                    ob[t, :, col] = np.where(u[k] < kp, ob[t, :, col] / kp, np.float32(0.0))
    return ob


def sig(x):
    return 1.0 / (1.0 + np.exp(-x))


FORGET_BIAS = 1.0   # TF1 LSTMCell default (LSTM/unique_lstm_cell/add/y in the reference graph)


def cell(x, c, h, Wl, bl):
    """One TF1 LSTMCell step: z = [x, h] Wl + bl split (i, j, f, o);
    c' = sig(f + forget_bias) c + sig(i) tanh(j); h' = sig(o) tanh(c').  Returns
    (c', h', (sig i, tanh j, sig(f + 1), sig o))."""
    z = np.concatenate([x, h], 1) @ Wl + bl
    i, j, f, o = np.split(z, 4, axis=1)
    gi, gj, gf, go = sig(i), np.tanh(j), sig(f + FORGET_BIAS), sig(o)
    c = gf * c + gi * gj
    return c, go * np.tanh(c), (gi, gj, gf, go)


def forward(p, ob, prev, state0=None):
    """ob [T,B,11] (already dropped), prev [T,B,4] -> dict with pdflat [T,B,4] and caches."""
    W = unpack(p)
    ob = np.asarray(ob, np.float64)
    prev = np.asarray(prev, np.float64)
    T, B, _ = ob.shape
    c = np.zeros((B, UNITS)) if state0 is None else np.asarray(state0[0], np.float64)
    h = np.zeros((B, UNITS)) if state0 is None else np.asarray(state0[1], np.float64)
    cache = dict(x=[], hprev=[], cprev=[], gi=[], gj=[], gf=[], go=[], c=[], h=[], acts=[])
    ys = []
    for t in range(T):
        pt = prev[t] @ W["Wp"] + W["bp"]
        x = np.concatenate([ob[t], pt], 1)
        cache["x"].append(x); cache["hprev"].append(h); cache["cprev"].append(c)
        c, h, (gi, gj, gf, go) = cell(x, c, h, W["Wl"], W["bl"])
        for k, v in (("gi", gi), ("gj", gj), ("gf", gf), ("go", go), ("c", c), ("h", h)):
            cache[k].append(v)
        a = [h]
        for k in range(1, 5):
            a.append(np.tanh(a[-1] @ W[f"h{t}/W{k}"] + W[f"h{t}/b{k}"]))
        ys.append(a[-1] @ W[f"h{t}/W5"] + W[f"h{t}/b5"])
        cache["acts"].append(a)
    return dict(pdflat=np.stack(ys), state=(c, h), cache=cache, prev=prev)


def loss_and_dout(pdflat, t_pdflat, loss, n_global):
    """Summed over T and B (KL) or MSE over n_global rows; pdflat [T,B,4]."""
    from oracle.refnet_np import loss_and_dout as lo
    T, B, _ = pdflat.shape
    L, d, sq = lo(pdflat.reshape(T * B, 4), np.asarray(t_pdflat).reshape(T * B, 4), loss, n_global)
    return L, d.reshape(T, B, 4), sq


def cell_backward(s, dh, dc_next):
    """Backward of one TF1 LSTMCell step (the cell's generated gradient ops: TanhGrad,
    SigmoidGrad, the f + forget_bias Add, Split_grad = concat of the gate gradients).
    s: that step's cache (gi, gj, gf, go = the gate activations, c = c_t, cprev = c_{t-1});
    dh: dL/dh_t (all consumers), dc_next: dL/dc_t from step t+1.
    Returns (dz [B, 4U] in (i, j, f, o) order, dc_prev = dL/dc_{t-1} through this step)."""
    gi, gj, gf, go = s["gi"], s["gj"], s["gf"], s["go"]
    tc = np.tanh(s["c"])
    dc = dh * go * (1 - tc ** 2) + dc_next
    dzo = dh * tc * go * (1 - go)
    dzi = dc * gj * gi * (1 - gi)
    dzj = dc * gi * (1 - gj ** 2)
    dzf = dc * s["cprev"] * gf * (1 - gf)
    return np.concatenate([dzi, dzj, dzf, dzo], 1), dc * gf


def bptt(steps, Wl, dh_out):
    """Back-propagation through time of the TF1 LSTMCell over T steps: steps[t] = the cache of
    step t (x, hprev, cprev, gates, c), dh_out[t] = dL/dh_t from the step's non-recurrent
    consumers (the head).  Returns (dWl, dbl, [dL/dx_t], dL/dc_0, dL/dh_0): the cell kernel's
    gradient is the sum over steps of [x_t, h_{t-1}]^T dz_t (TF: MatMul_grad per step, AddN),
    its bias's the sum of dz_t (BiasAddGrad, AddN).  Pinned to the reference graph's own
    generated BPTT (adam/gradients/AddN_6, AddN_7; tests/test_graph_pins.py)."""
    T = len(steps)
    nx = steps[0]["x"].shape[1]
    dWl, dbl = np.zeros_like(Wl), np.zeros(Wl.shape[1])
    dxs = [None] * T
    dh_next = np.zeros_like(np.asarray(steps[-1]["hprev"], np.float64))
    dc_next = np.zeros_like(dh_next)
    for t in range(T - 1, -1, -1):
        s = steps[t]
        dz, dc_next = cell_backward(s, dh_out[t] + dh_next, dc_next)
        xin = np.concatenate([s["x"], s["hprev"]], 1)
        dW, db, dxin = dense_backward(xin, dz, Wl)
        dWl += dW
        dbl += db
        dxs[t], dh_next = dxin[:, :nx], dxin[:, nx:]
    return dWl, dbl, dxs, dc_next, dh_next


def backward(p, fw, dout):
    W = unpack(p)
    lay, _ = layout(steps_of(p))
    g = {k: np.zeros(s) for k, (_, s) in lay.items()}
    C = fw["cache"]
    T = len(C["x"])
    dh_out = []
    for t in range(T):   # step t's own head (no recurrence through it)
        a = C["acts"][t]
        gW, gb, da = dense_backward(a[4], dout[t], W[f"h{t}/W5"])
        g[f"h{t}/W5"] += gW
        g[f"h{t}/b5"] += gb
        for k in range(4, 0, -1):
            gW, gb, da = dense_backward(a[k - 1], tanh_grad(a[k], da), W[f"h{t}/W{k}"])
            g[f"h{t}/W{k}"] += gW
            g[f"h{t}/b{k}"] += gb
        dh_out.append(da)
    steps = [dict(x=C["x"][t], hprev=C["hprev"][t], cprev=C["cprev"][t], gi=C["gi"][t], gj=C["gj"][t],
                  gf=C["gf"][t], go=C["go"][t], c=C["c"][t]) for t in range(T)]
    g["Wl"], g["bl"], dxs, _, _ = bptt(steps, W["Wl"], dh_out)
    for t in range(T):   # the prev_pdflat projection feeds x_t[11:43]
        gW, gb, _ = dense_backward(fw["prev"][t], dxs[t][:, 11:IN_X], W["Wp"])
        g["Wp"] += gW
        g["bp"] += gb
    return np.concatenate([g[k].ravel() for k in lay])


def loss_fn(p, ob, prev, t_pdflat, loss, n_global):
    return loss_and_dout(forward(p, ob, prev)["pdflat"], t_pdflat, loss, n_global)[0]

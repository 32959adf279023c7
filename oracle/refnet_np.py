"""ORACLE (test infrastructure only) -- numpy restatement of the reference's own MLP student
and its training step.

  student_mlp_graph (reference student_nn.py:51-57): input 16 = dropout(ob)[11] |
      prev_pdflat[4] | prev_rew[1] (mlp_train.py:38-52; dropout keep_prob = 1 here) ->
      dense 24 tanh -> dense 128 tanh -> dense 128 (linear) -> dense 32 tanh -> dense 4
      (pdflat = mean[2] | logstd[2], a state-dependent log-std);  tf.layers.dense kernels
      glorot_uniform, biases zero.
  kl_loss (reference loss.py:3-13): sum over rows and action dims of KL(s||t);
  MSE: mean over [n_global, 2] of (mu_s - mu_t)^2 / 2 (the BASELINE action-MSE, as the
      2x64 path defines it: dL/dmu = (mu_s - mu_t) / n_global).
  Adam: the TF1 form, policy_np.AdamTF1.

  dropout (tf.nn.dropout on the 11 ob inputs, mlp_train.py:50, KEEP_PROB config.py:30):
      the mask is the counter-based draw include/reacher_student_mlp.h defines (Philox4x32-10,
      Salmon et al. SC'11, restated here in numpy), so the oracle reproduces it exactly; TF's
      own RNG stream cannot be matched and is not claimed.

Parity status: the graph of student_nn.py:51-57 is not in the reference's logged GraphDefs,
but every piece of this backward is: the dense layer's MatMul_grad / BiasAddGrad
(dense_backward), TanhGrad (tanh_grad) and the kl loss gradient are pinned to the TF-generated
gradients of the logged LSTM student graph (tests/test_graph_pins.py);
the composition is checked against finite differences in tests/test_refnet_oracle.py.
"""
from __future__ import annotations

import numpy as np

DIMS = (16, 24, 128, 128, 32, 4)
ACT = (True, True, False, True, False)   # tanh after layers 1, 2, 4


def layout():
    """[(W offset, b offset, in, out)] of the flat parameter vector (W row-major [in][out])."""
    out, off = [], 0
    for a, b in zip(DIMS[:-1], DIMS[1:]):
        out.append((off, off + a * b, a, b))
        off += a * b + b
    return out, off


LAYOUT, P_REF = layout()   # P_REF = 24,380


def unpack(p):
    return [(p[w:bo].reshape(a, b), p[bo:bo + b]) for (w, bo, a, b) in LAYOUT]


def init(seed=2):
    """tf.layers.dense defaults: glorot_uniform kernels, zero biases."""
    rng = np.random.RandomState(seed)
    p = np.zeros(P_REF, np.float32)
    for (w, bo, a, b) in LAYOUT:
        lim = np.sqrt(6.0 / (a + b))
        p[w:bo] = rng.uniform(-lim, lim, a * b).astype(np.float32)
    return p


M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c, k0, k1):
    """c: uint32 [4, n] counters; k0, k1: key words.  Returns uint32 [4, n]."""
    c = [np.asarray(v, np.uint64) & M32 for v in c]
    k0, k1 = np.uint64(k0) & M32, np.uint64(k1) & M32
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        hi0, lo0, hi1, lo1 = p0 >> np.uint64(32), p0 & M32, p1 >> np.uint64(32), p1 & M32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return np.stack(c).astype(np.uint32)


def apply_mask(x, u, kp):
    """tf.nn.dropout's scale with our keep rule: x / kp where u < kp, else 0.  TF keeps
    where floor(kp + U) = 1, i.e. U >= 1 - kp: the same rule with u = 1 - U (pinned
    against the reference graph's LSTM/dropout ops by tests/test_graph_pins.py)."""
    return np.where(u < kp, x / kp, np.float32(0.0)).astype(np.float32)


def dropout(x, keep_prob, seed, step, row_base=0):
    """Training-time input dropout of rows x [n,16] (f32), columns 0..10 only."""
    x = np.array(x, np.float32)
    if keep_prob >= 1.0:
        return x
    n = x.shape[0]
    rows = np.arange(n, dtype=np.uint64) + np.uint64(row_base)
    kp = np.float32(keep_prob)
    for q in range(3):
        w = philox4x32_10([rows & M32, rows >> np.uint64(32), np.full(n, step, np.uint64),
                           np.full(n, q, np.uint64)], seed & 0xFFFFFFFF, seed >> 32)
        u = (w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        for k in range(4):
            col = 4 * q + k
            if col < 11:
                x[:, col] = apply_mask(x[:, col], u[k], kp)
    return x


def forward(p, x):
    """x [n,16] -> dict(hs=[h0..h5], pdflat [n,4])."""
    hs = [np.asarray(x, np.float64)]
    for (W, b), act in zip(unpack(np.asarray(p, np.float64)), ACT):
        z = hs[-1] @ W + b
        hs.append(np.tanh(z) if act else z)
    return dict(hs=hs, pdflat=hs[-1])


def loss_and_dout(pdflat, t_pdflat, loss, n_global):
    """Returns (loss, dL/dpdflat [n,4], sum sq mean error)."""
    ms, ls = pdflat[:, :2], pdflat[:, 2:]
    t = np.asarray(t_pdflat, np.float64)
    mt, lt = t[:, :2], t[:, 2:]
    diff = ms - mt
    sq = float((diff ** 2).sum())
    d = np.zeros_like(pdflat)
    if loss == "mse":
        d[:, :2] = diff / n_global
        return sq / (2.0 * n_global), d, sq
    vt, vs = np.exp(2 * lt), np.exp(2 * ls)
    kl = float((lt - ls + (vs + diff ** 2) / (2 * vt) - 0.5).sum())
    d[:, :2] = diff / vt
    d[:, 2:] = vs / vt - 1.0
    return kl, d, sq


def tanh_grad(y, dy):
    """TF's TanhGrad(y, dy) = dy (1 - y^2), from the layer's OUTPUT y (the op the reference's
    generated backward uses after every tanh layer; pinned by tests/test_graph_pins.py)."""
    return dy * (1.0 - y * y)


def dense_backward(a_in, dz, W):
    """Backward of a tf.layers.dense layer z = a_in W + b, as TF generates it: MatMul_grad
    (dW = a_in^T dz, da_in = dz W^T) and BiasAddGrad (db = dz summed over rows).  The
    building block of every oracle backward here (refnet_np, policy_np, lstm_np), pinned to
    the reference graph's adam/gradients/* by tests/test_graph_pins.py.
    Returns (dW, db, da_in)."""
    return a_in.T @ dz, dz.reshape(-1, dz.shape[-1]).sum(0), dz @ W.T


def backward(p, fw, dout):
    Ws = unpack(np.asarray(p, np.float64))
    hs = fw["hs"]
    g = [None] * len(Ws)
    dz = dout
    for li in range(len(Ws) - 1, -1, -1):
        W, _ = Ws[li]
        gw, gb, dh = dense_backward(hs[li], dz, W)
        g[li] = (gw, gb)
        if li > 0:
            dz = tanh_grad(hs[li], dh) if ACT[li - 1] else dh
    return np.concatenate([np.concatenate([gw.ravel(), gb]) for gw, gb in g])


def loss_fn(p, x, t_pdflat, loss, n_global):
    return loss_and_dout(forward(p, x)["pdflat"], t_pdflat, loss, n_global)[0]

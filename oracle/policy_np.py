"""ORACLE (test infrastructure only) -- numpy restatement of the policy side of the hot path.

  teacher query  baselines ppo1 MlpPolicy(hid_size=64, num_hid_layers=2) pol branch
                 (reference teacher.py:14-16; queried at mlp_train.py:123-125,165-167):
                 obz = clip((ob - mean) / std, -5, 5); h1 = tanh(obz W1 + b1);
                 h2 = tanh(h1 W2 + b2); mean = h2 W3 + b3; pdflat = [mean, logstd]
  student        the same 2x64 MlpPolicy structure (BASELINE configs 2-5; reference
                 backup/student_rollout.py:79-87 StudentAgent), logstd trainable
  loss           kl_loss (reference loss.py:3-13): sum over envs and action dims of
                 KL(s||t) = lt - ls + (es^2 + (ms - mt)^2) / (2 et^2) - 1/2, or the BASELINE
                 action-MSE mean((ms - mt)^2) over [N, 2]
  optimiser      tf.train.AdamOptimizer(1e-4, .9, .999, 1e-8) (reference mlp_train.py:73-80),
                 TF1 ApplyAdam functor: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
                 var -= m * lr*sqrt(1 - b2^t)/(1 - b1^t) / (sqrt(v) + eps), with
                 beta1_power/beta2_power float32 variables multiplied once per step.

Parity status: PINNED to the reference's own GraphDefs (src/~/reacher/data/viz/1 event
files, parsed and evaluated by oracle/tfgraph.py; goldens tests/golden/graph_golden.npz):
the MlpPolicy forward incl. the observation filter (pi/pol/concat on the teacher's own
initial weights and on seeded weights), the kl loss and TF's gradient of it, the Adam
constants and beta-power schedule (tests/test_graph_pins.py).  The backward is built from
refnet_np.dense_backward / tanh_grad, which are pinned to the TF-generated gradients of the
logged LSTM graph (adam/gradients/*: MatMul_grad, BiasAddGrad, TanhGrad), and is checked
against finite differences of the pinned forward (tests/test_policy_oracle.py).
TensorFlow/baselines themselves are not installed.
"""
from __future__ import annotations

import numpy as np

OBD, HID, ACD = 11, 64, 2
# flat parameter layout (shared with the HIP kernel and the C oracle)
P_W1 = 0
P_B1 = P_W1 + OBD * HID
P_W2 = P_B1 + HID
P_B2 = P_W2 + HID * HID
P_W3 = P_B2 + HID
P_B3 = P_W3 + HID * ACD
P_LS = P_B3 + ACD
P_TOT = P_LS + ACD  # 5060


# baselines RunningMeanStd as the reference's GraphDef computes it (pi/obfilter: count and
# runningsumsq start at 1e-2, runningsum at 0, sums in f64; the floor is on the VARIANCE,
# Maximum/y = 1e-2); pinned by tests/test_graph_pins.py against the graph itself
OBF_COUNT0, OBF_SUMSQ0, OB_CLIP = 1e-2, 1e-2, 5.0
OBF_VAR_FLOOR = float(np.float32(1e-2))   # a float32 Const in the graph


def obfilter(runningsum, runningsumsq, count):
    """(mean, std) of the observation filter from its running sums (pi/obfilter/*)."""
    mean = np.asarray(runningsum, np.float64) / count
    var = np.asarray(runningsumsq, np.float64) / count - mean ** 2
    return mean, np.sqrt(np.maximum(var, OBF_VAR_FLOOR))


def unpack(p):
    return dict(W1=p[P_W1:P_B1].reshape(OBD, HID), b1=p[P_B1:P_W2], W2=p[P_W2:P_B2].reshape(HID, HID),
                b2=p[P_B2:P_W3], W3=p[P_W3:P_B3].reshape(HID, ACD), b3=p[P_B3:P_LS], ls=p[P_LS:P_TOT])


def pack(W1, b1, W2, b2, W3, b3, ls):
    return np.concatenate([np.ravel(x) for x in (W1, b1, W2, b2, W3, b3, ls)])


def forward(p, obmu, obsd, ob):
    """ob [N,11] -> dict(z, h1, h2, mean [N,2], logstd [2])."""
    q = unpack(p)
    z = np.clip((ob - obmu) / obsd, -OB_CLIP, OB_CLIP)
    h1 = np.tanh(z @ q["W1"] + q["b1"])
    h2 = np.tanh(h1 @ q["W2"] + q["b2"])
    mean = h2 @ q["W3"] + q["b3"]
    return dict(z=z, h1=h1, h2=h2, mean=mean, logstd=q["ls"])


def bf16(x):
    """Round to the nearest bf16 (ties to even), returned as float64 values.  The kernel's
    v_cvt_pk_bf16_f32 rounds this way (include/reacher_distill.h RDD_DTYPE_BF16)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def forward_bf16(p, obmu, obsd, ob):
    """The bf16-student forward (RDD_DTYPE_BF16): weight matrices and the MFMA operands z, h1
    rounded to bf16; biases, tanh, layer-3 inputs (h2) and accumulations in f32 (f64 here).
    z is formed in f32 exactly as the kernel does ((ob - mu) * (1/sd), clipped)."""
    q = unpack(p)
    ob32 = np.asarray(ob, np.float32)
    rs = (np.float32(1) / np.asarray(obsd, np.float32)).astype(np.float32)
    z = np.clip((ob32 - np.asarray(obmu, np.float32)) * rs, np.float32(-5), np.float32(5)).astype(np.float32)
    zb = bf16(z)
    h1 = np.tanh(zb @ bf16(q["W1"]) + q["b1"])
    h2 = np.tanh(bf16(h1) @ bf16(q["W2"]) + q["b2"])
    mean = h2 @ bf16(q["W3"]) + q["b3"]
    return dict(z=z.astype(np.float64), zb=zb, h1=h1, h2=h2, mean=mean, logstd=q["ls"])


def backward_bf16(p, fs, dmean, dls):
    """Gradients of the bf16 student as the kernel forms them: dZ2 = (W3b dmean)(1 - h2^2);
    dW2 = bf16(h1)^T bf16(dZ2); db2 = sum dZ2; dH1 = bf16(W2) bf16(dZ2); dZ1 = dH1 (1 - h1^2);
    dW1 = bf16(z)^T bf16(dZ1); db1 = sum bf16(dZ1) (the bias row of the same product)."""
    q = unpack(p)
    g = dict(W3=fs["h2"].T @ dmean, b3=dmean.sum(0), ls=np.asarray(dls, np.float64))
    dz2 = (dmean @ bf16(q["W3"]).T) * (1 - fs["h2"] ** 2)
    dz2b = bf16(dz2)
    g["W2"] = bf16(fs["h1"]).T @ dz2b
    g["b2"] = dz2.sum(0)
    dz1 = (dz2b @ bf16(q["W2"]).T) * (1 - fs["h1"] ** 2)
    dz1b = bf16(dz1)
    g["W1"] = fs["zb"].T @ dz1b
    g["b1"] = dz1b.sum(0)
    return pack(g["W1"], g["b1"], g["W2"], g["b2"], g["W3"], g["b3"], g["ls"])


def loss_and_dmean(fs, ft, loss, n_global):
    """Returns (loss, dL/dmean_s [N,2], dL/dlogstd_s [2], sum sq action error)."""
    diff = fs["mean"] - ft["mean"]
    sq = float((diff ** 2).sum())
    if loss == "mse":
        return sq / (2.0 * n_global), diff / n_global, np.zeros(ACD), sq
    lt, ls = ft["logstd"], fs["logstd"]
    vt, vs = np.exp(2 * lt), np.exp(2 * ls)
    kl = (lt - ls + (vs + diff ** 2) / (2 * vt) - 0.5).sum()
    dls = (vs / vt - 1.0) * diff.shape[0]
    return float(kl), diff / vt, dls, sq


def backward(p, fs, dmean, dls):
    """The MlpPolicy backward from the pinned building blocks (refnet_np.dense_backward =
    TF's MatMul_grad + BiasAddGrad, refnet_np.tanh_grad = TanhGrad)."""
    from oracle.refnet_np import dense_backward, tanh_grad
    q = unpack(p)
    g = dict(ls=np.asarray(dls, np.float64))
    g["W3"], g["b3"], dh2 = dense_backward(fs["h2"], dmean, q["W3"])
    g["W2"], g["b2"], dh1 = dense_backward(fs["h1"], tanh_grad(fs["h2"], dh2), q["W2"])
    g["W1"], g["b1"], _ = dense_backward(fs["z"], tanh_grad(fs["h1"], dh1), q["W1"])
    return pack(g["W1"], g["b1"], g["W2"], g["b2"], g["W3"], g["b3"], g["ls"])


def loss_fn(sp, smu, ssd, tp, tmu, tsd, ob, loss, n_global):
    fs, ft = forward(sp, smu, ssd, ob), forward(tp, tmu, tsd, ob)
    return loss_and_dmean(fs, ft, loss, n_global)[0]


class AdamTF1:
    """tf.train.AdamOptimizer as the reference builds it (mlp_train.py:73-80)."""

    def __init__(self, n, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8, dtype=np.float32):
        self.lr, self.b1, self.b2, self.eps = dtype(lr), dtype(b1), dtype(b2), dtype(eps)
        self.m = np.zeros(n, dtype)
        self.v = np.zeros(n, dtype)
        self.b1p, self.b2p = dtype(b1), dtype(b2)   # beta powers start at beta (t = 1)
        self.dtype = dtype
        self.t = 0

    def step(self, var, g):
        d = self.dtype
        g = g.astype(d)
        one = d(1)
        alpha = self.lr * np.sqrt(one - self.b2p) / (one - self.b1p)
        self.m += (g - self.m) * (one - self.b1)
        self.v += (g * g - self.v) * (one - self.b2)
        var -= (self.m * alpha) / (np.sqrt(self.v) + self.eps)
        self.b1p = d(self.b1p * self.b1)
        self.b2p = d(self.b2p * self.b2)
        self.t += 1
        return var


def normc(rng, shape, std):
    """baselines.common.tf_util.normc_initializer."""
    out = rng.standard_normal(shape).astype(np.float32)
    out *= std / np.sqrt(np.square(out).sum(axis=0, keepdims=True))
    return out

"""ORACLE (test infrastructure only) -- numpy restatement of the reference teacher's PPO
training (reference teacher.py:23-37: baselines ppo1 ``pposgd_simple.learn`` with
MlpPolicy(hid_size=64, num_hid_layers=2), timesteps_per_actorbatch 2048, clip 0.2,
entcoeff 0, optim_epochs 10, optim_stepsize 3e-4, optim_batchsize 64, gamma 0.99,
lam 0.95, schedule 'linear').

baselines (commit 3900f2a, not in /root/reference; restated from its published algorithm):
  * MlpPolicy: obfilter = RunningMeanStd(sum, sumsq, count; count starts at 1e-2; std =
    sqrt(max(sumsq/count - mean^2, 1e-2))); obz = clip((ob - mean)/std, -5, 5); value net
    vf: 2 x 64 tanh + dense 1; policy pol: 2 x 64 tanh + dense 2 (mean) + free logstd[2].
  * add_vtarg_and_adv: GAE(lambda) with `new` flags (first step of an episode) and the
    bootstrap value of the observation after the segment (0 if it starts an episode).
  * loss: ratio = exp(logp - logp_old); pol_surr = -mean(min(ratio A, clip(ratio, 1 - e,
    1 + e) A)), e = clip_param * lrmult; vf_loss = mean((V - ret)^2); A standardized over
    the actor batch; entcoeff 0.  TF gradient conventions: min() passes to its first
    argument on ties; clip passes inside the closed interval.
  * MpiAdam (epsilon 1e-5, learn()'s adam_epsilon default): the TF1 form (a = lr sqrt(1 -
    b2^t) / (1 - b1^t), eps outside the sqrt) on the
    concatenated trainable vector [pol | vf] with stepsize optim_stepsize * lrmult,
    lrmult = max(1 - timesteps_so_far / max_timesteps, 0).
Parameter vectors here: pol = the 5,060-float MlpPolicy layout of policy_np (W1 b1 W2 b2
W3 b3 logstd); vf = V1[11][64] c1 V2[64][64] c2 V3[64][1] c3 (4,993 floats).

Parity status: UNPINNED beyond the formulas (TensorFlow/baselines absent; no reference test
covers PPO); checked by finite differences in tests/test_ppo_oracle.py.
"""
from __future__ import annotations

import numpy as np

OBD, HID = 11, 64
P_POL = OBD * HID + HID + HID * HID + HID + HID * 2 + 2 + 2     # 5060
P_VF = OBD * HID + HID + HID * HID + HID + HID + 1              # 4993
LOG2PI = np.log(2 * np.pi)


def unpack_pol(p):
    p = np.asarray(p, np.float64)
    o = 0
    out = []
    for shp in ((OBD, HID), (HID,), (HID, HID), (HID,), (HID, 2), (2,), (2,)):
        n = int(np.prod(shp))
        out.append(p[o:o + n].reshape(shp))
        o += n
    return out


def unpack_vf(p):
    p = np.asarray(p, np.float64)
    o = 0
    out = []
    for shp in ((OBD, HID), (HID,), (HID, HID), (HID,), (HID, 1), (1,)):
        n = int(np.prod(shp))
        out.append(p[o:o + n].reshape(shp))
        o += n
    return out


class RunningMeanStd:
    """baselines.common.mpi_running_mean_std.RunningMeanStd (float64 sums)."""

    def __init__(self, shape=(OBD,), epsilon=1e-2):
        self.sum = np.zeros(shape)
        self.sumsq = np.full(shape, epsilon)
        self.count = epsilon

    @property
    def mean(self):
        return self.sum / self.count

    @property
    def std(self):
        return np.sqrt(np.maximum(self.sumsq / self.count - np.square(self.mean), 1e-2))

    def update(self, x):
        x = np.asarray(x, np.float64).reshape(-1, self.sum.shape[0])
        self.sum += x.sum(0)
        self.sumsq += np.square(x).sum(0)
        self.count += x.shape[0]


def obz(ob, mean, std):
    return np.clip((np.asarray(ob, np.float64) - mean) / std, -5.0, 5.0)


def pol_forward(p, z):
    W1, b1, W2, b2, W3, b3, ls = unpack_pol(p)
    h1 = np.tanh(z @ W1 + b1)
    h2 = np.tanh(h1 @ W2 + b2)
    return dict(h1=h1, h2=h2, mean=h2 @ W3 + b3, logstd=ls)


def vf_forward(p, z):
    V1, c1, V2, c2, V3, c3 = unpack_vf(p)
    g1 = np.tanh(z @ V1 + c1)
    g2 = np.tanh(g1 @ V2 + c2)
    return dict(g1=g1, g2=g2, v=(g2 @ V3 + c3)[:, 0])


def logp(mean, logstd, a):
    std = np.exp(logstd)
    return -0.5 * (((a - mean) / std) ** 2).sum(1) - logstd.sum() - 0.5 * 2 * LOG2PI


def gae(rew, vpred, new, nextvpred, gamma=0.99, lam=0.95):
    """rew, vpred, new: [T, N]; nextvpred: [N] (already 0 where the next ob starts an
    episode).  Returns (adv, tdlamret) [T, N]."""
    T = rew.shape[0]
    new_ext = np.concatenate([new, np.zeros((1,) + new.shape[1:])], 0)
    v_ext = np.concatenate([vpred, nextvpred[None]], 0)
    adv = np.zeros_like(rew, dtype=np.float64)
    last = np.zeros(rew.shape[1:])
    for t in range(T - 1, -1, -1):
        nonterm = 1.0 - new_ext[t + 1]
        delta = rew[t] + gamma * v_ext[t + 1] * nonterm - vpred[t]
        last = delta + gamma * lam * nonterm * last
        adv[t] = last
    return adv, adv + vpred


def standardize(adv):
    return (adv - adv.mean()) / adv.std()


def loss_and_grads(pol, vf, z, a, logp_old, atarg, ret, clip_eps):
    """Minibatch loss terms and the gradient of pol_surr + vf_loss w.r.t. [pol | vf]."""
    n = z.shape[0]
    fp, fv = pol_forward(pol, z), vf_forward(vf, z)
    lp = logp(fp["mean"], fp["logstd"], a)
    ratio = np.exp(lp - logp_old)
    s1 = ratio * atarg
    rc = np.clip(ratio, 1.0 - clip_eps, 1.0 + clip_eps)
    s2 = rc * atarg
    pol_surr = -np.minimum(s1, s2).mean()
    vf_loss = np.square(fv["v"] - ret).mean()
    # d(-min)/dratio with TF's conventions
    take1 = s1 <= s2
    inside = (ratio >= 1.0 - clip_eps) & (ratio <= 1.0 + clip_eps)
    dr = np.where(take1, -atarg, np.where(inside, -atarg, 0.0)) / n
    dlp = dr * ratio
    std = np.exp(fp["logstd"])
    dmean = dlp[:, None] * (a - fp["mean"]) / std ** 2
    dls = (dlp[:, None] * (((a - fp["mean"]) / std) ** 2 - 1.0)).sum(0)
    W1, b1, W2, b2, W3, b3, _ = unpack_pol(pol)
    gW3 = fp["h2"].T @ dmean
    gb3 = dmean.sum(0)
    d2 = (dmean @ W3.T) * (1 - fp["h2"] ** 2)
    gW2 = fp["h1"].T @ d2
    gb2 = d2.sum(0)
    d1 = (d2 @ W2.T) * (1 - fp["h1"] ** 2)
    gW1 = z.T @ d1
    gb1 = d1.sum(0)
    gpol = np.concatenate([gW1.ravel(), gb1, gW2.ravel(), gb2, gW3.ravel(), gb3, dls])
    V1, c1, V2, c2, V3, c3 = unpack_vf(vf)
    dv = 2.0 * (fv["v"] - ret)[:, None] / n
    gV3 = fv["g2"].T @ dv
    gc3 = dv.sum(0)
    e2 = (dv @ V3.T) * (1 - fv["g2"] ** 2)
    gV2 = fv["g1"].T @ e2
    gc2 = e2.sum(0)
    e1 = (e2 @ V2.T) * (1 - fv["g1"] ** 2)
    gV1 = z.T @ e1
    gc1 = e1.sum(0)
    gvf = np.concatenate([gV1.ravel(), gc1, gV2.ravel(), gc2, gV3.ravel(), gc3])
    ent = (fp["logstd"] + 0.5 * np.log(2 * np.pi * np.e)).sum()
    kl = None
    return dict(pol_surr=pol_surr, vf_loss=vf_loss, ent=ent, gpol=gpol, gvf=gvf, ratio=ratio, kl=kl)


def total_loss(pol, vf, z, a, logp_old, atarg, ret, clip_eps):
    r = loss_and_grads(pol, vf, z, a, logp_old, atarg, ret, clip_eps)
    return r["pol_surr"] + r["vf_loss"]

"""The oracles' policy / loss / LSTM / Adam math pinned to the reference's own GraphDefs.

tests/golden/graph_golden.npz holds the reference graph (src/~/reacher/data/viz/1 event
files, TF 1.10) EVALUATED by oracle/tfgraph.py on seeded inputs, and graph_consts.json the
constants read out of it; tests/golden/make_graph_consts.py made both.  These tests check
that the oracles (policy_np, refnet_np, lstm_np, AdamTF1) and the product's defaults agree
with them.  What the graphs do NOT hold: trained weights (the teacher checkpoint is absent)
and the MLP student graph itself (student_nn.py:51-57 is not in the logged graphs; its
dense/tanh/kl pieces are).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

from oracle import lstm_np, policy_np, refnet_np

C = json.load(open(os.path.join(GOLDEN, "graph_consts.json")))
K = C["constants"]


@pytest.fixture(scope="module")
def gg():
    return dict(np.load(os.path.join(GOLDEN, "graph_golden.npz")))


def f32(x):
    return float(np.float32(x))


def test_every_event_file_agrees():
    files = C["files"]
    assert len(files) == 12 and all(f["graph_defs"] == 1 for f in files)
    assert all(f.get("constants_agree", True) for f in files)


def test_adam_constants_and_schedule():
    # tf.train.AdamOptimizer(beta1=.9, beta2=.999, epsilon=1e-8) as logged (adam/Adam/*)
    opt = policy_np.AdamTF1(4)
    assert (f32(opt.b1), f32(opt.b2), f32(opt.eps)) == (K["adam_beta1"], K["adam_beta2"], K["adam_epsilon"])
    # beta powers are variables initialised to beta and multiplied once per step after
    # the ApplyAdams (adam/Adam/mul = beta1_power * beta1)
    assert (f32(opt.b1p), f32(opt.b2p)) == (K["adam_beta1_power0"], K["adam_beta2_power0"])
    assert K["adam_beta1_power_update"] == ["adam/beta1_power/read", "adam/Adam/beta1"]
    assert K["adam_apply_inputs"][3:9] == ["adam/beta1_power/read", "adam/beta2_power/read", "adam/Adam/learning_rate",
                                           "adam/Adam/beta1", "adam/Adam/beta2", "adam/Adam/epsilon"]
    from reacherdistilation_amd.distill import DistillConfig
    from reacherdistilation_amd.student_lstm import StudentLstmConfig
    d = DistillConfig()
    assert (f32(d.beta1), f32(d.beta2), f32(d.eps)) == (K["adam_beta1"], K["adam_beta2"], K["adam_epsilon"])
    # the logged graph is the LSTM student's: its learning rate is lstm_train's (1e-3); the
    # MLP driver's 1e-4 (mlp_train.py:75) is not in any logged graph
    assert f32(StudentLstmConfig().lr) == K["adam_learning_rate"]


def test_obfilter_constants():
    assert K["obfilter_count0"] == policy_np.OBF_COUNT0
    assert K["obfilter_sum0_absmax"] == 0.0 and K["obfilter_sumsq0_absmax"] == policy_np.OBF_SUMSQ0
    assert K["obfilter_var_floor"] == f32(policy_np.OBF_VAR_FLOOR)
    assert (K["obz_clip_min"], K["obz_clip_max"]) == (-policy_np.OB_CLIP, policy_np.OB_CLIP)
    ops = K["obfilter_ops"]
    assert ops["pi/obfilter/Maximum"][0] == "Maximum" and ops["pi/obfilter/Maximum"][2] == "pi/obfilter/Maximum/y"
    assert ops["pi/obfilter/sub"] == ["Sub", "pi/obfilter/ToFloat_1", "pi/obfilter/Square"]   # E[x^2] - mean^2
    assert ops["pi/vf/truediv"] == ["RealDiv", "pi/vf/sub", "pi/obfilter/Sqrt"]


@pytest.mark.parametrize("which", ["init", "rand"])
def test_policy_forward_matches_graph(gg, which):
    """pi/pol/concat of the reference graph == policy_np.forward (with the filter from
    policy_np.obfilter), on the teacher's own initial weights and on seeded weights."""
    if which == "init":
        W1, W2, W3 = gg["pol_init_W1"], gg["pol_init_W2"], gg["pol_init_W3"]
        b1, b2, b3, ls = np.zeros(64), np.zeros(64), np.zeros(2), np.zeros(2)
        ob = gg["pol_ob"]
    else:
        W1, W2, W3 = gg["pol_rand_W1"], gg["pol_rand_W2"], gg["pol_rand_W3"]
        b1, b2, b3, ls = gg["pol_rand_b1"], gg["pol_rand_b2"], gg["pol_rand_b3"], gg["pol_rand_logstd"]
        ob = gg["pol_rand_ob"]
    mu, sd = policy_np.obfilter(gg[f"pol_{which}_rsum"], gg[f"pol_{which}_rsumsq"], float(gg[f"pol_{which}_count"]))
    p = policy_np.pack(W1, b1, W2, b2, W3, b3, ls).astype(np.float64)
    f = policy_np.forward(p, mu, sd, ob)
    want = gg[f"pol_{which}_pdflat"]
    got = np.concatenate([f["mean"], np.broadcast_to(f["logstd"], f["mean"].shape)], 1)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-14)
    if which == "rand":   # the seeded case exercises the clip and the variance floor
        assert (np.abs((ob - mu) / sd) > 5).any() and (sd == np.sqrt(policy_np.OBF_VAR_FLOOR)).any()


def test_policy_shapes_and_init():
    assert K["pol_fc1_kernel_shape"] == [policy_np.OBD, policy_np.HID]
    assert K["pol_fc2_kernel_shape"] == [policy_np.HID, policy_np.HID]
    assert K["pol_final_kernel_shape"] == [policy_np.HID, policy_np.ACD]
    assert K["pol_logstd_init"] == [[0.0, 0.0]] and K["pol_logstd_mul"] == 0.0
    # normc(1.0) hidden, normc(0.01) output columns, zero biases: the student's init
    from reacherdistilation_amd.policy import SLICES, student_init
    s = student_init(2)
    for name, key in (("W1", "fc1"), ("W2", "fc2"), ("W3", "final")):
        lo, hi = K[f"pol_{key}_normc_colnorm"]
        n = np.sqrt((s[name].astype(np.float64) ** 2).sum(0))
        assert lo - 1e-6 * hi <= n.min() and n.max() <= hi + 1e-6 * hi, name
        assert K[f"pol_{key}_bias_init_absmax"] == 0.0
    for b in ("b1", "b2", "b3", "logstd"):
        a, e, _ = SLICES[b]
        assert not s.flat[a:e].any()


def test_kl_loss_and_gradient_match_graph(gg):
    """LSTM/kstm_kl_loss (loss.py:3-13 as built) and TF's gradient of it w.r.t. the student
    pdflat == refnet_np.loss_and_dout (used by the reference-student and LSTM oracles)."""
    assert (K["kl_two"], K["kl_half"], K["kl_reduction_indices"]) == (2.0, 0.5, [2, 1, 0])
    for k in range(gg["kl_loss"].shape[0]):
        s = np.concatenate([gg["kl_s1"][k], gg["kl_s2"][k]], 0)                      # [T=2, 4]
        t = np.concatenate([gg["kl_tmean"][k].reshape(2, 2), gg["kl_tlogstd"][k].reshape(2, 2)], 1)
        kl, d, _ = refnet_np.loss_and_dout(s, t, "kl", 2)
        np.testing.assert_allclose(kl, gg["kl_loss"][k], rtol=1e-12)
        np.testing.assert_allclose(d, np.concatenate([gg["kl_grad1"][k], gg["kl_grad2"][k]], 0),
                                   rtol=1e-12, atol=1e-14)


def test_policy_np_kl_is_the_pinned_kl():
    """policy_np's KL (state-independent logstd, one value for all rows) equals the pinned
    per-row form with that logstd broadcast: dlogstd = the rows' sum."""
    rng = np.random.RandomState(5)
    n = 37
    fs = dict(mean=rng.uniform(-1, 1, (n, 2)), logstd=rng.uniform(-3, 0.5, 2))
    ft = dict(mean=rng.uniform(-1, 1, (n, 2)), logstd=rng.uniform(-3, 0.5, 2))
    kl, dm, dls, _ = policy_np.loss_and_dmean(fs, ft, "kl", n)
    s = np.concatenate([fs["mean"], np.tile(fs["logstd"], (n, 1))], 1)
    t = np.concatenate([ft["mean"], np.tile(ft["logstd"], (n, 1))], 1)
    kl2, d2, _ = refnet_np.loss_and_dout(s, t, "kl", n)
    np.testing.assert_allclose(kl, kl2, rtol=1e-13)
    np.testing.assert_allclose(dm, d2[:, :2], rtol=1e-13)
    np.testing.assert_allclose(dls, d2[:, 2:].sum(0), rtol=1e-13)


def test_lstm_cell_matches_graph(gg):
    """LSTM/unique_lstm_cell (TF1 LSTMCell: split i, j, f, o; forget bias on f) == lstm_np.cell."""
    assert K["lstm_forget_bias"] == lstm_np.FORGET_BIAS and K["lstm_split"] == 4
    assert K["lstm_gate_inputs"] == {"Sigmoid_1": "LSTM/unique_lstm_cell/split", "Tanh": "LSTM/unique_lstm_cell/split:1",
                                     "add": "LSTM/unique_lstm_cell/split:2", "Sigmoid_2": "LSTM/unique_lstm_cell/split:3"}
    c, h, _ = lstm_np.cell(gg["cell_x"], gg["cell_c0"], gg["cell_h0"], gg["cell_Wl"], gg["cell_bl"])
    np.testing.assert_allclose(c, gg["cell_c1"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(h, gg["cell_h1"], rtol=1e-12, atol=1e-14)


def test_glorot_limit_matches_graph():
    """tf.layers.dense / LSTMCell kernels: glorot_uniform, limit sqrt(6 / (fan_in + fan_out))
    (the limit refnet_np.init, lstm_np.init and policy.student_mlp_graph_params use)."""
    fi, fo = K["lstm_kernel_shape"]
    assert f32(np.sqrt(6.0 / (fi + fo))) == K["lstm_glorot_limit"]


def test_dropout_scale_matches_graph(gg):
    """tf.nn.dropout = x / kp * floor(kp + U): refnet_np.apply_mask with u = 1 - U."""
    assert K["dropout_uniform_range"] == [0.0, 1.0]
    x, U, kp = gg["drop_x"], gg["drop_u"], float(gg["drop_kp"])
    ok = np.abs(U - (1 - kp)) > 1e-9
    got = refnet_np.apply_mask(x, 1.0 - U, np.float32(kp))
    np.testing.assert_allclose(got[ok], gg["drop_out"][ok], rtol=1e-6)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="the reference is not on this box")
def test_goldens_regenerate_from_the_reference_graph(tmp_path, gg):
    """The committed goldens are what the reference's event files evaluate to."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mgc", os.path.join(GOLDEN, "make_graph_consts.py"))
    mgc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgc)
    from oracle import tfgraph
    g, _ = tfgraph.reference_graph()
    fresh = mgc.goldens(g)
    assert set(fresh) == set(gg)
    for k in gg:
        np.testing.assert_array_equal(fresh[k], gg[k], err_msg=k)
    assert mgc.constants(g) == K


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["init", "rand"])
def test_kernel_forward_matches_reference_graph(gg, which):
    """The product's f32 MFMA policy forward (rdd_forward, teacher and student images) on the
    reference graph's own inputs == the reference graph's pi/pol/concat.  Tolerance: f32
    accumulation + the kernel's 2-ulp tanh vs the graph evaluated in f64 on the same f32
    weights: means 5e-5 abs + 2e-5 rel; logstd exact."""
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    from reacherdistilation_amd.policy import MlpPolicyParams
    if which == "init":
        W = [gg["pol_init_W1"], np.zeros(64), gg["pol_init_W2"], np.zeros(64), gg["pol_init_W3"], np.zeros(2),
             np.zeros(2)]
        ob = gg["pol_ob"]
    else:
        W = [gg[f"pol_rand_{k}"] for k in ("W1", "b1", "W2", "b2", "W3", "b3", "logstd")]
        ob = gg["pol_rand_ob"]
    mu, sd = policy_np.obfilter(gg[f"pol_{which}_rsum"], gg[f"pol_{which}_rsumsq"], float(gg[f"pol_{which}_count"]))
    p = MlpPolicyParams(policy_np.pack(*W).astype(np.float32), mu.astype(np.float32), sd.astype(np.float32))
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=0), device="cuda:0", teacher=p, student=p)
    t, s = tr.forward(torch.tensor(ob, dtype=torch.float32))
    want = gg[f"pol_{which}_pdflat"]
    for out in (t, s):
        got = out.cpu().numpy().astype(np.float64)
        np.testing.assert_allclose(got[:, :2], want[:, :2], atol=5e-5, rtol=2e-5)
        assert np.array_equal(got[:, 2:], want[:, 2:].astype(np.float32))
    tr.close()


def _variant_grads(v, ph):
    """The logged LSTM graph (1-unit TF1 LSTMCell over T = 2 steps; per step a tanh 'lstm_step'
    layer feeding a reward head 64-32-64-1 and an action head 64-4 = pdflat; loss = kl_loss +
    the reward squared error) forward AND backward, built only from the oracle's primitives:
    lstm_np.cell / bptt, refnet_np.dense_backward / tanh_grad / loss_and_dout."""
    Wl, bl = v["unique_lstm_cell/kernel"], v["unique_lstm_cell/bias"]
    ob, act, P = ph["ob_combined_ph"], ph["action_combined_ph"], ph["Placeholder"]
    c, h = P[0], P[1]
    steps, heads, pd = [], [], []
    for t in range(2):
        x = np.concatenate([ob[t], act[t]], 1)      # dropout at keep_prob 1 is the identity
        cprev, hprev = c, h
        c, h, (gi, gj, gf, go) = lstm_np.cell(x, cprev, hprev, Wl, bl)
        steps.append(dict(x=x, hprev=hprev, cprev=cprev, gi=gi, gj=gj, gf=gf, go=go, c=c))
        k = t + 1
        a = np.tanh(h @ v[f"lstm_step{k}/kernel"] + v[f"lstm_step{k}/bias"])
        r = [a]
        for name in ("reward_hid", "reward_2hid", "reward_3hid"):
            r.append(np.tanh(r[-1] @ v[f"{name}{k}/kernel"] + v[f"{name}{k}/bias"]))
        rew = r[-1] @ v[f"reward_out{k}/kernel"] + v[f"reward_out{k}/bias"]
        q = np.tanh(a @ v[f"lstm_action{k}/kernel"] + v[f"lstm_action{k}/bias"])
        pd.append(q @ v[f"pd_step{k}/kernel"] + v[f"pd_step{k}/bias"])
        heads.append((h, a, r, rew, q))
    tp = np.concatenate([ph["t_mean_combined"], ph["t_logstd_combined"]], 2).reshape(2, 4)
    kl, dpd, _ = refnet_np.loss_and_dout(np.concatenate(pd, 0), tp, "kl", 2)
    rews = np.array([heads[t][3].item() for t in range(2)])
    diff = rews[None, :] - ph["reward_target"]            # [2 targets, 2 steps]: the graph's broadcast
    rloss, drew = float((diff ** 2).sum()), 2.0 * diff.sum(0)
    g, dh_out = {}, []
    for t in range(2):
        k = t + 1
        h, a, r, rew, q = heads[t]
        g[f"pd_step{k}/kernel"], g[f"pd_step{k}/bias"], dq = dense_backward(q, dpd[t:t + 1], v[f"pd_step{k}/kernel"])
        g[f"lstm_action{k}/kernel"], g[f"lstm_action{k}/bias"], da = dense_backward(
            a, refnet_np.tanh_grad(q, dq), v[f"lstm_action{k}/kernel"])
        g[f"reward_out{k}/kernel"], g[f"reward_out{k}/bias"], dr = dense_backward(
            r[3], np.array([[drew[t]]]), v[f"reward_out{k}/kernel"])
        for j, name in ((3, "reward_3hid"), (2, "reward_2hid"), (1, "reward_hid")):
            g[f"{name}{k}/kernel"], g[f"{name}{k}/bias"], dr = dense_backward(
                r[j - 1], refnet_np.tanh_grad(r[j], dr), v[f"{name}{k}/kernel"])
        g[f"lstm_step{k}/kernel"], g[f"lstm_step{k}/bias"], dh = dense_backward(
            h, refnet_np.tanh_grad(a, da + dr), v[f"lstm_step{k}/kernel"])
        dh_out.append(dh)
    g["unique_lstm_cell/kernel"], g["unique_lstm_cell/bias"], _, _, _ = lstm_np.bptt(steps, Wl, dh_out)
    return g, kl, rloss


def dense_backward(a, dz, W):
    return refnet_np.dense_backward(a, dz, W)


@pytest.mark.parametrize("case", range(4))
def test_oracle_backward_reproduces_tf_generated_gradients(gg, case):
    """the TF-generated backward of the reference's logged LSTM graph --
    the gradient input of each of its 30 ApplyAdam nodes (adam/gradients/AddN_6, AddN_7 = the
    cell's BPTT over two steps; every dense layer's MatMul_grad + BiasAddGrad through TanhGrad;
    the kl + reward losses), evaluated from the graph (tests/golden/make_graph_consts.py) --
    equals the oracle's own backward primitives composed the same way.  These primitives ARE
    lstm_np.backward (bptt, cell_backward), refnet_np.backward and policy_np.backward
    (dense_backward, tanh_grad, loss_and_dout), so the oracle backward that checks every GPU
    gradient rests on reference-held vectors.  Tolerance: rtol 1e-10 (both f64)."""
    names = [str(n) for n in gg["bptt_vars"]]
    v = {n[len("LSTM/"):]: gg[f"bptt{case}_var{j}"].astype(np.float64) for j, n in enumerate(names)}
    ph = {k: gg[f"bptt{case}_{k}"] for k in ("ob_combined_ph", "action_combined_ph", "Placeholder",
                                              "t_mean_combined", "t_logstd_combined", "reward_target")}
    g, kl, rloss = _variant_grads(v, ph)
    assert abs(kl - float(gg[f"bptt{case}_kl"])) <= 1e-10 * abs(kl)
    assert abs(rloss - float(gg[f"bptt{case}_rloss"])) <= 1e-10 * abs(rloss)
    assert sorted(g) == sorted(v)
    for j, n in enumerate(names):
        want = gg[f"bptt{case}_grad{j}"]
        got = g[n[len("LSTM/"):]]
        assert got.shape == want.shape, n
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-12 * np.abs(want).max(), err_msg=n)


def test_tf_gradient_goldens_cover_every_apply_adam(gg):
    """All 30 ApplyAdam gradient inputs of the logged graph are in the goldens (the cell's two
    AddN sums are its BPTT over the two unrolled steps)."""
    nodes = [str(n) for n in gg["bptt_grad_nodes"]]
    assert len(nodes) == 30 and int(gg["bptt_cases"]) == 4
    assert nodes[:2] == ["adam/gradients/AddN_7", "adam/gradients/AddN_6"]
    assert all(("MatMul_grad" in n) == ("kernel" in str(v)) for n, v in zip(nodes[2:], gg["bptt_vars"][2:]))

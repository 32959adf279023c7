#!/usr/bin/env python3
"""Generate tests/golden/graph_consts.json + graph_golden.npz from the reference's own
TensorBoard GraphDefs (the only reference-held evidence for the policy / loss / LSTM /
Adam math; SURVEY.md §8c, VERDICT r1 "Next round" item 1).

Input (read here, never on the GPU box):
    /root/reference/src/~/reacher/data/viz/1/events.out.tfevents.*   (12 files)
parsed as data by oracle/tfgraph.py (TFRecord framing + protobuf wire format; no
TensorFlow, nothing in the files is executed).

Output (data only: constants, shapes, and input/output vectors):
  graph_consts.json  -- per-file graph summary and the constants the oracles must use:
      adam/Adam/{learning_rate,beta1,beta2,epsilon}, adam/beta{1,2}_power initial values;
      pi/obfilter count / sums initial values, variance floor (Maximum/y), clip bounds;
      pi/pol fc1/fc2/final kernel shapes, logstd init, the column norms of the normc
      initial kernels; LSTMCell forget bias, gate split, glorot-uniform limit; the kl
      loss's constants and reduction axes.
  graph_golden.npz   -- the reference graph EVALUATED (float64 interpreter) on seeded inputs:
      pol_*   pi/pol/concat (pdflat) of the teacher MlpPolicy: its own initial weights and
              filter on the fixture observations ("init"), and seeded random weights with a
              non-trivial filter ("rand");
      kl_*    LSTM/kstm_kl_loss and its TF-generated gradient w.r.t. the student pdflat
              (adam/gradients/LSTM/split{,_1}_grad/concat), 64 instances of the graph's
              [T=2, B=1] shape;
      cell_*  one LSTM/unique_lstm_cell step (c', h') on seeded x, c, h, kernel, bias;
      drop_*  LSTM/dropout/mul with the RandomUniform draw fed;
      bptt{k}_*  the graph's WHOLE TF-generated backward: the gradient input of every one of
              its 30 ApplyAdam nodes (adam/gradients/AddN_6, AddN_7 -- the cell's BPTT over the
              T = 2 unrolled steps -- and each dense layer's MatMul_grad / BiasAddGrad, through
              TanhGrad, SigmoidGrad, the kl and reward losses) with every LSTM/* variable and
              placeholder fed from a seed (keep_prob 1).  k = 0 at the logged shapes (1 unit,
              B = 1, heads 128/64/32/64); k = 1..3 with narrower heads, which the graph's ops accept
              (heads 16/8/4/8; the unit count and B = 1 are baked into its Reshape constants).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import tfgraph  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT_JSON = os.path.join(HERE, "graph_consts.json")
OUT_NPZ = os.path.join(HERE, "graph_golden.npz")


def scalar(g, name):
    return float(np.asarray(g.const(name)).reshape(()))


def constants(g):
    c = {}
    for k in ("learning_rate", "beta1", "beta2", "epsilon"):
        c[f"adam_{k}"] = scalar(g, f"adam/Adam/{k}")
    c["adam_beta1_power0"] = scalar(g, "adam/beta1_power/initial_value")
    c["adam_beta2_power0"] = scalar(g, "adam/beta2_power/initial_value")
    # the beta powers advance by one multiply per step, after every ApplyAdam
    mul = g.nodes["adam/Adam/mul"]
    c["adam_beta1_power_update"] = [i for i in mul["inputs"] if not i.startswith("^")]
    c["adam_apply_inputs"] = g.nodes["adam/Adam/update_LSTM/unique_lstm_cell/kernel/ApplyAdam"]["inputs"][:9]
    c["obfilter_count0"] = scalar(g, "pi/obfilter/count/Initializer/Const")
    c["obfilter_sum0_absmax"] = float(np.abs(g.const("pi/obfilter/runningsum/Initializer/Const")).max())
    c["obfilter_sumsq0_absmax"] = float(np.abs(g.const("pi/obfilter/runningsumsq/Initializer/Const")).max())
    c["obfilter_var_floor"] = scalar(g, "pi/obfilter/Maximum/y")
    c["obz_clip_max"] = scalar(g, "pi/vf/clip_by_value/Minimum/y")
    c["obz_clip_min"] = scalar(g, "pi/vf/clip_by_value/y")
    # the filter: mean = sum / count, var = sumsq / count - mean^2, std = sqrt(max(var, floor))
    c["obfilter_ops"] = {n: [g.nodes[n]["op"]] + [i for i in g.nodes[n]["inputs"] if not i.startswith("^")]
                         for n in ("pi/obfilter/truediv", "pi/obfilter/truediv_1", "pi/obfilter/sub",
                                   "pi/obfilter/Maximum", "pi/obfilter/Sqrt", "pi/vf/truediv")}
    for layer in ("fc1", "fc2", "final"):
        k = g.const(f"pi/pol/{layer}/kernel/Initializer/Const")
        c[f"pol_{layer}_kernel_shape"] = list(k.shape)
        norms = np.sqrt((np.asarray(k, np.float64) ** 2).sum(0))
        c[f"pol_{layer}_normc_colnorm"] = [float(norms.min()), float(norms.max())]
        c[f"pol_{layer}_bias_init_absmax"] = float(np.abs(g.const(f"pi/pol/{layer}/bias/Initializer/zeros")).max())
    c["pol_logstd_init"] = np.asarray(g.const("pi/pol/logstd/Initializer/zeros")).tolist()
    c["pol_logstd_mul"] = scalar(g, "pi/pol/mul/y")        # pdflat = [mean, mean * 0 + logstd]
    c["lstm_forget_bias"] = scalar(g, "LSTM/unique_lstm_cell/add/y")
    c["lstm_split"] = g.nodes["LSTM/unique_lstm_cell/split"]["attr"]["num_split"]
    c["lstm_gate_inputs"] = {n: g.nodes[f"LSTM/unique_lstm_cell/{n}"]["inputs"][0]
                             for n in ("Sigmoid_1", "Tanh", "add", "Sigmoid_2")}   # i, j, f(+bias), o
    shp = [int(v) for v in g.const("LSTM/unique_lstm_cell/kernel/Initializer/random_uniform/shape")]
    c["lstm_kernel_shape"] = shp
    c["lstm_glorot_limit"] = scalar(g, "LSTM/unique_lstm_cell/kernel/Initializer/random_uniform/max")
    c["kl_two"] = scalar(g, "LSTM/mul/x")
    c["kl_half"] = scalar(g, "LSTM/sub_2/y")
    c["kl_reduction_indices"] = [int(v) for v in g.const("LSTM/kstm_kl_loss/reduction_indices")]
    c["dropout_uniform_range"] = [scalar(g, "LSTM/dropout/random_uniform/min"),
                                  scalar(g, "LSTM/dropout/random_uniform/max")]
    return c


def policy_feeds(W1, b1, W2, b2, W3, b3, ls, rsum, rsumsq, count, ob):
    return {"pi/ob": ob, "pi/obfilter/runningsum": rsum, "pi/obfilter/runningsumsq": rsumsq,
            "pi/obfilter/count": np.float64(count), "pi/pol/fc1/kernel": W1, "pi/pol/fc1/bias": b1,
            "pi/pol/fc2/kernel": W2, "pi/pol/fc2/bias": b2, "pi/pol/final/kernel": W3,
            "pi/pol/final/bias": b3, "pi/pol/logstd": np.asarray(ls).reshape(1, 2)}


def goldens(g):
    out = {}
    fx = np.load(os.path.join(HERE, "reacher_fixture.npz"))
    ob = fx["ob"][:2].reshape(-1, 11)            # the fixture's first two episodes (100 obs)
    # (1) the teacher MlpPolicy at its own initial weights and filter
    W = [np.asarray(g.const(f"pi/pol/{n}/kernel/Initializer/Const"), np.float64) for n in ("fc1", "fc2", "final")]
    rsum = np.asarray(g.const("pi/obfilter/runningsum/Initializer/Const"), np.float64)
    rsumsq = np.asarray(g.const("pi/obfilter/runningsumsq/Initializer/Const"), np.float64)
    cnt = scalar(g, "pi/obfilter/count/Initializer/Const")
    b = [np.zeros(64), np.zeros(64), np.zeros(2)]
    ls = np.zeros(2)
    out["pol_init_pdflat"] = g.run("pi/pol/concat", policy_feeds(W[0], b[0], W[1], b[1], W[2], b[2], ls,
                                                                  rsum, rsumsq, cnt, ob))
    for k, v in zip(("W1", "W2", "W3"), W):
        out[f"pol_init_{k}"] = v.astype(np.float32)
    out["pol_init_rsum"], out["pol_init_rsumsq"], out["pol_init_count"] = rsum, rsumsq, np.float64(cnt)
    out["pol_ob"] = ob
    # (2) seeded weights (f32 values) and a filter with some variances under the floor
    rng = np.random.RandomState(20241016)
    W1 = (rng.standard_normal((11, 64)) * 0.4).astype(np.float32)
    W2 = (rng.standard_normal((64, 64)) * 0.15).astype(np.float32)
    W3 = (rng.standard_normal((64, 2)) * 0.3).astype(np.float32)
    b1, b2, b3 = [(rng.standard_normal(n) * 0.1).astype(np.float32) for n in (64, 64, 2)]
    lsr = rng.uniform(-3.5, 0.5, 2).astype(np.float32)
    count = 1234.5
    mu = rng.uniform(-0.5, 0.5, 11)
    var = np.exp(rng.uniform(np.log(1e-3), np.log(2.0), 11))   # some below the 1e-2 floor
    rs, rss = mu * count, (var + mu ** 2) * count
    obr = ob + rng.standard_normal(ob.shape) * 0.3                 # include |z| > 5 clipping
    obr[::7, 3] += 40.0
    out["pol_rand_pdflat"] = g.run("pi/pol/concat", policy_feeds(W1, b1, W2, b2, W3, b3, lsr, rs, rss, count, obr))
    for k, v in dict(W1=W1, b1=b1, W2=W2, b2=b2, W3=W3, b3=b3, logstd=lsr, rsum=rs, rsumsq=rss, ob=obr).items():
        out[f"pol_rand_{k}"] = v
    out["pol_rand_count"] = np.float64(count)
    # (3) kl loss + TF's gradient w.r.t. the student's pdflat (shape [T=2, B=1] as built)
    K = 64
    s1, s2 = rng.uniform(-1, 1, (K, 1, 4)), rng.uniform(-1, 1, (K, 1, 4))
    s1[..., 2:] = rng.uniform(-3.5, 0.5, (K, 1, 2))
    s2[..., 2:] = rng.uniform(-3.5, 0.5, (K, 1, 2))
    tm = rng.uniform(-1, 1, (K, 2, 1, 2))
    tl = rng.uniform(-3.5, 0.5, (K, 2, 1, 2))
    kl, g1, g2 = [], [], []
    for k in range(K):
        r = g.run(["LSTM/kstm_kl_loss", "adam/gradients/LSTM/split_grad/concat",
                   "adam/gradients/LSTM/split_1_grad/concat"],
                  {"LSTM/pd_step1/BiasAdd": s1[k], "LSTM/pd_step2/BiasAdd": s2[k], "LSTM/t_mean_combined": tm[k],
                   "LSTM/t_logstd_combined": tl[k], "LSTM/t_std_combined": np.exp(tl[k]), "LSTM/Sum": 0.0})
        kl.append(float(r[0])); g1.append(r[1]); g2.append(r[2])
    out.update(kl_s1=s1, kl_s2=s2, kl_tmean=tm, kl_tlogstd=tl, kl_loss=np.array(kl),
               kl_grad1=np.stack(g1), kl_grad2=np.stack(g2))
    # (4) one LSTMCell step, 8 units (the cell's ops are shape-generic), 16 rows
    U, B, X = 8, 16, 13
    x, c0, h0 = rng.standard_normal((B, X)), rng.standard_normal((B, U)), rng.uniform(-1, 1, (B, U))
    Wl, bl = rng.standard_normal((X + U, 4 * U)) * 0.5, rng.standard_normal(4 * U) * 0.3
    c1, h1 = g.run(["LSTM/unique_lstm_cell/add_1", "LSTM/unique_lstm_cell/mul_2"],
                   {"LSTM/strided_slice_2": x, "LSTM/cm_state/control_dependency": c0,
                    "LSTM/cm_state/control_dependency_1": h0, "LSTM/unique_lstm_cell/kernel": Wl,
                    "LSTM/unique_lstm_cell/bias": bl})
    out.update(cell_x=x, cell_c0=c0, cell_h0=h0, cell_Wl=Wl, cell_bl=bl, cell_c1=c1, cell_h1=h1)
    # (5) tf.nn.dropout: x / kp * floor(kp + U)
    xo = rng.standard_normal((10, 20, 11)).astype(np.float32)
    u = rng.uniform(0, 1, xo.shape)
    kp = 0.5
    out.update(drop_x=xo, drop_u=u, drop_kp=np.float64(kp),
               drop_out=g.run("LSTM/dropout/mul", {"LSTM/ob_combined_ph": xo, "LSTM/keep_prob": kp,
                                                   "LSTM/dropout/random_uniform/RandomUniform": u}))
    out.update(bptt_goldens(g, rng))
    return out


# the logged graph's trainable LSTM/* variables, in creation order (= its ApplyAdam order)
def lstm_variables(g):
    return [n for n, d in g.nodes.items() if d["op"] == "VariableV2" and n.startswith("LSTM/") and "/Adam" not in n]


def bptt_feeds(g, rng, units, B, heads):
    """Seeded values for every LSTM/* variable and placeholder.  heads = (step, reward hid 1,
    2, 3, action) widths; units = the cell's.  Values are float32-representable."""
    H, R1, R2, R3, A = heads
    shapes = {"unique_lstm_cell/kernel": (13 + units, 4 * units), "unique_lstm_cell/bias": (4 * units,)}
    for k in (1, 2):
        for name, a, b in (("lstm_step", units, H), ("reward_hid", H, R1), ("reward_2hid", R1, R2),
                           ("reward_3hid", R2, R3), ("reward_out", R3, 1), ("lstm_action", H, A), ("pd_step", A, 4)):
            shapes[f"{name}{k}/kernel"], shapes[f"{name}{k}/bias"] = (a, b), (b,)
    f = {}
    for v in lstm_variables(g):
        shp = shapes[v[len("LSTM/"):]]
        scale = 1.5 / np.sqrt(shp[0]) if len(shp) == 2 else 0.3
        f[v] = (rng.standard_normal(shp) * scale).astype(np.float32).astype(np.float64)
    tl = rng.uniform(-1.5, 0.5, (2, B, 2)).astype(np.float32).astype(np.float64)
    f.update({"LSTM/ob_combined_ph": rng.standard_normal((2, B, 11)).astype(np.float32).astype(np.float64),
              "LSTM/action_combined_ph": rng.uniform(-1, 1, (2, B, 2)).astype(np.float32).astype(np.float64),
              "LSTM/Placeholder": (rng.standard_normal((2, B, units)) * 0.5).astype(np.float32).astype(np.float64),
              "LSTM/t_mean_combined": rng.uniform(-1, 1, (2, B, 2)).astype(np.float32).astype(np.float64),
              "LSTM/t_logstd_combined": tl, "LSTM/t_std_combined": np.exp(tl),
              "LSTM/reward_target": rng.standard_normal((2, 1)).astype(np.float32).astype(np.float64)})
    return f


def bptt_goldens(g, rng):
    names = lstm_variables(g)
    adam = {g.nodes[n]["inputs"][0]: g.nodes[n]["inputs"][9] for n, d in g.nodes.items() if d["op"] == "ApplyAdam"}
    assert sorted(adam) == sorted(names) and len(names) == 30
    out = {"bptt_vars": np.array(names), "bptt_grad_nodes": np.array([adam[v] for v in names])}
    cases = [(1, 1, (128, 64, 32, 64, 64))] + [(1, 1, (16, 8, 4, 8, 8))] * 3   # B, units baked into Reshape consts
    for k, (units, B, heads) in enumerate(cases):
        f = bptt_feeds(g, rng, units, B, heads)
        feeds = dict(f, **{"LSTM/keep_prob": 1.0,
                           "LSTM/dropout/random_uniform/RandomUniform": rng.uniform(0, 1, (2, B, 11))})
        vals = g.run([adam[v] for v in names] + ["LSTM/kstm_kl_loss", "LSTM/Sum"], feeds)
        for j, v in enumerate(names):
            out[f"bptt{k}_var{j}"] = f[v].astype(np.float32)   # f32-representable by construction
            out[f"bptt{k}_grad{j}"] = np.asarray(vals[j], np.float64)
        for ph in ("ob_combined_ph", "action_combined_ph", "Placeholder", "t_mean_combined", "t_logstd_combined",
                   "reward_target"):
            out[f"bptt{k}_{ph}"] = f[f"LSTM/{ph}"]
        out[f"bptt{k}_kl"], out[f"bptt{k}_rloss"] = np.float64(vals[-2]), np.float64(vals[-1])
    out["bptt_cases"] = np.array(len(cases))
    return out


def main():
    files = tfgraph.event_files()
    if not files:
        raise SystemExit(f"no event files under {tfgraph.REF_VIZ}")
    summary, consts = [], None
    for p in files:
        gds = tfgraph.graph_defs(p)
        entry = {"file": os.path.basename(p), "graph_defs": len(gds)}
        if gds:
            g = tfgraph.Graph(gds[0])
            c = constants(g)
            entry["nodes"] = len(g.nodes)
            if consts is None:
                consts = c
            else:   # every file must agree on what the oracles take from it
                entry["constants_agree"] = c == consts
                assert entry["constants_agree"], p
        summary.append(entry)
    g, src = tfgraph.reference_graph()
    gold = goldens(g)
    with open(OUT_JSON, "w") as fh:
        json.dump({"source": "reference src/~/reacher/data/viz/1/events.out.tfevents.* (GraphDef, TF 1.10)",
                   "golden_from": os.path.basename(src), "files": summary, "constants": consts}, fh, indent=1)
    np.savez_compressed(OUT_NPZ, **gold)
    print(f"wrote {OUT_JSON} and {OUT_NPZ} ({len(files)} event files, {len(gold)} arrays)")


if __name__ == "__main__":
    main()

"""GPU parity of the LSTM student (csrc/student_lstm.hip + csrc/rd_gemm.h) against
oracle/lstm_np.py (f64).

Tolerances (f32 kernels through T recurrent steps vs the f64 oracle): pdflat and final
state |err| <= 5e-5 + 1e-4 |ref|; gradient relative L2 error < 5e-4 and per element
<= 1e-3 max|g| + 1e-6; Adam step within 1e-6 + 1e-3 |update| where |g| > 1e-4 max|g|
(elsewhere Adam's ~lr sign(g) step is bounded by 2 lr).
"""
import numpy as np
import pytest
import torch

from oracle import lstm_np as ln
from oracle import policy_np as pn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _batch(T, B, seed=0):
    rs = np.random.RandomState(seed)
    ob = rs.uniform(-1, 1, (T, B, 11)).astype(np.float32)
    prev = np.concatenate([rs.uniform(-.5, .5, (T, B, 2)), rs.uniform(-1, 0, (T, B, 2))], 2).astype(np.float32)
    t = np.concatenate([rs.uniform(-.5, .5, (T, B, 2)), rs.uniform(-1.0, -0.2, (T, B, 2))], 2).astype(np.float32)
    return ob, prev, t


def _params(seed=6, T=10):
    p = ln.init(seed, T)
    rs = np.random.RandomState(seed + 1)
    for k, (o, s) in ln.layout(T)[0].items():
        if len(s) == 1:
            p[o:o + s[0]] = rs.uniform(-.1, .1, s[0]).astype(np.float32)
    return p


def _trainer(T=10, B=20, loss="kl", params=None, **kw):
    from reacherdistilation_amd.student_lstm import StudentLstmConfig, StudentLstmTrainer
    return StudentLstmTrainer(StudentLstmConfig(loss=loss, steps=T, max_windows=B, **kw), device=DEV,
                              params=_params(T=T) if params is None else params)


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


def _grad_check(g, want):
    g = np.asarray(g, np.float64)
    rel = np.linalg.norm(g - want) / np.linalg.norm(want)
    assert rel < 5e-4, rel
    assert np.abs(g - want).max() <= 1e-3 * np.abs(want).max() + 1e-6
    return rel


@pytest.mark.parametrize("T,B,with_state", [(10, 1, False), (10, 20, False), (10, 20, True), (3, 130, True)])
def test_forward_matches_oracle(T, B, with_state):
    tr = _trainer(T, B)
    ob, prev, _ = _batch(T, B, B)
    st = None
    if with_state:
        rs = np.random.RandomState(5)
        st = rs.uniform(-.5, .5, (2, B, 200)).astype(np.float32)
    y, fin = tr.forward(_t(ob), _t(prev), None if st is None else _t(st))
    want = ln.forward(tr.params().cpu().numpy(), ob, prev, st)
    np.testing.assert_allclose(y.cpu().numpy(), want["pdflat"], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(fin[0].cpu().numpy(), want["state"][0], atol=5e-5, rtol=1e-4)
    np.testing.assert_allclose(fin[1].cpu().numpy(), want["state"][1], atol=5e-5, rtol=1e-4)


@pytest.mark.parametrize("loss", ["mse", "kl"])
@pytest.mark.parametrize("T,B", [(10, 20), (10, 300), (4, 2000)])
def test_bptt_gradient_and_metrics_match_oracle(loss, T, B):
    tr = _trainer(T, B, loss)
    ob, prev, t = _batch(T, B, 3 + B)
    p = tr.params().cpu().numpy()
    g = tr.rollout(_t(ob), _t(prev), _t(t)).cpu().numpy()
    fw = ln.forward(p, ob, prev)
    L, d, sq = ln.loss_and_dout(fw["pdflat"], t, loss, T * B)
    _grad_check(g, ln.backward(p, fw, d))
    tr.apply()
    m = tr.metrics(1)[0]
    assert abs(m[0] - L) <= 2e-4 * abs(L) + 1e-6 and abs(m[1] - sq) <= 2e-4 * sq + 1e-6 and m[2] == T * B


def test_gradient_from_a_given_initial_state():
    T, B = 5, 40
    tr = _trainer(T, B, "kl")
    ob, prev, t = _batch(T, B, 1)
    st = np.random.RandomState(2).uniform(-.5, .5, (2, B, 200)).astype(np.float32)
    p = tr.params().cpu().numpy()
    g = tr.rollout(_t(ob), _t(prev), _t(t), _t(st)).cpu().numpy()
    fw = ln.forward(p, ob, prev, st)
    _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
    _grad_check(g, ln.backward(p, fw, d))


def test_adam_steps_match_oracle():
    T, B = 10, 20
    tr = _trainer(T, B, "kl")
    ob, prev, t = _batch(T, B, 8)
    p = tr.params().cpu().numpy().copy()
    opt = pn.AdamTF1(ln.P_LSTM, lr=1e-3)
    for k in range(3):
        fw = ln.forward(p, ob, prev)
        _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
        g = ln.backward(p, fw, d)
        before = p.copy()
        p = opt.step(p, g)
        tr.step(_t(ob), _t(prev), _t(t))
        got = tr.params().cpu().numpy()
        # Adam's update is ~lr * sign(g) where |g| is tiny, so f32 rounding of a near-zero
        # gradient can move it by up to 2 lr: compare tightly where the gradient is resolved
        strong = np.abs(g) > 1e-4 * np.abs(g).max()
        np.testing.assert_allclose(got[strong], p[strong], atol=1e-6 + 1e-3 * np.abs(p - before).max())
        assert np.abs(got - p).max() <= 2e-3 + 1e-6
        p = got.copy()
    assert tr.counter() == 3


def test_dropout_matches_oracle_mask():
    T, B = 10, 50
    tr = _trainer(T, B, "mse", keep_prob=0.5, seed=77)
    ob, prev, t = _batch(T, B, 4)
    for step in range(2):
        p = tr.params().cpu().numpy()
        g = tr.rollout(_t(ob), _t(prev), _t(t)).cpu().numpy()
        fw = ln.forward(p, ln.dropout(ob, 0.5, 77, step), prev)
        _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "mse", T * B)
        _grad_check(g, ln.backward(p, fw, d))
        tr.apply()


def test_sharded_windows_sum_to_the_full_batch():
    from reacherdistilation_amd.student_lstm import StudentLstmConfig, StudentLstmTrainer
    T, B = 10, 60
    ob, prev, t = _batch(T, B, 9)
    cfg = dict(loss="mse", steps=T, keep_prob=0.8, seed=3)
    full = StudentLstmTrainer(StudentLstmConfig(max_windows=B, **cfg), device=DEV, params=_params())
    gf = full.rollout(_t(ob), _t(prev), _t(t)).clone()
    a = StudentLstmTrainer(StudentLstmConfig(max_windows=25, **cfg), device=DEV, params=_params(), row_base=0)
    b = StudentLstmTrainer(StudentLstmConfig(max_windows=35, **cfg), device=DEV, params=_params(), row_base=25)
    ga = a.rollout(_t(ob[:, :25]), _t(prev[:, :25]), _t(t[:, :25]), windows_global=B).clone()
    gb = b.rollout(_t(ob[:, 25:]), _t(prev[:, 25:]), _t(t[:, 25:]), windows_global=B).clone()
    _grad_check((ga + gb).cpu().numpy(), gf.cpu().numpy().astype(np.float64))


def test_deterministic():
    T, B = 10, 500
    ob, prev, t = _batch(T, B, 2)
    g1 = _trainer(T, B).rollout(_t(ob), _t(prev), _t(t)).clone()
    g2 = _trainer(T, B).rollout(_t(ob), _t(prev), _t(t)).clone()
    assert torch.equal(g1, g2)


def test_learns_a_fixed_teacher_sequence():
    """KL to fixed target windows falls by > 5x in 150 Adam steps (lr 1e-3)."""
    T, B = 10, 64
    ob, prev, _ = _batch(T, B, 11)
    target = ln.forward(ln.init(99), ob, prev)["pdflat"].astype(np.float32)
    tr = _trainer(T, B, "kl")
    obt, prt, tgt = _t(ob).to(DEV), _t(prev).to(DEV), _t(target).to(DEV)
    for _ in range(150):
        tr.step(obt, prt, tgt)
    m = tr.metrics(150)
    assert np.all(np.isfinite(m[:, 0])) and m[-1, 0] < 0.2 * m[0, 0], (m[0, 0], m[-1, 0])


def test_bad_arguments_raise():
    tr = _trainer(10, 20)
    ob, prev, t = _batch(10, 21)
    with pytest.raises(ValueError):
        tr.forward(_t(ob), _t(prev))           # 21 windows > max_windows 20
    with pytest.raises(ValueError):
        tr.forward(_t(ob[:5, :4]), _t(prev[:5, :4]))   # T = 5 != 10


def test_graph_step_equals_eager():
    T, B = 10, 20
    ob, prev, t = _batch(T, B, 21)
    eager, graphed = _trainer(T, B, keep_prob=0.5, seed=4), _trainer(T, B, keep_prob=0.5, seed=4)
    step = graphed.graph_step(B)
    for _ in range(3):
        eager.step(_t(ob), _t(prev), _t(t))
        step(_t(ob).to(DEV), _t(prev).to(DEV), _t(t).to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(eager.params(), graphed.params())
    assert eager.counter() == graphed.counter() == 3
    np.testing.assert_array_equal(eager.metrics(3), graphed.metrics(3))


def test_final_state_of_a_training_step_is_the_pre_update_forward_state():
    """rdl_final_state after rdl_step = final_state_batch of the same sess.run (computed with
    the parameters before the update, backup/lstm_bbpt.py:147-155): equal to rdl_forward's
    state at those parameters, and to the oracle."""
    T, B = 10, 20
    ob, prev, t = _batch(T, B, 31)
    st0 = np.random.RandomState(4).uniform(-.5, .5, (2, B, 200)).astype(np.float32)
    tr = _trainer(T, B, "kl")
    p0 = tr.params().cpu().numpy()
    _, fin = tr.forward(_t(ob), _t(prev), _t(st0))
    tr.step(_t(ob), _t(prev), _t(t), _t(st0))
    got = tr.final_state(B)
    assert torch.equal(got, fin)
    want = ln.forward(p0, ob, prev, st0)["state"]
    np.testing.assert_allclose(got.cpu().numpy(), np.stack(want), atol=5e-5, rtol=1e-4)
    assert not np.array_equal(tr.params().cpu().numpy(), p0)
    with pytest.raises(RuntimeError):
        tr.final_state(B - 1)                   # the last pass had B windows


def test_carried_state_chain_matches_oracle():
    """Truncated BPTT as the variant driver runs it: window k starts from window k-1's final
    state (after that window's Adam step); gradients and carried states follow the oracle
    over three windows."""
    T, B = 10, 20
    tr = _trainer(T, B, "kl")
    s_dev, s_np = None, None
    for k in range(3):
        ob, prev, t = _batch(T, B, 40 + k)
        p = tr.params().cpu().numpy()
        g = tr.rollout(_t(ob), _t(prev), _t(t), s_dev).cpu().numpy()
        fw = ln.forward(p, ob, prev, s_np)
        _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
        _grad_check(g, ln.backward(p, fw, d))
        tr.apply()
        s_dev = tr.final_state(B)
        s_np = np.stack(fw["state"]).astype(np.float32)
        np.testing.assert_allclose(s_dev.cpu().numpy(), s_np, atol=5e-5, rtol=1e-4)
    assert tr.counter() == 3


def test_bptt_variant_driver_runs():
    """lstm_train.train_bptt (backup/lstm_bbpt.py): teacher warm-up, then per episode a
    40-window BPTT pass with carried state and an episode stepped by the student."""
    from reacherdistilation_amd import lstm_train
    st, ds, losses = lstm_train.train_bptt(episodes=5, warmup_episodes=2, keep_prob=0.5, log=lambda *a: None)
    assert ds.num_episodes() == 5 and len(losses) == 2
    assert st.counter() == 2 * 40
    assert all(np.isfinite(losses)) and all(x > 0 for x in losses)


@pytest.mark.parametrize("fmt", ["lstm.safetensors", "lstm_with_keep_probability_1.0.ckpt"])
def test_checkpoint_round_trip(tmp_path, fmt):
    """save/load = the reference's Saver over the 'LSTM' scope (lstm_train.py:86-107,199), as a
    safetensors file or as a TF checkpoint with the reference's variable names: params and
    Adam slots come back bitwise; the beta powers and step counter start afresh, so the
    restored trainer's next step equals a fresh optimiser's first step from the same params
    and slots."""
    T, B = 10, 20
    ob, prev, t = _batch(T, B, 51)
    a = _trainer(T, B, "kl")
    for _ in range(3):
        a.step(_t(ob), _t(prev), _t(t))
    path = str(tmp_path / fmt)
    a.save(path)
    m0, v0 = (x.cpu().numpy() for x in a._slots())
    b = _trainer(T, B, "kl", params=ln.init(99))
    b.load(path)
    assert torch.equal(a.params(), b.params()) and b.counter() == 0
    assert all(torch.equal(x.cpu(), torch.from_numpy(y)) for x, y in zip(b._slots(), (m0, v0)))
    # the next step from the restored state: m, v carried over, beta powers from t = 1
    p0 = b.params().cpu().numpy().copy()
    fw = ln.forward(p0, ob, prev)
    _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
    g = b.rollout(_t(ob), _t(prev), _t(t)).cpu().numpy()
    _grad_check(g, ln.backward(p0, fw, d))
    b.apply()
    m, v = m0, v0
    m = m + (g - m) * np.float32(0.1)
    v = v + (g * g - v) * np.float32(0.001)
    alpha = np.float32(1e-3) * np.sqrt(np.float32(1) - np.float32(0.999)) / (np.float32(1) - np.float32(0.9))
    want = p0 - (m * alpha) / (np.sqrt(v) + np.float32(1e-8))
    np.testing.assert_allclose(b.params().cpu().numpy(), want, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("name", ["student.safetensors", "student.ckpt"])
def test_driver_restores_and_saves_the_student(tmp_path, name):
    from reacherdistilation_amd import lstm_train
    path = str(tmp_path / name)
    msgs = []
    st, _, _ = lstm_train.train(episodes=4, warmup_episodes=2, restore=True, student_path=path, log=msgs.append)
    assert any("does not exist" in m for m in msgs)       # first run: nothing to restore, only a message
    saved = st.params().clone()
    st2, _, _ = lstm_train.train(train=False, restore=True, student_path=path, log=msgs.append)
    assert torch.equal(st2.params(), saved)


@pytest.mark.parametrize("T,B,with_state", [(10, 20, False), (10, 32, True), (1, 7, True), (3, 1, False),
                                             (16, 24, True), (40, 17, False)])
def test_persistent_recurrence_matches_per_step_launches(T, B, with_state):
    """B <= 32: the whole forward recurrence and the whole BPTT each run as one persistent
    launch (lstm_fwd_persist_kernel / lstm_bptt_persist_kernel).  Forward: bitwise the per-step
    kernels (same MFMA sequence and cell arithmetic); gradient: the dh sums over the 800 gate
    columns run in another order, so within 1e-5 of max|g| (and both within the oracle bound)."""
    ob, prev, t = _batch(T, B, 11 + B)
    st = np.random.RandomState(4).uniform(-.5, .5, (2, B, 200)).astype(np.float32) if with_state else None
    out = {}
    for mode in ("1", "0"):
        tr = _trainer(T, B, "kl", step_recurrence=mode == "0")
        y, fin = tr.forward(_t(ob), _t(prev), None if st is None else _t(st))
        g = tr.rollout(_t(ob), _t(prev), _t(t), None if st is None else _t(st)).cpu().numpy()
        out[mode] = (y.cpu().numpy(), fin[0].cpu().numpy(), fin[1].cpu().numpy(), g, tr.params().cpu().numpy())
        tr.close()
    for a, b in zip(out["1"][:3], out["0"][:3]):
        assert np.array_equal(a, b)
    g1, g0 = out["1"][3], out["0"][3]
    assert np.abs(g1 - g0).max() <= 1e-5 * np.abs(g0).max()
    p = out["1"][4]
    fw = ln.forward(p, ob, prev, st)
    _, d, _ = ln.loss_and_dout(fw["pdflat"], t, "kl", T * B)
    _grad_check(g1, ln.backward(p, fw, d))


@pytest.mark.parametrize("T,B", [(10, 20), (3, 130), (1, 5), (10, 4100), (4, 16384), (10, 16384)])
def test_fused_head_matches_the_layer_gemms(T, B):
    """At most 16,384 rows: the heads' forward is one launch (head_fwd_kernel) and its backward
    two (head_bwd_kernel + a fixed-order reduce).  Same MFMA k order and epilogues as the
    per-layer GEMMs for the activations and the data gradients, so the outputs, dh_head and
    everything BPTT derives from it (the LSTM's gradients) are bitwise those of
    layer_head=True; the head's weight gradients sum the rows in per-workgroup partials (16
    rows, or 2-8 tiles of 16 rows in registers for large batches: (10, 4100) has a ragged last
    workgroup and tile, (4, 16384) four tiles per workgroup, (10, 16384) eight -- the cap, the
    benchmarked size), so they agree to 1e-5 of their largest entry."""
    ob, prev, t = _batch(T, B, 21 + B)
    out = {}
    for mode in ("1", "0"):
        tr = _trainer(T, B, "mse", layer_head=mode == "0")
        assert tr.fused_head == (mode == "1")   # rdl_head_path: the path this trainer takes
        y, _ = tr.forward(_t(ob), _t(prev))
        g = tr.rollout(_t(ob), _t(prev), _t(t)).cpu().numpy()
        out[mode] = (y.cpu().numpy(), g)
        tr.close()
    assert np.array_equal(out["1"][0], out["0"][0])
    w1 = ln.CELL_PARAMS   # the heads' [W1 b1 ... W5 b5] x T range starts here
    assert np.array_equal(out["1"][1][:w1], out["0"][1][:w1])
    h1, h0 = out["1"][1][w1:], out["0"][1][w1:]
    assert np.abs(h1 - h0).max() <= 1e-5 * np.abs(h0).max()


def test_persistent_kernels_many_steps_stay_in_step_with_per_step_path():
    """500 training steps of the reference's 20 windows through the persistent kernels (50
    workgroups exchanging h granules / partial dh every unrolled step; the granule generation
    advances on the device per forward) and through the per-step launches: no hand-off timeout
    (rdl_get_counter raises on one), the same step count, two persistent runs bitwise equal, and
    parameters that stay within the accumulated f32 reordering of the two paths' gradient sums."""
    T, B = 10, 20
    ob, prev, t = _batch(T, B, 77)
    params = {}
    for mode in ("1", "1b", "0"):   # persistent twice (run to run: bitwise), then per-step
        tr = _trainer(T, B, "kl", step_recurrence=mode == "0")
        for _ in range(500):
            tr.step(_t(ob), _t(prev), _t(t))
        assert tr.counter() == 500
        params[mode] = tr.params().cpu().numpy().astype(np.float64)
        tr.close()
    assert np.array_equal(params["1"], params["1b"])   # fixed-order sums: deterministic
    d = np.abs(params["1"] - params["0"]).max()
    assert d <= 1e-4 * np.abs(params["0"]).max(), d


def test_persistent_forward_past_256_steps_two_calls():
    """the persistent forward's granule tags carry the unrolled step in their own
    12-bit field (the old 8-bit phase let step 257 of one call pass for step 1 of the next).  At
    T = 258 with 8 windows (persistent: B <= 32, T < 4,096) a trainer's second forward equals a
    fresh trainer's first forward on the same inputs bitwise -- nothing of the first call is taken
    for the second's -- and both agree with the per-step launches to f32 rounding (at 2,064 rows
    the per-step input product tiles its k sum differently)."""
    T, B = 258, 8
    ob, prev, _ = _batch(T, B, 91)
    ob2 = np.ascontiguousarray(ob[::-1])
    tr = _trainer(T, B, "kl")
    tr.forward(_t(ob), _t(prev))
    y2, fin2 = tr.forward(_t(ob2), _t(prev))
    y2, h2 = y2.cpu().numpy(), fin2[1].cpu().numpy()
    tr.close()
    tr = _trainer(T, B, "kl")
    y1, fin1 = tr.forward(_t(ob2), _t(prev))
    assert np.array_equal(y2, y1.cpu().numpy()) and np.array_equal(h2, fin1[1].cpu().numpy())
    tr.close()
    tr = _trainer(T, B, "kl", step_recurrence=True)
    y0, _ = tr.forward(_t(ob2), _t(prev))
    tr.close()
    assert np.abs(y2 - y0.cpu().numpy()).max() <= 1e-5 * max(1.0, np.abs(y2).max())

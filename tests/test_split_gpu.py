"""f32 on bf16 MFMAs (rdd_config.f32_split = 1, include/reacher_distill.h): parity with the f64
oracle at the f32 path's tolerances, and f32 accuracy measured against the exact f32 MFMA
path on the same inputs.

Tolerances: as tests/test_distill_gpu.py (tests/parity.py: means 2e-5, gradient per entry
2e-5 x M_e and 1e-5 x max|g|, states per component).  Accuracy: the split path's gradient
error vs the f64 oracle stays within 3x the exact-f32 path's error (both are f32 sums over the
batch; the split keeps every partial product of order >= 2^-16, so its rounding is f32's).
"""
import numpy as np
import pytest
import torch

from oracle import policy_np as pn
from tests.test_distill_gpu import _grad_check, _np_params, _obs_from_state, _trainer

pytestmark = pytest.mark.gpu


def _g64(tr, st0, sp, loss, n):
    ob = _obs_from_state(st0)
    fs = pn.forward(sp.astype(np.float64), *_np_params(tr.student)[1:], ob)
    ft = pn.forward(*_np_params(tr.teacher), ob)
    L, dmean, dls, sq = pn.loss_and_dmean(fs, ft, loss, n)
    return pn.backward(sp.astype(np.float64), fs, dmean, dls), fs, ft


@pytest.mark.parametrize("n", [17, 1000, 40001, 65536])
@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_split_gradient_matches_oracle(n, loss):
    tr = _trainer(n, loss=loss, f32_split=True)
    _grad_check(tr, loss, "teacher")


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_split_is_f32_accurate(loss):
    """Same envs, same weights: split and exact paths against the f64 oracle."""
    n = 65536
    out = {}
    for split in (False, True):
        tr = _trainer(n, loss=loss, f32_split=split)
        st0 = tr.env_state().cpu().numpy()
        sp = tr.student_params().cpu().numpy()
        tr.rollout()
        g = tr.grad().cpu().numpy().astype(np.float64)
        g64, fs, ft = _g64(tr, st0, sp, loss, n)
        out[split] = (np.abs(g - g64).max() / np.abs(g64).max(), g, tr.env_state().cpu().numpy())
        tr.close()
    e_exact, e_split = out[False][0], out[True][0]
    print(f"split accuracy {loss}: split {e_split:.2e} exact {e_exact:.2e}")
    assert e_split < 1e-5 and e_split <= 3 * e_exact + 1e-7, (e_split, e_exact)
    # the two paths differ by f32 rounding only
    ge, gs = out[False][1], out[True][1]
    assert np.abs(gs - ge).max() <= 2e-5 * np.abs(ge).max()
    np.testing.assert_allclose(out[True][2], out[False][2], atol=1e-5, rtol=1e-5)


def test_split_forward_means_in_rollout_match_exact():
    """The teacher means that step the envs: split teacher vs exact teacher, one step from
    the same state (the states after the step agree to f32 rounding of the actions)."""
    a = _trainer(4096, f32_split=False)
    b = _trainer(4096, f32_split=True)
    assert torch.equal(a.env_state(), b.env_state())
    a.rollout(); b.rollout()
    d = (a.env_state() - b.env_state()).abs().max().item()
    assert d < 1e-5, d


def test_split_dagger_adam_step():
    n = 4096
    tr = _trainer(n, loss="mse", act="student", f32_split=True)
    p0 = tr.student_params().cpu().numpy()
    g, g64, L, sq = _grad_check(tr, "mse", "student")
    tr.apply()
    p1 = tr.student_params().cpu().numpy()
    opt = pn.AdamTF1(pn.P_TOT)
    ref = p0.copy()
    opt.step(ref, g64.astype(np.float32))
    strong = np.abs(g64) > 1e-3 * np.abs(g64).max()
    np.testing.assert_allclose(p1[strong], ref[strong], atol=1e-6, rtol=0)
    m = tr.metrics(1)[0]
    assert m[3] == n and m[1] == pytest.approx(L, rel=1e-3) and m[2] == pytest.approx(sq, rel=1e-3)


def test_split_multistep_matches_c_oracle(oracle_c):
    """60 Adam steps across an episode boundary: loss curve and final student vs the C f32
    oracle (which runs exact f32 products), as test_multistep_matches_c_oracle."""
    n, seed, steps = 4096, 5, 60
    tr = _trainer(n, seed=seed, lr=1e-3, stagger=True, f32_split=True)
    tp, smu, ssd = tr.teacher.flat, tr.student.ob_mean, tr.student.ob_std
    sp = tr.student.flat.copy()
    st = oracle_c.philox_reset(n, 0, seed, 0)
    m = np.zeros(pn.P_TOT, np.float32); v = np.zeros(pn.P_TOT, np.float32)
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    ref_loss = []
    for k in range(steps):
        g, met = oracle_c.distill_step(st, k, (tp, tr.teacher.ob_mean, tr.teacher.ob_std), (sp, smu, ssd),
                                       seed=seed, loss="mse", stagger=True, nthreads=4)
        oracle_c.adam_tf1(sp, m, v, g, float(b1p), float(b2p), lr=1e-3)
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
        ref_loss.append(met[1])
        tr.step()
    got = tr.metrics(steps)[:, 1]
    np.testing.assert_allclose(got, ref_loss, rtol=2e-3)
    p = tr.student_params().cpu().numpy()
    assert np.abs(p - sp).max() < 2e-3 * max(1.0, np.abs(sp).max())


def test_split_student_learns_teacher():
    tr = _trainer(16384, lr=1e-3, f32_split=True)
    for _ in range(300):
        tr.step()
    m = tr.metrics(300)
    mse = m[:, 2] / (2 * m[:, 3])
    assert mse[-10:].mean() < 1e-3, mse[-10:].mean()


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_bf16_student_with_split_teacher(loss):
    """Config 5 arithmetic with the teacher's hidden layer on split bf16 MFMAs: the gradient
    still matches the bf16 student definition against the f64 teacher."""
    n = 65536
    tr = _trainer(n, loss=loss, act="student", student_dtype="bf16", f32_split=True)
    st0 = tr.env_state().cpu().numpy()
    sp = tr.student_params().cpu().numpy().astype(np.float64)
    tr.rollout()
    g = tr.grad().cpu().numpy()
    ob = _obs_from_state(st0).astype(np.float32)
    fs = pn.forward_bf16(sp, *_np_params(tr.student)[1:], ob)
    ft = pn.forward(*_np_params(tr.teacher), ob.astype(np.float64))
    L, dmean, dls, sq = pn.loss_and_dmean(fs, ft, loss, n)
    gb = pn.backward_bf16(sp, fs, dmean, dls)
    err_b = np.abs(g - gb).max() / np.abs(gb).max()
    from tests import parity
    rep = parity.grad_report(g, gb, parity.abs_scale(sp, fs, dmean, dls, bf16=True))
    print(f"bf16 + split teacher {loss}: {err_b:.2e} {rep}")
    assert err_b < 1e-4, err_b
    assert rep["entry"] <= parity.TOL_ENTRY_BF16, rep


def test_split_graph_replay_matches_eager():
    a = _trainer(8192, seed=1, f32_split=True)
    b = _trainer(8192, seed=1, f32_split=True)
    g = b.capture(steps=3)
    for _ in range(2):
        g.replay()
        for _ in range(3):
            a.step()
    torch.cuda.synchronize()
    assert torch.equal(a.student_params(), b.student_params())
    assert torch.equal(a.env_state(), b.env_state())

"""GPU parity of the fused rollout+distill kernels (through the C ABI) against the oracles.

Tolerances (round 4; tests/parity.py): action means 2e-5 abs; gradient
per entry <= 2e-5 x M_e (M_e = the sum over envs of |each env's contribution to entry e|) and
globally <= 1e-5 x max|g|; per-env contributions isolated at N = 64 / 128 (every lane of a
64-env group owns one env); env state after the step per component (angles / offsets 1e-5,
velocities 1e-5 + 1e-5 rel, targets bitwise) for limit-inactive envs, the round-3 bound for
the few near the joint limit; Adam updates compared where the gradient is not ~0 (a TF1 Adam
step is ~lr*sign(g), so sign noise on vanishing gradients is expected); resets and counters
bit-exact.  Every gradient check prints its measured errors (pytest -s).
"""
import numpy as np
import pytest
import torch

from oracle import policy_np as pn
from oracle import reacher_np as rn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainer(n, loss="mse", act="teacher", seed=3, **kw):
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    return DistillTrainer(DistillConfig(n_envs=n, seed=seed, loss=loss, act_with=act, **kw), device=DEV)


def _obs_from_state(st):
    st = st.astype(np.float64)
    z = np.zeros_like(st[0])
    ob = rn.observe(st[0], st[1], st[2], st[3], st[4], st[5], z, z)
    ob[:, 8], ob[:, 9] = st[6], st[7]
    return ob


def _np_params(p):
    return p.flat.astype(np.float64), p.ob_mean.astype(np.float64), p.ob_std.astype(np.float64)


@pytest.mark.parametrize("n", [1, 33, 1000, 4096])
def test_forward_matches_oracle(n):
    tr = _trainer(128)
    # non-trivial filters and biases
    rs = np.random.RandomState(n)
    tr.teacher.ob_mean[:] = rs.uniform(-.1, .1, 11); tr.teacher.ob_std[:] = rs.uniform(.5, 2, 11)
    tr.student.flat[pn.P_B1:pn.P_W2] = rs.uniform(-.2, .2, 64)
    tr.student.flat[pn.P_B2:pn.P_W3] = rs.uniform(-.2, .2, 64)
    tr.set_teacher(tr.teacher); tr.set_student(tr.student)
    ob = _obs_from_state(np.stack([rs.uniform(-3, 3, n), rs.uniform(-3, 3, n), rs.uniform(-9, 9, n),
                                   rs.uniform(-9, 9, n), rs.uniform(-.2, .2, n), rs.uniform(-.2, .2, n),
                                   rs.uniform(-.3, .3, n), rs.uniform(-.3, .3, n)]))
    t, s = tr.forward(torch.tensor(ob, dtype=torch.float32))
    ft = pn.forward(*_np_params(tr.teacher), ob.astype(np.float32).astype(np.float64))
    fs = pn.forward(*_np_params(tr.student), ob.astype(np.float32).astype(np.float64))
    np.testing.assert_allclose(t.cpu().numpy()[:, :2], ft["mean"], atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(s.cpu().numpy()[:, :2], fs["mean"], atol=2e-5, rtol=1e-5)
    assert np.all(t.cpu().numpy()[:, 2:] == tr.teacher.flat[pn.P_LS:].astype(np.float32))


def _grad_check(tr, loss, act, tol_entry=None):
    from tests import parity
    st0 = tr.env_state().cpu().numpy()
    sp = tr.student_params().cpu().numpy()
    c0 = tr.counter()   # env clock of this rollout (rdd_rollout advances it)
    tr.rollout()
    g = tr.grad().cpu().numpy()
    st1 = tr.env_state().cpu().numpy()
    ob = _obs_from_state(st0)
    g64, M, (fs, ft, L, sq) = parity.oracle_grad(sp, tr.teacher, tr.student, ob, loss, tr.n_global)
    ok, rep = parity.grad_ok(g, g64, M, tol_entry or parity.TOL_ENTRY)
    print(f"grad n={tr.n_local} {loss} split={tr.cfg.f32_split}: {rep}")
    assert ok, rep
    # the env moved with the chosen policy's mean (envs whose staggered episode ended at
    # this step were reset instead: test_staggered_resets_bit_exact covers those)
    a = (fs if act == "student" else ft)["mean"].astype(np.float32)
    ref = np.ascontiguousarray(st0.astype(np.float64))
    __import__("oracle.ref_c", fromlist=["x"]).step(ref, a, np.float64)
    n = st0.shape[1]
    off = (np.arange(n) // 32) % 50 if tr.cfg.stagger else np.zeros(n, np.int64)
    reset = (c0 + off) % 50 == 49
    near = np.abs(st0[1]) > 2.8
    keep = ~reset
    sok, worst = parity.state_ok(st1[:, keep], ref[:, keep], near[keep])
    print(f"state n={n}: {worst}")
    assert sok, worst
    return g, g64, L, sq


@pytest.mark.parametrize("n", [17, 1000, 4096, 40001, 65536])   # 16-, 16-, 16-, 32-, 64-env groups
@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_rollout_gradient_matches_oracle(n, loss):
    tr = _trainer(n, loss=loss)
    _grad_check(tr, loss, "teacher")
    # metrics of that step
    m = tr.metrics(0)  # counter not advanced by rollout alone
    assert m.shape == (0, 4)


@pytest.mark.parametrize("grid,n", [(7, 3000), (300, 300 * 4 * 64), (257, 20000)])
def test_gradient_over_explicit_grids(grid, n):
    """rdd_config.grid sets the workgroups (= partial rows of the column-chunked workspace the
    reduce sums): few rows, more rows than the 256 a reduce thread sums in its unrolled
    four-way loop (the remainder path), and a count that is no multiple of 64 -- the same
    gradient as the oracle; the grid changes only the summation order."""
    tr = _trainer(n, loss="kl", grid=grid)
    g, g64, _, _ = _grad_check(tr, "kl", "teacher")
    ref = _trainer(n, loss="kl")
    ref.rollout()
    gr = ref.grad().cpu().numpy()
    assert np.abs(g - gr).max() <= 1e-5 * np.abs(gr).max()


def test_dagger_rollout_and_adam_step():
    n = 4096
    tr = _trainer(n, loss="mse", act="student")
    p0 = tr.student_params().cpu().numpy()
    g, g64, L, sq = _grad_check(tr, "mse", "student")
    tr.apply()
    p1 = tr.student_params().cpu().numpy()
    assert tr.counter() == 1
    opt = pn.AdamTF1(pn.P_TOT)
    ref = p0.copy()
    opt.step(ref, g64.astype(np.float32))
    strong = np.abs(g64) > 1e-3 * np.abs(g64).max()
    np.testing.assert_allclose(p1[strong], ref[strong], atol=1e-6, rtol=0)
    assert np.abs(p1 - ref).max() <= 2.01 * opt.lr
    m = tr.metrics(1)[0]
    assert m[3] == n and m[1] == pytest.approx(L, rel=1e-3) and m[2] == pytest.approx(sq, rel=1e-3)


def test_episode_boundary_resets_bit_exact(oracle_c):
    n, seed = 2000, 9
    tr = _trainer(n, seed=seed, stagger=False)
    st = tr.env_state().cpu().numpy()
    assert np.array_equal(st[:6], oracle_c.philox_reset(n, 0, seed, 0)[:6])
    for k in range(50):
        tr.step()
    assert tr.counter() == 50
    st = tr.env_state().cpu().numpy()
    assert np.array_equal(st[:6], oracle_c.philox_reset(n, 0, seed, 1)[:6])
    m = tr.metrics(50)
    assert np.all(m[:, 3] == n)


@pytest.mark.parametrize("stagger", [False, True])
def test_multistep_matches_c_oracle(oracle_c, stagger):
    """60 steps (crossing an episode boundary) of teacher-driven MSE distillation with Adam:
    the loss curve and final student match the C f32 oracle run step for step."""
    n, seed, steps = 4096, 5, 60
    tr = _trainer(n, seed=seed, lr=1e-3, stagger=stagger)
    tp, smu, ssd = tr.teacher.flat, tr.student.ob_mean, tr.student.ob_std
    sp = tr.student.flat.copy()
    st = oracle_c.philox_reset(n, 0, seed, 0)
    m = np.zeros(pn.P_TOT, np.float32); v = np.zeros(pn.P_TOT, np.float32)
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    ref_loss = []
    for k in range(steps):
        g, met = oracle_c.distill_step(st, k, (tp, tr.teacher.ob_mean, tr.teacher.ob_std), (sp, smu, ssd),
                                       seed=seed, loss="mse", stagger=stagger, nthreads=4)
        oracle_c.adam_tf1(sp, m, v, g, float(b1p), float(b2p), lr=1e-3)
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
        ref_loss.append(met[1])
        tr.step()
    got = tr.metrics(steps)[:, 1]
    np.testing.assert_allclose(got, ref_loss, rtol=2e-3)
    p = tr.student_params().cpu().numpy()
    assert np.abs(p - sp).max() < 2e-3 * max(1.0, np.abs(sp).max())


def test_student_learns_teacher():
    """Staggered episodes: action-MSE falls by >10x and below the north-star 1e-3 within
    300 steps on 16k envs (lr 1e-3; the C oracle reaches ~3.5e-4 at 4k envs)."""
    tr = _trainer(16384, lr=1e-3)
    for _ in range(300):
        tr.step()
    m = tr.metrics(300)
    mse = m[:, 2] / (2 * m[:, 3])
    assert mse[-10:].mean() < 0.1 * mse[:10].mean(), (mse[:10].mean(), mse[-10:].mean())
    assert mse[-10:].mean() < 1e-3, mse[-10:].mean()


def test_staggered_resets_bit_exact(oracle_c):
    """With stagger, env g resets when (C + (g/32) % 50) % 50 == 49, from Philox episode
    (C + off)/50 + 1: the reset envs' states equal the oracle's draws bit for bit, every
    other env kept its episode going."""
    n, seed = 4096, 11
    tr = _trainer(n, seed=seed, stagger=True)
    off = (np.arange(n) // 32) % 50
    for k in range(7):
        tr.step()
    st = tr.env_state().cpu().numpy()
    C = 6                                      # the step just taken
    u = C + off
    hit = (u % 50) == 49
    assert hit.sum() == 64                     # groups 43 and 93 (offset 43)
    ep = u // 50 + 1
    for e in np.unique(ep[hit]):
        idx = np.flatnonzero(hit & (ep == e))
        ref = oracle_c.philox_draws(seed, idx, int(e))
        got = st[:6, idx].T
        assert np.array_equal(got[:, [0, 1, 2, 3, 4, 5]], ref), e
    # envs that did not reset are not at a fresh draw
    assert not np.array_equal(st[:6, ~hit], oracle_c.philox_reset(n, 0, seed, 0)[:6, ~hit])


def test_graph_capture_replay_matches_eager():
    """The step is capturable in a HIP graph (no host sync inside) and replays identically."""
    a = _trainer(8192, seed=1)
    b = _trainer(8192, seed=1)
    g = b.capture(steps=3)
    for _ in range(4):
        g.replay()
        for _ in range(3):
            a.step()
    torch.cuda.synchronize()
    assert b.counter() == a.counter() == 12
    assert torch.equal(a.student_params(), b.student_params())
    assert torch.equal(a.env_state(), b.env_state())


# ---------------------------------------------------------------- bf16 student (config 5)
# Tolerances: the kernel and oracle/policy_np.forward_bf16/backward_bf16 round the same
# operands to bf16; they differ by f32-vs-f64 accumulation order and the kernel's 2-ulp
# tanh, which can flip a bf16 rounding (one bf16 ulp = 2^-8 relative) of an activation now
# and then.  So: means within 1e-3 (max) and 2e-5 (median); the gradient within 1e-2 of its
# max entry.  Each check also asserts the kernel is much closer to the bf16 definition than
# to the f32 student, i.e. the bf16 arithmetic is the one implemented.

def test_bf16_forward_matches_bf16_oracle():
    n = 4096
    tr = _trainer(128, student_dtype="bf16")
    rs = np.random.RandomState(5)
    tr.student.flat[pn.P_B1:pn.P_W2] = rs.uniform(-.2, .2, 64)
    tr.student.flat[pn.P_W3:pn.P_B3] = rs.normal(0, .3, 128)
    tr.student.ob_mean[:] = rs.uniform(-.1, .1, 11); tr.student.ob_std[:] = rs.uniform(.5, 2, 11)
    tr.set_student(tr.student)
    ob = _obs_from_state(np.stack([rs.uniform(-3, 3, n), rs.uniform(-3, 3, n), rs.uniform(-9, 9, n),
                                   rs.uniform(-9, 9, n), rs.uniform(-.2, .2, n), rs.uniform(-.2, .2, n),
                                   rs.uniform(-.3, .3, n), rs.uniform(-.3, .3, n)])).astype(np.float32)
    _, s = tr.forward(torch.tensor(ob))
    got = s.cpu().numpy()[:, :2]
    p, mu, sd = _np_params(tr.student)
    fb = pn.forward_bf16(p, mu, sd, ob)
    f32 = pn.forward(p, mu, sd, ob.astype(np.float64))
    e_b = np.abs(got - fb["mean"])
    e_f = np.abs(got - f32["mean"])
    assert e_b.max() < 1e-3 and np.median(e_b) < 2e-5, (e_b.max(), np.median(e_b))
    assert np.median(e_f) > 10 * np.median(e_b), (np.median(e_f), np.median(e_b))


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_bf16_rollout_gradient_matches_bf16_oracle(loss):
    n = 65536
    tr = _trainer(n, loss=loss, act="student", student_dtype="bf16")
    st0 = tr.env_state().cpu().numpy()
    sp = tr.student_params().cpu().numpy().astype(np.float64)
    tr.rollout()
    g = tr.grad().cpu().numpy()
    ob = _obs_from_state(st0).astype(np.float32)
    fs = pn.forward_bf16(sp, *_np_params(tr.student)[1:], ob)
    ft = pn.forward(*_np_params(tr.teacher), ob.astype(np.float64))
    L, dmean, dls, sq = pn.loss_and_dmean(fs, ft, loss, n)
    gb = pn.backward_bf16(sp, fs, dmean, dls)
    fs32 = pn.forward(sp, *_np_params(tr.student)[1:], ob.astype(np.float64))
    g32 = pn.backward(sp, fs32, *pn.loss_and_dmean(fs32, ft, loss, n)[1:3])
    err_b = np.abs(g - gb).max() / np.abs(gb).max()
    err_f = np.abs(g - g32).max() / np.abs(g32).max()
    from tests import parity
    rep = parity.grad_report(g, gb, parity.abs_scale(sp, fs, dmean, dls, bf16=True))
    print(f"bf16 grad {loss}: global {err_b:.2e} vs f32 {err_f:.2e}; {rep}")
    assert err_b < 1e-4, err_b
    assert rep["entry"] <= parity.TOL_ENTRY_BF16, rep
    assert err_f > 2 * err_b, (err_f, err_b)


def test_bf16_dagger_student_learns():
    """DAgger with the bf16 student (config 5's arithmetic): action-MSE falls by >10x."""
    tr = _trainer(16384, act="student", lr=1e-3, student_dtype="bf16")
    for _ in range(300):
        tr.step()
    m = tr.metrics(300)
    mse = m[:, 2] / (2 * m[:, 3])
    assert mse[-10:].mean() < 0.1 * mse[:10].mean(), (mse[:10].mean(), mse[-10:].mean())


def test_accumulated_steps_sum_rollout_gradients():
    """accum_steps = K: the gradient of one optimiser step is the sum of K rollouts' gradients
    at frozen weights (KL: no normalisation, so bit-exact vs separate rollouts), the env clock
    advances every rollout, and Adam runs once per K env steps."""
    K = 3
    a = _trainer(2048, loss="kl", accum_steps=K)
    b = _trainer(2048, loss="kl")
    gs = []
    for k in range(K - 1):
        a.step()
        b.launch(b.STAGE_ROLLOUT)
        b.launch(b.STAGE_REDUCE)
        gs.append(b.grad().clone())
    assert torch.equal(a.grad(), gs[0] + gs[1])
    assert a.counters() == (K - 1, 0) and torch.equal(a.env_state(), b.env_state())
    p0 = a.student_params().clone()
    a.step()
    assert a.counters() == (K, 1) and not torch.equal(a.student_params(), p0)
    m = a.metrics(1)[0]
    assert m[3] == K * 2048   # the step's metrics slot sums its K rollouts


def test_accumulated_mse_normalises_over_k_rollouts():
    K = 2
    a = _trainer(1024, loss="mse", accum_steps=K)
    b = _trainer(1024, loss="mse")
    a.step()
    b.launch(b.STAGE_ROLLOUT)
    b.launch(b.STAGE_REDUCE)
    torch.testing.assert_close(a.grad() * K, b.grad(), rtol=1e-6, atol=1e-9)


def test_group_size_changes_only_the_summation_order():
    """16-, 32- and 64-env groups (chosen by batch size) step every env
    identically (bitwise) and give the same gradient up to f32 reordering of the sums."""
    n = 3000
    out = {}
    for gs in (16, 32, 64):
        tr = _trainer(n, loss="kl", group_envs=gs)
        tr.rollout()
        out[gs] = (tr.grad().cpu().numpy().astype(np.float64), tr.env_state().cpu().numpy())
        tr.close()
    g16, s16 = out[16]
    for gs in (32, 64):
        g, s_ = out[gs]
        assert np.array_equal(s_, s16)
        assert np.abs(g - g16).max() <= 1e-5 * np.abs(g16).max()


@pytest.mark.parametrize("n", [4096, 777, 8192])
@pytest.mark.parametrize("split,loss,act", [(True, "mse", "teacher"), (False, "mse", "teacher"),
                                            (True, "kl", "teacher"), (True, "mse", "student"),
                                            (False, "kl", "student")])
def test_helper_layout_matches_the_plain_layout(n, split, loss, act):
    """The helper-pair layout (automatic for <= two 16-env groups per CU: pairs 2, 3 of a
    workgroup run pairs 0, 1's teacher forwards, weight gradient dW2 and -- teacher acting --
    env steps) against the plain layout (group_envs = 16 fixed), one fused step: the env states
    bitwise (round 5: the env step's rounding is fixed by its source, rd_physics.h
    FP_SOURCE_ROUNDING, so the helper wave's inlined copy rounds like the owner's; r04 measured
    1-ulp differences in ~29 % of the envs before), the gradient to f32 reordering of the sums (the partial rows group the envs
    differently), the Adam update where the gradient is not ~0, the step's metrics."""
    out = {}
    for gs in (0, 16):
        tr = _trainer(n, loss=loss, act=act, f32_split=split, group_envs=gs, seed=5)
        tr.step()
        out[gs] = (tr.grad().cpu().numpy().astype(np.float64), tr.env_state().cpu().numpy(),
                   tr.student_params().cpu().numpy().astype(np.float64), tr.metrics(1))
        tr.close()
    (gh, sh, ph, mh), (gp, spl, pp, mp) = out[0], out[16]
    nd = int((sh != spl).any(0).sum())
    print(f"helper vs plain n={n} split={split} {loss} {act}: {nd} envs differ, max {np.abs(sh - spl).max():.3g}")
    assert nd == 0
    assert np.abs(gh - gp).max() <= 1e-5 * np.abs(gp).max()
    strong = np.abs(gp) > 1e-3 * np.abs(gp).max()
    assert np.abs(ph - pp)[strong].max() <= 1e-6
    assert mh[0, 3] == mp[0, 3] == n                               # envs stepped
    np.testing.assert_allclose(mh[0, :3], mp[0, :3], rtol=1e-5, atol=1e-7)


def _limit_states(n, rs):
    """Env states where the joint-1 limit (|q1| = 3) is active in every RK stage for half of
    the envs (|q1| in [3.05, 3.3], moving outward or inward slowly) and inactive in every stage
    for the other half (|q1| <= 2.85); targets and fingertip offsets consistent with q."""
    q0 = rs.uniform(-np.pi, np.pi, n)
    side = np.where(rs.uniform(size=n) < 0.5, -1.0, 1.0)
    active = np.arange(n) % 2 == 0
    q1 = np.where(active, side * rs.uniform(3.05, 3.3, n), rs.uniform(-2.85, 2.85, n))
    v0, v1 = rs.uniform(-1, 1, n), rs.uniform(-0.5, 0.5, n)
    tx, ty = rs.uniform(-.2, .2, n), rs.uniform(-.2, .2, n)
    dx = 0.1 * np.cos(q0) + 0.11 * np.cos(q0 + q1) - tx
    dy = 0.1 * np.sin(q0) + 0.11 * np.sin(q0 + q1) - ty
    return np.stack([q0, q1, v0, v1, tx, ty, dx, dy]).astype(np.float32), active


@pytest.mark.parametrize("split,act,sdt", [(False, "teacher", "f32"), (True, "teacher", "f32"),
                                           (True, "student", "f32"), (True, "student", "bf16")])
def test_fused_step_joint_limit_and_resets_match_oracle(oracle_c, split, act, sdt):
    """the fused rollout's own env step (rd::env_step<false>, the
    narrow-range-sincos instantiation inside rollout_kernel) on states with the joint-1 limit
    ACTIVE (|q1| > 3, every RK stage) and inactive, plus this step's staggered resets, against
    the oracle with NO exemption: every non-reset env against the f64 C oracle stepped with the
    oracle policy's actions -- limit-inactive envs per component (angles / offsets 1e-5,
    velocities 1e-5 + 1e-5 rel, targets bitwise; tests/parity.py), limit-active ones within
    3e-4 + 1e-4 rel --, every reset env's (q, v, target) the oracle's Philox draw bit for bit
    and its fingertip offset within 1e-6."""
    n, seed = 4096, 13
    tr = _trainer(n, seed=seed, loss="mse", act=act, stagger=True, f32_split=split, student_dtype=sdt)
    st0, active = _limit_states(n, np.random.RandomState(5))
    tr.set_env_state(torch.from_numpy(st0))
    sp = tr.student_params().cpu().numpy()
    tr.rollout()                         # env clock C = 0: groups with offset 49 reset
    st1 = tr.env_state().cpu().numpy()
    ob = _obs_from_state(st0)
    if sdt == "bf16":
        fs = pn.forward_bf16(sp.astype(np.float64), *_np_params(tr.student)[1:], ob)
    else:
        fs = pn.forward(sp.astype(np.float64), *_np_params(tr.student)[1:], ob)
    ft = pn.forward(*_np_params(tr.teacher), ob)
    a = (fs if act == "student" else ft)["mean"].astype(np.float32)
    ref = np.ascontiguousarray(st0.astype(np.float64))
    oracle_c.step(ref, a, np.float64)
    off = (np.arange(n) // 32) % 50
    reset = off == 49
    assert reset.sum() == 64 and (active & ~reset).sum() > 1900
    # the limit-active envs really are pushed back by the constraint (not a vacuous check)
    assert np.all(np.abs(ref[1][active & ~reset]) > 2.9)
    keep = ~reset
    from tests import parity
    sok, worst = parity.state_ok(st1[:, keep], ref[:, keep], active[keep],
                                 vtol=(3e-5, 1e-5) if sdt == "bf16" and act == "student" else (5e-6, 1e-6))
    print(f"fused step split={split} act={act} {sdt}: {worst}")
    assert sok, worst
    draws = oracle_c.philox_draws(seed, np.flatnonzero(reset), 1)
    assert np.array_equal(st1[:6, reset].T, draws)
    fresh = oracle_c.philox_reset(n, 0, seed, 1)
    np.testing.assert_allclose(st1[6:, reset], fresh[6:, reset], atol=1e-6)
    tr.close()


# ---------------------------------------------------------------- one env per lane
def _null_state(n):
    """A fixed, limit-free env state (the replacement env of the isolation test)."""
    q0, q1, v0, v1, tx, ty = 0.3, -0.2, 0.1, 0.15, 0.1, -0.05
    dx = 0.1 * np.cos(q0) + 0.11 * np.cos(q0 + q1) - tx
    dy = 0.1 * np.sin(q0) + 0.11 * np.sin(q0 + q1) - ty
    return np.array([q0, q1, v0, v1, tx, ty, dx, dy], np.float32)


@pytest.mark.parametrize("n,gs", [(64, 64), (64, 16), (128, 32), (64, 0), (128, 0)])
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_each_env_contribution_isolated(n, gs, split, loss):
    """Every env of a small batch, i.e. every lane 0..63 of a 64-env group (and of 16- / 32-env
    groups; gs = 0: the automatic choice, the helper-pair layout at these sizes), owns one env;
    its contribution to every gradient entry is isolated as
    g(batch) - g(batch with env e replaced by a fixed env z) = c(x_e) - c(z) and compared with
    the oracle's per entry: |error| <= 1e-5 x (M(x_e) + M(z)) + 5e-6 x M(batch) (the second term:
    the f32 round-off of the two batch sums; measured r04a: worst error 0.014 of the round's first,
    4x looser, bound).  One env's wrong lane -- a lost load in lanes
    48-63 -- moves c(x_e) by O(1) in the entries it touches, far past this bound
    (tests/test_parity_mutation.py)."""
    from tests import parity
    rs = np.random.RandomState(7 + n + gs)
    tr = _trainer(n, loss=loss, stagger=False, f32_split=split, group_envs=gs)
    st, _ = _limit_states(n, rs)
    st[1] = rs.uniform(-2.5, 2.5, n).astype(np.float32)        # limit-free
    z = _null_state(n)
    sp = tr.student_params().cpu().numpy()

    def grad_of(states):
        tr.set_env_state(torch.from_numpy(np.ascontiguousarray(states)))
        tr.rollout()
        return tr.grad().cpu().numpy().astype(np.float64)

    g_all = grad_of(st)
    ob = _obs_from_state(st)
    g64_all, M_all, _ = parity.oracle_grad(sp, tr.teacher, tr.student, ob, loss, n)
    ok, rep = parity.grad_ok(g_all, g64_all, M_all)
    assert ok, rep
    obz = _obs_from_state(z[:, None])
    worst = 0.0
    for e in range(n):
        se = st.copy()
        se[:, e] = z
        d_gpu = g_all - grad_of(se)
        obe = ob.copy()
        obe[e] = obz[0]
        g64_e, M_e, _ = parity.oracle_grad(sp, tr.teacher, tr.student, obe, loss, n)
        d64 = g64_all - g64_e
        _, Mx, _ = parity.oracle_grad(sp, tr.teacher, tr.student, ob[e:e + 1], loss, n)
        _, Mz, _ = parity.oracle_grad(sp, tr.teacher, tr.student, obz, loss, n)
        bound = 1e-5 * (Mx + Mz) + 5e-6 * np.maximum(M_all, M_e)
        r = np.abs(d_gpu - d64) / np.where(bound > 0, bound, 1.0)
        r[(bound == 0) & (np.abs(d_gpu - d64) > 0)] = np.inf
        worst = max(worst, float(r.max()))
        assert r.max() <= 1.0, (e, int(np.argmax(r)), float(r.max()))
    print(f"per-env n={n} gs={gs} split={split} {loss}: worst error / bound {worst:.3f}")
    tr.close()


@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_each_env_contribution_isolated_bf16(loss):
    """The same isolation for the bf16 student (DAgger, config 5's arithmetic) at 64 envs, with
    its rounding-flip tolerance: |error| <= 1e-4 x (M(x_e) + M(z)) + 2e-5 x M(batch)."""
    from tests import parity
    n = 64
    rs = np.random.RandomState(11)
    tr = _trainer(n, loss=loss, act="student", stagger=False, student_dtype="bf16", group_envs=64)
    st, _ = _limit_states(n, rs)
    st[1] = rs.uniform(-2.5, 2.5, n).astype(np.float32)
    z = _null_state(n)
    sp = tr.student_params().cpu().numpy()

    def grad_of(states):
        tr.set_env_state(torch.from_numpy(np.ascontiguousarray(states)))
        tr.rollout()
        return tr.grad().cpu().numpy().astype(np.float64)

    ob = _obs_from_state(st).astype(np.float32).astype(np.float64)
    obz = _obs_from_state(z[:, None]).astype(np.float32).astype(np.float64)
    g_all = grad_of(st)
    g64_all, M_all, _ = parity.oracle_grad(sp, tr.teacher, tr.student, ob, loss, n, bf16=True)
    _, Mz, _ = parity.oracle_grad(sp, tr.teacher, tr.student, obz, loss, n, bf16=True)
    worst = 0.0
    for e in range(n):
        se = st.copy()
        se[:, e] = z
        d_gpu = g_all - grad_of(se)
        obe = ob.copy()
        obe[e] = obz[0]
        g64_e, M_e, _ = parity.oracle_grad(sp, tr.teacher, tr.student, obe, loss, n, bf16=True)
        _, Mx, _ = parity.oracle_grad(sp, tr.teacher, tr.student, ob[e:e + 1], loss, n, bf16=True)
        bound = 1e-4 * (Mx + Mz) + 2e-5 * np.maximum(M_all, M_e)
        err = np.abs(d_gpu - (g64_all - g64_e))
        r = err / np.where(bound > 0, bound, 1.0)
        r[(bound == 0) & (err > 0)] = np.inf
        worst = max(worst, float(r.max()))
        assert r.max() <= 1.0, (e, int(np.argmax(r)), float(r.max()))
    print(f"per-env bf16 {loss}: worst error / bound {worst:.3f}")
    tr.close()


def test_set_env_state_rejects_angles_outside_the_rollout_range():
    """The fused rollout's joint trig is exact for |q0| < 8192 and |q1| <= 4 rad
    (include/reacher_distill.h): a caller's state outside that range, or not finite, raises and
    leaves the trainer's state as it was; the edges of the range are taken."""
    from reacherdistilation_amd import _native as nat
    n = 300
    tr = _trainer(n, seed=4)
    st, _ = _limit_states(n, np.random.RandomState(8))
    tr.set_env_state(torch.from_numpy(st))
    before = tr.env_state().cpu().numpy()
    for row, val in ((1, 4.5), (1, -100.0), (0, 8192.0), (0, -1e5), (1, np.nan), (0, np.inf)):
        bad = st.copy()
        bad[row, n - 1] = val
        with pytest.raises(nat.NativeError, match="outside the fused rollout's range"):
            tr.set_env_state(torch.from_numpy(bad))
        assert np.array_equal(tr.env_state().cpu().numpy(), before)
    edge = st.copy()
    edge[0, 0], edge[1, 0], edge[0, 1], edge[1, 1] = 8191.0, 4.0, -8191.0, -4.0
    tr.set_env_state(torch.from_numpy(edge))
    assert np.array_equal(tr.env_state().cpu().numpy(), edge)
    tr.close()

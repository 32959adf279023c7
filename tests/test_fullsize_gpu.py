"""BASELINE's full sizes (c4: 262,144 envs per GPU; c5: 131,072 envs per GPU x 8 = 1,048,576,
DAgger with the bf16 student) through size-independent properties, on one MI355X:

  * shard linearity: the rollout gradient over N envs equals the sum of the gradients of two
    contiguous shards (env_base keys, MSE normalised by the global N) -- the multi-GPU
    contract -- within f32 summation order (relative L2 < 1e-5); the shards' env states are
    the full batch's, bitwise (each env's step is independent of the batch split);
  * determinism: the same full-size rollout twice is bitwise identical;
  * (each with the exact f32 products and with f32_split, the split-bf16 hidden layers)
  * the whole c5 global batch (1,048,576 envs) on one GPU equals its eight 131,072-env
    shards summed (the 8-GPU step), the same way.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _tr(**kw):
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    rank, world = kw.pop("rank", 0), kw.pop("world_size", 1)
    return DistillTrainer(DistillConfig(seed=5, **kw), device=DEV, rank=rank, world_size=world)


def _rollout(tr):
    tr.rollout()
    return tr.grad().clone(), tr.env_state()


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("wl", ["c4", "c5"])
def test_full_size_shard_linearity_and_state(wl, split):
    kw = dict(loss="mse", act_with="teacher") if wl == "c4" else \
        dict(loss="mse", act_with="student", student_dtype="bf16")
    kw["f32_split"] = split
    N = 262144 if wl == "c4" else 2 * 131072
    g_full, s_full = _rollout(_tr(n_envs=N, **kw))
    parts = [_rollout(_tr(n_envs_global=N, rank=r, world_size=2, **kw)) for r in range(2)]
    g_sum = parts[0][0] + parts[1][0]
    rel = float((g_sum - g_full).norm() / g_full.norm())
    assert rel < 1e-5, rel
    assert torch.equal(torch.cat([parts[0][1], parts[1][1]], dim=1), s_full)


WL_KW = {"c2": dict(n_envs=4096), "c3": dict(n_envs=65536, loss="kl"), "c4": dict(n_envs=262144),
         "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16")}


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("wl", ["c2", "c3", "c4", "c5"])
def test_full_size_rollout_is_deterministic(wl, split):
    """Three fresh trainers, one rollout each: gradients and env states bitwise equal (every
    config steps the envs on the producer wave)."""
    kw = WL_KW[wl]
    a = _rollout(_tr(f32_split=split, **kw))
    for _ in range(2):
        b = _rollout(_tr(f32_split=split, **kw))
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_c5_global_batch_equals_eight_shards():
    kw = dict(loss="mse", act_with="student", student_dtype="bf16")
    N = 8 * 131072
    g_full, s_full = _rollout(_tr(n_envs=N, **kw))
    g_sum = torch.zeros_like(g_full)
    states = []
    for r in range(8):
        g, s = _rollout(_tr(n_envs_global=N, rank=r, world_size=8, **kw))
        g_sum += g
        states.append(s)
    rel = float((g_sum - g_full).norm() / g_full.norm())
    assert rel < 1e-5, rel
    assert torch.equal(torch.cat(states, dim=1), s_full)
    assert np.isfinite(g_full.cpu().numpy()).all()


@pytest.mark.parametrize("split", [False, True])
def test_c4_full_size_gradient_matches_oracle(split):
    """c4 at its full per-GPU size (262,144 envs, teacher-driven, staggered, MSE): the rollout
    gradient vs the f64 numpy oracle (policy_np, pinned to the reference graph) per entry within
    2e-5 x M_e and globally 1e-5 x max|g|, and every env's transition vs the f64 C oracle per
    component (tests/test_distill_gpu.py _grad_check, tests/parity.py)."""
    from tests.test_distill_gpu import _grad_check, _trainer
    tr = _trainer(262144, loss="mse", f32_split=split)
    assert tr.cfg.stagger
    _grad_check(tr, "mse", "teacher")


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("loss", ["mse", "kl"])
def test_c5_shard_gradient_matches_bf16_oracle(loss, split):
    """A c5 shard (rank 5 of 8: 131,072 of 1,048,576 envs, DAgger, bf16 student) vs the bf16
    oracle (policy_np.forward_bf16 / backward_bf16, MSE normalised by the global N), with the
    tolerances of tests/test_distill_gpu.py's bf16 tests."""
    from oracle import policy_np as pn
    from tests.test_distill_gpu import _np_params, _obs_from_state
    N, rank = 8 * 131072, 5
    tr = _tr(n_envs_global=N, rank=rank, world_size=8, loss=loss, act_with="student", student_dtype="bf16",
             f32_split=split)
    assert tr.n_local == 131072 and tr.env_base == rank * 131072
    st0 = tr.env_state().cpu().numpy()
    sp = tr.student_params().cpu().numpy().astype(np.float64)
    tr.rollout()
    g = tr.grad().cpu().numpy()
    ob = _obs_from_state(st0).astype(np.float32)
    fs = pn.forward_bf16(sp, *_np_params(tr.student)[1:], ob)
    ft = pn.forward(*_np_params(tr.teacher), ob.astype(np.float64))
    # MSE is normalised by the global N; the KL is a sum, so dlogstd is over this shard's rows
    L, dmean, dls, sq = pn.loss_and_dmean(fs, ft, loss, N)
    gb = pn.backward_bf16(sp, fs, dmean, dls)
    err = np.abs(g - gb).max() / np.abs(gb).max()
    from tests import parity
    rep = parity.grad_report(g, gb, parity.abs_scale(sp, fs, dmean, dls, bf16=True))
    print(f"c5 shard {loss} split={split}: {err:.2e} {rep}")
    assert err < 1e-4, err
    assert rep["entry"] <= parity.TOL_ENTRY_BF16, rep

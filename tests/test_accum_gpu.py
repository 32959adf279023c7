"""K env steps per optimiser step in ONE rollout launch (rdd_step_accum / rdd_rollout_accum,
SURVEY.md §8d's K = 50 reading) against the staged accumulation it replaces: K x (rollout
launch + reduction into the gradient) then Adam (rdd_launch_stage ROLLOUT, REDUCE(_ACCUM)).

The reference takes its MpiAdam step once per batch of env steps in the batched on-policy
loop (backup/student_rollout.py:658-659,709) and once per env step in mlp_train.py:143-161;
accum_steps = K is the first reading, and the K-step launch must not change what it computes:
  * env states after the K steps bitwise equal (same actions: the teacher is fixed and the
    student is frozen between optimiser steps; the same Philox resets at episode ends);
  * the gradient equal up to f32 reordering of the sums (the launch sums K steps in
    registers, the staged form adds K reduced gradients): globally <= 1e-5 x max|g|, and per
    entry <= 1e-5 x the entry's own scale (the sum of |staged per-step gradients|);
  * the counters (env clock += K, one optimiser step) and the metrics slot.
Sizes: config 3's 65,536 envs (one 64-env group per wave pair, state re-read), the 32,768-env
shard of config 4 at 8 GPUs (one 32-env group per pair: state kept in registers across the K
steps), a ragged batch with two groups on some pairs, DAgger and the bf16 student.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainer(n, K, **kw):
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    return DistillTrainer(DistillConfig(n_envs=n, seed=5, accum_steps=K, **kw), device=DEV)


def _staged_grad(tr, K):
    """K staged rollouts; returns the accumulated gradient and the per-step gradients' |sum|."""
    scale = torch.zeros_like(tr.grad(), dtype=torch.float64)
    prev = torch.zeros_like(tr.grad())
    for k in range(K):
        tr.launch(tr.STAGE_ROLLOUT)
        tr.launch(tr.STAGE_REDUCE_ACCUM if k else tr.STAGE_REDUCE)
        g = tr.grad().clone()
        scale += (g - prev).double().abs()
        prev = g
    return prev, scale


CASES = [
    # n, K, loss, act, split, student dtype
    (65536, 5, "kl", "teacher", True, "f32"),      # config 3
    (32768, 7, "mse", "teacher", True, "f32"),     # config 4's 8-GPU shard (register-resident state)
    (32768, 4, "mse", "teacher", False, "f32"),    # exact f32 MFMA path
    (20000, 6, "mse", "student", True, "f32"),     # ragged, DAgger, 16-env groups, 2 groups on some pairs
    (4096, 3, "kl", "teacher", True, "f32"),       # config 2's size (plain layout, not the helper pairs)
    (131072, 3, "mse", "student", True, "bf16"),   # config 5's shard: bf16 student, DAgger
]


@pytest.mark.parametrize("n,K,loss,act,split,sdt", CASES)
def test_k_step_launch_equals_staged_accumulation(n, K, loss, act, split, sdt):
    kw = dict(loss=loss, act_with=act, f32_split=split, student_dtype=sdt)
    a, b = _trainer(n, K, **kw), _trainer(n, K, **kw)
    a.rollout_accum()
    gb, scale = _staged_grad(b, K)
    assert a.counters() == b.counters() == (K, 0)
    assert torch.equal(a.env_state(), b.env_state()), "env states differ after the K steps"
    ga, gb = a.grad().double(), gb.double()
    err = (ga - gb).abs()
    glob = err.max().item() / gb.abs().max().item()
    ent = (err / (scale + 1e-30)).max().item()
    print(f"n={n} K={K} {loss}/{act}/split={split}/{sdt}: global {glob:.2e}, per entry {ent:.2e}")
    assert glob <= 1e-5 and ent <= 1e-5, (glob, ent)
    # Adam on both, the metrics slot of that optimiser step
    a.apply()
    b.launch(b.STAGE_APPLY)
    assert a.counters() == b.counters() == (K, 1)
    ma, mb = a.metrics(1)[0], b.metrics(1)[0]
    assert ma[3] == mb[3] == K * n
    np.testing.assert_allclose(ma[:3], mb[:3], rtol=1e-5)
    pa, pb = a.student_params(), b.student_params()
    assert (pa - pb).abs().max().item() <= 2.01 * a.cfg.lr


def test_k50_chain_crosses_episode_ends_bitwise():
    """Two optimiser steps of K = 50 env steps (every env passes an episode end: staggered
    Philox resets inside the launch) with the teacher acting: states bitwise equal to the
    staged form, both Adam steps applied, counters (100, 2)."""
    n, K = 32768, 50
    a, b = _trainer(n, K), _trainer(n, K)
    for _ in range(2):
        a.step_accum()
        for _ in range(K):
            b.step()
    assert a.counters() == b.counters() == (2 * K, 2)
    assert torch.equal(a.env_state(), b.env_state())
    pa, pb = a.student_params(), b.student_params()
    assert (pa - pb).abs().max().item() <= 4.02 * a.cfg.lr
    assert a.steps == b.steps == 2 * K


def test_k_step_graph_replay_is_eager():
    """step_accum captured in a HIP graph replays bitwise like eager calls."""
    n, K = 16384, 10
    a, b = _trainer(n, K), _trainer(n, K)
    g = a.capture(2, fused=True)
    g.replay()
    torch.cuda.synchronize()
    b.step_accum()
    b.step_accum()
    assert a.counters() == b.counters() == (2 * K, 2)
    assert torch.equal(a.student_params(), b.student_params())
    assert torch.equal(a.env_state(), b.env_state())


def test_k_step_launch_is_deterministic():
    n, K = 32768, 8
    outs = []
    for _ in range(2):
        t = _trainer(n, K)
        t.rollout_accum()
        outs.append((t.grad().clone(), t.env_state()))
        t.close()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_step_accum_inside_a_staged_accumulation_raises():
    t = _trainer(1024, 4)
    t.step()
    with pytest.raises(RuntimeError):
        t.step_accum()

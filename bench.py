#!/usr/bin/env python3
"""Benchmark of the hot path: batched Reacher-v2 rollout + distillation step on MI355X.

One "step" = one lockstep env-step of every env on every rank, fused with its teacher
query, student forward/backward, distillation loss and one TF1 Adam step (+ one RCCL
all-reduce of the 5060-float student gradient when N > 1) -- the reference's hot-loop
iteration (mlp_train.py:143-204) batched.  Unit: env-steps/s summed over all ranks.

  python bench.py [--gpus N --steps K --warmup W --workload c4|c2|c3|c5 --envs-per-gpu E]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Default workload: BASELINE config 4's 262,144 envs on EVERY GPU
(weak scaling: per-GPU work fixed as N grows), teacher-driven, MSE, fp32 -- the metric is
quoted at 1/2/4/8 MI355X, which is config 4.  Rank 0 prints one JSON line, with a
`roofline` object for the dominant kernel (rollout_kernel, timed with HIP events on its
stream inside the timed region) and a `cpu_baseline` (the C f32 restatement, OpenMP, on a
bounded sample; rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Reacher env-steps/sec (rollout+distill step) at 1/2/4/8 MI355X; student MSE"
# algorithmic work per env-step of the fused step: FLOPs of the
# GEMM-shaped parts (teacher fwd 9,856 + student fwd 9,856 + student bwd 18,304)
FLOP_PER_ENV_STEP = 2 * (11 * 64 + 64 * 64 + 64 * 2) * 2 + 2 * (64 * 2 * 2 + 64 * 64 * 2 + 11 * 64)
# HBM bytes per env-step of rollout_kernel: read state 32 B, write q, v, dx, dy 24 B
BYTES_PER_ENV_STEP = 56
PEAK_F32_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak (dense)
PEAK_HBM_GBS = 8000.0

WORKLOADS = {
    "c2": dict(envs=4096, loss="mse", act_with="teacher",
               desc="BASELINE config 2: 4,096 envs/GPU, 2x64 tanh MlpPolicy student, MSE, fp32"),
    "c3": dict(envs=65536, loss="kl", act_with="teacher",
               desc="BASELINE config 3: 65,536 envs/GPU, Gaussian KL(s||t) distillation, fp32"),
    "c4": dict(envs=262144, loss="mse", act_with="teacher",
               desc="BASELINE config 4: 262,144 envs per GPU, RCCL student-grad all-reduce, MSE, fp32"),
    "c5": dict(envs=131072, envs_global=1048576, loss="mse", act_with="student", student_dtype="bf16",
               desc="BASELINE config 5 shard: DAgger (student acts, teacher relabels), 1,048,576 envs over 8 GPUs "
                    "= 131,072 envs/GPU, bf16 student MLP (f32 master + Adam), f32 teacher, MSE"),
}
# FLOPs per env-step by MFMA precision: teacher forward f32; student fwd + bwd f32 or bf16
FLOP_TEACHER = 2 * (11 * 64 + 64 * 64 + 64 * 2)
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
# f32_split: the f32 products emulated on bf16 MFMAs (the K = 64 products -- teacher + student
# layer 2, student dH1 -- the env-K dW2 and both nets' layer 1; beside the bf16 student the
# teacher's layers 1 and 2) take six bf16 partial products each, so their f32-equivalent peak is
# the bf16 peak / 6; the rest stays on the f32 MFMA (dW1) or VALU (the 64x2 layer)
FLOP_SPLIT_PER_NET_L2 = 2 * 64 * 64
FLOP_L1 = 2 * 11 * 64
PEAK_SPLIT_TFLOPS = PEAK_BF16_TFLOPS / 6
# reference numbers quoted beside the fixture leg (derived from the fixture)
REF_LSTM_STUDENT_MSE = 0.0212
# the round-3 mixed peaks (mixed_peak() of the round-3 FLOP mix), frozen for a round-stable frac
FIXED_PEAK = {("f32", True): 376.9, ("f32", False): 157.3, ("bf16", True): 1058.0}      # the reference LSTM student vs the teacher on the fixture's episodes 21-24


def default_f32_mode():
    """The headline runs the library's default f32 mode (DistillConfig.f32_split)."""
    from reacherdistilation_amd.distill import DistillConfig
    return "split" if DistillConfig().f32_split else "exact"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed steps for this long before the W warm-up steps, so that the GPU's "
                         "clocks have left their idle state (reported as 'settle' in the line)")
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--envs-per-gpu", type=int, default=0)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--accum", type=int, default=50,
                    help="also time K env-steps per optimiser step (SURVEY §8d: K = 50 = one episode); 0 = skip")
    ap.add_argument("--conv-steps", type=int, default=5000,
                    help="convergence leg: optimiser steps allowed to reach student action-MSE < 1e-3; 0 = skip")
    ap.add_argument("--f32-mode", default=default_f32_mode(), choices=["exact", "split"],
                    help="f32 hidden-layer products: f32 emulated on bf16 MFMAs by exact 3-piece operand splits "
                         "(include/reacher_distill.h f32_split; default), or every product on the f32 MFMA")
    ap.add_argument("--no-exact-leg", action="store_true",
                    help="skip the secondary timing of the exact-f32-MFMA kernel beside the split one")
    ap.add_argument("--no-strong", action="store_true",
                    help="at N > 1 skip the strong-scaling leg (the workload's fixed global batch over the ranks)")
    ap.add_argument("--conv-small-envs", type=int, default=64,
                    help="env count of the second convergence run (the env-step reading of the budget: "
                         "scripts/conv_sweep.py measured 16/32/64/128 envs within it at lr 1e-4, 256 not)")
    ap.add_argument("--fixture-steps", type=int, default=250_000,
                    help="convergence_fixture leg: Adam steps of the 2x64 student on the fixture's teacher episodes "
                         "0-19 (the reference's budget: 5000 episodes x 50 steps); 0 = skip")
    ap.add_argument("--fixture-ref-steps", type=int, default=25_000,
                    help="the same leg's steps for the reference graph student (student_nn.py:51-57)")
    ap.add_argument("--no-workloads", action="store_true",
                    help="at N = 1 skip the `workloads` object (configs 2, 3 and the config-5 shard at K = 1 and 50)")
    ap.add_argument("--no-strong-projection", action="store_true",
                    help="at N = 1 skip timing c4's 2/4/8-GPU strong shards (strong_projection)")
    ap.add_argument("--teacher", default="synthetic", choices=["synthetic", "fitted", "ppo"],
                    help="fixed teacher of the run and its convergence legs: the seeded synthetic MlpPolicy, the "
                         "reference teacher's structure fitted to the fixture's 1,050 teacher records "
                         "(teacher.fit_teacher), or the teacher PPO-trained here with the reference's hyperparameters "
                         "(teacher.ppo_teacher, teachers/ppo_teacher.ckpt); the line carries fitted- and PPO-teacher "
                         "convergence blocks either way")
    return ap.parse_args()


def cpu_ref_loop(seconds):
    """BASELINE.md §2 "CPU-ref-loop (C1)": the reference's single-env loop structure on one
    core -- per env step: teacher query (B=1), one distillation Adam step on a window batch
    of 20 episodes x 10 steps (200 rows, f64 policy math), the student's query (B=1), f64
    env.step -- with the oracle's CPU restatement (numpy policy, C f64 env)."""
    import numpy as np

    from oracle import policy_np as pn
    from oracle import ref_c
    from reacherdistilation_amd.policy import student_init, synthetic_teacher
    t, s = synthetic_teacher(1), student_init(2)
    tp, tmu, tsd = t.flat.astype(np.float64), t.ob_mean.astype(np.float64), t.ob_std.astype(np.float64)
    sp = s.flat.copy()
    smu, ssd = s.ob_mean.astype(np.float64), s.ob_std.astype(np.float64)
    opt = pn.AdamTF1(pn.P_TOT)
    state = ref_c.philox_reset(1, 0, 0, 0).astype(np.float64)
    rng = np.random.RandomState(0)
    buf = np.zeros((40, 50, 11))                       # a filled dataset of 40 episodes
    buf[:] = rng.uniform(-1, 1, buf.shape)
    ob, _ = ref_c.step(state, np.zeros((1, 2), np.float32), np.float64)
    import threadpoolctl
    limit = threadpoolctl.threadpool_limits(1)         # one core: BLAS single-threaded
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ft1 = pn.forward(tp, tmu, tsd, ob)                              # teacher query
        eps, st = rng.randint(0, 40, 20), rng.randint(0, 41)
        win = buf[eps, st:st + 10].reshape(200, 11)                     # training window
        fs = pn.forward(sp.astype(np.float64), smu, ssd, win)
        ft = pn.forward(tp, tmu, tsd, win)
        _, dmean, dls, _ = pn.loss_and_dmean(fs, ft, "mse", 200)
        sp = opt.step(sp, pn.backward(sp.astype(np.float64), fs, dmean, dls))
        fa = pn.forward(sp.astype(np.float64), smu, ssd, ob)           # student acts
        ob, _ = ref_c.step(state, fa["mean"].astype(np.float32), np.float64)
        del ft1
        steps += 1
    el = time.perf_counter() - t0
    limit.restore_original_limits()
    return dict(value=steps / el, unit="env-steps/s", cores=1, kind="port",
                sample=f"{steps} env steps ({el:.1f} s) of the reference-shaped single-env loop")


def cpu_batched_env(seconds, n=65536):
    """BASELINE.md §2 "CPU-batched-env": the C restatement's OpenMP reacher_step, f32 and f64."""
    import numpy as np

    from oracle import ref_c
    out = {}
    for dt, name in ((np.float32, "f32"), (np.float64, "f64")):
        state = ref_c.philox_reset(n, 0, 0, 0).astype(dt)
        act = np.random.RandomState(1).uniform(-1, 1, (n, 2)).astype(np.float32)
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 2:
            ref_c.step(state, act, dt)
            steps += 1
        el = time.perf_counter() - t0
        out[name] = dict(value=n * steps / el, unit="env-steps/s",
                         cores=int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                         sample=f"{n} envs x {steps} steps ({el:.1f} s)")
    return out


def env_roofline(dev, n=1 << 24, iters=100, warmup=20):
    """The standalone env.step kernel (rd_step) at 16.8M envs: algorithmic 113 B per
    env-step (read act 8 + q,v 16 + target 8 + held offset 8; write q,v 16 + offset 8 +
    obs 44 + rew 4 + done 1) over its launch time, vs the 8 TB/s HBM peak."""
    import torch

    from reacherdistilation_amd.env import BatchedReacher
    env = BatchedReacher(n, seed=0, device=dev)
    env.reset()
    a = (torch.rand(n, 2, device=dev) * 2 - 1).contiguous()
    for _ in range(warmup):
        env.step(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    s.record()
    for _ in range(iters):
        env.step(a)
    e.record()
    torch.cuda.synchronize(dev)
    sec = s.elapsed_time(e) * 1e-3 / iters
    env.close()
    gbs = 113 * n / sec / 1e9
    return {"kernel": "rd_step_kernel", "bound": "hbm", "envs": n, "env_steps_per_s": n / sec,
            "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS}


def copy_ceiling(gib=1.0, reps=20):
    """The float4 copy ceiling measured in this run (scripts/micro/copy_bw.hip built as
    scripts/micro/libcopybw.so: grid-stride 16 B and one-shot float4 x4 / x8, plain and
    non-temporal; read + write bytes / s), the practical HBM ceiling the env kernel is quoted
    against (MI355X_MICROARCH.md: 6.29 TB/s measured for a float4 copy).  None if not built."""
    import ctypes
    path = os.path.join(ROOT, "scripts", "micro", "libcopybw.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.copy_bw_tbs.restype = ctypes.c_double
    lib.copy_bw_tbs.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.copy_bw_name.restype = ctypes.c_char_p
    lib.copy_bw_name.argtypes = [ctypes.c_int]
    nbytes = int(gib * (1 << 30))
    res = {}
    for v, blocks in ((1, 65536), (2, 65536), (3, 0), (4, 0), (5, 0), (6, 0)):
        res[lib.copy_bw_name(v).decode()] = 1e3 * lib.copy_bw_tbs(nbytes, v, blocks, reps)   # GB/s
    best = max(res, key=res.get)
    # the env step's own read:write mix (40 B read : 73 B written ~ 1 : 2), 16-B streaming
    mix = {lib.copy_bw_name(v).decode(): 1e3 * lib.copy_bw_tbs(nbytes, v, 0, reps) for v in (7, 8)}
    mbest = max(mix, key=mix.get)
    return {"best_gbs": res[best], "best": best, "variants_gbs": res, "bytes": nbytes,
            "mix_1r2w_best_gbs": mix[mbest], "mix_1r2w_best": mbest, "mix_1r2w_gbs": mix,
            "source": "scripts/micro/copy_bw.hip (libcopybw.so), this run"}


def copy_bandwidth(dev, gib=1.0, iters=40):
    """Measured device-to-device copy bandwidth (read + write bytes / s), the practical HBM
    ceiling the roofline is also quoted against."""
    import torch
    n = int(gib * (1 << 30)) // 4
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    for _ in range(10):
        b.copy_(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        b.copy_(a)
    e.record()
    torch.cuda.synchronize(dev)
    return 2 * 4 * n * iters / (s.elapsed_time(e) * 1e-3) / 1e9


def mixed_peak(sdt, split):
    """The MFMA-time-weighted peak of the kernel's FLOP mix (f32 MFMA, split-emulated f32,
    bf16): the roofline the kernel's algorithmic FLOP/s is quoted against."""
    if sdt == "bf16":   # bf16 student fwd + bwd; teacher f32 (layers 1 and 2 split, or exact)
        f_s = FLOP_PER_ENV_STEP - FLOP_TEACHER
        f_split = FLOP_SPLIT_PER_NET_L2 + FLOP_L1 if split else 0
        f_f32 = FLOP_TEACHER - f_split
        return FLOP_PER_ENV_STEP / (f_f32 / PEAK_F32_TFLOPS + f_split / PEAK_SPLIT_TFLOPS + f_s / PEAK_BF16_TFLOPS)
    if split:           # teacher L2 + student L2 + student dH1 + student dW2 + both nets' layer 1
        f_split = 4 * FLOP_SPLIT_PER_NET_L2 + 2 * FLOP_L1
        return FLOP_PER_ENV_STEP / ((FLOP_PER_ENV_STEP - f_split) / PEAK_F32_TFLOPS + f_split / PEAK_SPLIT_TFLOPS)
    return PEAK_F32_TFLOPS


SIMDS = 256 * 4             # MI355X: 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4             # the clock the dense TFLOP/s peaks assume (MI355X_MICROARCH.md)


def issue_roofline(avg, launch_s):
    """The rollout kernel's real bound on gfx950: one instruction stream per SIMD shared by the
    VALU and the MFMAs (an f32 MFMA holds it 32 cycles, a bf16 16x16x32 16 -- measured,
    scripts/micro/mfma_mix.hip; each VALU instruction >= 4 cycles, a transcendental 8).
    issue cycles >= SQ_VALU_MFMA_BUSY_CYCLES + 4 (SQ_INSTS_VALU - SQ_INSTS_MFMA) per launch
    (rocprofv3 PMC pass of this workload, profiles/pmc_*.json; transcendentals counted at 4),
    against the SIMDs' cycles over the live launch time at 2.4 GHz."""
    try:
        mfma_cyc = float(avg["SQ_VALU_MFMA_BUSY_CYCLES"])
        valu = float(avg["SQ_INSTS_VALU"]) - float(avg["SQ_INSTS_MFMA"])
    except (KeyError, TypeError):
        return None
    need = mfma_cyc + 4.0 * valu
    have = SIMDS * launch_s * CLOCK_GHZ * 1e9
    return {"bound": "simd-issue", "issue_cycles_per_launch": need, "available_cycles": have, "frac": need / have,
            "mfma_cycles": mfma_cyc, "valu_instructions": valu, "valu_per_mfma": valu / max(1.0, float(avg["SQ_INSTS_MFMA"])),
            "model": "MFMA busy cycles (counter) + 4 cycles per non-MFMA VALU instruction; 1,024 SIMDs x launch "
                     "time x 2.4 GHz; counters from the committed PMC pass (traffic_source)"}


def settle(step, dev, ms, world=1):
    """Untimed steps for about `ms` of wall time: on a GPU that idled (trainer set-up, the
    convergence leg's teardown) the first ~100 ms of steps run at ramping clocks -- c4 measured
    93.6 us per step after 2,000 warm-up steps, 98.9 after 20 and 105.4 in a 20-step region
    after 5.  The count is fixed after a 10-step probe and agreed over the ranks (MAX), since
    every sharded step is a collective."""
    import torch
    if ms <= 0:
        return {"steps": 0, "ms": 0.0}
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize(dev)
    probe = max(time.perf_counter() - t0, 1e-6)
    k = torch.tensor([max(10, int(math.ceil(10 * ms * 1e-3 / probe)))], dtype=torch.int64, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
    k = int(k.item())
    for _ in range(k - 10):
        step()
    torch.cuda.synchronize(dev)
    return {"steps": k, "ms": (time.perf_counter() - t0) * 1e3}


def time_leg(wl, n, sdt, split, dev, lr, steps, warmup, npass=100, settle_ms=0.0):
    """Secondary timing at world size 1: `steps` fused steps (no events), then the rollout
    kernel's event-timed launch (the other f32 mode beside the headline's)."""
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    tr = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                      student_dtype=sdt, f32_split=split), device=dev)
    settle(tr.step, dev, settle_ms)
    for _ in range(warmup):
        tr.step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(npass)]
    for a, b in evs:
        a.record()
        tr.launch(tr.STAGE_ROLLOUT)
        b.record()
        tr.launch(tr.STAGE_REDUCE_APPLY)
    torch.cuda.synchronize(dev)
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    tr.close()
    achieved = FLOP_PER_ENV_STEP * n / (kern_ms * 1e-3) / 1e12
    peak = mixed_peak(sdt, split)
    return {"f32_mode": "split" if split else "exact", "value": n * steps / el, "ms_per_step": el * 1e3 / steps,
            "launch_us": kern_ms * 1e3, "achieved_tflops": achieved, "peak_tflops": peak, "frac": achieved / peak,
            "frac_of_f32_mfma_peak": achieved / PEAK_F32_TFLOPS}


def workload_leg(name, dev, lr, steps, warmup, settle_ms, K=1, split=True, npass=50):
    """one BASELINE config at world size 1, timed like the headline (settle,
    warm-up, then exactly `steps` env steps between synchronizes, no events), plus an
    event-timed pass over the rollout launches for the mixed-peak fraction.  K = 1: rdd_step per
    env step; K > 1: rdd_step_accum (one K-env-step launch + reduce + Adam per optimiser step,
    SURVEY §8d's K = 50 reading), its launch timed with the reduce (rdd_rollout_accum)."""
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    wl = WORKLOADS[name]
    n, sdt = wl["envs"], wl.get("student_dtype", "f32")
    tr = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                      student_dtype=sdt, f32_split=split, accum_steps=K), device=dev)
    fn = tr.step if K == 1 else tr.step_accum
    calls = steps if K == 1 else max(4, steps // K)
    settle(fn, dev, settle_ms)
    for _ in range(max(1, warmup // K)):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    npass = npass if K == 1 else max(4, npass // 10)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(npass)]
    for a, b in evs:
        a.record()
        if K == 1:
            tr.launch(tr.STAGE_ROLLOUT)
        else:
            tr.rollout_accum()
        b.record()
        tr.launch(tr.STAGE_REDUCE_APPLY if K == 1 else tr.STAGE_APPLY)
    torch.cuda.synchronize(dev)
    launch_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    tr.close()
    env_steps = calls * K
    achieved = FLOP_PER_ENV_STEP * n * K / (launch_ms * 1e-3) / 1e12
    peak = mixed_peak(sdt, split)
    return {"workload": name, "envs": n, "accum_steps": K, "env_steps": env_steps,
            "us_per_env_step": el * 1e6 / env_steps, "env_steps_per_s": n * env_steps / el,
            "launch_us": launch_ms * 1e3, "launch_us_per_env_step": launch_ms * 1e3 / K,
            "launch": "rollout_kernel" if K == 1 else f"rollout_kernel, {K} env steps per launch, + its reduce",
            "achieved_tflops": achieved, "mixed_peak_tflops": peak, "frac": achieved / peak,
            "f32_mode": "split" if split else "exact", "student_dtype": sdt, "loss": wl["loss"],
            "act_with": wl["act_with"]}


def workloads(dev, lr, steps, warmup, settle_ms, accum=50, names=("c2", "c3", "c5")):
    """Every BASELINE config besides the headline's in the driver-run line: K = 1 and K = accum."""
    out = {"timing": "per leg: settle, warm-up, then `env_steps` env steps between synchronizes (the "
                     "headline's method); launch_us from HIP events around the rollout launches in a pass after",
           "flop_per_env_step": FLOP_PER_ENV_STEP}
    for name in names:
        out[name] = {"description": WORKLOADS[name]["desc"], "k1": workload_leg(name, dev, lr, steps, warmup, settle_ms)}
        if accum > 1:
            out[name][f"k{accum}"] = workload_leg(name, dev, lr, max(steps, 8 * accum), warmup, settle_ms, K=accum)
    return out


def exchange_latency(comm, dev, n=5060, iters=200, warmup=20):
    """Mean time of one in-place all-reduce of the student gradient's size (5,060 floats) on
    the bound communicator, back to back on the current stream (HIP events, all ranks)."""
    import torch
    import torch.distributed as dist
    x = torch.ones(n, dtype=torch.float32, device=dev)
    for _ in range(warmup):
        comm.allreduce_(x)
    torch.cuda.synchronize(dev)
    dist.barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        comm.allreduce_(x)
    b.record()
    torch.cuda.synchronize(dev)
    return {"floats": n, "us": a.elapsed_time(b) * 1e3 / iters, "iters": iters}


def _make_comm(kind, dev, world):
    """A native communicator of `kind` that passed its one-shot self-check on EVERY rank, or
    (None, reason).  Collective: every rank calls it in the same order."""
    import torch
    import torch.distributed as dist
    c, why = None, ""
    if kind == "rccl" and dist.get_backend() != "nccl":
        return None, "the process group is not RCCL (gloo rehearsal)"
    try:
        if kind == "rccl":
            from reacherdistilation_amd.dist import RcclComm
            c = RcclComm(dev)
        else:
            from reacherdistilation_amd.dist import XgmiComm
            # a 60-s deadline per wait (the library's default is 600 s): on a node where the IPC-mapped
            # pushes do not arrive, the self-check fails within the driver's 600-s run instead of
            # outlasting it, and the run goes on with RCCL (or torch's collective)
            c = XgmiComm(dev, timeout=60.0)
        ok = c.self_check()
        if not ok:
            why = "self-check sum mismatch"
    except Exception as e:   # noqa: BLE001  (reported in the line, never silent)
        ok, why = False, str(e).splitlines()[0][:200]
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return c, ""
    if c is not None:
        try:
            c.close()
        except Exception:   # noqa: BLE001
            pass
    return None, why or "failed its self-check on another rank"


def comm_view(comm, dev, world):
    """Every rank's communicator as the library sees it (rd_comm_query: RCCL's own
    ncclCommCount / ncclCommUserRank / ncclCommCuDevice, or an xGMI communicator's creation
    values), gathered to every rank: [{rank, count, user_rank, device, from_rccl}]."""
    import torch
    import torch.distributed as dist
    q = comm.query()
    mine = torch.tensor([dist.get_rank(), q["count"], q["user_rank"], q["device"], int(q["from_rccl"])],
                        dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
    allq = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allq, mine)
    rows = [dict(zip(("rank", "count", "user_rank", "device", "from_rccl"), t.cpu().tolist())) for t in allq]
    for r in rows:
        r["from_rccl"] = bool(r["from_rccl"])
    return {"ranks": rows, "consistent": all(r["count"] == world and r["user_rank"] == r["rank"] for r in rows),
            "distinct_devices": len({r["device"] for r in rows}) == world}


def strong_leg(wl, total, sdt, split, dev, lr, steps, warmup, rank, world, comm, settle_ms=0.0, accum=1):
    """BASELINE config 4's own wording, "262 144 envs sharded across 8 x MI355X": the
    workload's fixed global batch split over the ranks (`n_envs_global`, contiguous shards,
    Philox key = global env id), timed like the headline (barrier + synchronize around
    exactly `steps` fused steps, MAX over ranks).  Reported beside the weak-scaling value.
    accum = K > 1: one optimiser step (+ all-reduce) per K env steps in one K-step launch
    (rdd_step_accum, SURVEY §8d's K = 50 reading); `steps` env steps = steps / K calls."""
    import torch
    import torch.distributed as dist

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    tr = DistillTrainer(DistillConfig(n_envs_global=total, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                      student_dtype=sdt, f32_split=split, accum_steps=accum),
                        device=dev, rank=rank, world_size=world, comm=comm)
    K = max(1, accum)
    step = tr.step if K == 1 else tr.step_accum
    calls = max(1, steps // K)
    steps = calls * K
    settle(step, dev, settle_ms / K if K > 1 else settle_ms, world)
    for _ in range(max(1, warmup // K)):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    same = tr.replicas_identical() if world > 1 else True
    out = {"envs_total": total, "envs_per_gpu": tr.n_local, "steps": steps, "value": total * steps / el,
           "ms_per_step": el * 1e3 / steps, "replicas_identical": same, "scaling": "strong",
           "accum_steps": K, "launch": "rdd_step (one optimiser step per env step)" if K == 1 else
           f"rdd_step_accum (one {K}-env-step launch + reduce + all-reduce + Adam per optimiser step)"}
    tr.close()
    return out


def strong_projection(wl, sdt, split, dev, lr, steps, settle_ms, accum=50):
    """the compute side of c4's 1/2/4/8-GPU curve measured on one GPU --
    one-process steps at the 2/4/8-GPU strong shards of the 262,144-env global batch (131,072 /
    65,536 / 32,768 envs) and the sharded step's extra launch (rollout, reduce, [exchange], Adam:
    three launches instead of rdd_step's two), measured at each size -- plus a MODEL of the
    exchange: `exchange_us_model` low = the one-kernel xGMI push measured with two ranks on one
    GPU (profiles/r03a_n2_rehearsal.json), high = 25 us, an assumed small-message RCCL
    all-reduce over xGMI at 8 GPUs (never measured here: no multi-GPU box).
      strong (BASELINE config 4's wording, fixed 262,144 envs): speedup(N) = t(262,144) /
        (t(shard) + t(split) + exchange)   -- >= 6x at 8 needs t(32,768) + t(split) + exchange <= t1 / 6;
      weak (bench.py's value: 262,144 envs on EVERY GPU): speedup(N) = N t1 / (t1 + t(split) + exchange)."""
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    total = wl["envs"]
    xlo, xhi = 9.2, 25.0
    out = {"global_envs": total, "target_speedup_8": 6.0, "exchange_us_model": {"low": xlo, "high": xhi},
           "model": ("strong: t1 / (t_shard + t_split + x); weak: N t1 / (t1 + t_split(t1) + x); "
                     "t_* measured on one GPU here, x (the all-reduce) modelled"), "shards": {}}
    t1 = split1 = t1k = None
    K = accum
    out["accum_steps"] = K
    out["model_k"] = (f"K = {K} (one optimiser step per {K} env steps, one K-step launch, SURVEY §8d): per env step "
                      f"t_K(shard) + (t_split_K + x) / K against t1 (K = 1, the headline's step) and t1_K (262,144 "
                      f"envs at K = {K} on one GPU)")

    def timeit(fn, calls=steps, per=1, warm=20):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e6 / (calls * per)

    for N in (1, 2, 4, 8):
        n = total // N
        tr = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                          student_dtype=sdt, f32_split=split), device=dev)
        settle(tr.step, dev, settle_ms)

        def three():   # the sharded step's launches with a zero-cost exchange
            tr.launch(tr.STAGE_ROLLOUT)
            tr.launch(tr.STAGE_REDUCE)
            tr.launch(tr.STAGE_APPLY)
        us = timeit(tr.step)
        split_us = max(0.0, timeit(three) - us)
        tr.close()
        kus = ksplit = None
        if K > 1:   # the K-step launch: per env step, and its sharded form's extra launch per optimiser step
            tk = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                              student_dtype=sdt, f32_split=split, accum_steps=K), device=dev)
            kcalls = max(4, (steps * 2) // K)
            kus = timeit(tk.step_accum, kcalls, K, warm=2)

            def kthree():   # the K-step launch + reduce, then Adam: the sharded form with a zero-cost exchange
                tk.rollout_accum()
                tk.launch(tk.STAGE_APPLY)
            ksplit = max(0.0, timeit(kthree, kcalls, 1, warm=2) - kus * K)
            tk.close()
        if N == 1:
            t1, split1 = us, split_us
            out["t1_us"], out["t1_split_overhead_us"] = us, split_us
            if kus is not None:
                t1k = kus
                out["t1_k_us_per_env_step"] = kus
            continue
        sh = out["shards"][str(N)] = {
            "envs_per_gpu": n, "step_us": us, "split_overhead_us": split_us,
            "strong_speedup": {"x_high": t1 / (us + split_us + xhi), "x_low": t1 / (us + split_us + xlo)},
            "weak_speedup": {"x_high": N * t1 / (t1 + split1 + xhi), "x_low": N * t1 / (t1 + split1 + xlo)},
            "strong_step_budget_for_6x_at_8_us": t1 / 6.0}
        if kus is not None:
            per = {x: kus + (ksplit + xv) / K for x, xv in (("x_high", xhi), ("x_low", xlo))}
            sh["k"] = {"us_per_env_step": kus, "split_overhead_us_per_opt_step": ksplit,
                       "us_per_env_step_with_exchange": per,
                       "strong_speedup_vs_t1": {x: t1 / v for x, v in per.items()},
                       "strong_speedup_vs_t1_k": {x: t1k / v for x, v in per.items()}}
    s8 = out["shards"]["8"]
    out["meets_6x_at_8"] = {"strong": {k: v >= 6.0 for k, v in s8["strong_speedup"].items()},
                            "weak": {k: v >= 6.0 for k, v in s8["weak_speedup"].items()}}
    if "k" in s8:
        out["meets_6x_at_8"]["strong_k_vs_t1"] = {k: v >= 6.0 for k, v in s8["k"]["strong_speedup_vs_t1"].items()}
    return out


def convergence_fixture(dev, lr, steps, ref_steps):
    """distillation from the reference's REAL teacher data -- the fixture's
    teacher-stepped episodes (src/distilation/tests/data/dataset.json via
    tests/golden/reacher_fixture.npz: observations with the baselines teacher's recorded pdflat).
    Train on episodes 0-19 (rows mode: recorded t_pdflat as the target, 200-row windows as
    dataset.py:179-194 draws them, one Adam step each, lr as the reference) and report the
    held-out action-MSE on teacher episode 20 and on episodes 21-24 (the reference LSTM
    student's own trajectories, labelled by the teacher) beside that student's 0.0212 on them."""
    import numpy as np

    from reacherdistilation_amd import mlp_train
    path = os.path.join(ROOT, "tests", "golden", "reacher_fixture.npz")
    if not os.path.exists(path):
        return None
    d = np.load(path)
    ob, t, rew = d["ob"], d["t"], d["rew"]
    out = {"data": "reference fixture (dataset.json): 21 teacher-stepped episodes, 4 stepped by the reference LSTM "
                   "student; train = teacher episodes 0-19 (1,000 records), held out = episode 20 and episodes 21-24",
           "reference_lstm_student_mse_eps21_24": REF_LSTM_STUDENT_MSE, "lr": lr, "loss": "mse",
           "target_mse": 1e-3, "reference_budget_opt_steps": 5000 * 50}
    for student, k in (("policy", steps), ("mlp", ref_steps)):
        if k <= 0:
            continue
        t0 = time.perf_counter()
        tr, hist = mlp_train.fit_records(ob[:20], t[:20], rew[:20], student=student, steps=k, loss="mse", lr=lr,
                                         seed=0, device=dev, log_every=max(k // 10, 100))
        el = time.perf_counter() - t0
        out["student_2x64" if student == "policy" else "student_reference_graph"] = {
            "opt_steps": k, "seconds": el, "train_mse_curve": hist,
            "heldout_mse_ep20": mlp_train.action_mse(tr, ob[20:21], t[20:21], rew[20:21]),
            "heldout_mse_eps21_24": mlp_train.action_mse(tr, ob[21:25], t[21:25], rew[21:25]),
            "train_mse_eps0_19": mlp_train.action_mse(tr, ob[:20], t[:20], rew[:20])}
        tr.close()
    return out


def fitted_teacher(dev):
    """teacher.fit_teacher on the fixture's 21 teacher-stepped episodes (1,050 records): the
    reference teacher's structure (teacher.py:14-16) fitted to the reference's own teacher data,
    with its fit quality on those records and on the LSTM student's episodes 21-24."""
    import numpy as np
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    from reacherdistilation_amd.teacher import fit_teacher
    path = os.path.join(ROOT, "tests", "golden", "reacher_fixture.npz")
    if not os.path.exists(path):
        return None, None
    d = np.load(path)
    ob, t = d["ob"], d["t"]
    t0 = time.perf_counter()
    p, hist = fit_teacher(ob[:21], t[:21], seed=0, device=dev)
    el = time.perf_counter() - t0
    tr = DistillTrainer(DistillConfig(n_envs=64, seed=0), device=dev, teacher=p)

    def mse(lo, hi):
        tq, _ = tr.forward(torch.from_numpy(ob[lo:hi].reshape(-1, 11).astype(np.float32)).to(dev), student=False)
        return float(np.mean((tq[:, :2].double().cpu().numpy() - t[lo:hi].reshape(-1, 4)[:, :2]) ** 2))
    info = {"fit": "teacher.fit_teacher: obfilter of the records + 2x64 tanh MlpPolicy + the records' logstd, "
                   "rows mode (recorded pdflat as MSE target), 30,000 Adam steps at lr 1e-3 then 20,000 at 1e-4",
            "records": int(21 * 50), "seconds": el, "train_mse": mse(0, 21), "eps21_24_mse": mse(21, 25),
            "reference_lstm_student_mse_eps21_24": REF_LSTM_STUDENT_MSE}
    tr.close()
    return p, info


def ppo_teacher_info(dev, episodes=1024):
    """The committed PPO-trained teacher (teacher.ppo_teacher): its training record
    (profiles/r06_ppo_teacher.json, scripts/train_ppo_teacher.py) and its mean-action 50-step return
    measured in this run on fresh gym-seeded episodes, beside the reference teacher's -7.53."""
    from reacherdistilation_amd.teacher import PPO_TEACHER, episode_returns, ppo_teacher
    p = ppo_teacher()
    r = episode_returns(p, episodes, seed=777, device=dev)
    info = {"checkpoint": os.path.relpath(PPO_TEACHER, ROOT), "format": "TF1 V2 bundle, scope 'pi' (tf_checkpoint)",
            "return_mean_this_run": float(r.mean()), "return_std_this_run": float(r.std()), "episodes": episodes,
            "reference_teacher_return": -7.53}
    rec = os.path.join(ROOT, "profiles", "r06_ppo_teacher.json")
    if os.path.exists(rec):
        with open(rec) as fh:
            d = json.load(fh)
        info["training"] = {"config": d["config"], "train_seconds": d["train_seconds"],
                            "env_steps_per_s": d["env_steps_per_s_training"], "final": d["final"],
                            "record": os.path.relpath(rec, ROOT)}
    return p, info


def teacher_ppo(dev, n=4096, T=50, mb=4096, iters=5):
    """The teacher's PPO iteration (csrc/ppo.hip): n envs x T steps of rollout, GAE,
    the filter update and 10 epochs of mb-row minibatch steps (two launches each), timed over
    iters - 1 whole iterations after one warm-up; the longer run is scripts/bench_ppo.py."""
    import torch

    from reacherdistilation_amd.ppo import PPOConfig, PPOTrainer
    tr = PPOTrainer(PPOConfig(n_envs=n, horizon=T, optim_batchsize=mb, max_timesteps=n * T * 40), device=dev)
    tr.iterate()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters - 1):
        tr.iterate()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / (iters - 1)
    return {"n_envs": n, "horizon": T, "minibatch": mb, "epochs": 10, "iter_ms": dt * 1e3,
            "env_steps_per_s": n * T / dt, "ep_ret_mean_last": float(tr.metrics(1)[0][0])}


def cpu_baseline(workload, seconds, threads, n):
    """Time the oracle's C f32 rollout+distill step (OpenMP) at the workload's own env count
    (the same per-GPU batch as the timed GPU step), for a bounded number of steps."""
    import numpy as np

    from oracle import ref_c
    from reacherdistilation_amd.policy import student_init, synthetic_teacher
    t, s = synthetic_teacher(1), student_init(2)
    state = ref_c.philox_reset(n, 0, 0, 0)
    threads = threads or min(16, os.cpu_count() or 1)
    P = ref_c.param_count()
    m = np.zeros(P, np.float32); v = np.zeros(P, np.float32)
    sp = s.flat.copy()
    steps = 0
    b1p, b2p = 0.9, 0.999
    t0 = time.perf_counter()
    while True:
        g, _ = ref_c.distill_step(state, steps, (t.flat, t.ob_mean, t.ob_std), (sp, s.ob_mean, s.ob_std),
                                  loss=workload["loss"], act_student=workload["act_with"] == "student",
                                  stagger=True, nthreads=threads)
        ref_c.adam_tf1(sp, m, v, g, b1p, b2p)
        b1p *= 0.9; b2p *= 0.999
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds and steps >= 2:
            break
    return dict(value=n * steps / el, unit="env-steps/s", cores=threads, kind="port", envs=n,
                sample=f"{n} envs (the workload's per-GPU batch) x {steps} steps ({el:.1f} s), same step "
                       f"(env + teacher + student fwd/bwd "
                       f"+ {workload['loss']} + TF1 Adam), C f32 restatement oracle/reacher_ref.c, "
                       f"OpenMP {threads} threads")


def convergence(wl, n, sdt, dev, rank, world, lr, max_steps, target=1e-3, chunk=None, comm=None, split=False,
                teacher=None):
    """North-star check: optimiser steps (one per env step, the reference's lr 1e-4 TF1 Adam)
    until the student's action-MSE vs the teacher, averaged over the last 10 steps and all
    ranks, falls below 1e-3 -- against the reference's budget of 5000 episodes x 50 steps =
    250,000 Adam steps (mlp_train.py:143-204)."""
    import torch
    import torch.distributed as dist

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    tr = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=lr,
                                      student_dtype=sdt, f32_split=split), device=dev, rank=rank, world_size=world,
                        comm=comm, teacher=teacher)
    t0 = time.perf_counter()
    steps, mse, hit, first = 0, float("nan"), None, None
    if chunk is None:   # small batches: checked every 10 steps, as scripts/conv_sweep.py measures them
        chunk = 10 if n * world <= 256 else 100
    while steps < max_steps:
        for _ in range(chunk):
            tr.step()
        steps += chunk
        met = tr.metrics(10)
        mt = torch.tensor(met.sum(0), dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(mt)
        mse = float(mt[2] / (2 * mt[3]))
        if first is None:   # the untrained student's MSE (the first check): how far the leg had to go
            first = mse
        if mse < target:
            hit = steps
            break
    el = time.perf_counter() - t0
    tr.close()
    env_steps = None if hit is None else hit * n * world
    budget = 5000 * 50   # mlp_train.py:143-204: 5000 episodes x 50 steps, one Adam step per env step
    return {"target_mse": target, "lr": lr, "loss": wl["loss"], "envs_total": n * world,
            "steps_checked_every": chunk, "opt_steps_to_target": hit, "env_steps_to_target": env_steps,
            "env_count_choice": ("the small-batch env count is a sweep's pick (scripts/conv_sweep.py, "
                                 "profiles/r03_conv_sweep.jsonl, lr 1e-4): 16/32/64/128 envs per step reach < 1e-3 "
                                 "within 250,000 env steps, 256 do not") if n * world <= 256 else None,
            "reference_budget_opt_steps": budget, "reference_budget_env_steps": budget,
            "within_opt_step_budget": hit is not None and hit <= budget,
            "within_env_step_budget": env_steps is not None and env_steps <= budget,
            "student_mse_first_check": first, "student_mse_final": mse, "opt_steps_run": steps, "seconds": el}


def convergence_driver(dev, lr, max_episodes=5000, target=1e-3, teacher=None):
    """The env-step reading of the budget on the reference's OWN loop shape: mlp_train.train
    (one env, per env step one Adam step on a 200-row window from the dataset's training pool,
    the 2x64 student, MSE) until an episode's mean window action-MSE is < 1e-3; env steps
    counted from the first teacher warm-up step (mlp_train.py:116-204)."""
    from reacherdistilation_amd import mlp_train
    t0 = time.perf_counter()
    tr, ds, losses = mlp_train.train(episodes=max_episodes, loss="mse", lr=lr, log=lambda *a: None, device=dev,
                                     stop_loss=target, teacher=teacher)
    el = time.perf_counter() - t0
    hit = bool(losses) and losses[-1] / 50 < target
    env_steps = ds.num_episodes() * 50
    tr.close()
    budget = 5000 * 50
    return {"target_mse": target, "lr": lr, "loss": "mse", "driver": "mlp_train.train (1 env, 200-row windows)",
            "episodes": ds.num_episodes(), "env_steps_to_target": env_steps if hit else None,
            "opt_steps_to_target": 50 * len(losses) if hit else None, "reference_budget_env_steps": budget,
            "within_env_step_budget": hit and env_steps <= budget,
            "student_mse_first_episode": losses[0] / 50 if losses else None,
            "student_mse_final": losses[-1] / 50 if losses else None, "seconds": el}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # RD_BENCH_ONE_DEVICE=1 + RD_DIST_BACKEND=gloo rehearse the N > 1 path with every rank
    # on cuda:0 (a 1-GPU box); the driver's multi-GPU runs use one GPU per rank over RCCL.
    if os.environ.get("RD_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("RD_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    # N > 1: the gradient all-reduce is issued by the native step on the trainer's stream
    # (include/reacher_comm.h).  The default is the native RCCL communicator (north star: one
    # RCCL all-reduce over xGMI per optimiser step); RD_COMM=xgmi binds the one-kernel xGMI push
    # exchange instead, RD_COMM=torch keeps torch.distributed's collective.  Whatever runs, BOTH
    # native exchanges are timed beside it (`exchange.rccl_us`, `exchange.xgmi_us`, or the
    # reason one is unavailable).  A communicator failing its one-shot self-check is dropped
    # for the next one (reported in config.collective).
    comm, collective = None, "none"
    exchange = None
    want = os.environ.get("RD_COMM", "rccl")
    if world > 1:
        exchange = {}
        cands = {}
        for kind in ("rccl", "xgmi"):
            c, why = _make_comm(kind, dev, world)
            if c is None:
                exchange[f"{kind}_us"] = f"unavailable: {why}"
                continue
            exchange[f"{kind}_us"] = exchange_latency(c, dev)["us"]
            exchange[f"{kind}_view"] = comm_view(c, dev, world)
            cands[kind] = c
        exchange["floats"] = 5060
        exchange["timing"] = "200 back-to-back in-place all-reduces of 5,060 floats, HIP events, trainer stream"
        order = [want] + [k for k in ("rccl", "xgmi") if k != want] if want != "torch" else []
        for kind in order:
            if kind in cands:
                comm = cands.pop(kind)
                collective = ("rccl (native, trainer stream)" if kind == "rccl"
                              else "xgmi push (native, one kernel, trainer stream)")
                break
        for c in cands.values():   # the one not bound
            torch.cuda.synchronize(dev)
            dist.barrier()
            c.close()
        if comm is None:
            collective = "torch.distributed" + (" (native exchanges unavailable)" if want != "torch" else "")
    wl = WORKLOADS[args.workload]
    n = args.envs_per_gpu or wl["envs"]
    sdt = wl.get("student_dtype", "f32")
    split = args.f32_mode == "split"

    # The convergence leg runs first, on trainers of its own: it is the north star's student
    # action-MSE check, and its ~1,000 back-to-back steps also take the GPU out of its idle
    # clocks, so the short timed region below (the driver runs 20 steps of ~0.12 ms) measures
    # the kernels rather than the clock ramp.
    conv = conv_small = None
    fitted, fit_info = fitted_teacher(dev) if ((args.conv_steps > 0 and world == 1) or args.teacher == "fitted") \
        else (None, None)
    if args.teacher == "fitted" and fitted is None:
        raise SystemExit("--teacher fitted needs tests/golden/reacher_fixture.npz")
    ppo_t, ppo_info = ppo_teacher_info(dev) if ((args.conv_steps > 0 and world == 1) or args.teacher == "ppo") \
        else (None, None)
    teacher = fitted if args.teacher == "fitted" else ppo_t if args.teacher == "ppo" else None
    if args.conv_steps > 0:
        conv = convergence(wl, n, sdt, dev, rank, world, args.lr, args.conv_steps, comm=comm, split=split,
                           teacher=teacher)
        # the same check at a small per-GPU batch: the env-step reading of the reference's budget
        conv_small = convergence(wl, args.conv_small_envs, sdt, dev, rank, world, args.lr, args.conv_steps, comm=comm,
                                 split=split, teacher=teacher)

    cfg = DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=args.lr, student_dtype=sdt,
                        f32_split=split)
    tr = DistillTrainer(cfg, device=dev, rank=rank, world_size=world, comm=comm, teacher=teacher)

    def one_step(ev=None):
        if ev is None and (world == 1 or comm is not None):
            tr.step()     # rdd_step: rollout + reduce (+ RCCL all-reduce) + Adam, one host call
            return
        if ev is not None:
            ev[0].record()
        tr.launch(tr.STAGE_ROLLOUT)
        if ev is not None:
            ev[1].record()
        if world == 1:
            tr.launch(tr.STAGE_REDUCE_APPLY)
        else:   # the bound communicator's or torch's all-reduce, between reduce and Adam
            tr.launch(tr.STAGE_REDUCE)
            tr.allreduce_grad()
            tr.launch(tr.STAGE_APPLY)

    settled = settle(one_step, dev, args.settle_ms, world)
    for _ in range(args.warmup):
        one_step()
    # the timed region: exactly `steps` steps, nothing else on the stream (no timing events)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # rollout_kernel's launch time for the roofline: a separate pass right after the timed
    # region, HIP events on the trainer's stream around every rollout launch (an event pair
    # costs the stream a few us per step, so it is kept out of the timed region)
    npass = max(20, min(args.steps, 200))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(npass)]
    for k in range(npass):
        one_step(evs[k])
    torch.cuda.synchronize(dev)
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    replicas = tr.replicas_identical() if world > 1 else True   # SURVEY §8e checksum
    if comm is not None and hasattr(comm, "check"):
        comm.check()   # (xGMI) raise if any exchange of the run waited past its limit for a peer

    accum = None
    if args.accum > 1:   # secondary line: one optimiser step (+ all-reduce) per K env-steps
        K = args.accum
        accum = {"accum_steps": K}
        # fused: one K-step launch per optimiser step (rdd_step_accum); staged: K rollout launches
        # each reduced into the gradient, then (all-reduce +) Adam (rdd_launch_stage)
        for form, opt_steps in (("fused", max(4, (2 * args.steps) // K)), ("staged", 2)):
            tk = DistillTrainer(DistillConfig(n_envs=n, seed=0, loss=wl["loss"], act_with=wl["act_with"], lr=args.lr,
                                              student_dtype=sdt, accum_steps=K, f32_split=split),
                                device=dev, rank=rank, world_size=world, comm=comm)

            def opt_step():
                if form == "fused":
                    tk.step_accum()
                else:
                    for _ in range(K):
                        tk.step()
            opt_step()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for _ in range(opt_steps):
                opt_step()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            tt = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ksteps = opt_steps * K
            accum[form] = {"env_steps": ksteps, "opt_steps": opt_steps, "value": n * world * ksteps / float(tt.item()),
                           "us_per_env_step": float(tt.item()) * 1e6 / ksteps,
                           "replicas_identical": tk.replicas_identical() if world > 1 else True}
            tk.close()
        accum["value"] = accum["fused"]["value"]
        accum["ms_per_step"] = accum["fused"]["us_per_env_step"] * 1e-3

    # the strong-scaling reading of the workload (its fixed global batch over the ranks); at
    # one GPU it is the headline run itself (c4: 262,144 envs on one GPU)
    strong = None
    total = wl.get("envs_global", wl["envs"])
    if world > 1 and not args.no_strong and not args.envs_per_gpu:
        strong = strong_leg(wl, total, sdt, split, dev, args.lr, max(args.steps, 100), args.warmup, rank, world, comm,
                            settle_ms=min(args.settle_ms, 100.0))
        if args.accum > 1:   # the same fixed global batch at one optimiser step per K env steps (K-step launch)
            strong["accum"] = strong_leg(wl, total, sdt, split, dev, args.lr, max(args.steps, 2 * args.accum),
                                         args.warmup, rank, world, comm, settle_ms=min(args.settle_ms, 100.0),
                                         accum=args.accum)

    # student action-MSE vs teacher over the last steps (all ranks)
    met = tr.metrics(min(10, tr.counter()))
    mt = torch.tensor(met.sum(0), dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(mt)
    mse = float(mt[2] / (2 * mt[3]))

    if rank == 0:
        ms = elapsed * 1e3 / args.steps
        value = n * world * args.steps / elapsed
        launch_s = kern_ms * 1e-3
        achieved = FLOP_PER_ENV_STEP * n / launch_s / 1e12
        peak = mixed_peak(sdt, split)
        copy_gbs = copy_bandwidth(dev)
        # HBM bytes per rollout launch from rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
        # MI355X_MICROARCH.md §HBM); counters cannot be read from inside this process, so the
        # committed profile of this workload is used and named in traffic_source
        traffic, traffic_src, issue = None, None, None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}_n{n}_{args.f32_mode}.json")
        if not os.path.exists(pmc) and not split:
            pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}_n{n}.json")   # round-1 name
        if os.path.exists(pmc):
            with open(pmc) as fh:
                pj = json.load(fh)
            traffic = pj.get("hbm_bytes_per_launch")
            issue = issue_roofline(pj.get("avg", {}), launch_s)
            traffic_src = {"file": os.path.relpath(pmc, ROOT), "measured": pj.get("measured", "round 1 (r01i/r01q)"),
                           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes "
                                     "(scripts/profile_workload.sh, scripts/pmc_traffic.py)"}
        other = None
        if world == 1 and not args.no_exact_leg:   # the other f32 mode, same workload, for comparison
            other = time_leg(wl, n, sdt, not split, dev, args.lr, args.steps, args.warmup, settle_ms=args.settle_ms)
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "settle": settled, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32" if sdt == "f32" else "bf16 student (f32 accumulate) + f32 teacher",
            "data": "synthetic: Philox(seed 0) Reacher-v2 resets, seeded synthetic teacher (normc, fixture logstd) "
                    "and student (2x64 MlpPolicy)",
            "config": {"workload": args.workload, "description": wl["desc"], "envs_per_gpu": n,
                       "envs_total": n * world, "student": f"MlpPolicy 2x64 tanh (5060 params, {sdt})",
                       "teacher": "MlpPolicy 2x64 tanh", "loss": wl["loss"], "act_with": wl["act_with"],
                       "optimizer": f"TF1 Adam lr {args.lr}, 1 step per env-step",
                       "parallelism": f"dp{world}", "collective": collective, "f32_mode": args.f32_mode,
                       "f32_arith": ("hidden-layer products (K = 64) f32-emulated on bf16 MFMA: exact 3-piece bf16 "
                                     "operand split, six partial products, f32 accumulate; the rest exact f32"
                                     if split else "every product on v_mfma_f32_16x16x4_f32 (exact f32)")},
            # the north star's student action-MSE: after the convergence leg (< 1e-3 within its
            # budget); the timed run's own value (220 steps from init) is kept beside it
            "student_mse": conv["student_mse_final"] if conv is not None else mse,
            "student_mse_timed_run": mse,
            "roofline": {"kernel": "rollout_kernel", "bound": "mfma", "achieved": achieved,
                         "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                         "peak_basis": ("MFMA-time-weighted peak of the FLOP mix: f32 MFMA 157.3 TF; split-emulated "
                                        "f32 (six bf16 products) 2500/6 TF; bf16 2500 TF"),
                         "frac_of_f32_mfma_peak": achieved / PEAK_F32_TFLOPS,
                         # round-stable reading: the same FLOP mix's peak as in round
                         # 3 (c4 split 376.9 TF, c5 1,058 TF), held fixed while the mix is unchanged
                         "frac_fixed_basis": achieved / FIXED_PEAK.get((sdt, split), peak),
                         "fixed_peak": FIXED_PEAK.get((sdt, split), peak),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "flop_per_env_step": FLOP_PER_ENV_STEP, "launch_us": kern_ms * 1e3,
                         "launch_timing": f"HIP events around each of {npass} rollout launches, a pass after "
                                          "the timed region",
                         "hbm_gbs_algorithmic": BYTES_PER_ENV_STEP * n / launch_s / 1e9,
                         "hbm_peak_gbs": PEAK_HBM_GBS, "hbm_copy_gbs_measured": copy_gbs},
            "replicas_identical": replicas,
        }
        if issue is not None:
            out["roofline_issue"] = issue
        if other is not None:
            out["other_f32_mode"] = other
        if strong is not None:
            out["strong_scaling"] = strong
        if exchange is not None:
            out["exchange"] = exchange
        if accum is not None:
            out["accum"] = accum
        if conv is not None:
            out["convergence"] = conv
            out["convergence_small_batch"] = conv_small
            out["convergence_teacher"] = args.teacher
            if world == 1:
                out["convergence_reference_driver"] = convergence_driver(dev, args.lr, teacher=teacher)
        if fit_info is not None and world == 1 and args.conv_steps > 0:
            # the north star's student action-MSE against a teacher shaped like the
            # reference's (fitted to its 1,050 teacher records), beside the synthetic teacher's legs
            ft = {"teacher": fit_info}
            if args.teacher == "fitted":
                ft["convergence"], ft["convergence_small_batch"] = conv, conv_small
                ft["convergence_reference_driver"] = out["convergence_reference_driver"]
            else:
                ft["convergence"] = convergence(wl, n, sdt, dev, 0, 1, args.lr, args.conv_steps, split=split,
                                                teacher=fitted)
                ft["convergence_small_batch"] = convergence(wl, args.conv_small_envs, sdt, dev, 0, 1, args.lr,
                                                            args.conv_steps, split=split, teacher=fitted)
                ft["convergence_reference_driver"] = convergence_driver(dev, args.lr, teacher=fitted)
            out["convergence_fitted_teacher"] = ft
        if ppo_info is not None and world == 1 and args.conv_steps > 0:
            # the north star's student action-MSE against the teacher PPO-trained here
            pt = {"teacher": ppo_info}
            if args.teacher == "ppo":
                pt["convergence"], pt["convergence_small_batch"] = conv, conv_small
                pt["convergence_reference_driver"] = out["convergence_reference_driver"]
            else:
                pt["convergence"] = convergence(wl, n, sdt, dev, 0, 1, args.lr, args.conv_steps, split=split,
                                                teacher=ppo_t)
                pt["convergence_small_batch"] = convergence(wl, args.conv_small_envs, sdt, dev, 0, 1, args.lr,
                                                            args.conv_steps, split=split, teacher=ppo_t)
                pt["convergence_reference_driver"] = convergence_driver(dev, args.lr, teacher=ppo_t)
            out["convergence_ppo_teacher"] = pt
        if conv is not None and world == 1:
            # every convergence leg at a glance -- which reach the north star's
            # action-MSE < 1e-3 within the reference's 250,000 env steps, against which teacher
            legs = {}
            for tname, blk in (("synthetic", out), ("fitted", out.get("convergence_fitted_teacher")),
                               ("ppo", out.get("convergence_ppo_teacher"))):
                if not blk:
                    continue
                if tname == "synthetic" and args.teacher != "synthetic":
                    tname = args.teacher
                for leg in ("convergence", "convergence_small_batch", "convergence_reference_driver"):
                    c = blk.get(leg)
                    if c:
                        legs[f"{tname}/{leg.replace('convergence_', '').replace('convergence', 'headline_batch')}"] = {
                            k: c.get(k) for k in ("envs_total", "env_steps_to_target", "within_env_step_budget",
                                                  "student_mse_first_check", "student_mse_first_episode",
                                                  "student_mse_final") if c.get(k) is not None}
            out["student_mse_legs"] = legs
        out["roofline_env"] = env_roofline(dev)
        ceil = copy_ceiling()
        if ceil is not None:   # the float4 copy measured in this run
            out["roofline_env"]["copy_ceiling"] = ceil
            out["roofline_env"]["frac_of_measured_copy"] = out["roofline_env"]["achieved"] / ceil["best_gbs"]
            out["roofline_env"]["frac_of_measured_mix"] = out["roofline_env"]["achieved"] / ceil["mix_1r2w_best_gbs"]
        else:
            out["roofline_env"]["frac_of_measured_copy"] = out["roofline_env"]["achieved"] / copy_gbs
            out["roofline_env"]["copy_ceiling"] = "torch copy_ (scripts/micro/libcopybw.so not built)"
        if world == 1 and args.workload == "c4" and not args.no_strong_projection and not args.envs_per_gpu:
            out["strong_projection"] = strong_projection(wl, sdt, split, dev, args.lr, 200, min(args.settle_ms, 100.0),
                                                         accum=max(1, args.accum))
        if world == 1 and not args.no_workloads and not args.envs_per_gpu:
            out["workloads"] = workloads(dev, args.lr, max(args.steps, 200), args.warmup, min(args.settle_ms, 100.0),
                                         accum=max(1, args.accum),
                                         names=tuple(k for k in ("c2", "c3", "c5") if k != args.workload))
        if world == 1 and args.fixture_steps > 0:
            out["convergence_fixture"] = convergence_fixture(dev, args.lr, args.fixture_steps, args.fixture_ref_steps)
        if world == 1 and args.fixture_steps > 0:
            out["teacher_ppo"] = teacher_ppo(dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds, args.cpu_threads, n)
            out["cpu_baseline"]["ref_loop"] = cpu_ref_loop(min(4.0, args.cpu_seconds))
            out["cpu_baseline"]["batched_env"] = cpu_batched_env(min(4.0, args.cpu_seconds))
        # at N > 1 a communication library may have written to stdout without a newline
        # (gloo's "[Gloo] Rank 0 is connected ..."): start the JSON line on a line of its own
        sys.stdout.flush()
        print(("\n" if world > 1 else "") + json.dumps(out), flush=True)
    if world > 1:
        tr.close()
        if comm is not None:
            torch.cuda.synchronize(dev)
            dist.barrier()   # (xGMI) no peer still writes into this rank's exchange buffer
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

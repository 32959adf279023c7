#!/usr/bin/env python3
"""Phase breakdown of rollout_kernel from the RD_STAMPS diagnostic build (per-wave s_memtime
stamps, summed per phase over a wave's groups/tiles; s_memrealtime at kernel start/end gives
the shader clock).  Read SHARES, not absolute lengths: the stamps' waits forbid some overlap,
and the two waves of a pair share their SIMD, so a phase's interval includes the partner's
issue.
usage: RD_LIB=libreacher_stamps.so python scripts/stamps.py [N]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd import _native as nat  # noqa: E402
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

NSTAMP = 24


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    # RD_SPLIT=1: f32_split; RD_WL=c5: DAgger with the bf16 student
    c5 = os.environ.get("RD_WL") == "c5"
    tr = DistillTrainer(DistillConfig(n_envs=n, seed=0, f32_split=os.environ.get("RD_SPLIT") == "1",
                                      act_with="student" if c5 else "teacher", student_dtype="bf16" if c5 else "f32"),
                        device="cuda:0")
    lib = nat.load()
    lib.rdd_debug_stamps.restype = ctypes.c_int
    lib.rdd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(1 << 22, np.uint64)
    for _ in range(5):
        tr.step()
    lib.rdd_debug_stamps(tr._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)   # reset the sums
    iters = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        tr.launch(tr.STAGE_ROLLOUT)
        tr.launch(tr.STAGE_REDUCE_APPLY)
    ev[1].record()
    torch.cuda.synchronize()
    cnt = lib.rdd_debug_stamps(tr._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    st = buf[:cnt].reshape(-1, NSTAMP).astype(np.float64)
    active = st[:, 0] > 0
    widx = np.flatnonzero(active) % 8
    st = st[active]
    prod = widx < 4
    # RD_OWNERS=1 (the helper-pair layout of a small batch): the role statistics over
    # the owner pairs 0, 1; the helper producers' teacher forwards are stamps 18 -> 19 (waves 2, 3),
    # the helper consumers' dW2 wait / dW2 are 20 -> 21 -> 22 (waves 6, 7)
    owners = os.environ.get("RD_OWNERS") == "1"
    hp, hc = (widx == 2) | (widx == 3), (widx == 6) | (widx == 7)
    if owners:
        prod = (widx == 0) | (widx == 1)
    cons = ((widx == 4) | (widx == 5)) if owners else ~prod

    def d(a, b, sel=None):
        v = (st[:, b] - st[:, a]) / iters
        return float(np.median(v if sel is None else v[sel]))

    cycles = d(0, 7)
    real_ns = d(16, 17) * 10.0          # s_memrealtime ticks at 100 MHz
    res = {
        "n": n, "waves": int(active.sum()), "step_us_with_reduce": ev[0].elapsed_time(ev[1]) * 1e3 / iters,
        "kernel_cycles": cycles, "kernel_us_in_kernel_clock": real_ns * 1e-3,
        "shader_clock_ghz": cycles / real_ns if real_ns > 0 else None,
        "prologue": d(0, 1),
        "group_loop": d(1, 6),
        "producer_obs": d(8, 11, prod),
        "producer_fwd_tiles": d(10, 12, prod),
        "producer_wait": d(2, 3, prod),
        "producer_physics": d(4, 5, prod),
        "consumer_physics": d(4, 5, cons),
        "consumer_wait": d(2, 3, cons),
        "consumer_slot_read": d(3, 13, cons),
        "consumer_dw2_dh1": d(13, 14, cons),
        "consumer_dz1_dw1": d(14, 15, cons),
        "helper_teacher_start": d(0, 18, hp) if owners else None,
        "helper_teacher_fwd": d(18, 19, hp) if owners else None,
        "helper_env_step": d(19, 23, hp) if owners else None,
        "helper_dw2_wait": d(20, 21, hc) if owners else None,
        "helper_dw2": d(21, 22, hc) if owners else None,
        "epilogue_barrier_wait": d(6, 9),
        "epilogue_reduce": d(9, 7),
        # per wave slot (0-3 dispatched first; w and w+4 share a SIMD): time to reach the epilogue
        "loop_end_by_wave_slot": [float(np.median(((st[:, 6] - st[:, 0]) / iters)[widx == w])) for w in range(8)],
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Phase breakdown of rollout_kernel from the RD_STAMPS diagnostic build (per-wave s_memtime
stamps).  Read SHARES, not absolute lengths: the stamps' waits forbid some overlap.
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    tr = DistillTrainer(DistillConfig(n_envs=n, seed=0), device="cuda:0")
    lib = nat.load()
    lib.rdd_debug_stamps.restype = ctypes.c_int
    lib.rdd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(1 << 20, np.uint64)
    for _ in range(5):
        tr.step()
    lib.rdd_debug_stamps(tr._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    iters = 20
    for _ in range(iters):
        tr.launch(tr.STAGE_ROLLOUT)
        tr.launch(tr.STAGE_REDUCE_APPLY)
    torch.cuda.synchronize()
    cnt = lib.rdd_debug_stamps(tr._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    st = buf[:cnt].reshape(-1, 16).astype(np.float64)
    active = st[:, 2] > 0
    st = st[active]
    d = lambda a, b: (st[:, b] - st[:, a]) / iters  # noqa: E731
    res = {
        "n": n, "waves": int(active.sum()),
        "prologue_load_nets": float(np.median(d(0, 1))),
        "obs_per_wave": float(np.median(d(2, 3))),
        "tiles_per_wave": float(np.median(d(3, 4))),
        "physics_per_wave": float(np.median(d(4, 5))),
        "group_loop_total": float(np.median(d(2, 5))),
        "epilogue_barrier_wait": float(np.median(d(6, 9))),
        "epilogue_reduce": float(np.median(d(9, 7))),
        "total": float(np.median(d(0, 7))),
    }
    prod = (np.flatnonzero(active) % 8) < 4
    res["producer_teacher_fwd"] = float(np.median(d(10, 11)[prod]))
    res["producer_student_fwd"] = float(np.median(d(11, 12)[prod]))
    res["producer_loss_dz2_to_wait"] = float(np.median((d(12, 2))[prod]))
    res["producer_wait"] = float(np.median(d(2, 3)[prod]))
    res["producer_slot_write"] = float(np.median((d(3, 10) )[prod]))
    res["consumer_wait"] = float(np.median(d(2, 3)[~prod]))
    res["consumer_slot_read"] = float(np.median(d(3, 13)[~prod]))
    res["consumer_dw2_dh1"] = float(np.median(d(13, 14)[~prod]))
    res["consumer_dz1_dw1"] = float(np.median(d(14, 15)[~prod]))
    res["producer_physics"] = float(np.median(d(4, 5)[prod]))
    # per wave slot (0-3 dispatched first; w and w+4 share a SIMD): time to finish the groups
    widx = np.flatnonzero(active) % 8
    res["finish_by_wave_slot"] = [float(np.median(d(0, 6)[widx == w])) for w in range(8)]
    res["tiles_by_wave_slot"] = [float(np.median(d(3, 4)[widx == w])) for w in range(8)]
    print(json.dumps(res))


if __name__ == "__main__":
    main()

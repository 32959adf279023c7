#!/usr/bin/env python3
"""Step time per workload and envs-per-group (DistillConfig.group_envs: 16 / 32 / 64; 0 = auto),
eager steps after a settle (diagnostic for the group-size choice).
usage: python scripts/sweep_group_envs.py [workload ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

CFG = {"c2": dict(n_envs=4096), "c3": dict(n_envs=65536, loss="kl"), "c4": dict(n_envs=262144),
       "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16")}


def step_us(tr, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        tr.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6


def main():
    for wl in sys.argv[1:] or ["c3", "c5"]:
        trs = {g: DistillTrainer(DistillConfig(seed=0, group_envs=g, **CFG[wl]), device="cuda:0") for g in (0, 16, 32, 64)}
        for tr in trs.values():
            step_us(tr, 1500)   # settle
        res = {g: [] for g in trs}
        for _ in range(3):
            for g, tr in trs.items():
                res[g].append(step_us(tr, 1000))
        print(json.dumps({"workload": wl, **{f"gs{g}_us": round(min(v), 2) for g, v in res.items()}}), flush=True)
        for tr in trs.values():
            tr.close()


if __name__ == "__main__":
    main()

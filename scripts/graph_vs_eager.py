#!/usr/bin/env python3
"""Step time of the fused rollout+distill step, eager launches vs one HIP graph of K steps,
per workload (diagnostic: does the host launch path or the inter-kernel gap show in the step?).
usage: python scripts/graph_vs_eager.py [workload ...]   (c2 c3 c4 c5)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

CFG = {"c2": dict(n_envs=4096), "c3": dict(n_envs=65536, loss="kl"), "c4": dict(n_envs=262144),
       "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16")}


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    K = 200
    for wl in sys.argv[1:] or ["c2", "c5", "c4"]:
        tr = DistillTrainer(DistillConfig(seed=0, **CFG[wl]), device="cuda:0")
        for _ in range(300):
            tr.step()
        g = tr.capture(K)
        g.replay()
        res = {"workload": wl}
        for rep in range(3):   # alternate, after the clock has settled
            res[f"eager_us_{rep}"] = timed(lambda: [tr.step() for _ in range(K)], 5) / K * 1e6
            res[f"graph_us_{rep}"] = timed(g.replay, 5) / K * 1e6
        print(json.dumps(res), flush=True)
        del g
        tr.close()


if __name__ == "__main__":
    main()

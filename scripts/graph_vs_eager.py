#!/usr/bin/env python3
"""Step time of the fused rollout+distill step, eager launches vs one HIP graph of K steps,
per env count (diagnostic: is the small-N step launch-bound?).
usage: python scripts/graph_vs_eager.py [N ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ns = [int(x) for x in sys.argv[1:]] or [4096, 65536, 262144]
    K = 50
    for n in ns:
        tr = DistillTrainer(DistillConfig(n_envs=n, seed=0), device="cuda:0")
        for _ in range(20):
            tr.step()
        eager = timed(lambda: [tr.step() for _ in range(K)], 4) / K
        g = tr.capture(K)
        g.replay()
        graph = timed(g.replay, 4) / K
        print(json.dumps({"n": n, "eager_us": eager * 1e6, "graph_us": graph * 1e6}), flush=True)
        tr.close()


if __name__ == "__main__":
    main()

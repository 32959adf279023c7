#!/usr/bin/env python3
"""Rollout/reduce kernel time vs env count in one process (fixed + per-env cost fit).
HIP events on the trainer's stream around each stage launch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402


def time_stage(tr, stage, iters=50):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        tr.launch(stage)
        b.record()
        if stage == tr.STAGE_ROLLOUT:
            tr.launch(tr.STAGE_REDUCE_APPLY)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


def main():
    out = []
    for n in [int(x) for x in (sys.argv[1:] or ["512", "8192", "65536", "262144", "1048576"])]:
        tr = DistillTrainer(DistillConfig(n_envs=n, seed=0), device="cuda:0")
        for _ in range(10):
            tr.step()
        r = time_stage(tr, tr.STAGE_ROLLOUT)
        out.append(dict(n=n, rollout_us=r, ns_per_env=1e3 * r / n))
        print(json.dumps(out[-1]), flush=True)
        tr.close()


if __name__ == "__main__":
    main()

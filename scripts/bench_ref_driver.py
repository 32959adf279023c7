#!/usr/bin/env python3
"""Throughput of the reference-shaped single-env driver (mlp_train.train, reference
src/distilation/mlp_train.py:18-204) on one MI355X: env steps per second over the whole run
(teacher warm-up phase + training phase), for the 2x64 MlpPolicy student and the reference's
own student_mlp_graph.  The loop is the reference's shape -- one env, per-step teacher and
student queries, one Adam step per window batch -- so it is latency-bound by design; compare
with bench.py's cpu_baseline.ref_loop (the same loop on one CPU core)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd import mlp_train  # noqa: E402


def main():
    episodes = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    for student in ("policy", "mlp"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr, ds, losses = mlp_train.train(episodes=episodes, student=student, log=lambda *a: None)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        steps = ds.num_episodes() * 50
        print(json.dumps({"driver": "mlp_train.train", "student": student, "episodes": ds.num_episodes(),
                          "env_steps": steps, "seconds": el, "env_steps_per_s": steps / el,
                          "last_episode_loss": losses[-1] if losses else None}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Throughput of the reference-shaped single-env driver (mlp_train.train, reference
src/distilation/mlp_train.py:18-204) on one MI355X: env steps per second over the whole run
(teacher warm-up phase + training phase), for the 2x64 MlpPolicy student and the reference's
own student_mlp_graph, and of the LSTM driver (lstm_train.train, the reference's
"successful" configuration); each with the env I/O on the device and through the gym-API env
(gym_env=True, numpy every step as the reference does).  The rate is over the whole run:
the reference's 41 teacher warm-up episodes, then the training episodes.  The loop is the reference's shape -- one env, per-step teacher and
student queries, one Adam step per window batch -- so it is latency-bound by design; compare
with bench.py's cpu_baseline.ref_loop (the same loop on one CPU core)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd import mlp_train  # noqa: E402


def run(name, fn, **kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr, ds, losses = fn(log=lambda *a: None, **kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = ds.num_episodes() * 50
    print(json.dumps({"driver": name, **{k: v for k, v in kw.items() if k != "episodes"},
                      "episodes": ds.num_episodes(), "env_steps": steps, "seconds": el,
                      "env_steps_per_s": steps / el, "last_episode_loss": losses[-1] if losses else None}), flush=True)


def main():
    from reacherdistilation_amd import lstm_train
    episodes = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    # one short untimed run of each driver first (module loads, first-launch costs)
    mlp_train.train(episodes=3, warmup_episodes=1, log=lambda *a: None)
    mlp_train.train(episodes=3, warmup_episodes=1, student="mlp", log=lambda *a: None)
    lstm_train.train(episodes=3, warmup_episodes=1, log=lambda *a: None)
    for gym_env in (False, True):
        for student in ("policy", "mlp"):
            run("mlp_train.train", mlp_train.train, episodes=episodes, student=student, gym_env=gym_env)
        run("lstm_train.train", lstm_train.train, episodes=episodes, gym_env=gym_env)


if __name__ == "__main__":
    main()

"""Where the reduce+Adam launch's time goes (c2/c4/c5): HIP-event timing of loops of
  step         = ROLLOUT + REDUCE_APPLY (the product step)
  rollout      = ROLLOUT only
  reduce_apply = REDUCE_APPLY only (back to back)
  reduce       = REDUCE only, apply = APPLY only
so that step - rollout is the reduce's in-stream cost after a rollout.
usage: python scripts/reduce_probe.py [c2 c4 c5]   (GPU)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

CFG = {"c2": dict(n_envs=4096), "c3": dict(n_envs=65536, loss="kl"), "c4": dict(n_envs=262144),
       "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16")}


def timed(fn, iters=400, warm=100):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    wls = sys.argv[1:] or ["c2", "c4", "c5"]
    for wl in wls:
        kw = dict(loss="mse", f32_split=True)
        kw.update(CFG[wl])
        tr = DistillTrainer(DistillConfig(**kw), device="cuda:0")
        L = tr.launch   # the trainer runs on torch's current stream, which the events see
        tiny = torch.zeros(1, device="cuda:0")
        r = {"workload": wl,
             "step_us": timed(lambda: (L(1), L(4))),
             "rollout_us": timed(lambda: L(1)),
             "reduce_apply_us": timed(lambda: L(4)),
             "reduce_us": timed(lambda: L(2)),
             "apply_us": timed(lambda: L(3)),
             # the floor: a minimal dependent kernel (one-element torch add) after the rollout
             "rollout_tiny_us": timed(lambda: (L(1), tiny.add_(1.0))),
             "tiny_us": timed(lambda: tiny.add_(1.0)),
             "step_us_again": timed(lambda: (L(1), L(4)))}
        r["reduce_in_step_us"] = r["step_us"] - r["rollout_us"]
        r["tiny_in_step_us"] = r["rollout_tiny_us"] - r["rollout_us"]
        print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}), flush=True)
        tr.close()


if __name__ == "__main__":
    main()

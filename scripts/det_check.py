"""Determinism probe: the same rollout twice (fresh trainers), per f32 mode / physics wave."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402


def roll(**kw):
    tr = DistillTrainer(DistillConfig(seed=5, **kw), device="cuda:0")
    s0 = tr.env_state().clone()
    tr.rollout()
    g, s = tr.grad().clone(), tr.env_state().clone()
    c = tr.counter()   # raises on a timed-out hand-off
    m = tr.metrics(0)
    tr.close()
    return g, s, s0, c


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
CASES = {"c4s": dict(n_envs=262144, f32_split=True), "c4e": dict(n_envs=262144, f32_split=False),
         "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=True),
         "c5e": dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=False),
         "c2s": dict(n_envs=4096, f32_split=True), "c2e": dict(n_envs=4096, f32_split=False),
         "c3s": dict(n_envs=65536, loss="kl", f32_split=True),
         "grid300": dict(n_envs=300 * 4 * 64, grid=300, f32_split=True)}
for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["c4s", "c4e"]):
    kw = CASES[name]
    ref = roll(**kw)
    for r in range(reps):
        b = roll(**kw)
        bad = (ref[1] != b[1]).any(0).nonzero().flatten()
        if len(bad):
            e = bad[0].item()
            same_as_start = torch.equal(b[1][:, bad], b[2][:, bad])
            print(os.environ.get("RDD_PHYS"), kw, "rep", r, "bad envs", len(bad), "first", e, "last", bad[-1].item(),
                  "unstepped in bad run:", same_as_start, "grad entries differing", (ref[0] != b[0]).nonzero().flatten()[:8].tolist(),
                  "state rows differing", (ref[1][:, bad] != b[1][:, bad]).any(1).nonzero().flatten().tolist())
        elif not torch.equal(ref[0], b[0]):
            d = (ref[0] != b[0]).nonzero().flatten()
            print(os.environ.get("RDD_PHYS"), kw, "rep", r, "states identical, grad entries differ:",
                  d[:8].tolist(), "max", float((ref[0] - b[0]).abs().max()))
        else:
            print(os.environ.get("RDD_PHYS"), kw, "rep", r, "identical")

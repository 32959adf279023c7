"""Child process of tests/test_determinism_gpu.py: per config, two fresh trainers each run two
fused steps (rollout + reduce + Adam) from the same seed; prints one JSON line of sha256 digests
of (gradient, student parameters, env state) for both.  The first one is the first launch of its
kernel in this process -- the launch that differed in the r04 LDS-DMA build
(profiles/r04i_imgdma_nondeterminism.txt)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

CASES = {
    "c4_split": dict(n_envs=262144, f32_split=True),
    "grid300_split": dict(n_envs=300 * 4 * 64, grid=300, f32_split=True),
    "c5_bf16": dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=True),
    "c2_helper": dict(n_envs=4096, f32_split=True),
    "c3_kl": dict(n_envs=65536, loss="kl", f32_split=True),
    "c4_exact": dict(n_envs=262144, f32_split=False),
    # the K-step launch (rdd_step_accum): two optimiser steps of K env steps each
    "c3_k50": dict(n_envs=65536, loss="kl", f32_split=True, accum_steps=50),
    "shard8_k50": dict(n_envs=32768, f32_split=True, accum_steps=50),
}


def digest(tr):
    h = hashlib.sha256()
    for t in (tr.grad(), tr.student_params(), tr.env_state()):
        h.update(t.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def main(names):
    out = {}
    for name in names:
        runs = []
        for _ in range(2):
            tr = DistillTrainer(DistillConfig(seed=11, **CASES[name]), device="cuda:0")
            for _ in range(2):
                tr.step_accum() if CASES[name].get("accum_steps", 1) > 1 else tr.step()
            torch.cuda.synchronize()
            tr.counter()   # raises on a timed-out hand-off
            runs.append(digest(tr))
            tr.close()
        out[name] = runs
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else list(CASES))

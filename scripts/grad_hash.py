"""Bitwise fingerprint of a few optimiser steps per workload (gradient, student parameters, env
state), so two builds (RD_LIB) can be compared for identical results across processes.
  python scripts/grad_hash.py [steps] [workload,...]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

WL = {"c2": dict(n_envs=4096), "c2_2048": dict(n_envs=2048), "c3": dict(n_envs=65536, loss="kl"),
      "c4": dict(n_envs=262144), "c4x": dict(n_envs=262144, f32_split=False),
      "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16"),
      "k50_32768": dict(n_envs=32768, accum_steps=50), "g100": dict(n_envs=100 * 64 * 4, grid=100),
      "g300": dict(n_envs=300 * 64 * 4, grid=300)}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(WL)
    dev = torch.device("cuda", 0)
    out = {"lib": os.environ.get("RD_LIB", "libreacher.so")}
    for name in names:
        kw = dict(WL[name])
        tr = DistillTrainer(DistillConfig(seed=0, **kw), device=dev)
        fn = tr.step if kw.get("accum_steps", 1) == 1 else tr.step_accum
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        h = hashlib.sha256()
        for t in (tr.grad(), tr.student_params(), tr.env_state()):
            h.update(t.detach().cpu().numpy().tobytes())
        out[name] = h.hexdigest()[:16]
        tr.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

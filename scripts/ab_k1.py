"""Per-step time of the fused step (K = 1) for the BASELINE workloads and of the K = 50 launch at
the 32,768-env shard, in one process; RD_LIB selects the build (A/B runs alternate processes).
  python scripts/ab_k1.py [steps] [workload,...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

WL = {"c2": dict(n_envs=4096), "c3": dict(n_envs=65536, loss="kl"), "c4": dict(n_envs=262144),
      "c4x": dict(n_envs=262144, f32_split=False), "c3x": dict(n_envs=65536, loss="kl", f32_split=False),
      "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16"),
      "c5x": dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=False),
      "k50_c5": dict(n_envs=131072, act_with="student", student_dtype="bf16", accum_steps=50),
      "k50_32768": dict(n_envs=32768, accum_steps=50), "k50_c3": dict(n_envs=65536, loss="kl", accum_steps=50)}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(WL)
    dev = torch.device("cuda", 0)
    out = {"lib": os.environ.get("RD_LIB", "libreacher.so")}
    for name in names:
        kw = WL[name]
        tr = DistillTrainer(DistillConfig(seed=0, **kw), device=dev)
        K = kw.get("accum_steps", 1)
        fn = tr.step if K == 1 else tr.step_accum
        calls = steps if K == 1 else max(8, steps // K)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:   # clock settle
            fn()
            torch.cuda.synchronize(dev)
        for _ in range(max(2, calls // 10)):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        torch.cuda.synchronize(dev)
        out[name] = (time.perf_counter() - t0) * 1e6 / (calls * K)
        tr.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Per-env-step time of the fused step (K = 1), the staged K-step accumulation and the K-step
launch (rdd_step_accum) at c4 and its strong shards (one GPU).  Prints one JSON line per size.

  python scripts/accum_probe.py [--k 50] [--sizes 262144,131072,65536,32768,4096] [--split 1]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--sizes", default="262144,131072,65536,32768,4096")
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--loss", default="mse")
    ap.add_argument("--act", default="teacher")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--opt-steps", type=int, default=8)
    args = ap.parse_args()
    import torch

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    dev = torch.device("cuda", 0)
    K = args.k
    for n in [int(x) for x in args.sizes.split(",")]:
        kw = dict(n_envs=n, seed=0, loss=args.loss, act_with=args.act, f32_split=bool(args.split),
                  student_dtype=args.dtype)
        res = {"envs": n, "K": K, "split": args.split, "loss": args.loss, "act": args.act, "dtype": args.dtype}

        def timed(fn, calls, env_steps):
            for _ in range(max(2, calls // 4)):
                fn()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(calls):
                fn()
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) * 1e6 / env_steps

        t1 = DistillTrainer(DistillConfig(**kw), device=dev)
        res["k1_us_per_env_step"] = timed(t1.step, 400, 400)
        t1.close()
        ts = DistillTrainer(DistillConfig(accum_steps=K, **kw), device=dev)
        res["staged_us_per_env_step"] = timed(ts.step, K * args.opt_steps, K * args.opt_steps)
        ts.close()
        tf = DistillTrainer(DistillConfig(accum_steps=K, **kw), device=dev)
        res["fused_us_per_env_step"] = timed(tf.step_accum, args.opt_steps, K * args.opt_steps)
        # the launch alone (HIP events on the trainer's stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.opt_steps):
            tf.rollout_accum()
        b.record()
        torch.cuda.synchronize(dev)
        res["fused_rollout_reduce_us_per_env_step"] = a.elapsed_time(b) * 1e3 / (K * args.opt_steps)
        res["counters"] = tf.counters()
        tf.close()
        res["fused_env_steps_per_s"] = n / (res["fused_us_per_env_step"] * 1e-6)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

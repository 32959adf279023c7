#!/usr/bin/env python3
"""Cost of the N > 1 step structure on ONE GPU (diagnostic): world-size-1 RCCL process
group, per step (a) the fused single-rank step, (b) rollout + apply as two calls, (c) rollout
+ torch all_reduce of the 20 KB gradient + apply (the torch path), (d) the bare all_reduce,
(e) the fused step with the native RCCL communicator bound (rdd_step: the all-reduce on the
trainer's stream, one host call).  (c) - (b) is what the torch collective path adds beyond the exchange itself.
usage: python scripts/allreduce_overhead.py [N ...]"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd import _native as nat  # noqa: E402
from reacherdistilation_amd.dist import RcclComm  # noqa: E402
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402


def timed(fn, reps=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    ns = [int(x) for x in sys.argv[1:]] or [4096, 262144]
    for n in ns:
        tr = DistillTrainer(DistillConfig(n_envs=n, seed=0), device="cuda:0")
        lib, h, g = tr._lib, tr._h, tr._grad
        fused = timed(lambda: nat.check(lib.rdd_step(h), "rdd_step"))
        split = timed(lambda: (nat.check(lib.rdd_rollout(h), "r"), nat.check(lib.rdd_apply(h), "a")))

        def with_ar():
            nat.check(lib.rdd_rollout(h), "r")
            dist.all_reduce(g)
            nat.check(lib.rdd_apply(h), "a")
        ar_step = timed(with_ar)
        bare = timed(lambda: dist.all_reduce(g))
        comm = RcclComm(torch.device("cuda:0"))
        tr.bind_comm(comm)
        native = timed(lambda: nat.check(lib.rdd_step(h), "rdd_step"))
        tr.bind_comm(None)
        comm.close()
        print(json.dumps({"n": n, "fused_us": fused, "split_us": split, "torch_allreduce_step_us": ar_step,
                          "bare_allreduce_us": bare,
                          "native_rccl_step_us": native}), flush=True)
        tr.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

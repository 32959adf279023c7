#!/usr/bin/env python3
"""Diagnostic: two processes on ONE GPU build the native RCCL communicator
(dist.RcclComm) over a gloo group.  RCCL either accepts two ranks on one device (then the
self-check all-reduce and a bound trainer's sharded step are exercised) or refuses with an
error -- which must surface as an exception, not a hang (the bench then falls back to torch's
collective).  Prints one JSON line per rank."""
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, port):
    import torch.distributed as dist

    from reacherdistilation_amd.dist import RcclComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        comm = RcclComm(torch.device("cuda:0"))
        out["created"] = True
        out["self_check"] = comm.self_check()
        from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
        tr = DistillTrainer(DistillConfig(n_envs_global=8192, seed=7, lr=1e-3), device="cuda:0", rank=rank,
                            world_size=world, comm=comm)
        for _ in range(5):
            tr.step()
        out["replicas_identical"] = tr.replicas_identical()
        tr.close()
        comm.close()
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)[:300]
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_rank, args=(2, port), nprocs=2, join=True, start_method="spawn")


if __name__ == "__main__":
    main()

"""Data-parallel sharding of the env batch.

Envs are independent, so ranks take contiguous slices of the global env index space and
the Philox reset stream is keyed by the GLOBAL env id: the union of the shards is exactly
the single-GPU run.  The one exchange per optimiser step is an all_reduce(SUM) of the flat
student gradient (RCCL over xGMI via torch.distributed backend "nccl"; "gloo" in the CPU
tests).  The reference has no distributed path in src/distilation; its only collective is
MpiAdam's Allreduce(SUM) of the flat gradient (reference backup/student_rollout.py:658-659,709).
"""
from __future__ import annotations

import os


def shard(n_global: int, rank: int, world: int) -> tuple[int, int]:
    """(n_local, env_base) of `rank`: contiguous slices, the remainder on the first ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if n_global < world:
        raise ValueError(f"{n_global} envs cannot be sharded over {world} ranks")
    q, r = divmod(int(n_global), world)
    n_local = q + (1 if rank < r else 0)
    env_base = rank * q + min(rank, r)
    return n_local, env_base


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world) from the torchrun environment (1 process per GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_process_group(backend: str = "nccl", device=None):
    """torch.distributed init for the env:// rendezvous (MASTER_ADDR 127.0.0.1 on one node)."""
    import torch.distributed as dist
    if dist.is_initialized():
        return dist.group.WORLD
    kw = {}
    if device is not None and backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)
    return dist.group.WORLD


def allreduce_sum_(t, group=None):
    """In-place SUM all-reduce of one flat buffer (never per-tensor)."""
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def checksum(t) -> int:
    """Exact position-weighted checksum of a float32 tensor's bits (int64 arithmetic)."""
    import torch
    bits = t.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(1, bits.numel() + 1, dtype=torch.int64, device=bits.device)
    return int(((bits & 0xFFFFFFFF) * w).sum().item())


def replicas_identical(t, group=None) -> bool:
    """True iff `t` is bitwise identical on every rank (MIN and MAX of the checksum agree)."""
    import torch
    import torch.distributed as dist
    c = checksum(t)
    if not dist.is_initialized():
        return True
    lo = torch.tensor([c], dtype=torch.int64, device=t.device)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    return int(lo.item()) == int(hi.item())

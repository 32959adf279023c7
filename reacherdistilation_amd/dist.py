"""Data-parallel sharding of the env batch.

Envs are independent, so ranks take contiguous slices of the global env index space and
the Philox reset stream is keyed by the GLOBAL env id: the union of the shards is exactly
the single-GPU run.  The one exchange per optimiser step is an all_reduce(SUM) of the flat
student gradient (RCCL over xGMI via torch.distributed backend "nccl"; "gloo" in the CPU
tests).  The reference has no distributed path in src/distilation; its only collective is
MpiAdam's Allreduce(SUM) of the flat gradient (reference backup/student_rollout.py:658-659,709).

`RcclComm` is that exchange issued by the native library itself (include/reacher_comm.h): an
RCCL communicator of our own whose all-reduce runs on the trainer's stream, so the sharded
step is one host call with no cross-stream waits (torch's collective path costs a c4 step
~9 us and ~19 us of host time per call even at world size 1).
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


class RcclComm:
    """This rank's RCCL communicator (include/reacher_comm.h), created collectively over a
    torch.distributed group in three steps, each of which every rank reaches whatever the
    others did, so a failure anywhere raises on every rank instead of leaving one waiting:

      1. every rank probes whether it can join (RCCL resolvable, its HIP device selectable)
         and the group sums a one-hot vector of the answers: if any rank cannot, every rank
         raises NativeError naming it, before any RCCL call;
      2. rank 0 draws the RCCL unique id and the group broadcasts it with a success flag (rank
         0 joins the broadcast even when the draw failed);
      3. every rank creates the communicator; RCCL's init runs non-blocking with a deadline
         (`timeout` seconds), so a rank whose peers never arrive aborts and raises.

    Bind it to a trainer (`DistillTrainer(..., comm=...)`)."""

    def __init__(self, device, group=None, timeout: float = 60.0):
        import ctypes

        import torch
        import torch.distributed as dist

        from . import _native as nat
        self._lib = nat.load()
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:   # a bare "cuda" is the current device
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        on_dev = dist.get_backend(group) == "nccl"
        # 1. can every rank take part?
        rc = self._lib.rd_comm_probe(device.index if device.type == "cuda" else -1)
        why = "" if rc == 0 else self._lib.rd_last_error().decode(errors="replace")
        ok = torch.zeros(self.world, dtype=torch.int32)
        ok[self.rank] = 1 if rc == 0 else 0
        if on_dev:
            ok = ok.to(device)
        dist.all_reduce(ok, group=group)
        bad = [r for r, v in enumerate(ok.cpu().tolist()) if v != 1]
        if bad:
            raise nat.NativeError(f"RCCL communicator: rank(s) {bad} cannot join"
                                  f"{' (this rank: ' + why + ')' if why else ''}")
        # 2. the unique id, from rank 0, with its success flag
        idb = (ctypes.c_uint8 * 128)()
        ok0, why = 1, ""
        if self.rank == 0:
            if self._lib.rd_comm_unique_id(idb) != 0:
                ok0, why = 0, self._lib.rd_last_error().decode(errors="replace")
        t = torch.tensor(list(bytes(idb)) + [ok0], dtype=torch.uint8)
        if on_dev:
            t = t.to(device)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src=src, group=group)
        t = t.cpu()
        if int(t[-1]) != 1:
            raise nat.NativeError(f"rd_comm_unique_id failed on rank 0{': ' + why if why else ''}")
        idb = (ctypes.c_uint8 * 128)(*t[:128].tolist())
        # 3. every rank joins (bounded by `timeout`)
        h = ctypes.c_void_p()
        nat.check(self._lib.rd_comm_create(ctypes.byref(h), idb, self.world, self.rank, device.index,
                                           float(timeout)), "rd_comm_create")
        self.handle = h

    def allreduce_(self, t):
        """In-place SUM of a contiguous float32 device tensor, on the current stream."""
        import ctypes

        import torch

        from . import _native as nat
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("allreduce_ takes a contiguous float32 tensor on the communicator's device")
        nat.check(self._lib.rd_comm_allreduce_f32(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                                  nat.stream_handle(self.device)), "rd_comm_allreduce_f32")
        return t

    def query(self) -> dict:
        """RCCL's own view of this communicator (rd_comm_query: ncclCommCount, ncclCommUserRank,
        ncclCommCuDevice), not the values it was created with; an xGMI communicator reports
        those (from_rccl False)."""
        import ctypes

        from . import _native as nat
        c, r, d, f = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        nat.check(self._lib.rd_comm_query(self.handle, ctypes.byref(c), ctypes.byref(r), ctypes.byref(d),
                                          ctypes.byref(f)), "rd_comm_query")
        return {"count": c.value, "user_rank": r.value, "device": d.value, "from_rccl": bool(f.value),
                "created_rank": self.rank, "created_world": self.world}

    def self_check(self) -> bool:
        """One all-reduce of a known pattern: every element must come back as the sum over
        ranks (the bench falls back to torch's collective if not)."""
        import torch
        x = torch.arange(1024, dtype=torch.float32, device=self.device) + 1000.0 * self.rank
        self.allreduce_(x)
        want = torch.arange(1024, dtype=torch.float32, device=self.device) * self.world + \
            1000.0 * (self.world * (self.world - 1) // 2)
        return bool(torch.equal(x, want))

    def close(self):
        if getattr(self, "handle", None):
            self._lib.rd_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class XgmiComm(RcclComm):
    """The exchange as one xGMI push kernel (include/reacher_comm.h rd_xcomm_*): every rank
    exports an uncached exchange buffer, the group all-gathers the IPC handles, every rank maps
    the others'; an all-reduce then writes this rank's gradient into its slot of every rank's
    buffer, raises a flag there, waits for all flags and sums the slots in rank order (bitwise
    the same on every rank).  Created collectively like RcclComm: a failure on any rank (no
    IPC, a buffer that cannot be mapped) raises on every rank.  `cap` = floats per exchange;
    `timeout` = seconds an exchange waits for a peer before the communicator fails on every
    rank (the bound trainer then skips that optimiser step and raises NativeError on its next
    call; include/reacher_comm.h).  It also bounds rank-local host work between two exchanges:
    a rank held longer (checkpoint I/O, evaluation on rank 0 only) fails the communicator for
    good, hence the 10-minute default.  After such a failure re-broadcast the student and its
    Adam state from one rank before training on a new communicator: the outcome of the failed
    exchange is atomic per rank, not across ranks."""

    def __init__(self, device, group=None, cap: int = 8192, timeout: float = 600.0):
        import ctypes

        import torch
        import torch.distributed as dist

        from . import _native as nat
        self._lib = nat.load()
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        on_dev = dist.get_backend(group) == "nccl"
        # 1. every rank: its exchange buffer and IPC handle (+ a success byte)
        h = ctypes.c_void_p()
        hb = (ctypes.c_uint8 * 64)()
        rc = self._lib.rd_xcomm_create(ctypes.byref(h), self.world, self.rank, device.index, int(cap),
                                       float(timeout), hb)
        why = "" if rc == 0 else self._lib.rd_last_error().decode(errors="replace")
        self.handle = h if rc == 0 else None
        mine = torch.tensor(list(bytes(hb)) + [1 if rc == 0 else 0], dtype=torch.uint8)
        if on_dev:
            mine = mine.to(device)
        allh = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(allh, mine, group=group)
        allh = [t.cpu() for t in allh]
        bad = [r for r, t in enumerate(allh) if int(t[-1]) != 1]
        if bad:
            self.close()
            raise nat.NativeError(f"xGMI exchange: rank(s) {bad} could not export a buffer"
                                  f"{' (this rank: ' + why + ')' if why else ''}")
        # 2. every rank maps every other rank's buffer; the group agrees on the outcome
        flat = (ctypes.c_uint8 * (64 * self.world))(*[b for t in allh for b in t[:64].tolist()])
        rc = self._lib.rd_xcomm_connect(self.handle, flat)
        why = "" if rc == 0 else self._lib.rd_last_error().decode(errors="replace")
        ok = torch.zeros(self.world, dtype=torch.int32)
        ok[self.rank] = 1 if rc == 0 else 0
        if on_dev:
            ok = ok.to(device)
        dist.all_reduce(ok, group=group)
        bad = [r for r, v in enumerate(ok.cpu().tolist()) if v != 1]
        if bad:
            self.close()
            raise nat.NativeError(f"xGMI exchange: rank(s) {bad} could not map the peers' buffers"
                                  f"{' (this rank: ' + why + ')' if why else ''}")

    def check(self):
        """Raise if an exchange of this rank failed (a peer missed the deadline, or a peer
        failed first); no synchronisation."""
        from . import _native as nat
        nat.check(self._lib.rd_comm_check(self.handle), "rd_comm_check")

    def self_check(self) -> bool:
        ok = super().self_check()
        self.check()
        return ok


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

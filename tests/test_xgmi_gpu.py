"""The xGMI push exchange (include/reacher_comm.h rd_xcomm_*, csrc/rd_xgmi.hip) with 2, 4 and 8
ranks (the N = 8 path rehearsed before an 8-GPU node runs it): one per device
where enough are visible, else round-robin on the visible devices -- on a one-GPU box all on
cuda:0 (IPC within one device; the same kernel, the peers' buffers mapped through
hipIpcOpenMemHandle).  Checks: the SUM of
known patterns (exact in f32: small integers), repeated across both buffer parities and a
ragged length; the error word stays clear; and a DistillTrainer with the exchange bound
reproduces the single-rank run over the whole batch (student within 1e-5 after 5 Adam steps:
f32 summation order differs; the ranks' students bitwise identical).  Skipped, with the
reason, if this box cannot export or map the exchange buffers."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
N_GLOBAL, STEPS = 8192, 5


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out):
    import torch.distributed as dist

    from reacherdistilation_amd._native import NativeError
    from reacherdistilation_amd.dist import XgmiComm
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = XgmiComm(dev)
    except NativeError as e:
        out[rank] = ("skip", str(e))
        dist.destroy_process_group()
        return
    sums = []
    for k, n in enumerate([5060, 5060, 7, 5060, 4096, 1, 3, 5059]):   # both parities, ragged tails, n < 4
        base = torch.zeros(n + 1, dtype=torch.float32, device=dev)
        x = base[1:] if k == 7 else base[:n]   # k = 7: a gradient that is not 16-B aligned (scalar push)
        x.copy_(torch.arange(n, dtype=torch.float32, device=dev) % 97 + 1000.0 * rank + k)
        comm.allreduce_(x)
        want = (torch.arange(n, dtype=torch.float32, device=dev) % 97) * world + 1000.0 * (world * (world - 1) // 2) \
            + k * world
        sums.append(bool(torch.equal(x, want)))
    # a long chain of exchanges whose inputs depend on the previous sums: one corrupted
    # exchange anywhere (e.g. a sum overwriting the gradient before a slower block pushed it)
    # leaves the ranks with different bits at the end
    from reacherdistilation_amd.dist import replicas_identical
    y = torch.ones(5060, dtype=torch.float32, device=dev)
    for _ in range(3000):
        y.mul_(0.5).add_(rank + 1)
        comm.allreduce_(y)
    torch.cuda.synchronize(dev)
    chain_same = replicas_identical(y.cpu())
    comm.check()
    tr = DistillTrainer(DistillConfig(n_envs_global=N_GLOBAL, seed=7, lr=1e-3), device=dev, rank=rank,
                        world_size=world, comm=comm)
    for _ in range(STEPS):
        tr.step()
    out[rank] = ("ok", sums + [chain_same], tr.student_params().cpu().numpy(), tr.env_state().cpu().numpy(),
                 tr.metrics(STEPS), tr.replicas_identical())
    comm.check()
    tr.close()
    dist.barrier()   # no peer still writes into this rank's buffer
    comm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_exchange(world):
    """Exact sums over both epoch parities and ragged / unaligned lengths, a 3,000-exchange chain
    whose replicas stay bitwise identical, and a trainer bound to the exchange that reproduces the
    single-rank run over the whole batch (the shards' states concatenate to it)."""
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_rank, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
    rs = [out[r] for r in range(world)]
    skip = [r for r in rs if r[0] == "skip"]
    if skip:
        pytest.skip(f"xGMI exchange unavailable here: {skip[0][1]}")
    for r in rs:
        assert all(r[1]), r[1]
        assert r[5] and np.array_equal(r[2], rs[0][2])
    ref = DistillTrainer(DistillConfig(n_envs=N_GLOBAL, seed=7, lr=1e-3), device="cuda:0")
    for _ in range(STEPS):
        ref.step()
    np.testing.assert_allclose(rs[0][2], ref.student_params().cpu().numpy(), atol=1e-5)
    np.testing.assert_allclose(np.concatenate([r[3] for r in rs], axis=1), ref.env_state().cpu().numpy(), atol=1e-4)
    np.testing.assert_allclose(sum(r[4][:, 3] for r in rs), ref.metrics(STEPS)[:, 3])
    ref.close()


TIMEOUT_S, LATE_S = 2.0, 6.0


def _late_rank(rank, world, port, out):
    """The last rank reaches its third step LATE_S seconds after the others (host skew past the
    exchange's TIMEOUT_S deadline): the others' exchanges time out and poison every buffer, the
    late rank's then fails on the poison; no rank applies Adam, and all raise on their next step."""
    import time

    import torch.distributed as dist

    from reacherdistilation_amd._native import NativeError
    from reacherdistilation_amd.dist import XgmiComm
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = XgmiComm(dev, timeout=TIMEOUT_S)
    except NativeError as e:
        out[rank] = ("skip", str(e))
        dist.destroy_process_group()
        return
    tr = DistillTrainer(DistillConfig(n_envs_global=4096, seed=7, lr=1e-3), device=dev, rank=rank,
                        world_size=world, comm=comm)
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize(dev)
    before = tr.student_params().cpu().numpy()
    dist.barrier()
    if rank == world - 1:
        time.sleep(LATE_S)
    t0 = time.perf_counter()
    tr.step()            # rank 0: times out after TIMEOUT_S; rank 1: fails on the poison
    torch.cuda.synchronize(dev)
    waited = time.perf_counter() - t0
    after = tr.student_params().cpu().numpy()
    errs = []
    for call in (tr.step, comm.check, tr.counters):
        try:
            call()
            errs.append(None)
        except NativeError as e:
            errs.append(str(e))
    out[rank] = ("ok", before, after, errs, waited)
    dist.barrier()
    tr.close()
    comm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_exchange_late_peer_fails_every_rank_and_skips_adam(world):
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_late_rank, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
    rs = [out[r] for r in range(world)]
    skip = [r for r in rs if r[0] == "skip"]
    if skip:
        pytest.skip(f"xGMI exchange unavailable here: {skip[0][1]}")
    for r in rs:
        _, before, after, errs, _ = r
        assert np.array_equal(before, after)          # Adam skipped: parameters unchanged
        assert all(e is not None for e in errs), errs  # rdd_step, rd_comm_check, the counters
        assert np.array_equal(before, rs[0][1])
    assert TIMEOUT_S * 0.8 <= rs[0][4] < LATE_S + TIMEOUT_S   # an early rank waited for its deadline
    assert rs[-1][4] < TIMEOUT_S                              # the late rank failed at once on the poison

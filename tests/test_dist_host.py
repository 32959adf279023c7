"""Multi-rank path on CPU (gloo, world_size 2): env sharding + the one gradient all-reduce.

Each rank runs the C f32 oracle's rollout+distill step on its contiguous shard (global env
ids, MSE normalised by the GLOBAL env count, staggered clocks keyed by global id: the
contract rollout_kernel implements, include/reacher_distill.h), all-reduces the flat
gradient with torch.distributed (gloo) and applies TF1 Adam.  The result must equal the
single-rank full batch up to f32 summation order (rtol 1e-5 on the gradient).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from reacherdistilation_amd.dist import allreduce_sum_, shard


def test_shard_covers_all_envs():
    for n, w in [(8, 1), (10, 3), (262144, 8), (1048576, 8), (4097, 2)]:
        parts = [shard(n, r, w) for r in range(w)]
        assert sum(p[0] for p in parts) == n
        assert parts[0][1] == 0
        for (n0, b0), (n1, b1) in zip(parts, parts[1:]):
            assert b1 == b0 + n0 and abs(n1 - n0) <= 1
    with pytest.raises(ValueError):
        shard(1, 0, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


N_GLOBAL, SEED, STEPS = 1000, 4, 3


def _nets():
    from reacherdistilation_amd.policy import student_init, synthetic_teacher
    t, s = synthetic_teacher(1), student_init(2)
    return (t.flat, t.ob_mean, t.ob_std), s


def _run(rank, world, port, out):
    from oracle import ref_c
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, base = shard(N_GLOBAL, rank, world)
    tnet, s = _nets()
    sp = s.flat.copy()
    P = ref_c.param_count()
    m, v = np.zeros(P, np.float32), np.zeros(P, np.float32)
    state = ref_c.philox_reset(n, base, SEED, 0)
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    grads = []
    for k in range(STEPS):
        g, met = ref_c.distill_step(state, k, tnet, (sp, s.ob_mean, s.ob_std), seed=SEED, loss="mse",
                                    n_global=N_GLOBAL, env_base=base, stagger=True, nthreads=1)
        gt = torch.from_numpy(g)
        allreduce_sum_(gt)
        grads.append(gt.numpy().copy())
        ref_c.adam_tf1(sp, m, v, gt.numpy(), float(b1p), float(b2p), lr=1e-3)
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
    out[rank] = (np.stack(grads), sp, state)
    dist.destroy_process_group()


def test_two_rank_allreduce_equals_full_batch(oracle_c):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_run, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, p0, st0 = out[0]
    g1, p1, st1 = out[1]
    # every rank holds the same reduced gradient and therefore the same student
    assert np.array_equal(g0, g1) and np.array_equal(p0, p1)
    # ... which is the full single-rank batch
    tnet, s = _nets()
    sp = s.flat.copy()
    P = oracle_c.param_count()
    m, v = np.zeros(P, np.float32), np.zeros(P, np.float32)
    state = oracle_c.philox_reset(N_GLOBAL, 0, SEED, 0)
    b1p, b2p = np.float32(0.9), np.float32(0.999)
    for k in range(STEPS):
        g, _ = oracle_c.distill_step(state, k, tnet, (sp, s.ob_mean, s.ob_std), seed=SEED, loss="mse",
                                     stagger=True, nthreads=1)
        np.testing.assert_allclose(g0[k], g, rtol=1e-5, atol=1e-6 * np.abs(g).max())
        oracle_c.adam_tf1(sp, m, v, g, float(b1p), float(b2p), lr=1e-3)
        b1p, b2p = np.float32(b1p * np.float32(0.9)), np.float32(b2p * np.float32(0.999))
    np.testing.assert_allclose(p0, sp, atol=2e-5)
    # the shards' env states are the full batch's, split contiguously
    n0 = shard(N_GLOBAL, 0, world)[0]
    np.testing.assert_allclose(np.concatenate([st0, st1], axis=1), state, atol=2e-5)
    assert st0.shape[1] == n0


def _run_checksum(rank, world, port, out):
    from reacherdistilation_amd.dist import checksum, replicas_identical
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    same = torch.arange(5060, dtype=torch.float32) * 1e-3
    diff = same.clone()
    if rank == 1:
        diff[1234] = torch.nextafter(diff[1234], torch.tensor(1e9))   # one ulp on one rank
    out[rank] = (replicas_identical(same), replicas_identical(diff), checksum(same))
    dist.destroy_process_group()


def test_replica_checksum_detects_one_ulp():
    """student weights are asserted identical across ranks by a checksum."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_run_checksum, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert out[r][0] is True and out[r][1] is False
    assert out[0][2] == out[1][2]


def test_native_comm_host_contract():
    """include/reacher_comm.h without a GPU: the RCCL unique id comes back (128 bytes, not
    all zero); argument errors and a communicator on a missing device fail with a message
    (rc != 0, rd_last_error set) instead of crashing -- the error path on which bench.py
    falls back to torch's collective."""
    import ctypes

    from reacherdistilation_amd import _native as nat
    lib = nat.load()
    idb = (ctypes.c_uint8 * 128)()
    rc = lib.rd_comm_unique_id(idb)
    if rc != 0:   # no RCCL on this host: the failure is reported, not raised from C
        assert lib.rd_last_error()
        return
    assert any(bytes(idb))
    h = ctypes.c_void_p()
    assert lib.rd_comm_create(ctypes.byref(h), idb, 0, 0, 0, 60.0) != 0    # nranks 0
    assert b"bad argument" in lib.rd_last_error()
    assert lib.rd_comm_create(ctypes.byref(h), idb, 2, 2, 0, 60.0) != 0    # rank out of range
    assert lib.rd_comm_create(ctypes.byref(h), idb, 1, 0, 0, 0.0) != 0     # no deadline
    assert lib.rd_comm_allreduce_f32(None, None, 4, None) != 0
    assert lib.rd_comm_nranks(None) == 0 and lib.rd_comm_destroy(None) == 0
    if not torch.cuda.is_available():
        assert lib.rd_comm_create(ctypes.byref(h), idb, 1, 0, 0, 60.0) != 0   # no HIP device here
        assert lib.rd_last_error()
        assert lib.rd_comm_probe(0) != 0 and b"rd_comm_probe" in lib.rd_last_error()


def _comm_rank(rank, world, port, out, inject=None):
    import datetime

    import torch.distributed as dist

    from reacherdistilation_amd import _native as nat
    from reacherdistilation_amd.dist import RcclComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # a short collective timeout: a regression that leaves a rank waiting fails fast
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
    if inject == "rank0_id":   # every rank passes the probe; rank 0 cannot draw the id
        lib = nat.load()
        lib.rd_comm_probe = lambda device: 0
        if rank == 0:
            lib.rd_comm_unique_id = lambda buf: 1
            lib.rd_last_error = lambda: b"injected failure"
    try:
        RcclComm(torch.device("cpu"))
        out[rank] = ("created", "")
    except Exception as e:  # noqa: BLE001
        out[rank] = (type(e).__name__, str(e))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.skipif(torch.cuda.is_available(), reason="the no-device failure path is exercised on CPU hosts")
def test_native_comm_failure_reaches_every_rank():
    """Two gloo ranks build dist.RcclComm on a host without a HIP device: both fail the
    probe, the group agrees on it, and each raises NativeError naming the ranks that cannot
    join -- before any RCCL call, with no rank left waiting in a collective."""
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_comm_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    assert out[0][0] == out[1][0] == "NativeError"
    assert "[0, 1] cannot join" in out[0][1] and "[0, 1] cannot join" in out[1][1]


def test_rank0_id_failure_reaches_every_rank():
    """Rank 0 fails to draw the RCCL unique id (injected); rank 1 must not wait for it: both
    raise, and rank 1's message names rank 0."""
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_comm_rank, args=(2, _free_port(), out, "rank0_id"), nprocs=2, join=True,
                       start_method="spawn")
    assert out[0][0] == out[1][0] == "NativeError"
    assert "failed on rank 0" in out[1][1] and "injected failure" in out[0][1]


def _xcomm_rank(rank, world, port, out, inject=None):
    import datetime

    import torch.distributed as dist

    from reacherdistilation_amd import _native as nat
    from reacherdistilation_amd.dist import XgmiComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
    if inject == "rank1_map":   # every rank exports a buffer; rank 1 cannot map its peer's
        lib = nat.load()
        lib.rd_xcomm_create = lambda h, nranks, r, dev, cap, timeout, hb: 0
        lib.rd_xcomm_connect = (lambda c, hs: 1) if rank == 1 else (lambda c, hs: 0)
        lib.rd_last_error = lambda: b"injected map failure"
        lib.rd_comm_destroy = lambda c: 0
    try:
        XgmiComm(torch.device("cuda", 0))
        out[rank] = ("created", "")
    except Exception as e:  # noqa: BLE001
        out[rank] = (type(e).__name__, str(e))
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.is_available(), reason="the no-device failure path is exercised on CPU hosts")
def test_xgmi_comm_failure_reaches_every_rank():
    """include/reacher_comm.h rd_xcomm_*: two gloo ranks build dist.XgmiComm on a host
    without a HIP device: neither can export a buffer, the all-gather of the handles carries
    that, and both raise NativeError naming the ranks -- no rank left waiting."""
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_xcomm_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    assert out[0][0] == out[1][0] == "NativeError"
    assert "[0, 1] could not export" in out[0][1] and "[0, 1] could not export" in out[1][1]


def test_xgmi_map_failure_reaches_every_rank():
    """Rank 1 cannot map rank 0's exchange buffer (injected): the group agrees on the
    outcome, both ranks raise, and rank 0's message names rank 1."""
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_xcomm_rank, args=(2, _free_port(), out, "rank1_map"), nprocs=2, join=True,
                       start_method="spawn")
    assert out[0][0] == out[1][0] == "NativeError"
    assert "[1] could not map" in out[0][1] and "injected map failure" in out[1][1]


def test_xgmi_comm_host_contract():
    """rd_xcomm_* argument errors and a buffer on a missing device fail with a message."""
    import ctypes

    from reacherdistilation_amd import _native as nat
    lib = nat.load()
    h, hb = ctypes.c_void_p(), (ctypes.c_uint8 * 64)()
    assert lib.rd_xcomm_create(ctypes.byref(h), 9, 0, 0, 5060, 60.0, hb) != 0     # more than 8 ranks
    assert b"bad argument" in lib.rd_last_error()
    assert lib.rd_xcomm_create(ctypes.byref(h), 2, 2, 0, 5060, 60.0, hb) != 0     # rank out of range
    assert lib.rd_xcomm_create(ctypes.byref(h), 2, 0, 0, 0, 60.0, hb) != 0        # no capacity
    assert lib.rd_xcomm_connect(None, hb) != 0 and lib.rd_comm_check(None) != 0
    if not torch.cuda.is_available():
        assert lib.rd_xcomm_create(ctypes.byref(h), 1, 0, 0, 5060, 60.0, hb) != 0  # no HIP device here
        assert lib.rd_last_error()

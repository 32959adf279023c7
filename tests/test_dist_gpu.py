"""Two ranks on one MI355X (gloo carries the gradient all-reduce; RCCL needs one GPU per
rank): DistillTrainer's multi-rank step (rdd_rollout -> all_reduce(SUM) -> rdd_apply) over
a sharded env batch reproduces the single-rank run over the whole batch.  Tolerance: the
student after 5 Adam steps within 1e-5 (f32 gradient summation order differs: the kernel's
per-workgroup partials vs two shard sums); the ranks' students bitwise identical."""
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

    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = DistillTrainer(DistillConfig(n_envs_global=N_GLOBAL, seed=7, lr=1e-3), device="cuda:0",
                        rank=rank, world_size=world)
    for _ in range(STEPS):
        tr.step()
    out[rank] = (tr.student_params().cpu().numpy(), tr.env_state().cpu().numpy(), tr.metrics(STEPS))
    tr.close()
    dist.destroy_process_group()


def test_two_ranks_match_single_rank():
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_rank, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
    ref = DistillTrainer(DistillConfig(n_envs=N_GLOBAL, seed=7, lr=1e-3), device="cuda:0")
    for _ in range(STEPS):
        ref.step()
    p_ref, st_ref, m_ref = ref.student_params().cpu().numpy(), ref.env_state().cpu().numpy(), ref.metrics(STEPS)
    (p0, st0, m0), (p1, st1, m1) = out[0], out[1]
    assert np.array_equal(p0, p1)
    np.testing.assert_allclose(p0, p_ref, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([st0, st1], axis=1), st_ref, atol=1e-4)
    np.testing.assert_allclose(m0[:, 3] + m1[:, 3], m_ref[:, 3])
    np.testing.assert_allclose(m0[:, 1] + m1[:, 1], m_ref[:, 1], rtol=1e-4)


class _Comm1:
    """A one-rank native RCCL communicator (include/reacher_comm.h) without a process group."""

    def __init__(self):
        import ctypes

        from reacherdistilation_amd import _native as nat
        self._lib = nat.load()
        idb = (ctypes.c_uint8 * 128)()
        nat.check(self._lib.rd_comm_unique_id(idb), "rd_comm_unique_id")
        h = ctypes.c_void_p()
        nat.check(self._lib.rd_comm_create(ctypes.byref(h), idb, 1, 0, 0, 60.0), "rd_comm_create")
        self.handle, self.world, self.rank, self.device = h, 1, 0, torch.device("cuda:0")

    def close(self):
        self._lib.rd_comm_destroy(self.handle)


def test_native_rccl_allreduce_one_rank():
    """rd_comm_allreduce_f32 over one rank is the identity, on the caller's stream."""
    import ctypes

    from reacherdistilation_amd import _native as nat
    c = _Comm1()
    try:
        assert c._lib.rd_comm_nranks(c.handle) == 1
        x = torch.randn(5060, device="cuda:0")
        want = x.clone()
        nat.check(c._lib.rd_comm_allreduce_f32(c.handle, ctypes.c_void_p(x.data_ptr()), x.numel(),
                                               nat.stream_handle(x.device)), "allreduce")
        torch.cuda.synchronize()
        assert torch.equal(x, want)
        assert c._lib.rd_comm_allreduce_f32(c.handle, None, 4, None) != 0   # bad argument -> error
        # RCCL's own view of the communicator (ncclCommCount / UserRank / CuDevice)
        cnt, r, d, f = (ctypes.c_int() for _ in range(4))
        nat.check(c._lib.rd_comm_query(c.handle, ctypes.byref(cnt), ctypes.byref(r), ctypes.byref(d),
                                       ctypes.byref(f)), "rd_comm_query")
        assert (cnt.value, r.value, d.value, f.value) == (1, 0, 0, 1)
    finally:
        c.close()


@pytest.mark.parametrize("accum", [1, 3])
def test_bound_comm_step_is_bitwise_the_single_rank_step(accum):
    """With a communicator bound, rdd_step = rollout, reduce, RCCL all-reduce, Adam on the
    trainer's stream; over one rank that is bitwise the fused single-rank step (and the
    staged accumulation path with rdd_allreduce_grad likewise)."""
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    cfg = DistillConfig(n_envs=20000, seed=3, lr=1e-3, accum_steps=accum)
    c = _Comm1()
    try:
        a = DistillTrainer(cfg, device="cuda:0")
        b = DistillTrainer(cfg, device="cuda:0", comm=c)
        for _ in range(4 * accum):
            a.step()
            b.step()
        assert torch.equal(a.student_params(), b.student_params())
        assert torch.equal(a.env_state(), b.env_state())
        assert np.array_equal(a.metrics(4), b.metrics(4))
        a.close()
        b.close()
    finally:
        c.close()


def _rccl_rank(rank, world, port, out):
    import torch.distributed as dist

    from reacherdistilation_amd.dist import RcclComm
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    comm = RcclComm(dev, timeout=60.0)
    assert comm.self_check()
    q = comm.query()
    assert (q["count"], q["user_rank"], q["device"], q["from_rccl"]) == (world, rank, rank, True), q
    tr = DistillTrainer(DistillConfig(n_envs_global=N_GLOBAL, seed=7, lr=1e-3), device=dev,
                        rank=rank, world_size=world, comm=comm)
    for _ in range(STEPS):
        tr.step()
    out[rank] = (tr.student_params().cpu().numpy(), tr.env_state().cpu().numpy(), tr.metrics(STEPS),
                 tr.replicas_identical())
    tr.close()
    comm.close()
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two HIP devices (one per rank)")
def test_two_devices_native_rccl_match_single_rank():
    """Two ranks on two devices, the native RCCL communicator bound (the multi-GPU bench's
    path): the same student as one rank over the whole batch (within f32 summation order),
    bitwise-identical replicas."""
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    out = mp.get_context("spawn").Manager().dict()
    mp.start_processes(_rccl_rank, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
    ref = DistillTrainer(DistillConfig(n_envs=N_GLOBAL, seed=7, lr=1e-3), device="cuda:0")
    for _ in range(STEPS):
        ref.step()
    p_ref, st_ref = ref.student_params().cpu().numpy(), ref.env_state().cpu().numpy()
    (p0, st0, m0, same0), (p1, st1, m1, same1) = out[0], out[1]
    assert same0 and same1 and np.array_equal(p0, p1)
    np.testing.assert_allclose(p0, p_ref, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([st0, st1], axis=1), st_ref, atol=1e-4)
    np.testing.assert_allclose(m0[:, 3] + m1[:, 3], ref.metrics(STEPS)[:, 3])

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

"""A/B of two builds on the same steps: writes the student parameters and the last gradient
after a few fused steps of several configs to an .npz (the build is chosen with RD_LIB), so
two runs can be compared bit for bit.
usage: RD_LIB=libreacher_x.so python scripts/bitwise_ab.py out.npz  (GPU)
       python scripts/bitwise_ab.py --compare a.npz b.npz"""
import os
import sys

import numpy as np

CASES = {   # name: DistillConfig overrides
    "c2": dict(n_envs=4096),
    "c2_g16": dict(n_envs=4096, group_envs=16),   # the plain layout at c2 (auto picks helper pairs)
    "c2_exact": dict(n_envs=4096, f32_split=False),
    "small_777": dict(n_envs=777, loss="kl"),
    "c4": dict(n_envs=262144),
    "c5": dict(n_envs=131072, act_with="student", student_dtype="bf16"),
    "ragged_5003": dict(n_envs=5003, loss="kl"),
    "grid7_kl": dict(n_envs=3000, loss="kl", grid=7),
    "grid300": dict(n_envs=300 * 4 * 64, grid=300),
    "accum3": dict(n_envs=20000, accum_steps=3),
    "c3_exact": dict(n_envs=65536, loss="kl", f32_split=False),
    "c5_exact": dict(n_envs=131072, act_with="student", student_dtype="bf16", f32_split=False),
}


def run(out):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from reacherdistilation_amd.distill import DistillConfig, DistillTrainer
    res = {}
    for name, kw in CASES.items():
        cfg = dict(loss="mse", f32_split=True, seed=3)
        cfg.update(kw)
        tr = DistillTrainer(DistillConfig(**cfg), device="cuda:0")
        for _ in range(6):
            tr.step()
        torch.cuda.synchronize()
        res[name + "_params"] = tr.student_params().cpu().numpy()
        res[name + "_grad"] = tr.grad().cpu().numpy()
        res[name + "_state"] = tr.env_state().cpu().numpy()
        tr.close()
    np.savez(out, **res)
    print("wrote", out, flush=True)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        d = float(np.abs(A[k] - B[k]).max())
        print(f"{k:24s} bitwise_equal={same} max_abs_diff={d:.3g}")
        bad += not same
    print("ALL BITWISE EQUAL" if not bad else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    run(sys.argv[1])

"""Which action stepped the envs of a non-reproducible rollout?  For each env whose state
differs between two identical rollouts, step its pre-step state with the actions of every env
in its 64-env group (C f32 oracle) and report which env's action matches each run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_c  # noqa: E402
from reacherdistilation_amd.distill import DistillConfig, DistillTrainer  # noqa: E402

ref_c.build()
kw = dict(n_envs=262144, f32_split=True)


def roll():
    tr = DistillTrainer(DistillConfig(seed=5, **kw), device="cuda:0")
    s0 = tr.env_state().clone()
    # teacher actions (exact forward) from the pre-step observations
    from tests.test_distill_gpu import _obs_from_state
    ob = torch.tensor(_obs_from_state(s0.cpu().numpy()), dtype=torch.float32)
    t, _ = tr.forward(ob)
    tr.rollout()
    s1 = tr.env_state().clone()
    tr.close()
    return s0.cpu().numpy(), s1.cpu().numpy(), t.cpu().numpy()[:, :2]


a = roll()
for rep in range(6):
    b = roll()
    bad = np.flatnonzero((a[1] != b[1]).any(0))
    if not len(bad):
        print("rep", rep, "identical")
        continue
    print("rep", rep, "bad", len(bad), bad[:4], "...")
    s0, acts = a[0], a[2]
    for e in bad[:16:5]:
        gbase = e - e % 64
        cands = np.arange(gbase - 64, gbase + 128)
        st = np.repeat(s0[:, e:e + 1].astype(np.float64), len(cands), axis=1).copy()
        ref_c.step(st, acts[cands].astype(np.float32), np.float64)
        for name, run in (("a", a[1]), ("b", b[1])):
            d = np.abs(st[[0, 1, 2, 3]] - run[[0, 1, 2, 3], e:e + 1]).max(0)
            k = int(np.argmin(d))
            print(f"   env {e} (group {e // 64} row {e % 64}): run {name} matches action of env {cands[k]} "
                  f"(row {cands[k] % 64}, group {cands[k] // 64}) err {d[k]:.2e}")

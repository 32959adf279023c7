"""Diagnosis of the K-step launch's gradient (one process): staged vs fused at a size, and
repeated fused launches' digests.  RD_LIB selects the build."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from reacherdistilation_amd.distill import DistillConfig, DistillTrainer


def tr(n, K, **kw):
    return DistillTrainer(DistillConfig(n_envs=n, seed=5, accum_steps=K, **kw), device="cuda:0")


def region(p):
    edges = [(0, "W1"), (704, "b1"), (768, "W2"), (4864, "b2"), (4928, "W3"), (5056, "b3"), (5058, "ls")]
    name = "W1"
    for e, nm in edges:
        if p >= e:
            name = nm
    return name


def main():
    n, K = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    kw = dict(loss="mse", f32_split=True)
    b = tr(n, K, **kw)
    for k in range(K):
        b.launch(b.STAGE_ROLLOUT)
        b.launch(b.STAGE_REDUCE_ACCUM if k else b.STAGE_REDUCE)
    gb = b.grad().double().cpu().numpy()
    out = {"lib": os.environ.get("RD_LIB", "libreacher.so"), "n": n, "K": K, "runs": []}
    first = None
    for r in range(reps):
        a = tr(n, K, **kw)
        a.rollout_accum()
        ga = a.grad().double().cpu().numpy()
        d = np.abs(ga - gb)
        bad = np.nonzero(d > 1e-6 * np.abs(gb).max())[0]
        rec = {"rep": r, "digest": hashlib.sha1(a.grad().cpu().numpy().tobytes()).hexdigest()[:12],
               "state_equal": bool(torch.equal(a.env_state(), b.env_state())),
               "glob": float(d.max() / np.abs(gb).max()), "nbad": int(bad.size),
               "bad_regions": sorted({region(int(p)) for p in bad}),
               "bad_first": [int(p) for p in bad[:12]]}
        if first is None:
            first = ga
        else:
            dd = np.nonzero(ga != first)[0]
            rec["vs_first_n"] = int(dd.size)
            rec["vs_first_idx"] = [int(p) for p in dd[:12]]
        out["runs"].append(rec)
        a.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

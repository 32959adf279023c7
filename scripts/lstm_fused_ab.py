#!/usr/bin/env python3
"""A/B of the LSTM student's fused recurrence (diagnostic).  Run once per library build
(RD_LIB=libreacher.so / libreacher_lstm_unfused.so): writes the forward outputs, final
state and one rollout's gradient at each size to gpurun_out/lstm_ab_<tag>.npz and prints the
training-step time; `--compare A B` checks the two .npz files bitwise.
usage: python scripts/lstm_fused_ab.py TAG [B ...] | --compare TAG_A TAG_B"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def run(tag, sizes):
    import torch
    sys.path.insert(0, ROOT)
    from reacherdistilation_amd.student_lstm import StudentLstmConfig, StudentLstmTrainer
    T, res = 10, {}
    for B in sizes:
        g = torch.Generator().manual_seed(B)
        ob = (torch.rand(T, B, 11, generator=g) * 2 - 1).cuda()
        prev = (torch.rand(T, B, 4, generator=g) - 0.5).cuda()
        tgt = (torch.rand(T, B, 4, generator=g) - 0.5).cuda()
        st = (torch.rand(2, B, 200, generator=g) - 0.5).cuda()
        tr = StudentLstmTrainer(StudentLstmConfig(loss="kl", steps=T, max_windows=B), device="cuda:0")
        y, fin = tr.forward(ob, prev, st)
        res[f"y{B}"] = y.cpu().numpy()
        res[f"c{B}"] = fin[0].cpu().numpy()
        res[f"h{B}"] = fin[1].cpu().numpy()
        res[f"g{B}"] = tr.rollout(ob, prev, tgt, st).cpu().numpy().copy()
        tr.apply()
        for _ in range(3):
            tr.step(ob, prev, tgt)
        iters = max(5, min(50, int(5e5 // (B * T + 1000))))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            tr.step(ob, prev, tgt)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / iters * 1e3
        print(json.dumps({"tag": tag, "windows": B, "step_ms": ms}), flush=True)
        tr.close()
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"lstm_ab_{tag}.npz"), **res)


def compare(a, b):
    x = np.load(os.path.join(OUT, f"lstm_ab_{a}.npz"))
    y = np.load(os.path.join(OUT, f"lstm_ab_{b}.npz"))
    ok = True
    for k in sorted(x.files):
        same = np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32))
        d = float(np.abs(x[k].astype(np.float64) - y[k]).max())
        print(json.dumps({"array": k, "bitwise_equal": same, "max_abs_diff": d}))
        ok &= same
    print(json.dumps({"all_bitwise_equal": ok}))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], [int(s) for s in sys.argv[2:]] or [20, 1024, 16384])

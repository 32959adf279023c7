"""Throughput of the reference student's training step (csrc/student_mlp.hip) vs batch rows.

Prints one JSON line per size: rows/s of rdm_step (train kernel + reduce/Adam), the train
kernel's MFMA-bound roofline fraction (algorithmic f32 flops of the unpadded graph) and
forward-only rows/s.
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from reacherdistilation_amd.student_mlp import StudentMlpConfig, StudentMlpTrainer  # noqa: E402

DIMS = (16, 24, 128, 128, 32, 4)
MACS = sum(a * b for a, b in zip(DIMS[:-1], DIMS[1:]))          # 24,192 per row per pass
FLOP_TRAIN = 2 * MACS * 3 - 2 * DIMS[0] * DIMS[1]                 # fwd + dgrad (not layer 0) + wgrad
PEAK_F32_MFMA = 157.3e12


def timeit(fn, iters, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def cpu_baseline(n=200, seconds=3.0):
    """The oracle (numpy f64, one core) doing the same training step on n rows."""
    import threadpoolctl
    import numpy as np

    from oracle import policy_np as pn
    from oracle import refnet_np as rn
    rs = np.random.RandomState(0)
    x = rs.uniform(-1, 1, (n, 16))
    t = np.concatenate([rs.uniform(-.5, .5, (n, 2)), rs.uniform(-1, -.2, (n, 2))], 1)
    p = rn.init(2).astype(np.float32)
    opt = pn.AdamTF1(rn.P_REF)
    with threadpoolctl.threadpool_limits(1):
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            fw = rn.forward(p, x)
            _, d, _ = rn.loss_and_dout(fw["pdflat"], t, "kl", n)
            p = opt.step(p, rn.backward(p, fw, d))
            k += 1
        el = time.perf_counter() - t0
    return {"cpu_rows_per_s": n * k / el, "cpu_step_us": el / k * 1e6, "cpu_rows": n, "cpu_cores": 1,
            "cpu_kind": "oracle/refnet_np.py (numpy f64)"}


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [200, 4096, 65536, 262144, 1048576]
    if not sys.argv[1:]:
        print(json.dumps(cpu_baseline()), flush=True)
    tr = StudentMlpTrainer(StudentMlpConfig(loss="kl"), device="cuda:0")
    for n in sizes:
        x = torch.rand(n, 16, device="cuda:0") * 2 - 1
        t = torch.rand(n, 4, device="cuda:0") - 0.5
        iters = max(5, min(200, int(2e8 // (n * 100 + 1e5))))
        ts = timeit(lambda: tr.step(x, t), iters)
        gstep = tr.graph_step(n)
        tg = timeit(lambda: gstep(x, t), iters)
        tf = timeit(lambda: tr.forward(x), iters)
        print(json.dumps({"rows": n, "step_us": ts * 1e6, "rows_per_s": n / ts, "graph_step_us": tg * 1e6, "fwd_us": tf * 1e6,
                          "fwd_rows_per_s": n / tf, "tflops": FLOP_TRAIN * n / ts / 1e12,
                          "mfma_frac_step": FLOP_TRAIN * n / ts / PEAK_F32_MFMA}), flush=True)


if __name__ == "__main__":
    main()

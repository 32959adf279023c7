"""Throughput of the LSTM student's truncated-BPTT training step (csrc/student_lstm.hip) vs
windows per step (T = 10).  One JSON line per size: window-steps/s, MFMA f32 fraction of the
algorithmic FLOPs (1,337,472 per window-step: forward 451,776 + data grads 433,920 + weight
grads 451,776), forward-only rate."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from reacherdistilation_amd.student_lstm import StudentLstmConfig, StudentLstmTrainer  # noqa: E402

T = 10
FWD = 2 * (243 * 800 + 4 * 32 + 200 * 64 + 64 * 128 + 128 * 64 + 64 * 32 + 32 * 4)
DGRAD = 2 * (800 * (200 + 32) + 4 * 32 + 32 * 64 + 64 * 128 + 128 * 64 + 64 * 200)
FLOP = 2 * FWD + DGRAD
PEAK = 157.3e12


def timeit(fn, iters, warm=3):
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


def cpu_baseline(B=20, seconds=3.0):
    """The oracle (numpy f64, one core): the same truncated-BPTT step on [T, B] windows."""
    import threadpoolctl
    import numpy as np

    from oracle import lstm_np as ln
    from oracle import policy_np as pn
    rs = np.random.RandomState(0)
    ob, prev = rs.uniform(-1, 1, (T, B, 11)), rs.uniform(-1, 0, (T, B, 4))
    tgt = np.concatenate([rs.uniform(-.5, .5, (T, B, 2)), rs.uniform(-1, -.2, (T, B, 2))], 2)
    p = ln.init(3)
    opt = pn.AdamTF1(ln.P_LSTM, lr=1e-3)
    with threadpoolctl.threadpool_limits(1):
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            fw = ln.forward(p, ob, prev)
            _, d, _ = ln.loss_and_dout(fw["pdflat"], tgt, "kl", T * B)
            p = opt.step(p, ln.backward(p, fw, d))
            k += 1
        el = time.perf_counter() - t0
    return {"cpu_window_steps_per_s": B * T * k / el, "cpu_step_ms": el / k * 1e3, "cpu_windows": B,
            "cpu_cores": 1, "cpu_kind": "oracle/lstm_np.py (numpy f64)"}


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [20, 1024, 16384]
    if not sys.argv[1:]:
        print(json.dumps(cpu_baseline()), flush=True)
    for B in sizes:
        tr = StudentLstmTrainer(StudentLstmConfig(loss="kl", steps=T, max_windows=B), device="cuda:0")
        ob = torch.rand(T, B, 11, device="cuda:0") * 2 - 1
        prev = torch.rand(T, B, 4, device="cuda:0") - 0.5
        tgt = torch.rand(T, B, 4, device="cuda:0") - 0.5
        iters = max(3, min(50, int(5e5 // (B * T + 1000))))
        ts = timeit(lambda: tr.step(ob, prev, tgt), iters)
        gstep = tr.graph_step(B)
        tg = timeit(lambda: gstep(ob, prev, tgt), iters)
        tf = timeit(lambda: tr.forward(ob, prev), iters)
        print(json.dumps({"windows": B, "T": T, "step_ms": ts * 1e3, "window_steps_per_s": B * T / ts,
                          "graph_step_ms": tg * 1e3,
                          "fwd_ms": tf * 1e3, "tflops": FLOP * B * T / ts / 1e12,
                          "mfma_frac": FLOP * B * T / ts / PEAK}), flush=True)
        tr.close()


if __name__ == "__main__":
    main()

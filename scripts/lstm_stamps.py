"""Phase stamps of the LSTM student's 20-window training step (diagnostic build
libreacher_lstmst.so: profiles/r05l_lstm_stamps_50wg.diff applied, -DRDL_STAMPS).  Workgroup 0's
s_memrealtime (100 MHz) at the phases of lstm_fwd_persist_kernel (0) and lstm_bptt_persist_kernel
(1) of the last of N steps; prints one JSON line.

  RD_LIB=libreacher_lstmst.so python scripts/lstm_stamps.py [windows] [steps]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    import numpy as np
    import torch

    from reacherdistilation_amd import _native as nat
    from reacherdistilation_amd.student_lstm import StudentLstmConfig, StudentLstmTrainer
    T = 10
    dev = torch.device("cuda", 0)
    tr = StudentLstmTrainer(StudentLstmConfig(loss="kl", steps=T, max_windows=B), device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    ob = torch.randn(T, B, 11, generator=g).to(dev)
    prev = torch.randn(T, B, 4, generator=g).to(dev) * 0.1
    tgt = torch.randn(T, B, 4, generator=g).to(dev) * 0.1
    lib = nat.load()
    rd = lib.rdl_read_stamps
    rd.restype, rd.argtypes = ctypes.c_int, [ctypes.c_void_p]
    for _ in range(n):
        tr.step(ob, prev, tgt)
    torch.cuda.synchronize(dev)
    st = np.zeros((8, 64), dtype=np.uint64)
    assert rd(st.ctypes.data) == 0
    us = lambda a, b: round(float(int(b) - int(a)) / 100.0, 3)   # 100 MHz ticks -> us
    f, bp = st[0], st[1]
    out = {"windows": B, "T": T, "steps": n,
           "fwd": {"prologue_and_inputs0": us(f[0], f[1]),
                   "steps": [{"wait_h": us(f[1] if s == 0 else f[5 + 4 * (s - 1)], f[2 + 4 * s]),
                              "mfma": us(f[2 + 4 * s], f[3 + 4 * s]), "cell": us(f[3 + 4 * s], f[4 + 4 * s]),
                              "inputs_next": us(f[4 + 4 * s], f[5 + 4 * s])} for s in range(T)],
                   "total": us(f[0], f[5 + 4 * (T - 1)])},
           "bptt": {"start_after_fwd_start": us(f[0], bp[0]), "prologue": us(bp[0], bp[1]),
                    "steps": [{"dh_in": us(bp[1] if j == 0 else bp[6 + 5 * (j - 1)], bp[2 + 5 * j]),
                               "cell_and_loads": us(bp[2 + 5 * j], bp[3 + 5 * j]),
                               "mfma_store": us(bp[3 + 5 * j], bp[4 + 5 * j]),
                               "arrive_dwl": us(bp[4 + 5 * j], bp[5 + 5 * j]),
                               "wait": us(bp[5 + 5 * j], bp[6 + 5 * j])} for j in range(T - 1)],
                    "last_cell": us(bp[6 + 5 * (T - 2)], bp[60])}}
    print(json.dumps(out), flush=True)
    tr.close()


if __name__ == "__main__":
    main()

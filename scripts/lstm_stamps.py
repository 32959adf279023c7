"""Phase stamps of the LSTM student's 20-window training step (diagnostic build
libreacher_lstmst.so: profiles/r05l_lstm_stamps.diff applied, -DRDL_STAMPS).  Workgroup 0's
s_memrealtime (100 MHz) at the phases of lstm_fwd_persist_kernel (0), lstm_bptt_persist_kernel
(1), head_bwd_kernel (2) and head_fwd_kernel (3) of the last of N steps; prints one JSON line.

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
    f, bp, hb, hf = st[0], st[1], st[2], st[3]
    t0 = int(f[0])
    out = {"windows": B, "T": T, "steps": n,
           "fwd": {"prologue": us(f[0], f[1]),
                   "steps": [{"wait_h": us(f[1] if s == 0 else f[4 + 3 * (s - 1)], f[2 + 3 * s]),
                              "mfma": us(f[2 + 3 * s], f[3 + 3 * s]), "cell": us(f[3 + 3 * s], f[4 + 3 * s])}
                             for s in range(T)],
                   "total": us(f[0], f[4 + 3 * (T - 1)]),
                   "shader_clock_ghz": round((int(st[4][1]) - int(st[4][0])) / (float(int(f[4 + 3 * (T - 1)]) - int(f[0])) * 10.0), 3)},
           "head_fwd": {"start_after_fwd_start": us(t0, hf[0]), "stage": us(hf[0], hf[1]),
                        "layers": [us(hf[k], hf[k + 1]) for k in range(1, 6)], "total": us(hf[0], hf[6])},
           "head_bwd": {"start_after_fwd_start": us(t0, hb[0]), "stage": us(hb[0], hb[1]),
                        "dgrad": [us(hb[k], hb[k + 1]) for k in range(1, 6)], "wgrad_issue": us(hb[6], hb[7]),
                        "wgrad_drain": us(hb[7], hb[8]), "total": us(hb[0], hb[8])},
           "bptt": {"start_after_fwd_start": us(t0, bp[0]), "prologue": us(bp[0], bp[1]),
                    "steps": [{"dh_in": us(bp[1] if j == 0 else bp[4 + 4 * (j - 1)], bp[2 + 4 * j]),
                               "cell": us(bp[2 + 4 * j], bp[3 + 4 * j]), "mfma_store": us(bp[3 + 4 * j], bp[4 + 4 * j])}
                              for j in range(T - 1)],
                    "last_cell_and_sums": us(bp[4 + 4 * (T - 2)], bp[60]),
                    "total_to_sums": us(bp[0], bp[60])}}
    if int(st[5][0]):   # the cell-split build (profiles/r05l_lstm_stamps.diff, second part)
        c5 = st[5]
        out["fwd_cell_split"] = [{"z_to_h": us(c5[6 * s], c5[6 * s + 1]), "stores": us(c5[6 * s + 1], c5[6 * s + 2]),
                                  "q1_z_to_h": us(c5[6 * s + 3], c5[6 * s + 4]) if int(c5[6 * s + 3]) else None,
                                  "q1_stores": us(c5[6 * s + 4], c5[6 * s + 5]) if int(c5[6 * s + 3]) else None,
                                  "after_mfma_to_z": us(f[3 + 3 * s], c5[6 * s]),
                                  "tail": us(c5[6 * s + 5] if int(c5[6 * s + 3]) else c5[6 * s + 2], f[4 + 3 * s])}
                                 for s in range(T)]
    print(json.dumps(out), flush=True)
    tr.close()


if __name__ == "__main__":
    main()

"""Phase stamps of head_bwd_kernel<false, 16> (workgroup 0, last of N 20-window steps) in the
diagnostic build libreacher_lstmst.so (profiles/r05p_lstm_head_stamps.diff, -DRDL_STAMPS).

  RD_LIB=libreacher_lstmst.so python scripts/lstm_stamps_head.py [windows] [steps]
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
    us = lambda a, b: round(float(int(b) - int(a)) / 100.0, 3)
    h = st[2]
    print(json.dumps({"windows": B, "stage": us(h[0], h[1]), "dgrad": [us(h[k], h[k + 1]) for k in range(1, 6)],
                      "wgrad_issue": us(h[6], h[7]), "wgrad_drain": us(h[7], h[8]), "total": us(h[0], h[8])}))
    tr.close()


if __name__ == "__main__":
    main()

"""Phase stamps of the PPO minibatch tile kernel (diagnostic build libreacher_ppost.so:
profiles/r05x_ppo_stamps.diff applied, -DRDP_STAMPS).  Workgroups 0-3's s_memrealtime (100 MHz)
at the phases of their first tile in the last minibatch of one iteration; one JSON line.

  RD_LIB=libreacher_ppost.so python scripts/ppo_stamps.py [minibatch]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["params", "gather", "layers1-2", "-", "loss", "head_bwd", "l2_bwd+dW2", "dW1", "writes", "stats"]


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    import numpy as np
    import torch

    from reacherdistilation_amd import _native as nat
    from reacherdistilation_amd.ppo import PPOConfig, PPOTrainer
    tr = PPOTrainer(PPOConfig(n_envs=4096, horizon=50, optim_batchsize=mb, optim_epochs=1 if mb < 1024 else 10,
                              max_timesteps=10 ** 8), device="cuda:0")
    lib = nat.load()
    rd = lib.rdp_read_stamps
    rd.restype, rd.argtypes = ctypes.c_int, [ctypes.c_void_p]
    tr.iterate()
    torch.cuda.synchronize()
    st = np.zeros((4, 16), dtype=np.uint64)
    assert rd(st.ctypes.data) == 0
    out = {"minibatch": mb}
    for w in range(4 if mb >= 128 else mb // 32):
        s = st[w]
        out[f"wg{w}"] = {PHASES[k]: round((int(s[k + 1]) - int(s[k])) / 100.0, 2) for k in range(10)}
        out[f"wg{w}"]["total_us"] = round((int(s[10]) - int(s[0])) / 100.0, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Micro-benchmark of the standalone env kernel (rd_step) at several N; HIP-event timing on
the stream the kernel is launched on (torch's current stream)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.env import BatchedReacher  # noqa: E402

BYTES_PER_ENV_STEP = 113  # read 40 + write 73


def run(n, iters=200):
    env = BatchedReacher(n, seed=0, device="cuda:0")
    env.reset()
    a = (torch.rand(n, 2, device="cuda:0") * 2 - 1).contiguous()
    for _ in range(20):
        env.step(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        env.step(a)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return dict(n=n, us_per_step=ms * 1e3, env_steps_per_s=n / (ms * 1e-3),
                gbps=BYTES_PER_ENV_STEP * n / (ms * 1e-3) / 1e9)


if __name__ == "__main__":
    for n in [int(x) for x in (sys.argv[1:] or ["4096", "65536", "262144", "1048576", "4194304"])]:
        print(json.dumps(run(n)), flush=True)

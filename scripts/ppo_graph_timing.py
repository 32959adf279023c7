"""(Record of a rejected variant, r04z: needs that build's PPOTrainer.set_graph.) PPO iteration time with the optimize phase's minibatch loop replayed from its graph vs
launched kernel by kernel (default PPOConfig and the DESIGN table's 4,096 x 50 config)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from reacherdistilation_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402


def run(cfg, graph, iters=10, warm=2):
    t = PPOTrainer(cfg)
    t.set_graph(graph)
    for _ in range(warm):
        t.iterate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        t.iterate()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    S = cfg.n_envs * cfg.horizon
    t.close()
    return {"ms_per_iteration": round(ms, 2), "env_steps_per_s": S / ms * 1e3}


for name, cfg in (("default_2048x32_mb4096", PPOConfig()),
                  ("design_4096x50_mb4096", PPOConfig(n_envs=4096, horizon=50, optim_batchsize=4096))):
    out = {"config": name, "graph": run(cfg, True), "launched": run(cfg, False)}
    print(json.dumps(out), flush=True)

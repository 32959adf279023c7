"""PPO teacher training throughput (csrc/ppo.hip): env steps per second of whole iterations
(rollout + GAE + filter + 10 epochs of minibatch Adam), and the learning curve."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from reacherdistilation_amd.ppo import METRICS, PPOConfig, PPOTrainer  # noqa: E402


def main():
    n, T, mb, iters = 4096, 50, 4096, 40
    tr = PPOTrainer(PPOConfig(n_envs=n, horizon=T, optim_batchsize=mb, max_timesteps=n * T * iters), device="cuda:0")
    tr.iterate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters - 1):
        tr.iterate()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = tr.metrics(iters)
    print(json.dumps({"n_envs": n, "horizon": T, "minibatch": mb, "iter_ms": dt * 1e3 / (iters - 1),
                      "env_steps_per_s": n * T * (iters - 1) / dt,
                      "ep_ret_mean_first": m[0, 0], "ep_ret_mean_last": m[-1, 0],
                      "curve": [round(float(x), 3) for x in m[:, 0]]}), flush=True)
    print(json.dumps(dict(zip(METRICS, map(float, m[-1])))), flush=True)


if __name__ == "__main__":
    main()

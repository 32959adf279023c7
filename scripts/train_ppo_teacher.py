"""Train the distillation teacher by PPO: the reference's
teacher.train (teacher.py:23-37, baselines ppo1 pposgd_simple.learn) with its hyperparameters --
timesteps_per_actorbatch 2048 (here n_envs x horizon), optim_batchsize 64, optim_epochs 10,
optim_stepsize 3e-4, schedule 'linear' over max_timesteps, gamma 0.99, lam 0.95, clip 0.2,
entcoeff 0 -- on csrc/ppo.hip, then evaluate the trained policy's MEAN action (the way the
reference's collect_reward steps it, teacher.py:39-62) on fresh episodes: the mean 50-step
return against the reference teacher's -7.53 on the fixture.  Writes the curve
and the result as JSON, and the policy as the reference Saver's scope-'pi' TF checkpoint.

  python scripts/train_ppo_teacher.py --timesteps 1000000 --n-envs 16 --horizon 128 --out X.json --ckpt PREFIX
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reacherdistilation_amd.ppo import METRICS, PPOConfig, PPOTrainer  # noqa: E402

REF_TEACHER_RETURN = -7.53   # the fixture's 21 teacher-stepped episodes


def evaluate(teacher, episodes, seed, dev):
    from reacherdistilation_amd.teacher import episode_returns
    return episode_returns(teacher, episodes, seed, dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timesteps", type=int, default=1_000_000)
    ap.add_argument("--n-envs", type=int, default=16)
    ap.add_argument("--horizon", type=int, default=128)
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--eval-every", type=int, default=0, help="iterations between evaluations (0: ~20 per run)")
    ap.add_argument("--eval-episodes", type=int, default=1024)
    ap.add_argument("--out", required=True)
    ap.add_argument("--ckpt", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = PPOConfig(n_envs=a.n_envs, horizon=a.horizon, seed=a.seed, optim_batchsize=a.mb, optim_epochs=a.epochs,
                    optim_stepsize=a.lr, max_timesteps=a.timesteps)
    tr = PPOTrainer(cfg, device=dev)
    iters = -(-a.timesteps // tr.S)
    every = a.eval_every or max(1, iters // 20)
    curve, evals = [], []
    t0 = time.perf_counter()
    train_s = 0.0
    for it in range(1, iters + 1):
        t1 = time.perf_counter()
        tr.iterate()
        train_s += time.perf_counter() - t1
        m = tr.metrics(1)[0]
        curve.append([int(m[7]), round(float(m[0]), 4)])
        if it % every == 0 or it == iters:
            r = evaluate(tr.teacher(), a.eval_episodes, 10_000 + it, dev)
            evals.append({"iteration": it, "timesteps": int(m[7]), "train_ep_ret_mean": float(m[0]),
                          "eval_return_mean": float(r.mean()), "eval_return_std": float(r.std())})
            print(json.dumps(evals[-1]), flush=True)
    teacher = tr.teacher()
    r = evaluate(teacher, 4096, 123_456, dev)
    out = {"config": {"n_envs": a.n_envs, "horizon": a.horizon, "actor_batch": tr.S, "optim_batchsize": a.mb,
                      "optim_epochs": a.epochs, "optim_stepsize": a.lr, "schedule": "linear",
                      "max_timesteps": a.timesteps, "gamma": cfg.gamma, "lam": cfg.lam, "clip_param": cfg.clip_param,
                      "entcoeff": cfg.entcoeff, "adam_epsilon": 1e-5, "seed": a.seed,
                      "reference": "teacher.py:30-36 (timesteps_per_actorbatch 2048, optim_batchsize 64, "
                                   "optim_epochs 10, optim_stepsize 3e-4, linear; num_timesteps 1e6 = "
                                   "mujoco_arg_parser's default)"},
           "iterations": iters, "train_seconds": train_s, "wall_seconds": time.perf_counter() - t0,
           "env_steps_per_s_training": iters * tr.S / train_s,
           "curve_train_ep_ret_mean": curve[:: max(1, len(curve) // 200)] + [curve[-1]],
           "evals": evals,
           "final": {"episodes": 4096, "eval": "policy mean action, fresh gym-seeded envs (seed 123456 + i)",
                     "return_mean": float(r.mean()), "return_std": float(r.std()),
                     "return_p10_p50_p90": [float(x) for x in np.percentile(r, [10, 50, 90])],
                     "reference_teacher_return": REF_TEACHER_RETURN,
                     "reaches_reference": bool(r.mean() >= REF_TEACHER_RETURN),
                     "logstd": [float(x) for x in teacher.flat[-2:]]},
           "metrics_last": dict(zip(METRICS, [float(x) for x in tr.metrics(1)[0]]))}
    if a.ckpt:
        from reacherdistilation_amd import tf_checkpoint
        tf_checkpoint.save_teacher(a.ckpt, teacher)
        out["checkpoint"] = a.ckpt
    tr.close()
    with open(a.out, "w") as fh:
        json.dump(out, fh)
    print(json.dumps(out["final"]), "train %.1f s, %.3g env-steps/s" % (train_s, out["env_steps_per_s_training"]),
          flush=True)


if __name__ == "__main__":
    main()

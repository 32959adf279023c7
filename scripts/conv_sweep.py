"""North-star convergence under the env-step reading of the reference's budget (VERDICT r2
item 6): env steps until the student's action-MSE vs the teacher is < 1e-3, against the
reference's 250,000 (mlp_train.py:143-204: 5,000 episodes x 50 steps).
  (a) the batched trainer at small batches and a few learning rates (bench.convergence);
  (b) the reference-shaped single-env driver (mlp_train.train: one env step + one Adam step on
      a 200-row dataset window per step, the reference's own loop), MSE loss.
usage: python scripts/conv_sweep.py [out.jsonl] [--teacher fitted] [--quick]
  --teacher fitted: the reference teacher's structure fitted to the fixture's 1,050 teacher records
  (teacher.fit_teacher) instead of the synthetic teacher."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = open(args[0], "w") if args else sys.stdout
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["c2"]
    teacher = None
    if "--teacher" in sys.argv and sys.argv[sys.argv.index("--teacher") + 1] == "fitted":
        teacher, info = bench.fitted_teacher(dev)
        out.write(json.dumps({"teacher": info}) + "\n")
    sizes = (8, 16, 32, 64) if "--quick" in sys.argv else (16, 32, 64, 128, 256)
    for n in sizes:
        for lr in (1e-4, 3e-4, 1e-3):
            r = bench.convergence(wl, n, "f32", dev, 0, 1, lr, max_steps=min(40000, 2_000_000 // n), chunk=10,
                                  split=True, teacher=teacher)
            r["leg"] = "batched"
            r["teacher"] = "fitted" if teacher is not None else "synthetic"
            out.write(json.dumps(r) + "\n")
            out.flush()
    from reacherdistilation_amd import mlp_train
    for lr in (1e-4, 3e-4, 1e-3):
        t0 = time.perf_counter()
        tr, ds, losses = mlp_train.train(episodes=5000, warmup_episodes=40, loss="mse", lr=lr, log=lambda *a: None,
                                         stop_loss=1e-3, teacher=teacher)
        el = time.perf_counter() - t0
        hit = len(losses) if losses and losses[-1] / 50 < 1e-3 else None
        env_steps = ds.num_episodes() * 50
        out.write(json.dumps({"leg": "reference-shaped driver", "lr": lr, "loss": "mse", "episodes": ds.num_episodes(),
                              "env_steps": env_steps, "hit": hit is not None,
                              "final_mean_window_mse": losses[-1] / 50 if losses else None,
                              "first_losses": [l / 50 for l in losses[:5]], "seconds": el}) + "\n")
        out.flush()
        tr.close()


if __name__ == "__main__":
    main()

#!/bin/bash
# r06h: PPO teacher at the reference's hyperparameters (actor batch 2048, minibatch 64, 10 epochs,
# 3e-4 linear over 1e6 steps, Adam eps 1e-5) in three env layouts of the 2048-step actor batch
set -o pipefail
OUT=gpurun_out/r06h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ppo_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ppo.log 2>&1 || { tail -30 $OUT/pytest_ppo.log; exit 1; }
tail -1 $OUT/pytest_ppo.log
for cfg in "16 128" "64 32" "1 2048"; do
  set -- $cfg
  timeout -k 10 400 python3 -u scripts/train_ppo_teacher.py --timesteps 1000000 --n-envs $1 --horizon $2 --out $OUT/ppo_$1x$2.json --ckpt $OUT/teacher_$1x$2.ckpt > $OUT/ppo_$1x$2.log 2>&1 || { tail -20 $OUT/ppo_$1x$2.log; exit 1; }
  echo "== $1 x $2"; grep -E "eval_return|return_mean" $OUT/ppo_$1x$2.log | cut -c1-200 | tail -6
done

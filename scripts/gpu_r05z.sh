#!/bin/bash
# A/B of PPO variants: product libreacher.so vs RD_LIB variants, bench_ppo (4,096-row minibatches), 3 alternations
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r05z_ab.jsonl; : > $out
for rep in 1 2 3; do
  for lib in libreacher.so "$@"; do
    echo "{\"lib\": \"$lib\"}" >> $out
    RD_LIB=$lib timeout -k 10 120 python -u scripts/bench_ppo.py --no-cpu --iters 20 2>/dev/null | head -1 | cut -c1-140 >> $out || exit 1
  done
done
cat $out

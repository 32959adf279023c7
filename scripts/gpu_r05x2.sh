#!/bin/bash
# PPO fused minibatch step: kernel stats at 4,096-row and 64-row minibatches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05x_prof -o ppo -- python3 scripts/bench_ppo.py --no-cpu --iters 6 > gpurun_out/r05x_prof.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05x_prof64 -o ppo -- python3 scripts/bench_ppo.py --no-cpu --mb 64 --iters 2 > gpurun_out/r05x_prof64.log 2>&1 || exit 1
find gpurun_out/r05x_prof gpurun_out/r05x_prof64 -name "*kernel_stats.csv"

#!/bin/bash
# PPO fused minibatch step: parity tests, bench (4,096-row and 64-row minibatches), kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo_gpu.py \
  > gpurun_out/r05x_ppo_tests.log 2>&1 || { tail -30 gpurun_out/r05x_ppo_tests.log; exit 1; }
tail -3 gpurun_out/r05x_ppo_tests.log
timeout -k 10 240 python -u scripts/bench_ppo.py --no-cpu > gpurun_out/r05x_ppo_bench.jsonl 2>&1 || exit 1
timeout -k 10 240 python -u scripts/bench_ppo.py --no-cpu --mb 64 --iters 6 >> gpurun_out/r05x_ppo_bench.jsonl 2>&1 || exit 1
cat gpurun_out/r05x_ppo_bench.jsonl | cut -c1-400
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05x_prof -o ppo -- python3 scripts/bench_ppo.py --no-cpu --iters 6 > gpurun_out/r05x_prof.log 2>&1 || exit 1
find gpurun_out/r05x_prof -name "*kernel_stats.csv" | head -3

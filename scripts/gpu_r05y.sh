#!/bin/bash
# PPO tile-kernel phase stamps (diagnostic variant) + PPO parity on the product library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RD_LIB=libreacher_ppost.so timeout -k 10 120 python -u scripts/ppo_stamps.py 4096 > gpurun_out/r05y_ppo_stamps.jsonl 2>&1 || exit 1
RD_LIB=libreacher_ppost.so timeout -k 10 120 python -u scripts/ppo_stamps.py 64 >> gpurun_out/r05y_ppo_stamps.jsonl 2>&1 || exit 1
cat gpurun_out/r05y_ppo_stamps.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ppo_gpu.py > gpurun_out/r05y_ppo_tests.log 2>&1 || { tail -30 gpurun_out/r05y_ppo_tests.log; exit 1; }
tail -2 gpurun_out/r05y_ppo_tests.log

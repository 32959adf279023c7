#!/bin/bash
# r03t: step time vs envs per group (16 / 32 / 64, 0 = the auto choice) per workload
set -o pipefail
OUT=gpurun_out/r03t; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/sweep_group_envs.py c3 c5 c4 c2 | tee $OUT/sweep_group_envs.jsonl

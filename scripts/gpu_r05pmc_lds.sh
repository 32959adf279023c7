#!/bin/bash
# LDS activity / bank-conflict pass over the PPO iteration (product build)
set -o pipefail
OUT=gpurun_out/r05pmc_lds; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o run -- python3 scripts/bench_ppo.py --no-cpu --iters 2 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }

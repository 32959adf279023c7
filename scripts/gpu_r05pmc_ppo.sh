#!/bin/bash
# PMC passes over the PPO iteration (bench_ppo, 2 iterations, 4,096 x 50): MFMA busy, VALU/MFMA
# instruction counts, LDS activity and bank conflicts, HBM fetch / write bytes; one counter set per pass
set -o pipefail
OUT=gpurun_out/r05pmc_ppo; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- python3 scripts/bench_ppo.py --no-cpu --iters 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head

#!/bin/bash
# r06zf: c4 rollout counters beyond FETCH/WRITE and MFMA busy -- LDS conflicts and waits, VALU /
# MFMA co-execution, instruction mix -- three separate --pmc passes (<= 8 SQ counters each)
set -o pipefail
OUT=gpurun_out/r06zf; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for c in "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pass$i -o run -- \
    python3 bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection --no-workloads > $OUT/pass$i.log 2>&1 || { tail -20 $OUT/pass$i.log; exit 1; }
  echo "pass $i ok"
done
python3 scripts/pmc_traffic.py $OUT/pmc_c4_counters.json rollout_kernel $OUT/pass1 $OUT/pass2 $OUT/pass3
find $OUT -name "*counter_collection.csv" -delete

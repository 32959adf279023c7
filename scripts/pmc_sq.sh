#!/bin/bash
# SQ counter passes on the c4 bench (each pass its own rocprofv3 run).  usage: pmc_sq.sh TAG
TAG=${1:-sq}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i exit $rc"; tail -5 $OUT/p$i.log; exit $rc; }
done
python3 scripts/pmc_traffic.py $OUT/sq.json rollout_kernel $OUT/p*/

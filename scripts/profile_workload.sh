#!/bin/bash
# Bench line + rocprofv3 kernel-trace summary + FETCH/WRITE PMC passes for one workload.
# usage: profile_workload.sh TAG WORKLOAD [extra bench args, e.g. --f32-mode exact]
TAG=$1; WL=$2; shift 2; EXTRA="$@"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload $WL $EXTRA --no-cpu-baseline --fixture-steps 0 --no-strong-projection > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --workload $WL $EXTRA --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  t=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$t -o run -- \
    python3 bench.py --workload $WL $EXTRA --steps 20 --warmup 3 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/pmc_$t.log 2>&1 || exit $?
done
python3 scripts/pmc_traffic.py $OUT/pmc_rollout.json rollout_kernel $OUT/pmc_*/

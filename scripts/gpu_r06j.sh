#!/bin/bash
# r06j: round-6 kernel evidence at HEAD -- rocprofv3 kernel stats + PMC passes (FETCH_SIZE,
# WRITE_SIZE, MFMA busy / VALU / MFMA instruction counts) of the rollout kernel for configs 2, 3, 5
# and 4 (K = 1, the bench's own timed loop) and of the K-step launch (K = 50) at config 3 and
# config 4's 8-GPU shard (scripts/accum_probe.py)
set -o pipefail
OUT=gpurun_out/r06j; mkdir -p $OUT; export TMPDIR=/tmp
BARGS="--steps 100 --warmup 200 --no-workloads --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection"
PARGS="--steps 20 --warmup 3 --no-workloads --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection"
for W in c2 c3 c5 c4 c4x; do
  WL=${W%x}; MODE=$([ "$W" = "c4x" ] && echo exact || echo split)
  mkdir -p $OUT/$W
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$W/prof -o run -- python3 bench.py --workload $WL --f32-mode $MODE $BARGS > $OUT/$W/bench.json 2> $OUT/$W/prof.err || { tail $OUT/$W/prof.err; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    t=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$W/pmc_$t -o run -- python3 bench.py --workload $WL --f32-mode $MODE $PARGS > $OUT/$W/pmc_$t.log 2>&1 || { tail $OUT/$W/pmc_$t.log; exit 1; }
  done
  WL=$W
  python3 scripts/pmc_traffic.py $OUT/$WL/pmc_rollout.json "rollout_kernel" $OUT/$WL/pmc_*/ > /dev/null
  echo "$WL done"
done
# the K-step launch: c3 (65,536 envs, KL) and the 32,768-env shard (MSE), K = 50
for cfg in "65536 kl" "32768 mse"; do
  set -- $cfg; N=$1; L=$2; D=$OUT/k50_$N; mkdir -p $D
  PA="--k 50 --sizes $N --loss $L --opt-steps 8"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 scripts/accum_probe.py $PA > $D/probe.jsonl 2> $D/prof.err || { tail $D/prof.err; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    t=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/pmc_$t -o run -- python3 scripts/accum_probe.py $PA > $D/pmc_$t.log 2>&1 || { tail $D/pmc_$t.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $D/pmc_rollout_k.json "0, true, false>(" $D/pmc_*/ > /dev/null
  echo "k50 $N done"
done
# keep the summaries (kernel stats, the PMC json) under the 64 MiB that travels back
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -name "*counter_collection.csv" -delete
du -sh $OUT

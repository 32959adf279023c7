#!/bin/bash
# A/B timing of diagnostic library builds (RD_LIB) on one GPU: bench.py lines per variant
# and workload; every run has its own time limit and a failure ends the script.
# usage: bash scripts/ab_variants.sh TAG "workloads" variant...   (variant "base" = libreacher.so)
TAG=$1; WLS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for wl in $WLS; do
  for v in "$@"; do
    lib=libreacher.so; [ "$v" = base ] || lib=libreacher_$v.so
    RD_LIB=$lib timeout -k 10 180 python3 bench.py --workload $wl --steps 300 --warmup 30 --accum 0 --no-cpu-baseline \
      > $OUT/${wl}_$v.json 2> $OUT/${wl}_$v.err || { echo "FAIL $wl $v"; tail -5 $OUT/${wl}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], '%.4g'%d['value'], 'launch_us %.2f'%r['launch_us'], 'step_ms %.4f'%d['ms_per_step'], 'frac %.3f'%r['frac'])" $OUT/${wl}_$v.json $wl $v
  done
done

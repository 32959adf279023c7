#!/bin/bash
# Quick bench lines (no convergence / CPU legs) for a list of workloads, optionally with a
# diagnostic library: usage quick_ab.sh TAG [RD_LIB] -- workloads...
TAG=$1; LIB=${2:-libreacher.so}; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
for wl in "$@"; do
  RD_LIB=$LIB timeout -k 10 200 python3 bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg \
    --accum 0 --conv-steps 0 > $OUT/$wl.json 2> $OUT/$wl.err || { tail -5 $OUT/$wl.err; exit 1; }
  python3 -c "import json,sys; b=json.load(open('$OUT/$wl.json')); print('$wl', '%.4g' % b['value'], 'step_us %.2f' % (b['ms_per_step']*1e3), 'launch_us %.2f' % b['roofline']['launch_us'])"
done

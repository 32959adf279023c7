#!/bin/bash
# Alternating A/B of two builds on the bench step time: ab_libs.sh OUT LIB_A LIB_B [workloads...]
# (LIB_* are file names under reacherdistilation_amd/, selected with RD_LIB; 1000 steps after 300 warm-up)
OUT=gpurun_out/$1; A=$2; B=$3; shift 3; mkdir -p $OUT
for wl in "$@"; do
  for rep in 1 2; do
    for lib in $A $B; do
      RD_LIB=$lib timeout -k 10 120 python3 bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/$wl.$lib.$rep.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.load(open('$OUT/$wl.$lib.$rep.json'));print('$wl', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
    done
  done
done

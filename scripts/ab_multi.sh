#!/bin/bash
# Alternating A/B/... of several builds on the bench step time:
# ab_multi.sh OUT "LIB1 LIB2 ..." workloads...  (LIB* under reacherdistilation_amd/, selected with RD_LIB;
# 1000 steps after 300 warm-up, two rounds)
OUT=gpurun_out/$1; LIBS=$2; shift 2; mkdir -p $OUT
for wl in "$@"; do
  for rep in 1 2; do
    for lib in $LIBS; do
      RD_LIB=$lib timeout -k 10 120 python3 bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/$wl.$lib.$rep.json 2>$OUT/$wl.$lib.$rep.err || { tail -5 $OUT/$wl.$lib.$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/$wl.$lib.$rep.json'));print('$wl %-22s' % '$lib', $rep, 'value %.4g' % d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
    done
  done
done

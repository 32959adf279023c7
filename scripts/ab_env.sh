#!/bin/bash
# A/B over an environment variable: ab_env.sh TAG VAR "v1 v2 .." "wl1 wl2 .." REPS [extra bench args]
# (alternating runs; 1000 timed steps after 300 warm-up; an empty value leaves VAR unset)
TAG=$1; VAR=$2; VALS=$3; WLS=$4; REPS=$5; shift 5; EXTRA="$@"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 $REPS); do for wl in $WLS; do for v in $VALS; do
  f=$OUT/${wl}_${v}_$rep.json
  env $VAR=$v timeout -k 10 120 python bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 $EXTRA > $f 2>$OUT/err.txt || exit 1
  python3 -c "import json;d=json.load(open('$f'));print('$wl $VAR=$v rep $rep', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
done; done; done

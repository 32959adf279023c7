#!/bin/bash
# Step time vs envs per GPU (groups per pair = envs / 65,536): sweep_envs.sh TAG "wl1 .." "n1 n2 .." [extra]
TAG=$1; WLS=$2; NS=$3; shift 3; EXTRA="$@"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for wl in $WLS; do for n in $NS; do
  f=$OUT/${wl}_$n.json
  timeout -k 10 120 python bench.py --workload $wl --envs-per-gpu $n --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 $EXTRA > $f 2>$OUT/err.txt || exit 1
  python3 -c "import json;d=json.load(open('$f'));print('$wl n=$n', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
done; done

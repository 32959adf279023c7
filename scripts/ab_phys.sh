#!/bin/bash
# A/B: which wave of a pair steps the envs (RDD_PHYS), alternating runs, f32_split default.
mkdir -p gpurun_out/ab_phys
for rep in 1 2 3; do for wl in c4 c5 c3; do for p in producer consumer; do
  RDD_PHYS=$p timeout -k 10 120 python bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > gpurun_out/ab_phys/${wl}_${p}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_phys/${wl}_${p}_$rep.json'));print('$wl $p $rep', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
done; done; done

#!/bin/bash
# A/B: which wave of a pair steps the envs (RDD_PHYS), c4 and c5, f32_split.
mkdir -p gpurun_out/ab_phys
for wl in c4 c5; do for p in producer consumer; do
  RDD_PHYS=$p timeout -k 10 120 python bench.py --workload $wl --steps 300 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > gpurun_out/ab_phys/${wl}_$p.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_phys/${wl}_$p.json'));print('$wl $p', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
done; done

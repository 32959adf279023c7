#!/bin/bash
# c2 / c3 timing (both f32 modes) and c2 stamps.
mkdir -p gpurun_out/small
for wl in c2 c3; do
  timeout -k 10 200 python bench.py --workload $wl --steps 500 --warmup 300 --no-cpu-baseline --accum 0 --conv-steps 0 > gpurun_out/small/$wl.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/small/$wl.json'));o=d['other_f32_mode']
print('$wl split', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'], '| exact', '%.4g'%o['value'], 'step_us %.2f'%(1e3*o['ms_per_step']), 'launch_us %.2f'%o['launch_us'])"
done
RD_LIB=libreacher_stamps.so RD_SPLIT=1 timeout -k 10 60 python scripts/stamps.py 4096 2>/dev/null
RD_LIB=libreacher_stamps.so RD_SPLIT=0 timeout -k 10 60 python scripts/stamps.py 4096 2>/dev/null

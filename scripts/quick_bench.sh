#!/bin/bash
# Distill parity tests, then every workload's step time (1000 steps after 300 warm-up).
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests/test_distill_gpu.py tests/test_split_gpu.py tests/test_fullsize_gpu.py tests/test_c1_gpu.py tests/test_dataset_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/quick/pytest.log 2>&1 || { tail -30 gpurun_out/quick/pytest.log; exit 1; }
tail -1 gpurun_out/quick/pytest.log
for wl in c2 c3 c4 c5; do
  timeout -k 10 120 python bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > gpurun_out/quick/$wl.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/quick/$wl.json'));print('$wl', '%.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
done

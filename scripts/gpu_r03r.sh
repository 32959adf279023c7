#!/bin/bash
# r03r: fused apply (each step's reduce + Adam at the head of the next rollout): bitwise tests, then the
# step time with and without it, alternating
set -o pipefail
OUT=gpurun_out/r03r; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_apply_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_fused.log 2>&1 || { tail -40 $OUT/pytest_fused.log; exit 1; }
tail -3 $OUT/pytest_fused.log
for wl in c2 c5 c3 c4; do
  for rep in 1 2; do
    for f in 0 1; do
      timeout -k 10 120 python3 bench.py --workload $wl --fused-apply $f --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/$wl.f$f.$rep.json 2>$OUT/$wl.f$f.$rep.err || { tail -5 $OUT/$wl.f$f.$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/$wl.f$f.$rep.json'));print('$wl fused=$f', $rep, 'value %.4g' % d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
    done
  done
done

#!/bin/bash
# r05u: GPU suite + smoke + the default bench line, end of round 5
set -o pipefail
OUT=gpurun_out/r05u; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
t1=$(date +%s.%N)
echo "bench default wall $(python3 -c "print($t1 - $t0)") s"
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('value', d['value'], 'us/step', d['ms_per_step']*1e3, 'frac', d['roofline']['frac'], 'accum', d.get('accum',{}).get('fused')); print(json.dumps(d.get('convergence_fitted_teacher',{}).get('convergence_small_batch')))"

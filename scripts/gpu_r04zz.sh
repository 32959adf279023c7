#!/bin/bash
# r04zz: round-4 final state (after the multi-tile LSTM head backward):
# full GPU suite, smoke, the default bench line
set -o pipefail
OUT=gpurun_out/r04zz; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['value'], d['ms_per_step']*1e3, 'us', d['roofline']['frac'], d['cpu_baseline'])"

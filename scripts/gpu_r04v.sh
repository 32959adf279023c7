#!/bin/bash
# r04v: the round-4 product after the LSTM per-step heads: full GPU
# suite, smoke, 10 repeated rollouts per config, the default bench line, c4 bench + rocprof + PMC
set -o pipefail
OUT=gpurun_out/r04v; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s,c4e > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
bash scripts/profile_workload.sh r04v/c4 c4 > /dev/null || { echo "profile c4 failed"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4/pmc_rollout.json')); print('c4 pmc', {k: d[k] for k in d if k != 'avg'})"
bash scripts/profile_workload.sh r04v/c2 c2 > /dev/null || { echo "profile c2 failed"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2/pmc_rollout.json')); print('c2 pmc', {k: d[k] for k in d if k != 'avg'})"

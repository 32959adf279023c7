#!/bin/bash
# r06zc: the gym-API env's joint-1 trig beyond 4 rad through sincos_q0 (wide-angle accuracy):
# the new wide-angle test first, the GPU suite, then the default bench line (env.step roofline)
set -o pipefail
OUT=gpurun_out/r06zc; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -v --timeout 120 --timeout-method thread > $OUT/pytest_env.log 2>&1 || { tail -40 $OUT/pytest_env.log; exit 1; }
grep -E "wide_angles|passed|failed" $OUT/pytest_env.log | tail -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - $OUT/bench_default.json <<'P'
import json, sys
b = json.load(open(sys.argv[1]))
print("value %.4g ms %.4f launch %.2f | env %.0f GB/s" % (b["value"], b["ms_per_step"], b["roofline"]["launch_us"], b["roofline_env"]["achieved"]))
P

#!/bin/bash
# Round-5 LSTM redesign check: LSTM GPU tests, the 20/32/1024-window bench, kernel stats at 20 windows
set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_student_lstm_gpu.py tests/test_c1_gpu.py > $OUT/pytest_lstm.log 2>&1 || { tail -30 $OUT/pytest_lstm.log; exit 1; }
tail -2 $OUT/pytest_lstm.log
timeout -k 10 300 python -u scripts/bench_student_lstm.py 20 32 1024 16384 > $OUT/bench.jsonl 2> $OUT/bench.err || { cat $OUT/bench.err | tail; exit 1; }
cat $OUT/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/prof_bench.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r05l/prof/**/run_kernel_stats.csv", recursive=True))[-1]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY

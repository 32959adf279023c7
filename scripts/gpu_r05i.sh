#!/bin/bash
# r05i: the LSTM persistent kernels with granule exchange (no grid barrier): LSTM GPU tests,
# then the training step at the reference's 20 windows (and 32 / 1,024) under rocprofv3
set -o pipefail
OUT=gpurun_out/r05i; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_student_lstm_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_lstm.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/pytest_lstm.log | head; tail -20 $OUT/pytest_lstm.log; exit 1; }
tail -1 $OUT/pytest_lstm.log
timeout -k 10 200 python -u scripts/bench_student_lstm.py 20 32 1024 > $OUT/lstm_bench.jsonl 2> $OUT/lstm_bench.err || { tail $OUT/lstm_bench.err; exit 1; }
cat $OUT/lstm_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof20 -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/prof20.log 2>&1 || { tail $OUT/prof20.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05i/prof20/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>6}  {r['Name'][:90]}")
PY

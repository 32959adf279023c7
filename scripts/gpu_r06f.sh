#!/bin/bash
# r06f: LSTM GPU tests + per-kernel rocprof of the 20-window step after the branch-free BPTT loads,
# round-5 library vs this build, alternating
set -o pipefail
OUT=gpurun_out/r06f; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_student_lstm_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_lstm.log 2>&1 || { tail -40 $OUT/pytest_lstm.log; exit 1; }
tail -1 $OUT/pytest_lstm.log
for r in 1 2; do
for lib in libreacher_head.so libreacher.so; do
  RD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib.$r -o run -- python3 scripts/bench_student_lstm.py 20 1024 > $OUT/$lib.$r.jsonl 2> $OUT/$lib.err || { tail $OUT/$lib.err; exit 1; }
  echo "== $lib"; cut -c1-100 $OUT/$lib.$r.jsonl
  python3 - $OUT/$lib.$r <<'P'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "persist" in r["Name"]: print("  %-60s %7s avg_us %.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
P
done
done

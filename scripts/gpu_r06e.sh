#!/bin/bash
# r06e: per-kernel rocprof of the LSTM's 20-window step, round-5 library vs the no-SLP build
set -o pipefail
OUT=gpurun_out/r06e; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher_head.so libreacher.so; do
  RD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/$lib.jsonl 2> $OUT/$lib.err || { tail $OUT/$lib.err; exit 1; }
  echo "== $lib"; cat $OUT/$lib.jsonl | cut -c1-120
  python3 - $OUT/$lib <<'P'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-70s %7s avg_us %.2f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
P
done

#!/bin/bash
# kernel stats of the 20-window LSTM step (round-5 redesign)
set -o pipefail
OUT=gpurun_out/r05l2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/prof_bench.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r05l2/prof/**/run_kernel_stats.csv", recursive=True))[-1]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY

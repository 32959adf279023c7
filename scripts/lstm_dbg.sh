#!/bin/bash
OUT=gpurun_out/lstm_dbg; mkdir -p $OUT; export TMPDIR=/tmp
for d in 0 1 2 4 7; do
  RDL_PR_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$d -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/b$d.log 2>&1 || exit 1
  f=$(ls $OUT/p$d/*/run_kernel_stats.csv $OUT/p$d/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'persist' in r['Name']: print('dbg $d', r['Name'][22:50], 'avg_us %.1f' % (float(r['AverageNs'])/1e3))"
done

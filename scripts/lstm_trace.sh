#!/bin/bash
# rocprofv3 kernel trace of the LSTM student's 20-window step; per-step timeline summary
OUT=gpurun_out/${1:-lstm_tr}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 scripts/bench_student_lstm.py 20 > $OUT/bench.log 2>&1 || exit $?
cat $OUT/bench.log | grep windows
python3 scripts/lstm_timeline.py $(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1)

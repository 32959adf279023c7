#!/bin/bash
# Benches + rocprofv3 kernel summaries of the widened paths (reference student MLP, LSTM
# student, PPO teacher).  Kernel traces are deleted after the summaries are written (the
# PPO trace alone exceeds the 64 MiB gpurun_out budget).
set -u
OUT=gpurun_out/${1:-sec}
mkdir -p "$OUT"
export TMPDIR=/tmp
for b in student_mlp student_lstm ppo; do
  timeout -k 10 300 python scripts/bench_$b.py > "$OUT/bench_$b.jsonl" 2> "$OUT/bench_$b.err" || { echo "bench $b failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_mlp" -o run -- \
  python3 scripts/bench_student_mlp.py 262144 > /dev/null 2>&1 || { echo "prof mlp failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lstm" -o run -- \
  python3 scripts/bench_student_lstm.py 16384 > /dev/null 2>&1 || { echo "prof lstm failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ppo" -o run -- \
  python3 scripts/bench_ppo.py --no-cpu > /dev/null 2>&1 || { echo "prof ppo failed"; exit 1; }
find "$OUT" -name '*kernel_trace.csv' -delete
cat "$OUT"/bench_*.jsonl
echo DONE

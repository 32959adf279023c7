#!/bin/bash
# r06c: GPU suite on the no-packed-f32 / per-site-fence / no-SLP build, then an A/B of the
# reference-student and LSTM benches (their sources are now built without SLP) vs HEAD
set -o pipefail
OUT=gpurun_out/r06c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for r in 1 2; do
  for lib in libreacher_head.so libreacher.so; do
    RD_LIB=$lib timeout -k 10 200 python3 scripts/bench_student_mlp.py 200 65536 262144 > $OUT/mlp_$lib.$r.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    RD_LIB=$lib timeout -k 10 200 python3 scripts/bench_student_lstm.py 20 1024 16384 > $OUT/lstm_$lib.$r.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    echo "== $lib $r"; cat $OUT/mlp_$lib.$r.jsonl $OUT/lstm_$lib.$r.jsonl | cut -c1-220
  done
done

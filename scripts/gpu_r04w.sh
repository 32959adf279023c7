#!/bin/bash
# r04w: the reduce kernel's one-round-trip partial sums (<= 256 rows): bitwise A/B against the
# previous build, the distill + LSTM GPU tests, c2 / c4 benches and rocprof kernel stats
set -o pipefail
OUT=gpurun_out/r04w; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 env RD_LIB=libreacher_ab0.so python3 -u scripts/bitwise_ab.py /tmp/ab0.npz > $OUT/ab0.log 2>&1 || { tail -20 $OUT/ab0.log; exit 1; }
timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/ab1.npz > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
python3 scripts/bitwise_ab.py --compare /tmp/ab0.npz /tmp/ab1.npz | tee $OUT/ab_compare.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_distill_gpu.py tests/test_student_lstm_gpu.py tests/test_tf_checkpoint.py tests/test_determinism_gpu.py -m "gpu or not gpu" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in c2 c4; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --fixture-steps 0 --no-strong-projection > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step']*1e3, 'us', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/prof_c2.log 2>&1 || { echo "rocprof c2 failed"; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" -exec head -4 {} \;

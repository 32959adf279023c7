#!/bin/bash
# r06d: GPU suite at HEAD of the round-6 work; the T = 258 LSTM test against the round-5 library
# (expected to fail there: its 8-bit tag phase); reference-student / LSTM A/B (no-SLP builds)
# vs round 5; one bench line with the new `workloads` object
set -o pipefail
OUT=gpurun_out/r06d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
RD_LIB=libreacher_head.so timeout -k 10 300 python -u -m pytest tests/test_student_lstm_gpu.py -k past_256 -q --timeout 200 --timeout-method thread > $OUT/lstm258_round5_lib.log 2>&1
echo "round-5 library on the T=258 test: rc=$? (1 = failed, as expected)"; tail -3 $OUT/lstm258_round5_lib.log
for r in 1 2; do
  for lib in libreacher_head.so libreacher.so; do
    RD_LIB=$lib timeout -k 10 200 python3 scripts/bench_student_mlp.py 200 65536 262144 > $OUT/mlp_$lib.$r.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    RD_LIB=$lib timeout -k 10 200 python3 scripts/bench_student_lstm.py 20 1024 16384 > $OUT/lstm_$lib.$r.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    echo "== $lib $r"; cat $OUT/mlp_$lib.$r.jsonl $OUT/lstm_$lib.$r.jsonl | cut -c1-200
  done
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --conv-steps 0 --fixture-steps 0 --no-cpu-baseline --no-strong-projection > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; b=json.load(open('$OUT/bench.json')); print('c4', b['value'], b['ms_per_step'], b['roofline']['launch_us'], 'exact', b['other_f32_mode']['ms_per_step'], b['other_f32_mode']['launch_us'])
for k, v in b['workloads'].items():
    if isinstance(v, dict): print(k, {kk: (round(vv['us_per_env_step'], 2), round(vv['launch_us_per_env_step'], 2), round(vv['frac'], 3)) for kk, vv in v.items() if isinstance(vv, dict)})"

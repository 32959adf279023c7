#!/bin/bash
# r06s: joint-0 angles on 2-pi-reduced hardware sin/cos (sincos_q0, libreacher_q0hw.so): its accuracy
# (scripts/micro/trig_acc), the whole GPU suite on the variant, then an alternating A/B vs HEAD
set -o pipefail
OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 5 120 ./scripts/micro/trig_acc > $OUT/trig_acc.jsonl || exit 1
cat $OUT/trig_acc.jsonl
RD_LIB=libreacher_q0hw.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_q0hw.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c5,c3,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

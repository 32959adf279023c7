#!/bin/bash
# r06o: every joint-1 angle (RK4 stages, kq1, the observation's q1) on the hardware v_sin/v_cos
# GPU suite on the variant (parity vs the f64 oracle / fixture at unchanged tolerances), then an
# alternating A/B against HEAD
set -o pipefail
OUT=gpurun_out/r06o; mkdir -p $OUT
RD_LIB=libreacher_hwtrig2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher_hwtrig.so libreacher_hwtrig2.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c5,c3,c2,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

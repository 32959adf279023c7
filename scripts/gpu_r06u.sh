#!/bin/bash
# r06u: qacc_sc with fewer VALU (M11 one fma, shared HC s, elimination, |q1| > 3) (libreacher_qa.so)
# the whole GPU suite on the variant, then an alternating A/B vs HEAD
set -o pipefail
OUT=gpurun_out/r06u; mkdir -p $OUT
RD_LIB=libreacher_qa.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_qa.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c5,c3,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

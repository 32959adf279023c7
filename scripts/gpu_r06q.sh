#!/bin/bash
# r06q: the split consumer's dW2+dH1 scheduling region after dw2_split32: 72 x (1 MFMA, 3 VALU)
# (product) vs 24 x (1, 5) + 48 x (1, 2) (s52) vs 72 x (1, 2) (s2); alternating processes
set -o pipefail
OUT=gpurun_out/r06q; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher.so libreacher_s52.so libreacher_s2.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c3,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

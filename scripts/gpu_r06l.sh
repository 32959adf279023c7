#!/bin/bash
# r06l: c5 (TC kernel) -- which tiles' teacher forward the consumer runs: odd tiles (HEAD), tile 3
# only (tc3), tile 1 only (tc1); alternating processes
set -o pipefail
OUT=gpurun_out/r06l; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher.so libreacher_tc3.so libreacher_tc1.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 3000 c5 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

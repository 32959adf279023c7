#!/bin/bash
# r06a: alternating A/B of HEAD (round-5 product) vs the no-packed-f32 rollout builds
set -o pipefail
OUT=gpurun_out/r06a; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher_head.so libreacher_nopk_last2.so libreacher_nopk_nofence.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c4x,c3,c3x,c5,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

#!/bin/bash
# r06b: exact-f32 fence placement A/B (layer-2 k-steps fenced per RD_FM mask) vs the unfenced build
set -o pipefail
OUT=gpurun_out/r06b; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher_fm0x8a00.so libreacher_fm0xaa00.so libreacher_fm0xaaaa.so libreacher_nopk_nofence.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4x,c3x,c4 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

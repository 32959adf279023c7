#!/bin/bash
# Narrowing the consumer-side hazard: c4 split, RDD_PHYS=consumer, 20 repeated
# rollouts per build: MFMA-to-MFMA latency filled with s_nops, and one s_nop before every instruction.
OUT=gpurun_out/cpbis; mkdir -p $OUT
for lib in libreacher_mfmapad.so libreacher_snop1.so libreacher.so; do
  RD_LIB=$lib RDD_PHYS=consumer timeout -k 10 300 python3 -u scripts/det_check.py 20 c4s > $OUT/det_$lib.txt 2>&1 || exit 1
  echo "$lib c4s consumer identical $(grep -c identical $OUT/det_$lib.txt) of 20"
done

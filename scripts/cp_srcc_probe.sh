#!/bin/bash
# One probe of the consumer-side env step's run-to-run differences against the
# static finding of scripts/isa/hazards.py: the variant as built (LDS loads 0-1 wait states
# after an f32 MFMA into its SrcC registers) vs the same variant with every f32 MFMA fenced
# (RD_MFMA_SRCC_FENCE: no load issues before the MFMA completes).  20 repeated rollouts each.
OUT=gpurun_out/srcc; mkdir -p $OUT
for lib in cp cpfence; do
  RD_LIB=libreacher_$lib.so RDD_PHYS=consumer timeout -k 10 400 python3 -u scripts/det_check.py 20 c4s,c5 > $OUT/det_$lib.txt 2>&1 || exit 1
  echo "$lib: $(grep -c " identical$" $OUT/det_$lib.txt) identical of $(grep -c rep $OUT/det_$lib.txt)"
done

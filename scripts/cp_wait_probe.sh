#!/bin/bash
# Consumer-side env step with every outstanding counter drained before the consumer frees the
# slot (RD_CP_WAIT build) vs the product, c4 split, 20 repeated rollouts each.
OUT=gpurun_out/cpw; mkdir -p $OUT
for lib in libreacher_cpwait.so libreacher.so; do
  RD_LIB=$lib RDD_PHYS=consumer timeout -k 10 300 python3 -u scripts/det_check.py 20 c4s > $OUT/det_$lib.txt 2>&1 || exit 1
  echo "$lib c4s consumer identical $(grep -c identical $OUT/det_$lib.txt) of 20"
done

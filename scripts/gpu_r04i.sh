#!/bin/bash
# r04i: the c4 first-rollout-of-a-process difference (r04g: r04e product 0/8 repeats identical,
# the TC build 8/8): r04e product vs its register-staged image copy (regcopy), vs every f32
# MFMA group SrcC-fenced (fenceall), vs TC, vs the helper-pair product
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher_notc.so libreacher_regcopy.so libreacher_fenceall.so libreacher_tc.so libreacher.so; do
  RD_LIB=$lib timeout -k 10 300 python3 -u scripts/det_check.py 6 c4s,c4e,grid300 > $OUT/det_$lib.txt 2>&1 || { tail $OUT/det_$lib.txt; exit 1; }
  echo "$lib det: $(grep -c ' identical$' $OUT/det_$lib.txt) identical of $(grep -c rep $OUT/det_$lib.txt)"
done

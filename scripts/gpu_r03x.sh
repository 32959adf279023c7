#!/bin/bash
# r03x2: repeated rollouts (det_check: each rep a fresh trainer, compared with the first) with the product (asm nt
# partial row from 128 workgroups up + consumer interleave), cs2plain (plain partial-row stores) and ntb
# (__builtin_nontemporal_store partial row at every grid)
OUT=gpurun_out/r03x2; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_cs2plain.so libreacher_ntb.so; do
  for c in c4s c2s c3s; do
    RD_LIB=$lib timeout -k 10 300 python3 -u scripts/det_check.py 20 $c > $OUT/det_${lib}_$c.txt 2>&1 || { tail -5 $OUT/det_${lib}_$c.txt; exit 1; }
    echo "$lib $c: $(grep -c ' identical$' $OUT/det_${lib}_$c.txt) identical of $(grep -c rep $OUT/det_${lib}_$c.txt)"
  done
done

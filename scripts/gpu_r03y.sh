#!/bin/bash
# r03y: product = consumer interleave schedule + plain partial-row stores (inline-asm nt removed): GPU suite, smoke,
# determinism (product, the builtin-nt partial row wsnt, the producer layer-2 pattern ps2), A/B against the previous commit
set -o pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03y || exit 1
for lib in libreacher.so libreacher_wsnt.so libreacher_ps2.so; do
  for c in c4s c5 c3s c2s c4e; do
    RD_LIB=$lib timeout -k 10 300 python3 -u scripts/det_check.py 12 $c > $OUT/det_${lib}_$c.txt 2>&1 || { tail -5 $OUT/det_${lib}_$c.txt; exit 1; }
    echo "$lib $c: $(grep -c ' identical$' $OUT/det_${lib}_$c.txt) identical of $(grep -c rep $OUT/det_${lib}_$c.txt)"
  done
done
bash scripts/ab_multi.sh r03y/ab "libreacher_prev.so libreacher.so libreacher_wsnt.so libreacher_ps2.so" c4 c5 c3 c2

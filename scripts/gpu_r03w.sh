#!/bin/bash
# r03w: the product with the consumer interleave schedule: GPU suite, smoke, determinism, A/B against the previous
# commit's library (libreacher_prev.so) on every workload
set -o pipefail
OUT=gpurun_out/r03w; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03w || exit 1
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c3s,c2s,c4e,c5 > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_multi.sh r03w/ab "libreacher_prev.so libreacher.so libreacher_ps2.so" c4 c3 c2 c5

#!/bin/bash
# r03ze: the producer's layer-2 pattern with 1 (pp1) or 3 (pp3) VALU per MFMA instead of 2 (the product)
set -o pipefail
OUT=gpurun_out/r03ze; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/ab_multi.sh r03ze/ab "libreacher_prev.so libreacher_pp1.so libreacher_pp3.so" c4 c3

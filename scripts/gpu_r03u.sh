#!/bin/bash
# r03u: f32-split consumer backward scheduling variants (cs1: dH1 split ahead of the dW2 MFMAs; cs2: + MFMA/VALU
# interleave pattern) vs the product; parity of cs2 first
set -o pipefail
OUT=gpurun_out/r03u; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_cs2.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_cs2.log 2>&1 || { tail -30 $OUT/pytest_cs2.log; exit 1; }
tail -1 $OUT/pytest_cs2.log
bash scripts/ab_multi.sh r03u/ab "libreacher.so libreacher_cs1.so libreacher_cs2.so" c4 c3 c2

#!/bin/bash
# r03zc: the pair's layer 1 + tanh with an interleave pattern (l1s) vs the product (libreacher_prev.so = c644bc8)
set -o pipefail
OUT=gpurun_out/r03zc; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_l1s.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_l1s.log 2>&1 || { tail -30 $OUT/pytest_l1s.log; exit 1; }
tail -1 $OUT/pytest_l1s.log
RD_LIB=libreacher_l1s.so timeout -k 10 300 python3 -u scripts/det_check.py 12 c4s > $OUT/det_l1s.txt 2>&1 || { tail -5 $OUT/det_l1s.txt; exit 1; }
echo "l1s c4s: $(grep -c ' identical$' $OUT/det_l1s.txt) identical of $(grep -c rep $OUT/det_l1s.txt)"
bash scripts/ab_multi.sh r03zc/ab "libreacher_prev.so libreacher_l1s.so" c4 c3 c2

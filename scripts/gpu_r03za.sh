#!/bin/bash
# r03za: the split teacher's layer 2 beside the bf16 student in three scheduling regions with an interleave pattern
# (ts1) and the pair's last K step with the tanh in its MFMA gaps (ps3) vs the product (libreacher_prev.so = 4b33943)
set -o pipefail
OUT=gpurun_out/r03za; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_ts1.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ts1.log 2>&1 || { tail -30 $OUT/pytest_ts1.log; exit 1; }
tail -1 $OUT/pytest_ts1.log
RD_LIB=libreacher_ts1.so timeout -k 10 300 python3 -u scripts/det_check.py 12 c5 > $OUT/det_ts1.txt 2>&1 || { tail -5 $OUT/det_ts1.txt; exit 1; }
echo "ts1 c5: $(grep -c ' identical$' $OUT/det_ts1.txt) identical of $(grep -c rep $OUT/det_ts1.txt)"
bash scripts/ab_multi.sh r03za/ab "libreacher_prev.so libreacher_ts1.so" c5 && bash scripts/ab_multi.sh r03za/ab2 "libreacher_prev.so libreacher_ps3.so" c4 c3 c2

#!/bin/bash
# r03zd: c5 -- the teacher's last K step and the bf16 student's MFMAs with VALU in their gaps (ts2) vs the product
set -o pipefail
OUT=gpurun_out/r03zd; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_ts2.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ts2.log 2>&1 || { tail -30 $OUT/pytest_ts2.log; exit 1; }
tail -1 $OUT/pytest_ts2.log
RD_LIB=libreacher_ts2.so timeout -k 10 300 python3 -u scripts/det_check.py 12 c5 > $OUT/det_ts2.txt 2>&1 || { tail -5 $OUT/det_ts2.txt; exit 1; }
echo "ts2 c5: $(grep -c ' identical$' $OUT/det_ts2.txt) identical of $(grep -c rep $OUT/det_ts2.txt)"
bash scripts/ab_multi.sh r03zd/ab "libreacher_prev.so libreacher_ts2.so" c5 c5

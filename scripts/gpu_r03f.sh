#!/bin/bash
# r03f: the split variant libreacher_s2.so -- dW2 of the f32 student (RDD_DW2_SPLIT) and the
# teacher's layer 1 beside the bf16 student (RDD_L1_SPLIT) on split bf16 MFMAs: split and
# distill parity tests with the variant, repeated-rollout determinism, then an alternating A/B
# against the product on c4/c3/c5/c2.
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_s2.so timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/pytest_s2.log 2>&1 || { tail -40 $OUT/pytest_s2.log; exit 1; }
tail -2 $OUT/pytest_s2.log
RD_LIB=libreacher_s2.so timeout -k 10 300 python3 -u scripts/det_check.py 10 c5,c4s,c2s > $OUT/det_s2.txt 2>&1 || { tail -20 $OUT/det_s2.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det_s2.txt) identical of $(grep -c rep $OUT/det_s2.txt)"
bash scripts/ab_libs.sh r03f/ab libreacher.so libreacher_s2.so c4 c5 c3 c2

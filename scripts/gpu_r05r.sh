#!/bin/bash
# r05r: c5 A/B of a distill.hip change (product) vs the previous build (libreacher_c5old.so)
set -o pipefail
OUT=gpurun_out/${AB_OUT:-r05r}; mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 120 python scripts/ab_k1.py 2000 c5 >> $OUT/ab.jsonl || exit 1
  RD_LIB=libreacher_c5old.so timeout -k 10 120 python scripts/ab_k1.py 2000 c5 >> $OUT/ab.jsonl || exit 1
done
cat $OUT/ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_distill_gpu.py tests/test_determinism_gpu.py tests/test_accum_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log

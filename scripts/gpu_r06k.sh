#!/bin/bash
# r06k: the CP kernels' last group stepped by the producer (libreacher_hyb.so) vs HEAD: the
# distill / full-size / accum / determinism GPU tests on the variant, then an alternating A/B
set -o pipefail
OUT=gpurun_out/r06k; mkdir -p $OUT
RD_LIB=libreacher_hyb.so timeout -k 10 600 python -u -m pytest tests/test_distill_gpu.py tests/test_fullsize_gpu.py tests/test_accum_gpu.py tests/test_determinism_gpu.py tests/test_split_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_hyb.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c5,c4,c3 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

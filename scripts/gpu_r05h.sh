#!/bin/bash
# r05h: c5 (bf16 student, DAgger): the teacher forward of odd tiles on the consumer wave (TC),
# with the consumer-side env step (RD_TC) or the producer-side one (RD_TC_NOCP): bf16 parity
# tests on each build, then alternating A/B timings of c5 against the product
set -o pipefail
OUT=gpurun_out/r05h; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher_tc.so libreacher_tcnocp.so; do
  RD_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_distill_gpu.py tests/test_split_gpu.py tests/test_fullsize_gpu.py -k "bf16 or student or c5 or shard" -x -q --timeout 240 --timeout-method thread > $OUT/pytest_$lib.log 2>&1 || { tail -30 $OUT/pytest_$lib.log; exit 1; }
  tail -1 $OUT/pytest_$lib.log
done
for rep in 1 2 3; do for lib in libreacher.so libreacher_tc.so libreacher_tcnocp.so; do
  RD_LIB=$lib timeout -k 10 100 python -u scripts/ab_k1.py 1000 c5 >> $OUT/ab_tc.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
done; done
cat $OUT/ab_tc.jsonl

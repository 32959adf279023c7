#!/bin/bash
# r05e: the no-SLP distill build + physics rounding fixed by source + K-step launch + LDS-DMA
# image fill: the whole GPU suite, smoke, the K-step probe, A/B of the image fill
set -o pipefail
OUT=gpurun_out/r05e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
grep -E "n=[0-9]+ K=|fitted teacher" $OUT/pytest_gpu.log | head -30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
for rep in 1 2; do for lib in libreacher_regcopy.so libreacher.so; do
  RD_LIB=$lib timeout -k 10 200 python -u scripts/ab_k1.py 1000 >> $OUT/ab_imgdma.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
done; done
cat $OUT/ab_imgdma.jsonl

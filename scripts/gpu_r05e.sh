#!/bin/bash
# r05e: the no-SLP distill build + physics rounding fixed by source + K-step launch: the whole
# GPU suite, smoke, the K-step probe
set -o pipefail
OUT=gpurun_out/r05e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
grep -E "n=[0-9]+ K=|helper vs plain" $OUT/pytest_gpu.log | head -30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 400 python -u scripts/accum_probe.py --k 50 > $OUT/accum_probe.jsonl 2> $OUT/accum_probe.err || { tail $OUT/accum_probe.err; exit 1; }
cat $OUT/accum_probe.jsonl

#!/bin/bash
# r05j: the GPU suite + smoke on the build with the c5 TC kernel, then the round-5 profiles
set -o pipefail
OUT=gpurun_out/r05j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
bash scripts/gpu_r05f.sh

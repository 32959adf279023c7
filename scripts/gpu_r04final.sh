#!/bin/bash
# round-4 closing check of the committed tree: full GPU suite and smoke
set -o pipefail
OUT=gpurun_out/r04final; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log

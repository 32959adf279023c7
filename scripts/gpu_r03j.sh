#!/bin/bash
# r03j: re-entry check of the restored tree (fresh container build): GPU suite, smoke, quick lines.
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash scripts/quick_ab.sh r03j/q libreacher.so c4 c5 c3 c2

#!/bin/bash
# r03m: the rollout partial row with NT stores (inline-asm, not tail-merged) from 128 workgroups up
# GPU suite, smoke, determinism, A/B against the previous commit's library (libreacher_prev.so)
set -o pipefail
OUT=gpurun_out/r03m; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_multi.sh r03m/ab "libreacher_prev.so libreacher.so libreacher_ntws.so" c5 c4 c3 c2

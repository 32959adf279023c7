#!/bin/bash
# r03i: the student's LDS image built by each rollout's prologue from its f32 parameters (no
# prepacked student image, no image refresh in the reduce+Adam kernel): bit-for-bit A/B of 9
# configs against the previous commit's library (libreacher_prev.so = dc58d01), the GPU suite,
# then the step-time A/B on c4/c5/c3/c2.
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_prev.so timeout -k 10 300 python3 -u scripts/bitwise_ab.py $OUT/prev.npz > $OUT/bw_prev.log 2>&1 || { tail -20 $OUT/bw_prev.log; exit 1; }
timeout -k 10 300 python3 -u scripts/bitwise_ab.py $OUT/new.npz > $OUT/bw_new.log 2>&1 || { tail -20 $OUT/bw_new.log; exit 1; }
python3 scripts/bitwise_ab.py --compare $OUT/prev.npz $OUT/new.npz > $OUT/bitwise.txt; tail -1 $OUT/bitwise.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/ab_libs.sh r03i/ab libreacher_prev.so libreacher.so c4 c5 c3 c2

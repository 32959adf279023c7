#!/bin/bash
# r03v: consumer interleave-pattern variants (cs2: 40 VALU, then 80 x (MFMA, 3 VALU); cs2b: 96 x (MFMA, 2 VALU);
# cs2c: 60, 60 x (MFMA, 4 VALU); cs2ps: cs2 + the producer's layer-2 pattern) vs the product
set -o pipefail
OUT=gpurun_out/r03v; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher_cs2ps.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_cs2ps.log 2>&1 || { tail -30 $OUT/pytest_cs2ps.log; exit 1; }
tail -1 $OUT/pytest_cs2ps.log
bash scripts/ab_multi.sh r03v/ab "libreacher.so libreacher_cs2.so libreacher_cs2b.so libreacher_cs2c.so libreacher_cs2ps.so" c4 c3

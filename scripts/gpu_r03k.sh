#!/bin/bash
# r03k3: partial-row NT stores always (ntws), + NT state stores (ntwsst), the runtime-threshold product, the previous commit
set -o pipefail
OUT=gpurun_out/r03k3; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/ab_multi.sh r03k3/ab "libreacher_prev.so libreacher.so libreacher_ntws.so libreacher_ntwsst.so" c5 c4 c3 c2

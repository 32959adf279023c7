#!/bin/bash
# r03n: standalone env kernel with non-temporal output stores (envnt) vs the product, alternating
set -o pipefail
OUT=gpurun_out/r03n; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in libreacher.so libreacher_envnt.so; do
    echo "## $lib rep $rep"
    RD_LIB=$lib timeout -k 10 120 python3 scripts/bench_env.py 16777216 4194304 1048576 || exit 1
  done
done

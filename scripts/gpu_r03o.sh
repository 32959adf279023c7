#!/bin/bash
# r03o: nt env stores (product) parity; nt loads in the env kernel (envntld) and the rollout's state loads (ldst);
# nt partial-row stores in the reference-student kernel (mlpnt); alternating A/B against the product
set -o pipefail
OUT=gpurun_out/r03o; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py tests/test_distill_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_env.log 2>&1 || { tail -30 $OUT/pytest_env.log; exit 1; }
tail -1 $OUT/pytest_env.log
for rep in 1 2; do
  for lib in libreacher.so libreacher_envntld.so; do
    echo "## env $lib rep $rep"
    RD_LIB=$lib timeout -k 10 120 python3 scripts/bench_env.py 16777216 4194304 1048576 || exit 1
  done
done
for rep in 1 2; do
  for lib in libreacher.so libreacher_mlpnt.so; do
    echo "## student_mlp $lib rep $rep"
    RD_LIB=$lib timeout -k 10 120 python3 scripts/bench_student_mlp.py 262144 1048576 || exit 1
  done
done
bash scripts/ab_multi.sh r03o/ab "libreacher.so libreacher_ldst.so" c5 c4

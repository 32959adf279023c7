#!/bin/bash
# r06zd: rdd_set_env_state's range check (check_state_kernel): the new test, then the GPU suite
set -o pipefail
OUT=gpurun_out/r06zd; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_distill_gpu.py -v -k "set_env_state or limit or isolated" --timeout 120 --timeout-method thread > $OUT/pytest_state.log 2>&1 || { tail -40 $OUT/pytest_state.log; exit 1; }
grep -E "rollout_range|passed|failed" $OUT/pytest_state.log | tail -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log

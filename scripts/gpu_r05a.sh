#!/bin/bash
# r05a: the K-step rollout launch (rdd_step_accum): parity vs the staged accumulation, and
# per-env-step times of c4 and its strong shards at K = 1 / staged K = 50 / fused K = 50
set -o pipefail
OUT=gpurun_out/r05a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_accum_gpu.py tests/test_distill_gpu.py -k "accum or k_step or k50 or helper" -v -s --timeout 240 --timeout-method thread > $OUT/pytest_accum.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|global|differ" $OUT/pytest_accum.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_env.log 2>&1 || { tail -30 $OUT/pytest_env.log; exit 1; }
tail -1 $OUT/pytest_env.log
timeout -k 10 400 python -u scripts/accum_probe.py --k 50 > $OUT/accum_probe.jsonl 2> $OUT/accum_probe.err || { tail $OUT/accum_probe.err; exit 1; }
cat $OUT/accum_probe.jsonl

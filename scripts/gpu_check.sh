#!/bin/bash
# One gpurun call: GPU parity tests, a bench line, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
# usage: bash scripts/gpu_check.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_stop() {  # $1 = exit code, $2 = step; test failures (1) continue, faults stop
  case "$1" in
    0|1) return 0 ;;
    *) echo "STOP after $2: exit $1"; exit "$1" ;;
  esac
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; ok_or_stop $rc pytest
timeout -k 10 420 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; [ $rc -eq 0 ] || { echo "bench exit $rc"; exit $rc; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --accum 0 --conv-steps 0 "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; [ $rc -eq 0 ] || { echo "rocprof exit $rc"; tail -20 "$OUT/prof.err"; exit $rc; }
find "$OUT/prof" -name '*stats*'
if [ "${PMC:-1}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"; do
    tagc=$(echo $c | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$tagc" -o run -- \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --accum 0 --conv-steps 0 "$@" > "$OUT/pmc_$tagc.json" 2> "$OUT/pmc_$tagc.err"
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $c exit $rc"; tail -5 "$OUT/pmc_$tagc.err"; exit $rc; }
  done
  python3 scripts/pmc_traffic.py "$OUT/pmc_rollout.json" rollout_kernel "$OUT"/pmc_*/
fi
echo DONE

#!/bin/bash
# r04r: helper layout with the two-phase image copy (helpers start on the teacher image) vs r04n's
# helper build (libreacher_hlp2.so): helper / distill / determinism tests, A/B, stamps
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_distill_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
RD_LIB=libreacher.so timeout -k 10 300 python3 -u scripts/det_check.py 6 c2s,c2e > $OUT/det.txt 2>&1 || { tail $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
for n in 4096; do RD_LIB=libreacher_stamps.so RD_SPLIT=1 RD_OWNERS=1 timeout -k 10 120 python3 scripts/stamps.py $n >> $OUT/stamps.jsonl 2>/dev/null || exit 1; done
run() {   # name lib rep args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for spec in "c2|--workload c2" "c2x|--workload c2 --f32-mode exact" "n2048|--workload c2 --envs-per-gpu 2048"; do
  name=${spec%%|*}; args=${spec#*|}
  for rep in 1 2 3; do
    for lib in libreacher.so libreacher_hlp2.so; do run $name $lib $rep $args; done
  done
done
cat $OUT/stamps.jsonl

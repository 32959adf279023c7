#!/bin/bash
# r04j: helper pairs on the register-staged image copy: determinism (new GPU test + det_check),
# bitwise vs the regcopy build of r04e (non-helper configs), step-time A/B vs regcopy
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_determinism_gpu.py -x -q --timeout 500 --timeout-method thread > $OUT/det_test.log 2>&1 || { tail -30 $OUT/det_test.log; exit 1; }
tail -2 $OUT/det_test.log
RD_LIB=libreacher.so timeout -k 10 300 python3 -u scripts/det_check.py 6 c4s,grid300,c5,c2s > $OUT/det.txt 2>&1 || { tail $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
for lib in libreacher.so libreacher_regcopy.so; do
  RD_LIB=$lib timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/bw_$lib.npz > $OUT/bw_$lib.log 2>&1 || { tail $OUT/bw_$lib.log; exit 1; }
done
python3 scripts/bitwise_ab.py --compare /tmp/bw_libreacher.so.npz /tmp/bw_libreacher_regcopy.so.npz | grep -E "False|ALL|differ"
run() {   # name lib rep args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for spec in "c2|--workload c2" "c4|--workload c4" "c5|--workload c5" "n2048|--workload c2 --envs-per-gpu 2048"; do
  name=${spec%%|*}; args=${spec#*|}
  for rep in 1 2; do
    for lib in libreacher.so libreacher_regcopy.so; do run $name $lib $rep $args; done
  done
done

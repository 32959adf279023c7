#!/bin/bash
# r04p: c5's producer with the split teacher and the bf16 student interleaved (product) vs the
# sequential forwards (libreacher_c5seq.so): bitwise, determinism, step-time A/B
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_c5seq.so; do
  RD_LIB=$lib timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/bw_$lib.npz > $OUT/bw_$lib.log 2>&1 || { tail $OUT/bw_$lib.log; exit 1; }
done
python3 scripts/bitwise_ab.py --compare /tmp/bw_libreacher.so.npz /tmp/bw_libreacher_c5seq.so.npz | grep -E "False|ALL|differ"
RD_LIB=libreacher.so timeout -k 10 300 python3 -u scripts/det_check.py 6 c5 > $OUT/det.txt 2>&1 || { tail $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
run() {   # name lib rep args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for rep in 1 2 3; do
  for lib in libreacher.so libreacher_c5seq.so; do run c5 $lib $rep --workload c5; done
done

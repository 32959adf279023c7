#!/bin/bash
# r03h: (1) the f32 student's consumer-side env step (libreacher_cp.so, RDD_PHYS=consumer; the
# consumer's dW1 SrcC-fenced, the producer has no f32 MFMA left): parity, determinism, A/B;
# (2) the reduce+Adam kernel without the student-image refresh (libreacher_nopack.so, timing
# only): what the refresh costs per step.
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT/ab; export TMPDIR=/tmp
RD_LIB=libreacher_cp.so RDD_PHYS=consumer timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_cp.log 2>&1 || { tail -40 $OUT/pytest_cp.log; exit 1; }
tail -1 $OUT/pytest_cp.log
RD_LIB=libreacher_cp.so RDD_PHYS=consumer timeout -k 10 300 python3 -u scripts/det_check.py 10 c4s,c2s,c3s > $OUT/det_cp.txt 2>&1 || { tail -20 $OUT/det_cp.txt; exit 1; }
echo "det cp: $(grep -c ' identical$' $OUT/det_cp.txt) identical of $(grep -c rep $OUT/det_cp.txt)"
run() {  # tag lib workload rep [env]
  env RD_LIB=$2 $5 timeout -k 10 120 python3 bench.py --workload $3 --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg \
    --accum 0 --conv-steps 0 > $OUT/ab/$3.$1.$4.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab/$3.$1.$4.json'));print('$3', '$1'.ljust(8), $4, 'value %.4g'%d['value'], 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for wl in c4 c3 c2; do
  for rep in 1 2; do
    run prod libreacher.so $wl $rep
    run cp libreacher_cp.so $wl $rep RDD_PHYS=consumer
    run nopack libreacher_nopack.so $wl $rep
  done
done
for rep in 1 2; do
  run prod libreacher.so c5 $rep
  run nopack libreacher_nopack.so c5 $rep
done

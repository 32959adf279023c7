#!/bin/bash
# Consumer-side env step with every physics transcendental's first reader held >= 5 wait
# states back (RD_TRANS_NOP build) vs the product: repeated-rollout reproducibility + c5/c4 speed.
OUT=gpurun_out/cptn; mkdir -p $OUT
RD_LIB=libreacher_transnop.so RDD_PHYS=consumer timeout -k 10 400 python3 -u scripts/det_check.py 40 c4s,c5 > $OUT/det_transnop.txt 2>&1 || exit 1
echo "transnop consumer identical $(grep -c identical $OUT/det_transnop.txt) of 80"
for wl in c5 c4; do
  for lib in libreacher.so libreacher_transnop.so; do
    for phys in producer consumer; do
      RD_LIB=$lib RDD_PHYS=$phys timeout -k 10 120 python3 bench.py --workload $wl --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/${wl}_${lib}_$phys.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.load(open('$OUT/${wl}_${lib}_$phys.json'));print('$wl $lib $phys', 'step_us %.2f'%(1e3*d['ms_per_step']))"
    done
  done
done

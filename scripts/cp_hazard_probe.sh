#!/bin/bash
# Consumer-side env step (RDD_PHYS=consumer) reproducibility under three builds: the product,
# -mllvm -amdgpu-mfma-vgpr-form (MFMA dst/srcC in VGPRs) and -mllvm -amdgpu-snop-padding=4
# (an s_nop 4 before every instruction: a wait-state bug would vanish).  DESIGN.md §3.
OUT=gpurun_out/cphaz; mkdir -p $OUT
for lib in libreacher.so libreacher_vgprform.so libreacher_snop.so; do
  RD_LIB=$lib RDD_PHYS=consumer timeout -k 10 300 python3 -u scripts/det_check.py 20 c5,c4s > $OUT/det_$lib.txt 2>&1 || exit 1
  echo "$lib identical $(grep -c identical $OUT/det_$lib.txt) of 40"
done
for lib in libreacher.so libreacher_vgprform.so; do
  for phys in producer consumer; do
    RD_LIB=$lib RDD_PHYS=$phys timeout -k 10 120 python3 bench.py --workload c5 --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/c5_${lib}_$phys.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$OUT/c5_${lib}_$phys.json'));print('c5 $lib $phys', 'step_us %.2f'%(1e3*d['ms_per_step']))"
  done
done

#!/bin/bash
# r06zg: the AMDGPU machine scheduler's strategy (-mllvm -amdgpu-sched-strategy=max-ilp / max-memory-clause,
# libreacher_ilp.so / libreacher_mmc.so; both ISAs hazard-clean by scripts/isa/check_isa.py) against the default
# (max-occupancy): alternating A/B
set -o pipefail
OUT=gpurun_out/r06zg; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher.so libreacher_ilp.so libreacher_mmc.so; do
    RD_LIB=$lib timeout -k 10 150 python3 scripts/ab_k1.py 2000 c2,c3,c4,c5,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

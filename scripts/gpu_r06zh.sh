#!/bin/bash
# r06zh: diagnostic -- what the env step costs inside the fused rollout: a build whose env step is a
# trivial update (libreacher_nophys.so, -DRD_DIAG_NOPHYS, never the product) against the product
set -o pipefail
OUT=gpurun_out/r06zh; mkdir -p $OUT
for r in 1 2 3; do
  for lib in libreacher.so libreacher_nophys.so; do
    RD_LIB=$lib timeout -k 10 150 python3 scripts/ab_k1.py 2000 c2,c3,c4,c5,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

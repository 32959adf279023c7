#!/bin/bash
# r06r: the bf16 student's dW2 on v_mfma_f32_32x32x16_bf16 (libreacher_b32.so)
# GPU suite on the variant (parity vs the f64 oracle / fixture at unchanged tolerances), then an
# alternating A/B against HEAD
set -o pipefail
OUT=gpurun_out/r06r; mkdir -p $OUT
RD_LIB=libreacher_b32.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_b32.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c5,k50_c5,c5x >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

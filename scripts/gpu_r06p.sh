#!/bin/bash
# r06p: the split consumer's dW2 on v_mfma_f32_32x32x16_bf16 (dw2_split32, libreacher_d32.so)
# GPU suite on the variant (parity vs the f64 oracle / fixture at unchanged tolerances), then an
# alternating A/B against HEAD
set -o pipefail
OUT=gpurun_out/r06p; mkdir -p $OUT
RD_LIB=libreacher_d32.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_d32.so; do
    RD_LIB=$lib timeout -k 10 120 python3 scripts/ab_k1.py 2000 c4,c3,c2,k50_32768,c3x >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

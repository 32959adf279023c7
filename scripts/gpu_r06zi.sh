#!/bin/bash
# r06zi: the producer loads the next group's env state one group ahead (libreacher_pf.so): bitwise
# fingerprints of both builds, the GPU suite on the variant, an alternating A/B against HEAD
set -o pipefail
OUT=gpurun_out/r06zi; mkdir -p $OUT
for lib in libreacher.so libreacher_pf.so; do
  RD_LIB=$lib timeout -k 10 300 python3 scripts/grad_hash.py 3 > $OUT/hash_$lib.json 2> $OUT/hash.err || { tail -20 $OUT/hash.err; exit 1; }
  cat $OUT/hash_$lib.json
done
RD_LIB=libreacher_pf.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lib in libreacher.so libreacher_pf.so; do
    RD_LIB=$lib timeout -k 10 150 python3 scripts/ab_k1.py 2000 c2,c3,c4,c5,k50_32768 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl
  done
done

#!/bin/bash
# r04g: which build's c4 is not reproducible (r04f: TC vs NO_TC differ in c4 only)
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher_tc.so libreacher_notc.so; do
  RD_LIB=$lib timeout -k 10 300 python3 -u scripts/det_check.py 8 c4s > $OUT/det_$lib.txt 2>&1 || { tail $OUT/det_$lib.txt; exit 1; }
  echo "$lib det: $(grep -c ' identical$' $OUT/det_$lib.txt) identical of $(grep -c rep $OUT/det_$lib.txt)"
  for r in 1 2; do
    RD_LIB=$lib timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/bw_$lib.$r.npz > $OUT/bw_$lib.$r.log 2>&1 || { tail $OUT/bw_$lib.$r.log; exit 1; }
  done
  python3 scripts/bitwise_ab.py --compare /tmp/bw_$lib.1.npz /tmp/bw_$lib.2.npz | grep -E "False|ALL|differ"
done
python3 scripts/bitwise_ab.py --compare /tmp/bw_libreacher_tc.so.1.npz /tmp/bw_libreacher_notc.so.1.npz | grep -E "False|ALL|differ"

#!/bin/bash
# r05c: the dW3 lanes-48-63 differences of the split K-step kernel: dW3 accumulation fenced /
# unpacked (RD_PK_FENCE), no SLP packing, against the product build
set -o pipefail
OUT=gpurun_out/r05c; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher_pkfence.so libreacher_noslp.so libreacher.so; do
  for cfg in "32768 7" "65536 5"; do
    RD_LIB=$lib timeout -k 10 120 python -u scripts/kstep_diag.py $cfg 4 >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r05c/diag.jsonl'):
    d=json.loads(l)
    print(d['lib'], d['n'], d['K'], [(r['digest'], '%.1e'%r['glob'], r['nbad'], r['bad_first'][:4], r.get('vs_first_n')) for r in d['runs']])
PY

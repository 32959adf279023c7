#!/bin/bash
# r05b: diagnosis of the split K-step kernel's gradient differences (one process per build)
set -o pipefail
OUT=gpurun_out/r05b; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_ksnores.so libreacher_ksfence.so libreacher_ksalways.so; do
  for cfg in "32768 7" "65536 5" "32768 1"; do
    RD_LIB=$lib timeout -k 10 120 python -u scripts/kstep_diag.py $cfg 3 >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r05b/diag.jsonl'):
    d=json.loads(l)
    print(d['lib'], d['n'], d['K'], [(r['digest'], r['state_equal'], '%.1e'%r['glob'], r['nbad'], r['bad_regions'], r.get('vs_first_n')) for r in d['runs']])
PY

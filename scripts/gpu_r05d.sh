#!/bin/bash
# r05d: cost of removing the packed dW3 accumulation (RD_PK_FENCE: scalar FMAs + fence;
# -fno-slp-vectorize: no SLP packing at all) vs the product, K = 1 and K = 50, alternating
set -o pipefail
OUT=gpurun_out/r05d; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
for lib in libreacher.so libreacher_pkfence.so libreacher_noslp.so; do
  RD_LIB=$lib timeout -k 10 200 python -u scripts/accum_probe.py --k 50 --sizes 262144,65536,32768 --opt-steps 6 > $OUT/ab_${lib}_$rep.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
  RD_LIB=$lib timeout -k 10 200 python -u scripts/accum_probe.py --k 50 --sizes 131072 --act student --dtype bf16 --opt-steps 6 >> $OUT/ab_${lib}_$rep.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r05d/ab_*.jsonl')):
    for l in open(f):
        d=json.loads(l)
        print(f.split('/')[-1][3:-6].ljust(26), d['envs'], d['dtype'], 'k1 %.2f fused %.2f staged %.2f' % (d['k1_us_per_env_step'], d['fused_us_per_env_step'], d['staged_us_per_env_step']))
PY

#!/bin/bash
# r04s: reduce_adam_kernel with every partial row of a thread loaded at once (nblk <= 256) vs the
# r04n product (libreacher_prevred.so): bitwise over bitwise_ab's cases, rocprof reduce time, step A/B
set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_prevred.so; do
  RD_LIB=$lib timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/bw_$lib.npz > $OUT/bw_$lib.log 2>&1 || { tail $OUT/bw_$lib.log; exit 1; }
done
python3 scripts/bitwise_ab.py --compare /tmp/bw_libreacher.so.npz /tmp/bw_libreacher_prevred.so.npz | grep -E "False|ALL|differ"
for lib in libreacher.so libreacher_prevred.so; do
  for wl in c2 c4; do
    RD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib.$wl -o run -- \
      python3 bench.py --workload $wl --steps 300 --warmup 100 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$lib.$wl.json 2>/dev/null || exit 1
    f=$(find $OUT/$lib.$wl -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
r=[x for x in rows if 'reduce_adam' in x['Name']][0]
print('$lib $wl reduce_avg_us %.2f min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
  done
done
run() {   # name lib rep args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']))"
}
for spec in "c2|--workload c2" "c4|--workload c4" "c3|--workload c3"; do
  name=${spec%%|*}; args=${spec#*|}
  for rep in 1 2 3; do
    for lib in libreacher.so libreacher_prevred.so; do run $name $lib $rep $args; done
  done
done

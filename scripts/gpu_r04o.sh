#!/bin/bash
# r04o: where reduce_adam_kernel's ~4.7 us go: the product vs a build without the student-image
# refresh (red1) vs one without the partial-row loads (red2) -- diagnostic builds, wrong results
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_red1.so libreacher_red2.so; do
  for wl in c2 c4; do
    RD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$lib.$wl -o run -- \
      python3 bench.py --workload $wl --steps 300 --warmup 100 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$lib.$wl.json 2>/dev/null || exit 1
    f=$(find $OUT/$lib.$wl -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,json
rows=list(csv.DictReader(open('$f')))
d=json.load(open('$OUT/$lib.$wl.json'))
r=[x for x in rows if 'reduce_adam' in x['Name']][0]; k=[x for x in rows if 'rollout_kernel' in x['Name']][0]
print('$lib $wl step_us %.2f reduce_avg_us %.2f min %.2f rollout_avg_us %.2f' % (1e3*d['ms_per_step'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(k['AverageNs'])/1e3))"
  done
done

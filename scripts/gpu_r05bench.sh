#!/bin/bash
# default bench line twice + rocm-smi clocks (box-variance check)
set -o pipefail
OUT=gpurun_out/r05bench; mkdir -p $OUT; export TMPDIR=/tmp
(rocm-smi --showclocks --showpower --showtemp 2>&1 | head -40) > $OUT/smi_before.txt || true
for i in 1 2; do
  timeout -k 10 600 python3 bench.py > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('value', d['value'], 'us/step', d['ms_per_step']*1e3, 'accum', d.get('accum',{}).get('us_per_env_step'))"
done
(rocm-smi --showclocks --showpower --showtemp 2>&1 | head -40) > $OUT/smi_after.txt || true
grep -i "sclk\|mclk\|power\|temp" $OUT/smi_after.txt | head -8

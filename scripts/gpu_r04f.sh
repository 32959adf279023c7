#!/bin/bash
# r04f: the pair's first-tile teacher forward on the consumer wave (TC) vs the r04e product
# (libreacher_notc.so = -DRD_NO_TC): bitwise A/B over scripts/bitwise_ab.py's cases, then
# alternating step-time A/B (1000 steps after 300 warm-up) on c2, c3, c4, c5, c4's 8-GPU shard
# (32,768 envs) and c4 exact.
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT; export TMPDIR=/tmp
RD_LIB=libreacher.so timeout -k 10 300 python3 -u scripts/bitwise_ab.py $OUT/tc.npz > $OUT/bw_tc.log 2>&1 || { tail $OUT/bw_tc.log; exit 1; }
RD_LIB=libreacher_notc.so timeout -k 10 300 python3 -u scripts/bitwise_ab.py $OUT/notc.npz > $OUT/bw_notc.log 2>&1 || { tail $OUT/bw_notc.log; exit 1; }
python3 scripts/bitwise_ab.py --compare $OUT/tc.npz $OUT/notc.npz | tail -12
run() {   # name lib args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for spec in "c2|--workload c2" "c3|--workload c3" "c4|--workload c4" "c5|--workload c5" "s32k|--workload c4 --envs-per-gpu 32768" "c4x|--workload c4 --f32-mode exact"; do
  name=${spec%%|*}; args=${spec#*|}
  for rep in 1 2 3; do
    for lib in libreacher.so libreacher_notc.so; do run $name $lib $rep $args; done
  done
done

#!/bin/bash
# r04h: helper pairs (MD_HELPER: pairs 2, 3 run pairs 0, 1's teacher forwards on the other SIMDs
# at one 16-env tile per group) vs the r04e product (libreacher_notc.so); determinism of both
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libreacher.so libreacher_notc.so; do
  for r in 1 2; do
    RD_LIB=$lib timeout -k 10 300 python3 -u scripts/bitwise_ab.py /tmp/bw_$lib.$r.npz > $OUT/bw_$lib.$r.log 2>&1 || { tail $OUT/bw_$lib.$r.log; exit 1; }
  done
  echo "== $lib run 1 vs run 2"; python3 scripts/bitwise_ab.py --compare /tmp/bw_$lib.1.npz /tmp/bw_$lib.2.npz | grep -E "False|ALL|differ"
done
echo "== helper vs r04e"; python3 scripts/bitwise_ab.py --compare /tmp/bw_libreacher.so.1.npz /tmp/bw_libreacher_notc.so.1.npz | grep -E "False|ALL|differ"
run() {   # name lib rep args...
  local name=$1 lib=$2 rep=$3; shift 3
  RD_LIB=$lib timeout -k 10 120 python3 bench.py "$@" --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/$name.$lib.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/$name.$lib.$rep.json'));print('$name', '$lib', $rep, 'step_us %.2f'%(1e3*d['ms_per_step']), 'launch_us %.2f'%d['roofline']['launch_us'])"
}
for spec in "c2|--workload c2" "c2x|--workload c2 --f32-mode exact" "c5|--workload c5" "n2048|--workload c2 --envs-per-gpu 2048" "n8192|--workload c2 --envs-per-gpu 8192"; do
  name=${spec%%|*}; args=${spec#*|}
  for rep in 1 2 3; do
    for lib in libreacher.so libreacher_notc.so; do run $name $lib $rep $args; done
  done
done

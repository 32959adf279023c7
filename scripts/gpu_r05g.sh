#!/bin/bash
# r05g: the default bench line (N = 1) and the two-rank rehearsal of the N > 1 path on one GPU
# (gloo process group, RD_BENCH_ONE_DEVICE: both ranks on cuda:0; RCCL refuses two ranks on one
# device, so the native xGMI exchange is the bound collective), each with its wall time
set -o pipefail
OUT=gpurun_out/r05g; mkdir -p $OUT; export TMPDIR=/tmp
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
t1=$(date +%s.%N)
echo "bench default wall $(python3 -c "print($t1 - $t0)") s"
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('value', d['value'], 'us/step', d['ms_per_step']*1e3, 'frac', d['roofline']['frac'], 'accum', d.get('accum',{}).get('fused'), 'k', d.get('strong_projection',{}).get('shards',{}).get('8',{}).get('k'))"
t0=$(date +%s.%N)
RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo RD_COMM=xgmi timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/n2.out 2> $OUT/n2.err || { tail -30 $OUT/n2.err; exit 1; }
t1=$(date +%s.%N)
echo "n2 rehearsal wall $(python3 -c "print($t1 - $t0)") s"
grep '^{' $OUT/n2.out | tail -1 > $OUT/n2_rehearsal.json
python3 - <<PY
import json
d = json.load(open("$OUT/n2_rehearsal.json"))
d["rehearsal"] = {"wall_s": $t1 - $t0, "command": "RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo RD_COMM=xgmi torchrun --nproc-per-node 2 bench.py --gpus 2 --steps 20 --warmup 5", "box": "one MI355X, both ranks on cuda:0"}
json.dump(d, open("$OUT/n2_rehearsal.json", "w"))
print({k: d.get(k) for k in ("value", "ms_per_step", "exchange", "strong_scaling", "accum", "replicas_identical")})
PY

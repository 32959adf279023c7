#!/bin/bash
# r05v: the two-rank rehearsal of the N > 1 path on one GPU (gloo group, both ranks on cuda:0,
# native xGMI exchange) on the end-of-round build, with its wall time; then the LSTM GPU tests
set -o pipefail
OUT=gpurun_out/r05v; mkdir -p $OUT; export TMPDIR=/tmp
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
print({k: d.get(k) for k in ("value", "ms_per_step", "replicas_identical")}, d["exchange"].get("xgmi_view", {}).get("consistent"), d["strong_scaling"]["accum"]["value"])
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_student_lstm_gpu.py tests/test_c1_gpu.py > $OUT/pytest_lstm.log 2>&1 || { tail -30 $OUT/pytest_lstm.log; exit 1; }
tail -1 $OUT/pytest_lstm.log

#!/bin/bash
# r03a: GPU suite + smoke after the hygiene / exchange-safety changes, then the default bench
# line and the N=2 one-GPU rehearsal (gloo group; RCCL reports unavailable, xGMI over IPC).
set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03a || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
tail -c 600 $OUT/bench_default.json
RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --accum 0 --conv-steps 0 \
  --workload c3 > $OUT/n2.json 2> $OUT/n2.err || { tail -20 $OUT/n2.err; exit 1; }
grep -o '"exchange": {[^}]*}' $OUT/n2.json; grep -o '"collective": "[^"]*"' $OUT/n2.json

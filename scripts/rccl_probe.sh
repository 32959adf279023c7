#!/bin/bash
# GPU probe of the native RCCL path: the comm tests, then bench.py at N=2 with both ranks
# on cuda:0 over RCCL (if RCCL refuses two ranks on one device, that is reported and the
# script stops), then the same with torch's collective for comparison.
OUT=gpurun_out/rccl; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_dist_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
for c in rccl torch; do
  RD_COMM=$c RD_BENCH_ONE_DEVICE=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --accum 0 --conv-steps 0 \
    --workload c3 > $OUT/n2_$c.json 2> $OUT/n2_$c.err
  rc=$?; tail -2 $OUT/n2_$c.json; grep -i "error\|refus\|duplicate" $OUT/n2_$c.err | head -5; [ $rc -eq 0 ] || exit $rc
done

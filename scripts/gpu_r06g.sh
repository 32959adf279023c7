#!/bin/bash
# r06g: the N > 1 path at 4 and 8 ranks on one GPU: the xGMI tests at world
# sizes 2/4/8, then the bench's N = 4 and N = 8 rehearsals (gloo group, every rank on cuda:0,
# native xGMI exchange bound) with their wall times
set -o pipefail
OUT=gpurun_out/r06g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $OUT/pytest_xgmi.log 2>&1 || { tail -40 $OUT/pytest_xgmi.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" $OUT/pytest_xgmi.log | tail -8
for N in 4 8; do
  t0=$(date +%s.%N)
  RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo RD_COMM=xgmi timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2953$N bench.py --gpus $N --steps 20 --warmup 5 > $OUT/n$N.out 2> $OUT/n$N.err || { tail -30 $OUT/n$N.err; exit 1; }
  t1=$(date +%s.%N)
  grep '^{' $OUT/n$N.out | tail -1 > $OUT/n${N}_rehearsal.json
  python3 - $OUT/n${N}_rehearsal.json $N $t0 $t1 <<'PY'
import json, sys
p, N, t0, t1 = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])
d = json.load(open(p))
d["rehearsal"] = {"wall_s": t1 - t0, "command": f"RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo RD_COMM=xgmi torchrun --nproc-per-node {N} bench.py --gpus {N} --steps 20 --warmup 5",
                  "box": f"one MI355X, all {N} ranks on cuda:0 (the per-rank step runs {N}x serialised on the one GPU)"}
json.dump(d, open(p, "w"))
x = d["exchange"]
print(N, "wall %.1f s" % (t1 - t0), "value %.4g" % d["value"], "replicas", d["replicas_identical"], "xgmi_us", x.get("xgmi_us"),
      "view", {k: x.get("xgmi_view", {}).get(k) for k in ("consistent", "distinct_devices")}, [r["count"] for r in x.get("xgmi_view", {}).get("ranks", [])],
      "rccl", str(x.get("rccl_us"))[:60], "strong", d["strong_scaling"]["replicas_identical"], "strong_accum", "accum" in d["strong_scaling"],
      d["strong_scaling"].get("accum", {}).get("replicas_identical"))
PY
done

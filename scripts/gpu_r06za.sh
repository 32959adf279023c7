#!/bin/bash
# r06za: HEAD after the measured xGMI communicator's 60 s exchange timeout -- the N = 8 rehearsal
# (gloo group, all ranks on cuda:0, native xGMI exchange) and the default N = 1 bench line
set -o pipefail
OUT=gpurun_out/r06za; mkdir -p $OUT; export TMPDIR=/tmp
N=8
t0=$(date +%s.%N)
RD_BENCH_ONE_DEVICE=1 RD_DIST_BACKEND=gloo RD_COMM=xgmi timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus $N --steps 20 --warmup 5 > $OUT/n$N.out 2> $OUT/n$N.err || { tail -30 $OUT/n$N.err; exit 1; }
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
      "strong", d["strong_scaling"]["replicas_identical"], "strong_accum", d["strong_scaling"].get("accum", {}).get("replicas_identical"))
PY
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print($t1 - $t0)") s"
python3 - $OUT/bench_default.json <<'P'
import json, sys
b = json.load(open(sys.argv[1]))
print("value %.4g ms %.4f launch %.2f frac %.3f issue %.3f | exact %.4g launch %.2f" % (b["value"], b["ms_per_step"], b["roofline"]["launch_us"], b["roofline"]["frac"], b["roofline_issue"]["frac"], b["other_f32_mode"]["value"], b["other_f32_mode"]["launch_us"]))
print("workloads", {k: {kk: round(vv["us_per_env_step"], 2) for kk, vv in v.items() if isinstance(vv, dict)} for k, v in b["workloads"].items() if isinstance(v, dict)})
P

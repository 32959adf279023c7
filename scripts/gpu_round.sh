#!/bin/bash
# One GPU session: full GPU suite, smoke, then bench + rocprof + PMC per workload.
# usage: scripts/gpu_round.sh TAG [workload ...]   (run from the repo root on the GPU box)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for wl in "$@"; do
  bash scripts/profile_workload.sh $TAG/$wl $wl > /dev/null || { echo "profile $wl failed"; exit 1; }
  python3 - $OUT/$wl <<'P'
import json, sys, csv, glob
d = sys.argv[1]
b = json.load(open(d + "/bench.json"))
print(d, "value %.4g" % b["value"], "ms/step %.4f" % b["ms_per_step"], "launch_us %.1f" % b["roofline"]["launch_us"],
      "frac %.3f" % b["roofline"]["frac"], "other", {k: round(v, 4) if isinstance(v, float) else v for k, v in b.get("other_f32_mode", {}).items()})
for f in glob.glob(d + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout_kernel" in r["Name"] or "reduce_adam" in r["Name"]:
            print("  rocprof", r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
P
done

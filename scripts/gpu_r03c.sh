#!/bin/bash
# r03c: the bf16-student kernels step the envs on the consumer (SrcC-fenced teacher layer 1):
# GPU suite, reproducibility of the product (20 repeated rollouts per config), c5 / c4 bench
# lines with rocprof kernel stats.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python3 -u scripts/det_check.py 20 c5,c5e,c4s > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
for wl in c5 c4; do
  bash scripts/profile_workload.sh r03c/$wl $wl > /dev/null || { echo "profile $wl failed"; exit 1; }
done
python3 - <<'P'
import json, csv, glob
for wl in ("c5", "c4"):
    d = f"gpurun_out/r03c/{wl}"
    b = json.load(open(d + "/bench.json"))
    print(wl, "value %.4g" % b["value"], "ms/step %.4f" % b["ms_per_step"], "launch_us %.1f" % b["roofline"]["launch_us"],
          "frac %.3f" % b["roofline"]["frac"])
    for f in glob.glob(d + "/prof/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rollout_kernel" in r["Name"] or "reduce_adam" in r["Name"]:
                print("  rocprof", r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
P

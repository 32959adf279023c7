#!/bin/bash
# r03z: the final round-3 product (consumer + producer interleave schedules, nt row in the bf16-student kernels):
# GPU suite, smoke, determinism, A/B against the previous commit, then per workload the bench line + rocprof
# kernel stats + PMC passes, and the driver-style default line
set -o pipefail
OUT=gpurun_out/r03z; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03z || exit 1
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s,c4e > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_multi.sh r03z/ab "libreacher_prev.so libreacher.so" c4 c5 c3 c2 || exit 1
for wl in c4 c5 c3 c2; do
  bash scripts/profile_workload.sh r03z/$wl $wl > /dev/null || { echo "profile $wl failed"; exit 1; }
done
python3 - <<'P'
import json, csv, glob
for wl in ("c4", "c5", "c3", "c2"):
    d = f"gpurun_out/r03z/{wl}"
    b = json.load(open(d + "/bench.json"))
    print(wl, "value %.4g" % b["value"], "ms/step %.4f" % b["ms_per_step"], "launch_us %.1f" % b["roofline"]["launch_us"],
          "frac %.3f" % b["roofline"]["frac"])
    for f in glob.glob(d + "/prof/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rollout_kernel" in r["Name"] or "reduce_adam" in r["Name"]:
                print("  rocprof", r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
    p = json.load(open(d + "/pmc_rollout.json"))
    a = p["avg"]
    print("  pmc hbm_bytes %.4g" % p["hbm_bytes_per_launch"], "write %.4g" % p["write_bytes"], "valu %.4g mfma %.4g busy %.4g" % (
        float(a["SQ_INSTS_VALU"]), float(a["SQ_INSTS_MFMA"]), float(a["SQ_VALU_MFMA_BUSY_CYCLES"])))
P
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench_driver_style.err || { tail -5 $OUT/bench_driver_style.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver_style.json')); print('driver-style', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_issue']['frac'])"

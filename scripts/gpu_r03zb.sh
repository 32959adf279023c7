#!/bin/bash
# r03zb: the final library (+ the teacher's layer-2 schedule): GPU suite, smoke, determinism, A/B vs the previous
# commit, the c5 profile (bench + rocprof + PMC) and the driver-style default line
set -o pipefail
OUT=gpurun_out/r03zb; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03zb || exit 1
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s,c5e > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_multi.sh r03zb/ab "libreacher_prev.so libreacher.so" c5 c4 || exit 1
bash scripts/profile_workload.sh r03zb/c5 c5 > /dev/null || { echo "profile c5 failed"; exit 1; }
python3 - <<'P'
import json, csv, glob
d = "gpurun_out/r03zb/c5"
b = json.load(open(d + "/bench.json"))
print("c5", "value %.4g" % b["value"], "ms/step %.4f" % b["ms_per_step"], "launch_us %.1f" % b["roofline"]["launch_us"], "frac %.3f" % b["roofline"]["frac"])
for f in glob.glob(d + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout_kernel" in r["Name"] or "reduce_adam" in r["Name"]:
            print("  rocprof", r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
p = json.load(open(d + "/pmc_rollout.json")); a = p["avg"]
print("  pmc hbm_bytes %.4g" % p["hbm_bytes_per_launch"], "valu %.4g mfma %.4g busy %.4g" % (float(a["SQ_INSTS_VALU"]), float(a["SQ_INSTS_MFMA"]), float(a["SQ_VALU_MFMA_BUSY_CYCLES"])))
P
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench_driver_style.err || { tail -5 $OUT/bench_driver_style.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver_style.json')); print('driver-style', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_issue']['frac'])"

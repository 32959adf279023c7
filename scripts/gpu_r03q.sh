#!/bin/bash
# r03q: profile of the product after the nt partial row / nt env stores: per workload the bench line, the
# rocprofv3 kernel stats and the FETCH/WRITE/SQ PMC passes (scripts/profile_workload.sh), then the
# driver-style default line (python bench.py --steps 20 --warmup 5) and the env roofline micro-benchmark
set -o pipefail
OUT=gpurun_out/r03q; mkdir -p $OUT; export TMPDIR=/tmp
for wl in c4 c5 c3 c2; do
  bash scripts/profile_workload.sh r03q/$wl $wl > /dev/null || { echo "profile $wl failed"; exit 1; }
done
python3 - <<'P'
import json, csv, glob
for wl in ("c4", "c5", "c3", "c2"):
    d = f"gpurun_out/r03q/{wl}"
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
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_env']['achieved'])"

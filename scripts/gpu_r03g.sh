#!/bin/bash
# r03g: the product with dW2 / both nets' layer 1 on split bf16 MFMAs (slot-carried dW1 inputs,
# single-buffered producer scratch): GPU suite, smoke, determinism, A/B against the previous
# commit's library (libreacher_prev.so), then the c4 and c5 bench lines with rocprof kernel
# stats and the FETCH/WRITE/SQ PMC passes.
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c4e,c5,c2s > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_libs.sh r03g/ab libreacher_prev.so libreacher.so c4 c5 c3 c2 || exit 1
for lib in libreacher_prev.so libreacher.so; do
  RD_LIB=$lib timeout -k 10 120 python3 bench.py --workload c4 --f32-mode exact --steps 1000 --warmup 300 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/ab/c4e.$lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab/c4e.$lib.json'));print('c4 exact', '$lib', 'step_us %.2f'%(1e3*d['ms_per_step']))"
done
for wl in c4 c5; do
  bash scripts/profile_workload.sh r03g/$wl $wl > /dev/null || { echo "profile $wl failed"; exit 1; }
done
python3 - <<'P'
import json, csv, glob
for wl in ("c4", "c5"):
    d = f"gpurun_out/r03g/{wl}"
    b = json.load(open(d + "/bench.json"))
    print(wl, "value %.4g" % b["value"], "ms/step %.4f" % b["ms_per_step"], "launch_us %.1f" % b["roofline"]["launch_us"],
          "frac %.3f" % b["roofline"]["frac"])
    for f in glob.glob(d + "/prof/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rollout_kernel" in r["Name"] or "reduce_adam" in r["Name"]:
                print("  rocprof", r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
    p = json.load(open(d + "/pmc_rollout.json"))
    a = p["avg"]
    print("  pmc hbm_bytes %.4g" % p["hbm_bytes_per_launch"], "valu %.4g mfma %.4g busy %.4g" % (
        float(a["SQ_INSTS_VALU"]), float(a["SQ_INSTS_MFMA"]), float(a["SQ_VALU_MFMA_BUSY_CYCLES"])))
P

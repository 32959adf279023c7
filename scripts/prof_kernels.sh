#!/bin/bash
# rocprofv3 kernel summary of one workload's timed loop: prof_kernels.sh TAG WORKLOAD [extra bench args]
TAG=$1; WL=$2; shift 2; OUT=gpurun_out/$TAG/$WL; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --workload $WL "$@" --steps 400 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/prof.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
f = glob.glob(out + "/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(out, r["Name"][:60], r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
b = [l for l in open(out + "/prof.log") if l.startswith("{")]
if b:
    d = json.loads(b[-1]); print(out, "step_us %.2f" % (1e3 * d["ms_per_step"]))
PY

#!/bin/bash
# r06zz: final validation of the committed tree -- GPU suite, smoke(), the default bench line (as the
# driver runs it) and a rocprofv3 kernel-trace summary of the headline workload
set -o pipefail
OUT=gpurun_out/r06zz; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print($t1 - $t0)") s"
python3 - $OUT/bench_default.json <<'P'
import json, sys
b = json.load(open(sys.argv[1]))
print("value %.4g ms %.4f launch %.2f frac %.3f | exact %.4g launch %.2f | env %.0f GB/s" % (b["value"], b["ms_per_step"], b["roofline"]["launch_us"], b["roofline"]["frac"], b["other_f32_mode"]["value"], b["other_f32_mode"]["launch_us"], b["roofline_env"]["achieved"]))
print("workloads", {k: {kk: round(vv["us_per_env_step"], 2) for kk, vv in v.items() if isinstance(vv, dict)} for k, v in b["workloads"].items() if isinstance(v, dict)})
P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --workload c4 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection --no-workloads > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/c4_kernel_stats.csv; head -3 $OUT/c4_kernel_stats.csv | cut -c1-200
find $OUT/prof -name "*kernel_trace.csv" -delete

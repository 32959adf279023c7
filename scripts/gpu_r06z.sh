#!/bin/bash
# r06z: end-of-round validation at HEAD -- the GPU suite, smoke(), and the default bench line (as
# the driver runs them), with the bench's wall time
set -o pipefail
OUT=gpurun_out/r06z; mkdir -p $OUT
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
print("value %.4g ms %.4f launch %.2f frac %.3f | exact %.4g launch %.2f | accum %.4g" % (b["value"], b["ms_per_step"], b["roofline"]["launch_us"], b["roofline"]["frac"], b["other_f32_mode"]["value"], b["other_f32_mode"]["launch_us"], b["accum"]["value"]))
print("workloads", {k: {kk: round(vv["us_per_env_step"], 2) for kk, vv in v.items() if isinstance(vv, dict)} for k, v in b["workloads"].items() if isinstance(v, dict)})
print("legs", json.dumps(b.get("student_mse_legs"))[:1500])
print("env", round(b["roofline_env"]["achieved"]), "cpu", b["cpu_baseline"]["value"], "ppo", b["teacher_ppo"]["iter_ms"])
P

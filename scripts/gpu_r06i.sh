#!/bin/bash
# r06i: PPO tests (the committed teacher's return) and the full default bench line (all legs,
# the new workloads and convergence_ppo_teacher blocks), with its wall time
set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ppo_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ppo.log 2>&1 || { tail -30 $OUT/pytest_ppo.log; exit 1; }
tail -1 $OUT/pytest_ppo.log
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print($t1 - $t0)") s"
python3 - $OUT/bench.json <<'P'
import json, sys
b = json.load(open(sys.argv[1]))
print("value %.4g ms %.4f launch %.2f frac %.3f exact_launch %.2f" % (b["value"], b["ms_per_step"], b["roofline"]["launch_us"], b["roofline"]["frac"], b["other_f32_mode"]["launch_us"]))
pt = b["convergence_ppo_teacher"]
print("ppo teacher", pt["teacher"]["return_mean_this_run"])
for k in ("convergence", "convergence_small_batch", "convergence_reference_driver"):
    c = pt[k]; print(" ", k, {x: c.get(x) for x in ("envs_total", "opt_steps_to_target", "env_steps_to_target", "within_env_step_budget", "student_mse_final", "seconds")})
for k in ("convergence", "convergence_small_batch", "convergence_reference_driver"):
    c = b[k] if k != "convergence_reference_driver" else b[k]; print(" synth", k, {x: c.get(x) for x in ("env_steps_to_target", "within_env_step_budget", "student_mse_final")})
print("workloads", {k: {kk: round(vv["us_per_env_step"], 2) for kk, vv in v.items() if isinstance(vv, dict)} for k, v in b["workloads"].items() if isinstance(v, dict)})
P

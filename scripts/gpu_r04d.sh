#!/bin/bash
# r04d: the product with the LDS-DMA rollout image and the 16-B staged env step: full GPU suite + smoke,
# env-kernel A/B vs the 4-B-per-lane step (libreacher_envold.so), default bench line + rocprof of c4
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_env_gpu.py tests/test_rows_gpu.py tests/test_split_gpu.py tests/test_student_lstm_gpu.py tests/test_student_mlp_gpu.py tests/test_xgmi_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for rep in 1 2; do for lib in libreacher_envold.so libreacher.so; do
  echo "== $lib $rep" >> $OUT/env_ab.jsonl
  RD_LIB=$lib timeout -k 10 120 python3 scripts/bench_env.py 1048576 4194304 16777216 >> $OUT/env_ab.jsonl 2>&1 || exit 1
done; done
grep -v amdgpu.ids $OUT/env_ab.jsonl
timeout -k 10 900 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 - $OUT/bench_default.json <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.4g ms/step %.4f frac %.3f fixed %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["frac_fixed_basis"]))
print("env", {k: d["roofline_env"][k] for k in ("achieved", "frac", "frac_of_measured_copy")})
print("strong", json.dumps(d.get("strong_projection"))[:1500])
P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 --fixture-steps 0 --no-strong-projection > $OUT/c4prof.log 2>&1 || exit 1
find $OUT/c4prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {}'

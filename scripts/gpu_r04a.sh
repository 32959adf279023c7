#!/bin/bash
# r04a: tightened parity suite (per-entry gradient bounds, per-env isolation, per-component state), smoke,
# and the reference student's fenced weight gradient vs the unfenced build (libreacher_prevmlp.so)
set -o pipefail
OUT=gpurun_out/${TAG:-r04a}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for lib in libreacher_prevmlp.so libreacher.so libreacher_prevmlp.so libreacher.so; do
  echo "== $lib" >> $OUT/student_mlp_ab.jsonl
  RD_LIB=$lib timeout -k 10 120 python3 scripts/bench_student_mlp.py 4096 65536 262144 1048576 >> $OUT/student_mlp_ab.jsonl 2>&1 || exit 1
done
grep -v cpu $OUT/student_mlp_ab.jsonl | python3 -c "
import sys, json
lib = None
for l in sys.stdin:
    if l.startswith('=='): lib = l.split()[1]; continue
    d = json.loads(l); print(lib, d['rows'], 'step_us %.1f' % d['step_us'])"
timeout -k 10 900 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 - $OUT/bench_default.json <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.4g ms/step %.4f frac %.3f fixed %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["frac_fixed_basis"]))
print("env", {k: d["roofline_env"][k] for k in ("achieved", "frac", "frac_of_measured_copy")}, d["roofline_env"].get("copy_ceiling"))
print("strong", json.dumps(d.get("strong_projection")))
print("fixture", json.dumps(d.get("convergence_fixture")))
P

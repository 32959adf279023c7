set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_distill_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02b/pytest_split.log 2>&1 || { tail -30 gpurun_out/r02b/pytest_split.log; exit 1; }
tail -3 gpurun_out/r02b/pytest_split.log
for m in exact split; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --f32-mode $m --no-cpu-baseline --conv-steps 0 --accum 0 > gpurun_out/r02b/c4_$m.json 2> gpurun_out/r02b/c4_$m.err || exit 1
  timeout -k 10 200 python bench.py --workload c5 --steps 200 --warmup 20 --f32-mode $m --no-cpu-baseline --conv-steps 0 --accum 0 > gpurun_out/r02b/c5_$m.json 2> gpurun_out/r02b/c5_$m.err || exit 1
done
python - <<'P'
import json
for w in ("c4","c5"):
    for m in ("exact","split"):
        d=json.load(open(f"gpurun_out/r02b/{w}_{m}.json"))
        print(w, m, "%.3e"%d["value"], "ms/step %.4f"%d["ms_per_step"], "launch_us %.1f"%d["roofline"]["launch_us"])
P

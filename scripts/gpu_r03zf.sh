#!/bin/bash
# r03zf: final library (producer pattern with 3 VALU per MFMA): GPU suite, smoke, determinism, c4 bench line + rocprof,
# driver-style default line
set -o pipefail
OUT=gpurun_out/r03zf; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03zf || exit 1
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s,c4e > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
bash scripts/ab_multi.sh r03zf/ab "libreacher_prev.so libreacher.so" c4 c2 || exit 1
timeout -k 10 300 python3 bench.py --workload c4 --no-cpu-baseline > $OUT/c4_bench.json 2> $OUT/c4_bench.err || exit 1
export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > $OUT/c4prof.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench_driver_style.err || { tail -5 $OUT/bench_driver_style.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver_style.json')); print('driver-style', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_issue']['frac'])"
python3 -c "import json; d=json.load(open('$OUT/c4_bench.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['roofline']['frac'])"

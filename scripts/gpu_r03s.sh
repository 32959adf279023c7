#!/bin/bash
# r03s: the round-3 library as committed (nt partial row, nt env outputs): full GPU suite, smoke,
# determinism, the driver-style default line (python bench.py --steps 20 --warmup 5, with the CPU baseline)
set -o pipefail
OUT=gpurun_out/r03s; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_round.sh r03s || exit 1
timeout -k 10 400 python3 -u scripts/det_check.py 10 c4s,c5,c3s,c2s,c4e > $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 1; }
echo "det: $(grep -c ' identical$' $OUT/det.txt) identical of $(grep -c rep $OUT/det.txt)"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_style.json 2> $OUT/bench_driver_style.err || { tail -5 $OUT/bench_driver_style.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver_style.json')); print('driver-style', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_issue']['frac'], d['cpu_baseline']['value'])"

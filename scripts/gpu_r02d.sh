mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
(RD_LIB=libreacher_stamps.so RD_SPLIT=1 timeout -k 10 60 python scripts/stamps.py 262144 && RD_LIB=libreacher_stamps.so RD_WL=c5 RD_SPLIT=1 timeout -k 10 60 python scripts/stamps.py 131072 && RD_LIB=libreacher_stamps.so RD_WL=c5 RD_SPLIT=0 timeout -k 10 60 python scripts/stamps.py 131072) > gpurun_out/r02d/stamps.jsonl 2>/dev/null || exit 1
cat gpurun_out/r02d/stamps.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02d/prof_c4 -o run -- python3 bench.py --workload c4 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > gpurun_out/r02d/c4.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02d/prof_c5 -o run -- python3 bench.py --workload c5 --steps 100 --warmup 200 --no-cpu-baseline --no-exact-leg --accum 0 --conv-steps 0 > gpurun_out/r02d/c5.json 2>&1 || exit 1
grep -h "rollout_kernel\|reduce_adam" gpurun_out/r02d/prof_c*/run_kernel_stats.csv | cut -d, -f1-4,6,7
grep -h '"metric"' gpurun_out/r02d/c4.json gpurun_out/r02d/c5.json | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'], d['value'], d['roofline']['launch_us'])"

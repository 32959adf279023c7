#!/bin/bash
# r03p: eager per-step launches vs a HIP graph of 200 steps, per workload
set -o pipefail
OUT=gpurun_out/r03p; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/graph_vs_eager.py c2 c5 c3 c4 | tee $OUT/graph_vs_eager.jsonl

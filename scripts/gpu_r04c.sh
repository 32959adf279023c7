#!/bin/bash
# r04c: r04a's validation (suite, smoke, student-MLP fence A/B, default bench with the new legs), then the
# LDS-DMA image fill A/B (libreacher_imgdma.so) at c2/c3/c4/c5 and stamp breakdowns at c2, the 32,768-env
# shard, c3 and c5 (libreacher_stamps.so)
set -o pipefail
export TMPDIR=/tmp
TAG=r04c bash scripts/gpu_r04a.sh || exit 1
OUT=gpurun_out/r04c
bash scripts/ab_libs.sh r04c/ab libreacher.so libreacher_imgdma.so c2 c3 c5 c4 > $OUT/ab_imgdma.txt 2>&1 || { cat $OUT/ab_imgdma.txt; exit 1; }
cat $OUT/ab_imgdma.txt
for n in 4096 32768 65536; do
  RD_SPLIT=1 RD_LIB=libreacher_stamps.so timeout -k 10 120 python3 scripts/stamps.py $n >> $OUT/stamps.jsonl 2>&1 || exit 1
done
RD_WL=c5 RD_SPLIT=1 RD_LIB=libreacher_stamps.so timeout -k 10 120 python3 scripts/stamps.py 131072 >> $OUT/stamps.jsonl 2>&1 || exit 1
tail -c 3000 $OUT/stamps.jsonl

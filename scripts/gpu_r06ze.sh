#!/bin/bash
# r06ze: the SQ counters this rocprofv3 offers on gfx950 (for an LDS / wait-state pass)
set -o pipefail
OUT=gpurun_out/r06ze; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 5 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || { tail -20 $OUT/avail.txt; exit 1; }
grep -oE "\bSQ_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/sq_names.txt
wc -l $OUT/sq_names.txt
grep -E "LDS|WAIT|BANK|ACTIVE_INST|INST_CYCLES|BUSY" $OUT/sq_names.txt | tr '\n' ' '

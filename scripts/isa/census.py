#!/usr/bin/env python3
"""Instruction census of one kernel's ISA between the RD_STAMPS markers (s_memtime):
usage: census.py FILE.s SYMBOL_SUBSTRING.  Counts per segment: VALU (non-MFMA v_*), MFMA,
transcendental (v_exp/v_rcp/v_sin/v_cos/v_log/v_sqrt), LDS (ds_*), global/buffer memory, SALU,
branches.  Build: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -DRD_STAMPS."""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and sym in l.split(":")[0] and ":" in l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
seg, segs = None, []


def new(label):
    return {"at": label, "valu": 0, "mfma": 0, "trans": 0, "lds": 0, "vmem": 0, "scr": 0, "salu": 0, "br": 0, "labels": []}


seg = new(start)
for i in range(start, end + 1):
    l = lines[i].strip()
    if not l or l.startswith(";") or l.startswith("."):
        continue
    if l.endswith(":"):
        seg["labels"].append(l[:-1])
        continue
    op = l.split()[0]
    if op == "s_memtime":
        segs.append(seg)
        seg = new(i)
        continue
    if op.startswith("v_mfma"):
        seg["mfma"] += 1
    elif op.startswith("v_"):
        seg["valu"] += 1
        if re.match(r"v_(exp|rcp|sin|cos|log|sqrt|rsq)", op):
            seg["trans"] += 1
    elif op.startswith("ds_"):
        seg["lds"] += 1
    elif op.startswith("scratch_") or (op.startswith("buffer_") and "off, s[0:3]" in l):
        seg["scr"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        seg["vmem"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        seg["br"] += 1
    elif op.startswith("s_"):
        seg["salu"] += 1
segs.append(seg)
for k, s in enumerate(segs):
    print(f"seg {k:2d} line {s['at']:6d}: valu {s['valu']:5d} mfma {s['mfma']:4d} trans {s['trans']:4d} "
          f"lds {s['lds']:4d} vmem {s['vmem']:4d} scratch {s['scr']:3d} salu {s['salu']:4d} br {s['br']:3d} labels {s['labels'][:4]}")

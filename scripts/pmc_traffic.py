#!/usr/bin/env python3
"""Per-launch HBM traffic (and MFMA activity) of one kernel from rocprofv3 --pmc passes.

usage: pmc_traffic.py OUT.json KERNEL_SUBSTR pass_dir [pass_dir ...]
Each pass dir holds a run_counter_collection.csv.  FETCH_SIZE / WRITE_SIZE are KiB per
dispatch (summed over XCDs).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE
reports 1/2 of the bytes of WIDE (16 B/lane) coalesced reads; our kernels read with
4-B/lane loads, for which the guide gives no calibration, so both the raw value and the
x2-corrected upper bound are recorded.  WRITE_SIZE is exact for streaming stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, kname, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if kname in row.get("Kernel_Name", ""):
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items() if v}
    res = {"kernel": kname, "dispatches": {k: len(v) for k, v in vals.items()}, "avg": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fb, wb = avg["FETCH_SIZE"] * 1024, avg["WRITE_SIZE"] * 1024
        # bench.py reads hbm_bytes_per_launch: FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM
        res.update(fetch_bytes_raw=fb, write_bytes=wb, hbm_bytes_per_launch_raw=fb + wb,
                   hbm_bytes_per_launch=2 * fb + wb)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        res["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (avg["GRBM_GUI_ACTIVE"] / 8)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

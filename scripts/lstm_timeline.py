"""Per-step timeline of a rocprofv3 kernel trace of scripts/bench_student_lstm.py (one size):
the last step's kernels (from the last adam_kernel back to the previous one), their
durations and the gaps between them."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] and "lstm" not in r["Kernel_Name"]]
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
busy = 0
prev_end = t0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.2f} us  dur {(e - s) / 1e3:7.2f}  gap {(s - prev_end) / 1e3:6.2f}  {r['Kernel_Name'][:80]}")
    prev_end = e
span = int(step[-1]["End_Timestamp"]) - t0
print(f"kernels {len(step)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  gaps {(span - busy) / 1e3:.1f} us")

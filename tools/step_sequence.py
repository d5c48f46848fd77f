"""The kernels of one steady bench step in launch order, with durations and the idle gap before each:
    python tools/step_sequence.py p_kernel_trace.csv   (the step window step_breakdown.py picks last)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "cim_fwd_v3_kernel<8" in r["Kernel_Name"]]
steps = []
for a, b in zip(marks, marks[1:]):
    wall = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b])
    if busy > 0.95 * wall and b - a > 50:
        steps.append((a, b))
a, b = steps[-1]
prev_end = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e
    print(f"{(e - s) / 1e3:8.1f} us  gap {gap:5.1f}  {r['Kernel_Name'].split('(')[0].replace('void ', '')[:80]}")

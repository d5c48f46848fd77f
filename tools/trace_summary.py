#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: per (kernel, grid) mean duration and share."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
d = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"][:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["VGPR_Count"],
           r["LDS_Block_Size"])
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in d.values())
print(f"total kernel time {tot / 1000:.2f} ms over {len(rows)} dispatches")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / tot * 100:5.1f}%  n={len(v):5d}  mean={sum(v) / len(v):8.1f}us  {k}")

#!/usr/bin/env python
"""Mean duration per libcimq kernel from a rocprofv3 kernel-trace CSV."""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "cimq" in r["Kernel_Name"]:
        d[r["Kernel_Name"].split("(")[0][-48:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {sum(v) / len(v):8.1f} us  n={len(v):3d}  {k}")

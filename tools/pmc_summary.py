#!/usr/bin/env python
"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel, counters per dispatch
and per wave (SQ_WAVES must be in one of the passes)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:60]
        if "cimq" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, path)].add(r["Dispatch_Id"])
for k, c in acc.items():
    nd = max(len(v) for (kk, _), v in disp.items() if kk == k)
    waves = c.get("SQ_WAVES", 0) / nd if nd else 0
    print(f"== {k}  dispatches/pass={nd}  waves/dispatch={waves:.0f}")
    for name, val in sorted(c.items()):
        per = val / nd
        pw = per / waves if waves else float("nan")
        print(f"   {name:28s} {per:14.0f} /dispatch  {pw:12.1f} /wave")

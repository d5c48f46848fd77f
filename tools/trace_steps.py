#!/usr/bin/env python
"""Per-step kernel breakdown of a rocprofv3 kernel trace of bench.py (steps counted by the
first layer's forward launches)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "cim_fwd_v3_kernel<8"
steps = max(1, sum(1 for r in rows if marker in r["Kernel_Name"]))
d = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].split("(")[0][:64]
    d[n][0] += 1
    d[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in d.values())
print(f"{len(rows)} dispatches, {steps} step-equivalents, {tot / steps / 1e3:.3f} ms kernel time per step")
for n, (c, t) in sorted(d.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{t / tot * 100:5.1f}% {c / steps:6.1f}/step {t / c:8.1f}us {t / steps / 1e3:6.3f}ms/step  {n}")

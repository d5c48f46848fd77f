"""Kernel time of one graph-replayed bench step, by kernel, from a rocprofv3 kernel trace:
    python tools/step_breakdown.py p_kernel_trace.csv  (the steady-state step windows of the
    timed HIP-graph region: step windows between first-layer forward launches whose wall time is
    within 5% of their busy time)"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "cim_fwd_v3_kernel<8" in r["Kernel_Name"]]
steps = []
for a, b in zip(marks, marks[1:]):
    wall = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b])
    # a training step's window holds backward kernels (the forward-only graph windows do not)
    if busy > 0.95 * wall and any("cim_bwd_" in r["Kernel_Name"] for r in rows[a:b]):
        steps.append((a, b, wall))
d = collections.defaultdict(float)
cnt = collections.defaultdict(int)
for a, b, _ in steps:
    for r in rows[a:b]:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        d[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
ns = len(steps)
if ns == 0:
    sys.exit("no steady step windows found")
print(f"{ns} steady steps, wall {sum(s[2] for s in steps) / ns / 1e3:.1f} us/step")
for n, t in sorted(d.items(), key=lambda kv: -kv[1]):
    print(f"{t / ns:8.1f} us/step  {cnt[n] / ns:5.1f}x  {n}")

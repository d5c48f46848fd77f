"""Per-kernel average durations of a rocprofv3 --stats csv, optionally against a baseline csv:
    python tools/kstats.py new.csv [base.csv]"""
import csv
import sys


def load(p):
    return {r["Name"]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(p))}


new = load(sys.argv[1])
base = load(sys.argv[2]) if len(sys.argv) > 2 else {}
for name, (calls, avg) in sorted(new.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:24]:
    b = base.get(name)
    extra = f"  base {b[1]:8.1f}us ({avg / b[1] - 1:+.1%})" if b else ""
    print(f"{calls * avg / 1e3:8.2f}ms {calls:5d}x {avg:8.1f}us{extra}  {name[:90]}")

#!/usr/bin/env python
"""Per-kernel stats (the rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

    python tools/db_stats.py gpurun_out/prof/run_results.db > profiles/rNN/kernel_stats.csv
"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                   "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for n, c, s, a, lo, hi in rows:
    w.writerow([n, c, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])

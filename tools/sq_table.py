#!/usr/bin/env python
"""Compact table from tools/pmc_summary.py outputs (<layer>.sq.txt): per kernel the wave cycles and the shares of
SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY in them (quad-cycle counters, as MI355X_MICROARCH.md says),
VALU / MFMA / LDS instructions per wave and LDS bank-conflict cycles per wave.

    python tools/sq_table.py gpurun_out/r06_sq/*.sq.txt
"""
import re
import sys

for path in sys.argv[1:]:
    cur, rows = None, {}
    for line in open(path):
        m = re.match(r"== (?:void )?([^(]+)\(", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.match(r"\s+(\S+)\s+(\S+) /dispatch\s+(\S+) /wave", line)
        if m and cur:
            rows[cur][m.group(1)] = float(m.group(3))
    print(f"# {path}")
    print(f"{'kernel':58s} {'cyc/wave':>9s} {'WAIT_ANY':>8s} {'WAIT_INST':>9s} {'ACTIVE':>7s} {'VALU':>7s} {'MFMA':>6s} {'LDS':>6s} {'bankcf':>7s}")
    for k, c in rows.items():
        if "cimq" not in k or c.get("SQ_WAVE_CYCLES", 0) == 0:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        f = lambda n: c.get(n, float("nan")) / wc  # noqa: E731
        print(f"{k[:58]:58s} {4 * wc:9.0f} {f('SQ_WAIT_ANY'):8.2f} {f('SQ_WAIT_INST_ANY'):9.2f} {f('SQ_ACTIVE_INST_ANY'):7.2f} "
              f"{c.get('SQ_INSTS_VALU', 0):7.0f} {c.get('SQ_INSTS_MFMA', 0):6.0f} {c.get('SQ_INSTS_LDS', 0):6.0f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0):7.0f}")

#!/usr/bin/env python
"""HBM traffic per launch of every libcimq kernel from two rocprofv3 --pmc passes.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir_f> -o p -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir_w> -o p -- python bench.py ...
    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d <dir_v> -o p -- python bench.py ...   (optional)
    python tools/pmc_traffic.py <dir_f>/p_counter_collection.csv <dir_w>/p_counter_collection.csv \
        [<dir_v>/p_counter_collection.csv] > traffic.json

Per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B / lane) streaming read, so
traffic = 2 * FETCH_SIZE + WRITE_SIZE.  Output: {kernel symbol: mean bytes per dispatch and the
dispatch count}, plus "_meta": the sha of the kernel sources measured (bench.py reports the
traffic only while the sources still match).
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_kernel(path, counter):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "cimq" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: acc[k] / len(disp[k]) for k in acc}, {k: len(disp[k]) for k in acc}


fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
write, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
valu = per_kernel(sys.argv[3], "SQ_INSTS_VALU")[0] if len(sys.argv) > 3 else {}
waves = per_kernel(sys.argv[3], "SQ_WAVES")[0] if len(sys.argv) > 3 else {}
from bench import source_sha  # noqa: E402

out = {"_meta": {"source_sha": source_sha()}}
for k in sorted(set(fetch) | set(write)):
    out[k] = {"fetch_kib": fetch.get(k), "write_kib": write.get(k), "dispatches": nf.get(k, 0),
              "traffic_bytes": (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024.0,
              "valu_insts": valu.get(k), "waves": waves.get(k)}
json.dump(out, sys.stdout, indent=1)

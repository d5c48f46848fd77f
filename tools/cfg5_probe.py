"""Time / profile the BASELINE cfg5 layer (QuantLinear 1024->1024 w4a4 xbar128, B=4096) alone:
    rocprofv3 --kernel-trace --stats -d <dir> -- python tools/cfg5_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    print(bench.bench_cfg5(dev, int(sys.argv[1]) if len(sys.argv) > 1 else 3, 1), flush=True)

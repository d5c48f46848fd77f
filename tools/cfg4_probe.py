#!/usr/bin/env python
"""BASELINE cfg4 (ResNet-56 w2a2 xbar64 adc1.5, 55 convs, B=256) fwd+bwd for a kernel trace:
    rocprofv3 --kernel-trace --stats -d <dir> -o p -- python tools/cfg4_probe.py [--shift] [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    shift = "--shift" in sys.argv
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 3
    r = bench.bench_layers(torch.device("cuda:0"), bench.resnet56_convs(), 256, 64, 1.5, steps, 1, adc_shift=shift)
    print(r, flush=True)


if __name__ == "__main__":
    main()

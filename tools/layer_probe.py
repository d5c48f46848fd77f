#!/usr/bin/env python
"""Run fwd+bwd of ONE ResNet-20 CiM layer shape repeatedly (for rocprofv3 PMC passes).

    python tools/layer_probe.py --layer layer1.0.conv1 --iters 5
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="layer1.0.conv1")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    names = [r[0] for r in bench.RESNET20]
    idx = names.index(a.layer)
    bench.RESNET20[:] = [bench.RESNET20[idx]]
    layers, xs, gs = bench.build(torch.device("cuda:0"), a.batch)
    m, x, g = layers[0], xs[0], gs[0]
    for _ in range(a.iters + 1):
        y = m(x.requires_grad_(True))
        y.backward(g)
    torch.cuda.synchronize()
    print("ok", a.layer, tuple(y.shape))


if __name__ == "__main__":
    main()

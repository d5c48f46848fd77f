"""Build container only: time the reference's own get_cim_output_signed (CPU, through the
CUDA-allocation shim of tests/golden/make_golden.py) against oracle/cim_torch_port.py -- the
op-faithful torch-CPU port bench.py times as its cpu_baseline on the GPU box -- on the same
inputs, and check they agree.  Prints one JSON line (recorded in DESIGN.md).

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_port_ratio.py
"""
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from make_golden import _import_reference  # noqa: E402

from oracle import cim_oracle as co  # noqa: E402
from oracle import cim_torch_port as tp  # noqa: E402


def case(B, C, O, H, s, bits, xbar=128, seed=0):
    rng = np.random.default_rng(seed)
    sa, sw = np.float32(0.11), np.float32(0.07)
    qn, qp = co.lsq_weight_params(bits)
    x = torch.from_numpy((rng.integers(0, 2 ** bits, (B, C, H, H)).astype(np.float32) * sa).astype(np.float32))
    w = torch.from_numpy((rng.integers(qn, qp + 1, (O, C, 3, 3)).astype(np.float32) * sw).astype(np.float32))
    T = math.ceil(C * 9 / xbar)
    a = torch.from_numpy(co.alpha_quantize(((rng.random((1, T, bits, bits, 1, O)) * 3 + 0.1) * sa * sw)
                                           .astype(np.float32), 8))
    ho = (H + 2 - 3) // s + 1
    g = torch.from_numpy(rng.standard_normal((B, ho * ho, O)).astype(np.float32))
    bm = torch.from_numpy(co.make_binary_mask(bits, bits, 1, 1))
    return x, w, a, g, bm, torch.tensor([sw]), torch.tensor([sa])


def main():
    ref = _import_reference()
    torch.set_num_threads(8)
    res = {}
    for name, (B, C, O, H, s, bits) in {"layer1_s1_16x16_32": (256, 16, 16, 32, 1, 3),
                                        "layer3_s1_64x64_8": (256, 64, 64, 8, 1, 3)}.items():
        x, w, a, g, bm, sw, sa = case(B, C, O, H, s, bits)
        times = {}
        for who in ("reference", "port"):
            best = 1e9
            for _ in range(2):
                t0 = time.perf_counter()
                if who == "reference":
                    xx, ww, aa = x.clone().requires_grad_(True), w.clone().requires_grad_(True), a.clone().requires_grad_(True)
                    out = ref.get_cim_output_signed.apply(xx, ww, (s, s), (1, 1), (1, 1), bits, 1, bits, 1, 1.5, 128, bm, aa,
                                                          sw, sa, False, torch.zeros(1))
                    out.backward(g)
                    r = (out.detach(), xx.grad, ww.grad, aa.grad)
                else:
                    out, c = tp.cim_forward(x, w, (s, s), (1, 1), bits, 1, bits, 1, 1.5, 128, bm, a, sw, sa)
                    gx, gw, ga = tp.cim_backward(c, g)
                    p = (out, gx, gw, ga)
                best = min(best, time.perf_counter() - t0)
            times[who] = best
        err = max(float((u - v).abs().max() / (v.abs().max() + 1e-30)) for u, v in zip(p, r))
        res[name] = dict(reference_s=round(times["reference"], 3), port_s=round(times["port"], 3),
                         port_over_reference=round(times["port"] / times["reference"], 3), max_rel_diff=err)
    res["threads"] = torch.get_num_threads()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

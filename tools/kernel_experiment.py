#!/usr/bin/env python
"""Time libcimq kernels of one ResNet-20 layer shape for several experiment builds.

    python tools/kernel_experiment.py --build            # (CPU) compile the variant libraries
    python tools/kernel_experiment.py --layer layer1.0.conv1   # (GPU) time them

Variant libraries live in exp/ (git-ignored); they skip parts of a kernel to attribute its
time and give wrong results by design -- never used by the product path or the tests.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# name -> preprocessor defines; kernels carry CIMQ_EXP_* knobs only while an experiment runs
VARIANTS = {
    "base": [],
    "gw_noga": ["CIMQ_EXP_GW_NOGA"],
    "gw_nomfma": ["CIMQ_EXP_GW_NOMFMA"],
    "gw_nostage": ["CIMQ_EXP_GW_NOSTAGE"],
    "gw_nod": ["CIMQ_EXP_GW_NOD"],
    "gw_noga_nomfma": ["CIMQ_EXP_GW_NOGA", "CIMQ_EXP_GW_NOMFMA"],
    "gw_noga_nomfma_nod": ["CIMQ_EXP_GW_NOGA", "CIMQ_EXP_GW_NOMFMA", "CIMQ_EXP_GW_NOD"],
    "gx_nomfma": ["CIMQ_EXP_GX_NOMFMA"],
    "gx_noring": ["CIMQ_EXP_GX_NORING"],
    "gx_nowload": ["CIMQ_EXP_GX_NOWLOAD"],
    "fwd_nost": ["CIMQ_EXP_FWD_NOST"],
    "gx_nofold": ["CIMQ_EXP_GX_NOFOLD"],
    "gx_nostate": ["CIMQ_EXP_GX_NOSTATE"],
    "gx_nofold_nomfma": ["CIMQ_EXP_GX_NOFOLD", "CIMQ_EXP_GX_NOMFMA"],
    "fwd_noadc": ["CIMQ_EXP_FWD_NOADC"],
    "fwd_nopro": ["CIMQ_EXP_FWD_NOPRO"],
    "fwd_nostage": ["CIMQ_EXP_FWD_NOSTAGE"],
    "fwd_nogather": ["CIMQ_EXP_FWD_NOGATHER"],
    "prep_noact": ["CIMQ_EXP_PREP_NOACT"],
    "prep_nowt": ["CIMQ_EXP_PREP_NOWT"],
    "prep_nowt_nocomp": ["CIMQ_EXP_PREP_NOWT", "CIMQ_EXP_PREP_NOCOMP"],
    "prep_nofrag": ["CIMQ_EXP_PREP_NOACT", "CIMQ_EXP_PREP_NOFRAG"],
    "prep_noparams": ["CIMQ_EXP_PREP_NOACT", "CIMQ_EXP_PREP_NOPARAMS"],
}
if os.environ.get("CIMQ_EXP_VARIANTS"):
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["CIMQ_EXP_VARIANTS"].split(",")}


def lib_path(name):
    return os.path.join(REPO, os.environ.get("CIMQ_EXP_DIR", "exp"), f"libcimq_{name}.so")


def do_build():
    from cim_quantization_amd import build as B
    os.makedirs(os.path.dirname(lib_path("base")), exist_ok=True)
    with cf.ThreadPoolExecutor(len(VARIANTS)) as ex:
        futs = {ex.submit(B.build, True, False, lib_path(n), list(d) + ["CIMQ_TUNING"]): n
                for n, d in VARIANTS.items()}
        for f in cf.as_completed(futs):
            f.result()
            print("built", futs[f], flush=True)


def do_time(layer, iters):
    import torch
    import bench
    from cim_quantization_amd import _lib
    if not hasattr(bench, "_ALL_LAYERS"):
        bench._ALL_LAYERS = list(bench.RESNET20)
    names = [r[0] for r in bench._ALL_LAYERS]
    bench.RESNET20[:] = [bench._ALL_LAYERS[names.index(layer)]]
    layers, xs, gs = bench.build(torch.device("cuda:0"), 256)
    m, x, g = layers[0], xs[0], gs[0]
    for name in VARIANTS:
        _lib._lib = _lib.load(lib_path(name))
        x1 = x.detach().requires_grad_(True)
        m(x1).backward(g)  # warm (alpha init etc.)
        torch.cuda.synchronize()
        res = {}
        for kern in ("fwd", "bwd_gx", "bwd_gw", "prep_act"):
            with _lib.KernelTimer(kern) as kt:
                for _ in range(iters):
                    x1 = x.detach().requires_grad_(True)
                    m(x1).backward(g)
                torch.cuda.synchronize()
            res[kern] = kt.total_ms / max(kt.launches, 1) * 1000
        print(f"{layer:16s} {name:10s} " + "  ".join(f"{k}={v:8.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--layer", action="append")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    if a.build:
        do_build()
    else:
        for L in a.layer or ["layer1.0.conv1"]:
            do_time(L, a.iters)

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

# name -> preprocessor defines.  The attribution knobs of rounds 1-2 (CIMQ_EXP_FWD_NOADC, _GX_NOMFMA,
# _GW_NOGA, ... : skip one part of a kernel) are no longer in the shipped kernel sources; an attribution
# run adds its #ifdef to a scratch copy of the kernel and its define here.  Their measurements are in
# DESIGN.md section 4.
VARIANTS = {
    "base": [],
    "cur": [],  # the working tree (a copy of base built later)
    # round 4: the fused backward (cimq_fused.hip) and the first conv's (cimq_c1.hip)
    "f_nogx": ["CIMQ_EXP_F_NOGX"],
    "f_nogw": ["CIMQ_EXP_F_NOGW"],
    "f_nostage": ["CIMQ_EXP_F_NOSTAGE"],
    "f_nogxgw": ["CIMQ_EXP_F_NOGX", "CIMQ_EXP_F_NOGW"],
    "c1_nopairs": ["CIMQ_EXP_C1_NOPAIRS"],
    "f_pf2": ["CIMQ_EXP_F_PF2"],
    "c1_ldsadd": ["CIMQ_EXP_C1_LDSADD"],  # round 6: c1's grad_alpha sums as no-return LDS adds (slower: not kept)
    "c1_xpf": ["CIMQ_EXP_C1_XPF"],  # round 6: c1's fold x loaded at the step's start (neutral: not kept)
    "fold_xb4": ["CIMQ_FOLD_XB=4"],  # round 6: the grad_x folds' x loads four elements per thread at a time
    "f_cbu2": ["CIMQ_EXP_F_CBU2"],  # round 6: the fused grad_x's (c, kh)-block loop unrolled by two (-0.8 us: not kept)
    "c1_sb2": ["CIMQ_EXP_C1_SB2"],  # round 6: c1's scheduling fence after every second slice (+1 us: not kept)
    "gxw5_il": ["CIMQ_EXP_GXW5_ORDER=1"],  # round 6: the merged launch's two roles interleaved (slower: not kept)
    "gxw5_wf": ["CIMQ_EXP_GXW5_ORDER=2"],  # round 6: grad_w's workgroups first (slower: not kept)
    "gx5_noploop": ["CIMQ_EXP_GX5_NOPLOOP"],  # round 6: gx5 without its A reads and MFMAs (timing only)
    "gx5_nosync": ["CIMQ_EXP_GX5_NOSYNC"],  # round 6: gx5 without its step barriers (timing only)
    "gx5_noepi": ["CIMQ_EXP_GX5_NOEPI"],  # round 6: gx5 without the per-m-tile x read / gx store (timing only)
    "gx5_bare": ["CIMQ_EXP_GX5_NOPLOOP", "CIMQ_EXP_GX5_NOBUILD", "CIMQ_EXP_GX5_NOLOAD", "CIMQ_EXP_GX5_NOEPI"],
    "c1_both": ["CIMQ_EXP_C1_LDSADD", "CIMQ_EXP_C1_XPF"],  # round 6: the fused grad_x's weight blocks two (c, kh)-blocks ahead
    # forward staging: the weight side (fragments + ADC parameters per tile) / the activation rows
    "fwd_nostagew": ["CIMQ_EXP_FWD_NOSTAGEW"],
    "fwd_nostagex": ["CIMQ_EXP_FWD_NOSTAGEX"],
    "fwd_nostage": ["CIMQ_EXP_FWD_NOSTAGEW", "CIMQ_EXP_FWD_NOSTAGEX"],
    # round 5: the compute phase of the forward -- without the LDS gather / the ADC and state bits /
    # the state bits only, and the staging-free skeletons
    "fwd_nogather": ["CIMQ_EXP_FWD_NOGATHER"],
    "fwd_noadc": ["CIMQ_EXP_FWD_NOADC"],
    "fwd_nostate": ["CIMQ_EXP_FWD_NOSTATE"],
    "fwd_ns_ng": ["CIMQ_EXP_FWD_NOSTAGEW", "CIMQ_EXP_FWD_NOSTAGEX", "CIMQ_EXP_FWD_NOGATHER"],
    "fwd_ns_ng_na": ["CIMQ_EXP_FWD_NOSTAGEW", "CIMQ_EXP_FWD_NOSTAGEX", "CIMQ_EXP_FWD_NOGATHER", "CIMQ_EXP_FWD_NOADC"],
    "fwd_ns_nst": ["CIMQ_EXP_FWD_NOSTAGEW", "CIMQ_EXP_FWD_NOSTAGEX", "CIMQ_EXP_FWD_NOSTATE"],
    # the module epilogue's grad_w role: without the weight quantiser's loads / stores, without the
    # slab sums (tools/tail_sweep.sh with CIMQ_LIB_PATH=<variant lib>)
    "tail_noepi": ["CIMQ_EXP_TAIL_NOEPI"],
    "tail_noslab": ["CIMQ_EXP_TAIL_NOSLAB"],
    # round 5: the per-input-pixel grad_x (cimq_gx5.hip) without the G build / with one A read per K-step
    # (LDS read traffic / 9 and one plane) / without the MFMAs
    "gx5_nobuild": ["CIMQ_EXP_GX5_NOBUILD"],
    "gx5_noaread": ["CIMQ_EXP_GX5_NOAREAD"],
    "gx5_nomfma": ["CIMQ_EXP_GX5_NOMFMA"],
    "gx5_noaread_nomfma": ["CIMQ_EXP_GX5_NOAREAD", "CIMQ_EXP_GX5_NOMFMA"],
    # round 6: the recompute backward (cimq_r6.hip) without its phase-A MFMAs / G writes / gw MFMAs / gx MFMAs /
    # finish (exchange rows, act-LSQ backward, gx stores)
    "r6_noa": ["CIMQ_EXP_R6_NOA"],
    "r6_nog": ["CIMQ_EXP_R6_NOG"],
    "r6_nogw": ["CIMQ_EXP_R6_NOGW"],
    "r6_nogx": ["CIMQ_EXP_R6_NOGX"],
    "r6_nofin": ["CIMQ_EXP_R6_NOFIN"],
    "r6_nogwgx": ["CIMQ_EXP_R6_NOGW", "CIMQ_EXP_R6_NOGX"],
    "gw5_noload": ["CIMQ_EXP_GW5_NOLOAD"],  # gw5 without its global reads (timing only)
    "gw5_noga": ["CIMQ_EXP_GW5_NOGA"],
    "gw5_nomfma": ["CIMQ_EXP_GW5_NOMFMA"],
    "gw5_noepi": ["CIMQ_EXP_GW5_NOEPI"],
    "gw5_skel": ["CIMQ_EXP_GW5_NOLOAD", "CIMQ_EXP_GW5_NOGA", "CIMQ_EXP_GW5_NOMFMA", "CIMQ_EXP_GW5_NOEPI"],
    "dense_noadc": ["CIMQ_EXP_DENSE_NOADC", "CIMQ_EXP_DENSE_NOSTORE"],  # cfg5 forward attribution (timing only)
    "dense_nostore": ["CIMQ_EXP_DENSE_NOSTORE"],
    "dense_noprm": ["CIMQ_EXP_DENSE_NOPRM"],
    "dense_skel_nox": ["CIMQ_EXP_DENSE_NOADC", "CIMQ_EXP_DENSE_NOSTORE", "CIMQ_EXP_DENSE_NOX"],
    "dense_skel_nostage": ["CIMQ_EXP_DENSE_NOADC", "CIMQ_EXP_DENSE_NOSTORE", "CIMQ_EXP_DENSE_NOSTAGE"],
    "dense_skel_none": ["CIMQ_EXP_DENSE_NOADC", "CIMQ_EXP_DENSE_NOSTORE", "CIMQ_EXP_DENSE_NOSTAGE", "CIMQ_EXP_DENSE_NOX"],
    "gw5_empty": ["CIMQ_EXP_GW5_EMPTY"],  # gw5's prologue + epilogue only
    "gw5_empty_noepi": ["CIMQ_EXP_GW5_EMPTY", "CIMQ_EXP_GW5_NOEPI"],
    "fwd5_noadc": ["CIMQ_EXP_FWD5_NOADC"],  # fwd5 attribution (timing only)
    "fwd5_nomfma": ["CIMQ_EXP_FWD5_NOMFMA"],
    "fwd5_nostage": ["CIMQ_EXP_FWD5_NOSTAGE"],
    "fwd5_skel": ["CIMQ_EXP_FWD5_NOADC", "CIMQ_EXP_FWD5_NOMFMA", "CIMQ_EXP_FWD5_NOSTAGE"],
    "gx5_nobuild": ["CIMQ_EXP_GX5_NOBUILD"],  # gx5 attribution (timing only)
    "gx5_nomfma": ["CIMQ_EXP_GX5_NOMFMA"],
    "gx5_noload": ["CIMQ_EXP_GX5_NOLOAD"],
    "gx5_skel": ["CIMQ_EXP_GX5_NOBUILD", "CIMQ_EXP_GX5_NOMFMA", "CIMQ_EXP_GX5_NOLOAD"],
    "gx5_dpp": ["CIMQ_EXP_GX5_DPP"],  # gx5's kw shifts by DPP instead of nine A reads per K-step (slower)
    "gx5_chains": ["CIMQ_EXP_GX5_CHAINS"],  # gx5's two K-steps in separate MFMA accumulators
    "r6_nopf": ["CIMQ_EXP_R6_NO_WFPF", "CIMQ_EXP_R6_NO_XFPF"],  # without the weight-fragment / x prefetches
    "r6_skel": ["CIMQ_EXP_R6_NOA", "CIMQ_EXP_R6_NOG", "CIMQ_EXP_R6_NOGW", "CIMQ_EXP_R6_NOGX", "CIMQ_EXP_R6_NOFIN"],
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

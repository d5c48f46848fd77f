"""Golden vectors for the scale + shift ADC Functions and the reference's own self-consistency
configurations, generated from the REAL reference test scripts.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_shift.py

It loads, unmodified and read-only, ``test/test_backward_cimlayer_scale_shift.py`` and
``test/test_backward_cimlayer.py`` from /root/reference.  Both are module-level scripts: loading
one runs its own check once (on the CPU, through the same CUDA-allocation shim as
make_golden.py) before its Functions become available.  For each case the script runs the
reference Functions, runs the numpy oracle (oracle/cim_shift_oracle.py) on the same inputs,
asserts agreement, and writes inputs + reference outputs as an .npz (data only).

Cases:
  ss_ver2_ref_cfg      get_analog_partial_sums_autograd_ver2 and its autograd twin at the
                       script's own configuration (scale_shift.py:700-739)
  ss_adcless_ref_cfg   get_adcless_cim_output at the same configuration
  ss_ver2_adc4_float   ver2, 4-bit ADC, non-integer alpha / beta
  ss_ver2_xbar128_wrap ver2, 128-row tiles driven to ps = 128 (the int8 buffer wraps it)
  ss_adcless_w2a2      adcless, w2a2, two images
  bk_adc4_ref_cfg      test_backward_cimlayer.py's ver2 Function and its autograd twin at that
                       script's configuration (:398-440: adc 4, alpha = 1, grad = 1)
"""
from __future__ import annotations

import contextlib
import importlib.util
import io
import json
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("CIMQ_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import cim_shift_oracle as so  # noqa: E402
sys.path.insert(0, HERE)
from make_golden import _install_cpu_shim  # noqa: E402

F32 = np.float32


def _load(relpath, name):
    _install_cpu_shim()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(io.StringIO()):  # the script prints its own check
        spec.loader.exec_module(mod)
    return mod


CASES = [
    ("ss_ver2_ref_cfg", dict(fn="ver2", B=1, C=16, O=32, H=32, k=3, s=2, p=1, wb=3, ab=3, xbar=64, adc=1,
                             alpha="int13", beta="int14", x="randint", w="randint", grad="randn", auto=True)),
    ("ss_adcless_ref_cfg", dict(fn="adcless", B=1, C=16, O=32, H=32, k=3, s=2, p=1, wb=3, ab=3, xbar=64, adc=1,
                                alpha="int13", beta="int14", x="randint", w="randint", grad="randn")),
    ("ss_ver2_adc4_float", dict(fn="ver2", B=2, C=8, O=8, H=6, k=3, s=1, p=1, wb=3, ab=3, xbar=64, adc=4,
                                alpha="float", beta="float", x="randint", w="randint", grad="randn")),
    ("ss_ver2_xbar128_wrap", dict(fn="ver2", B=1, C=16, O=8, H=6, k=3, s=1, p=1, wb=3, ab=3, xbar=128, adc=1,
                                  alpha="int13", beta="int14", x="sevens", w="threes", grad="randn")),
    ("ss_adcless_w2a2", dict(fn="adcless", B=2, C=16, O=16, H=8, k=3, s=1, p=1, wb=2, ab=2, xbar=64, adc=1,
                             alpha="int13", beta="float", x="randint", w="randint", grad="randn")),
    ("bk_adc4_ref_cfg", dict(fn="bk_ver2", B=1, C=16, O=32, H=32, k=3, s=2, p=1, wb=3, ab=3, xbar=64, adc=4,
                             alpha="ones_tile", beta=None, x="randint", w="randint", grad="ones", auto=True)),
]


def case_inputs(cfg, seed):
    g = torch.Generator().manual_seed(seed)
    B, C, O, H, k = cfg["B"], cfg["C"], cfg["O"], cfg["H"], cfg["k"]
    nbw, nba = cfg["wb"], cfg["ab"]
    T = math.ceil(C * k * k / cfg["xbar"])
    if cfg["x"] == "randint":  # scale_shift.py:734, test_backward_cimlayer.py:427
        x = torch.randint(0, 2 ** cfg["ab"] - 1, (B, C, H, H), generator=g).float()
    else:
        x = torch.full((B, C, H, H), 7.0)
        x[:, :, 0, 0] = 3.0
    if cfg["w"] == "randint":  # scale_shift.py:735
        w = torch.randint(-(2 ** (cfg["wb"] - 1)), 2 ** (cfg["wb"] - 1) - 1, (O, C, k, k), generator=g).float()
    else:
        w = torch.randint(-4, 3, (O, C, k, k), generator=g).float()
        w[: O // 2] = 3.0
    shp = (1, T, nbw, nba, 1, O)
    a = {"int13": lambda: torch.randint(1, 3, shp, generator=g).float(),  # scale_shift.py:726
         "float": lambda: torch.rand(shp, generator=g) * 2.0 + 0.5,
         "ones_tile": lambda: torch.ones(1, T, 1, 1, 1, O)}[cfg["alpha"]]()  # test_backward_cimlayer.py:425
    b = None
    if cfg["beta"] is not None:
        b = {"int14": lambda: torch.randint(1, 4, shp, generator=g).float(),  # scale_shift.py:729
             "float": lambda: torch.rand(shp, generator=g) * 4.0 - 2.0}[cfg["beta"]]()
    Ho = (H + 2 * cfg["p"] - k) // cfg["s"] + 1
    grad = torch.randn(B, Ho * Ho, O, generator=g) if cfg["grad"] == "randn" else torch.ones(B, Ho * Ho, O)
    bm = torch.ones(nbw, nba)  # scale_shift.py:716-720: float mask 2^(j) * 2^(k)
    for i in range(nba):
        for j in range(nbw):
            bm[j, i] = (2 ** i) * (2 ** j)
    bm = bm.view(1, 1, nbw, nba, 1, 1)
    return dict(x=x, w=w, alpha=a, beta=b, grad=grad, binary_mask=bm)


def run_ref(fn, cfg, inp, autograd=False):
    x = inp["x"].clone().requires_grad_(True)
    w = inp["w"].clone().requires_grad_(True)
    a = inp["alpha"].clone().requires_grad_(True)
    b = None if inp["beta"] is None else inp["beta"].clone().requires_grad_(True)
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    args = (x, w, st, pd, (1, 1), cfg["ab"], 1, cfg["wb"], 1, cfg["adc"], cfg["xbar"], inp["binary_mask"], a)
    if b is not None:
        args = args + (b,)
    with contextlib.redirect_stdout(io.StringIO()):  # test_backward_cimlayer.py's backward prints
        out = fn(*args) if autograd else fn.apply(*args)
        out.backward(inp["grad"])
    res = dict(out=out.detach().numpy().copy(), grad_x=x.grad.numpy().copy(), grad_w=w.grad.numpy().copy(),
               grad_alpha=a.grad.numpy().copy())
    if b is not None:
        res["grad_beta"] = b.grad.numpy().copy()
    return res


def _err(mine, ref_val, terms):
    d = np.abs(mine.astype(np.float64) - ref_val.astype(np.float64))
    scale = np.maximum(np.abs(ref_val.astype(np.float64)), terms) + 1e-30
    return float(np.nanmax(d / scale)) if d.size else 0.0


def check_oracle(name, cfg, inp, res):
    variant = so.VARIANT_SIGN if cfg["fn"] == "adcless" else so.VARIANT_ROUND
    T = math.ceil(cfg["C"] * cfg["k"] ** 2 / cfg["xbar"])
    shp = (1, T, cfg["wb"], cfg["ab"], 1, cfg["O"])
    a = np.broadcast_to(inp["alpha"].numpy(), shp).astype(F32)
    b = np.zeros(shp, F32) if inp["beta"] is None else inp["beta"].numpy()
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    out, c = so.shift_forward(inp["x"].numpy(), inp["w"].numpy(), st, pd, cfg["ab"], 1, cfg["wb"], 1, cfg["adc"],
                              cfg["xbar"], inp["binary_mask"].numpy(), a, b, variant)
    gx, gw, ga, gb = so.shift_backward(c, inp["grad"].numpy())
    ax, aw, aa, ab = so.shift_backward(c, inp["grad"].numpy(), absolute=True)
    ga_r = res["grad_alpha"]
    if ga_r.shape != ga.shape:  # alpha broadcast over (k, j): autograd sums the grad to its shape
        ga, aa = ga.sum(axis=(2, 3), keepdims=True), aa.sum(axis=(2, 3), keepdims=True)
    out_terms = np.abs(c.code.astype(np.float64) * a + b) * np.abs(c.binary_mask)
    out_terms = out_terms.sum(axis=(1, 2, 3))
    errs = dict(out=_err(out, res["out"], out_terms), gx=_err(gx, res["grad_x"], ax), gw=_err(gw, res["grad_w"], aw),
                ga=_err(ga, ga_r, aa))
    if "grad_beta" in res:
        errs["gb"] = _err(gb, res["grad_beta"], ab)
    print(f"  {name}: " + "  ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    assert max(errs.values()) < 1e-5, (name, errs)
    extra = dict(abs_out=out_terms.astype(F32), abs_grad_x=ax, abs_grad_w=aw, abs_grad_alpha=aa)
    if "grad_beta" in res:
        extra["abs_grad_beta"] = ab
    return extra


def main():
    ss = _load("test/test_backward_cimlayer_scale_shift.py", "ref_scale_shift")
    bk = _load("test/test_backward_cimlayer.py", "ref_backward_cimlayer")
    torch.set_num_threads(4)
    manifest = {}
    for idx, (name, cfg) in enumerate(CASES):
        seed = 3000 + idx
        inp = case_inputs(cfg, seed)
        if cfg["fn"] == "ver2":
            res = run_ref(ss.get_analog_partial_sums_autograd_ver2, cfg, inp)
            auto = run_ref(ss.get_analog_partial_sums, cfg, inp, autograd=True) if cfg.get("auto") else None
        elif cfg["fn"] == "adcless":
            res = run_ref(ss.get_adcless_cim_output, cfg, inp)
            auto = None
        else:
            res = run_ref(bk.get_analog_partial_sums_autograd_ver2, cfg, inp)
            auto = run_ref(bk.get_analog_partial_sums, cfg, inp, autograd=True)
        extra = check_oracle(name, cfg, inp, res)
        arrays = {("in_" + k): v.numpy() for k, v in inp.items() if v is not None}
        arrays.update({("ref_" + k): v for k, v in res.items()})
        arrays.update({("ref_" + k): v for k, v in extra.items()})
        if auto is not None:
            arrays.update({("auto_" + k): v for k, v in auto.items()})
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        manifest[name] = dict(kind="shift_function", cfg=cfg, seed=seed)
    with open(os.path.join(HERE, "manifest_shift.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest), "scale/shift golden cases")


if __name__ == "__main__":
    main()

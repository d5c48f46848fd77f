"""Golden vectors for the plain LSQ modules (ActLSQ -> Conv2dLSQ, LinearLSQ), generated from
the REAL reference modules (models/_modules/lsq.py:389-436, :591-662).

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_plain.py

Each case builds the reference modules, runs one training-mode forward (the first-step alpha
initialisation included) and a backward of a seeded grad_out, runs the numpy oracle
(oracle/lsq_plain_oracle.py) on the same inputs and post-initialisation alphas, asserts
agreement, and writes inputs, the initialised alphas and the reference outputs / gradients as
an .npz (data only).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import lsq_plain_oracle as po  # noqa: E402
from make_golden import _import_reference  # noqa: E402

CONV_CASES = [
    ("plain_conv_a4w4_s1", dict(B=2, C=16, O=16, H=8, k=3, s=1, p=1, na=4, nw=4, signed=False, bias=False)),
    ("plain_conv_a8w8_signed_s2_bias", dict(B=2, C=3, O=8, H=9, k=3, s=2, p=1, na=8, nw=8, signed=True, bias=True)),
    ("plain_conv_a8u_w4", dict(B=2, C=8, O=16, H=6, k=3, s=1, p=1, na=8, nw=4, signed=False, bias=False)),
    ("plain_conv_1x1_a3w3", dict(B=4, C=32, O=64, H=4, k=1, s=1, p=0, na=3, nw=3, signed=False, bias=False)),
]
LINEAR_CASES = [
    ("plain_linear_w4_bias", dict(N=8, IN=64, OUT=32, nw=4, bias=True)),
    ("plain_linear_w2", dict(N=16, IN=48, OUT=24, nw=2, bias=False)),
]


def _rel(mine, ref, terms):
    """max |mine - ref| / max(terms): ``terms`` is the tensor's max |ref| (normwise, the
    contractions cancel) or a scale gradient's sum of absolute terms"""
    d = np.abs(np.asarray(mine, np.float64) - np.asarray(ref, np.float64))
    return float(np.max(d) / (np.max(terms) + 1e-30))


def conv_case(ref, cfg, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(cfg["B"], cfg["C"], cfg["H"], cfg["H"], generator=g)
    if not cfg["signed"]:
        x = x.clamp_min(0)
    act = ref.ActLSQ(nbits_a=cfg["na"])
    conv = ref.Conv2dLSQ(cfg["C"], cfg["O"], cfg["k"], stride=cfg["s"], padding=cfg["p"], bias=cfg["bias"],
                         nbits_w=cfg["nw"])
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        if cfg["bias"]:
            conv.bias.copy_(torch.randn(cfg["O"], generator=g) * 0.1)
    act.train()
    conv.train()
    xr = x.clone().requires_grad_(True)
    y = conv(act(xr))
    gout = torch.randn(y.shape, generator=g)
    y.backward(gout)
    res = dict(in_x=x.numpy(), in_weight=conv.weight.detach().numpy().copy(), in_grad=gout.numpy(),
               in_alpha_a=act.alpha.detach().numpy().copy(), in_alpha_w=conv.alpha.detach().numpy().copy(),
               in_signed=act.signed.numpy().copy(),
               ref_y=y.detach().numpy(), ref_grad_x=xr.grad.numpy(), ref_grad_weight=conv.weight.grad.numpy(),
               ref_grad_alpha_a=act.alpha.grad.numpy(), ref_grad_alpha_w=conv.alpha.grad.numpy())
    if cfg["bias"]:
        res["in_bias"] = conv.bias.detach().numpy().copy()
        res["ref_grad_bias"] = conv.bias.grad.numpy()
    o = po.act_conv_chain(x.numpy(), res["in_alpha_a"][0], cfg["na"], bool(res["in_signed"][0]), res["in_weight"],
                          res["in_alpha_w"][0], cfg["nw"], res.get("in_bias"), (cfg["s"],) * 2, (cfg["p"],) * 2,
                          gout.numpy())
    errs = dict(y=_rel(o["y"], res["ref_y"], np.abs(res["ref_y"]).max()),
                gx=_rel(o["grad_x"], res["ref_grad_x"], np.abs(res["ref_grad_x"]).max()),
                gw=_rel(o["grad_weight"], res["ref_grad_weight"], np.abs(res["ref_grad_weight"]).max()),
                ga=_rel(o["grad_alpha_a"], res["ref_grad_alpha_a"][0], o["abs_alpha_a"]),
                gaw=_rel(o["grad_alpha_w"], res["ref_grad_alpha_w"][0], o["abs_alpha_w"]))
    res["ref_abs_alpha_a"] = np.float64(o["abs_alpha_a"])
    res["ref_abs_alpha_w"] = np.float64(o["abs_alpha_w"])
    return res, errs


def linear_case(ref, cfg, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(cfg["N"], cfg["IN"], generator=g)
    lin = ref.LinearLSQ(cfg["IN"], cfg["OUT"], bias=cfg["bias"], nbits_w=cfg["nw"])
    with torch.no_grad():
        lin.weight.copy_(torch.randn(lin.weight.shape, generator=g) * 0.2)
        if cfg["bias"]:
            lin.bias.copy_(torch.randn(cfg["OUT"], generator=g) * 0.1)
    lin.train()
    xr = x.clone().requires_grad_(True)
    y = lin(xr)
    gout = torch.randn(y.shape, generator=g)
    y.backward(gout)
    res = dict(in_x=x.numpy(), in_weight=lin.weight.detach().numpy().copy(), in_grad=gout.numpy(),
               in_alpha_w=lin.alpha.detach().numpy().copy(),
               ref_y=y.detach().numpy(), ref_grad_x=xr.grad.numpy(), ref_grad_weight=lin.weight.grad.numpy(),
               ref_grad_alpha_w=lin.alpha.grad.numpy())
    if cfg["bias"]:
        res["in_bias"] = lin.bias.detach().numpy().copy()
        res["ref_grad_bias"] = lin.bias.grad.numpy()
    o = po.linear_lsq(x.numpy(), res["in_weight"], res["in_alpha_w"][0], cfg["nw"], res.get("in_bias"), gout.numpy())
    errs = dict(y=_rel(o["y"], res["ref_y"], np.abs(res["ref_y"]).max()),
                gx=_rel(o["grad_x"], res["ref_grad_x"], np.abs(res["ref_grad_x"]).max()),
                gw=_rel(o["grad_weight"], res["ref_grad_weight"], np.abs(res["ref_grad_weight"]).max()),
                gaw=_rel(o["grad_alpha"], res["ref_grad_alpha_w"][0], o["abs_alpha"]))
    res["ref_abs_alpha_w"] = np.float64(o["abs_alpha"])
    return res, errs


def main():
    ref = _import_reference()
    torch.set_num_threads(4)
    manifest = {}
    for idx, (name, cfg) in enumerate(CONV_CASES + LINEAR_CASES):
        seed = 5000 + idx
        res, errs = (conv_case if name.startswith("plain_conv") else linear_case)(ref, cfg, seed)
        print(f"  {name}: " + "  ".join(f"{k} {v:.1e}" for k, v in errs.items()))
        assert max(errs.values()) < 1e-5, (name, errs)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
        manifest[name] = dict(kind="conv" if name.startswith("plain_conv") else "linear", cfg=cfg, seed=seed)
    with open(os.path.join(HERE, "manifest_plain.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest), "plain LSQ golden cases")


if __name__ == "__main__":
    main()

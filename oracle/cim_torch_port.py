"""Op-faithful torch-CPU restatement of the CiM partial-sum Function -- the CPU BASELINE leg.

TEST / MEASUREMENT INFRASTRUCTURE ONLY: ``bench.py``'s ``cpu_baseline`` times it on the GPU
box's host cores (the reference itself cannot travel there); nothing in ``cim_quantization_amd``
imports it.  It issues the reference's op sequence of ``get_cim_output_signed`` (lsq.py:92-386)
on torch CPU tensors -- im2col with ``F.unfold``, the floor/remainder bit slicing, one matmul per
(tile, a-slice, w-slice) into an fp16 partial-sum buffer, the ADC, the shift-and-add, and the
backward's repeat / mask / per-tile matmuls / ``F.fold`` -- so its time tracks the reference's CPU
path (the in-container ratio to the reference).  Numerics follow ``cim_oracle`` (the
numpy restatement pinned by the golden vectors); this module is timed, not used as a checker.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _slices(t: torch.Tensor, n: int, bs: int) -> torch.Tensor:
    """floor(t / 2^(bs*i)) then remainder 2^bs, LSB first (lsq.py:466-480)."""
    s = t.unsqueeze(0).repeat(n, *([1] * t.dim()))
    for i in range(1, n):
        s[i] = torch.floor(s[i] / (2 ** bs) ** i)
    return torch.remainder(s, 2 ** bs)


def _slices_signed(t: torch.Tensor, n: int, bs: int) -> torch.Tensor:
    """positive and negated-negative parts sliced separately (lsq.py:438-464, 483-509)."""
    pos = t.clone()
    pos[pos.le(0)] = 0
    neg = t.clone()
    neg[neg.ge(0)] = 0
    return _slices(pos, n, bs) - _slices(-1 * neg, n, bs)


def cim_forward(x_q, w_q, stride, padding, act_bits, act_bs, w_bits, w_bs, adc_bits, arr, binary_mask, alpha, sw, sa,
                signed_act=False):
    """get_cim_output_signed.forward (lsq.py:92-237) on CPU tensors; returns (out [B, P, O], ctx)."""
    x_int = x_q / sa
    w_int = w_q / sw
    ctx = {"x_int8": x_int.to(torch.int8)}
    nbw, nba = int(w_bits / w_bs), int(act_bits / act_bs)
    O, k = w_int.shape[0], w_int.shape[2]
    x_unf = F.unfold(x_int, k, padding=padding, stride=stride).transpose(1, 2)
    B, P, K = x_unf.shape
    xs = (_slices_signed if signed_act else _slices)(x_unf, nba, act_bs).transpose(0, 1)  # [B, nba, P, K]
    ws = _slices_signed(w_int.view(O, -1).t(), nbw, w_bs)                                 # [nbw, K, O]
    ctx["w_sliced8"] = ws.to(torch.int8)
    T = math.ceil(K / arr)
    ps = torch.empty(B, T, nbw, nba, P, O, dtype=torch.float16)
    for i in range(T):
        lo, hi = i * arr, min(K, (i + 1) * arr)
        for j in range(nba):
            for kk in range(nbw):
                ps[:, i, kk, j] = torch.matmul(xs[:, j, :, lo:hi], ws[kk, lo:hi, :])
    ctx["ps"] = ps
    u = ps * sw * sa
    if adc_bits == 1.5:
        adc = torch.round(u / alpha).clamp(-1, 1) * alpha
    elif adc_bits == 1:
        adc = torch.sign(u) * alpha
    else:
        qp, qn = 2 ** (adc_bits - 1) - 1, -(2 ** (adc_bits - 1))
        adc = torch.round(u / (sw * sa)).clamp(qn, qp) * sw * sa
    out = torch.sum(adc * binary_mask, dim=(1, 2, 3))
    ctx.update(shape=(B, T, nbw, nba, P, O, K), k=k, stride=stride, padding=padding, hw=x_q.shape[2:], arr=arr,
               act_bits=act_bits, act_bs=act_bs, w_bs=w_bs, adc_bits=adc_bits, alpha=alpha, sw=sw, sa=sa,
               binary_mask=binary_mask, signed=signed_act)
    return out, ctx


def cim_backward(ctx, grad_out):
    """get_cim_output_signed.backward (lsq.py:244-386) on CPU tensors: (grad_x, grad_w, grad_alpha)."""
    B, T, nbw, nba, P, O, K = ctx["shape"]
    sw, sa, alpha = ctx["sw"], ctx["sa"], ctx["alpha"]
    w_sl = ctx["w_sliced8"].float() * sw
    x_unf = F.unfold(ctx["x_int8"].float(), ctx["k"], padding=ctx["padding"], stride=ctx["stride"]).transpose(1, 2)
    xs = (_slices_signed if ctx["signed"] else _slices)(x_unf, nba, ctx["act_bs"]).transpose(0, 1) * sa
    adc_bits = ctx["adc_bits"]
    ps = ctx["ps"].float() * sw * sa / alpha if adc_bits in (1, 1.5) else ctx["ps"].float()
    qp, qn = (1, -1) if adc_bits in (1, 1.5) else (2 ** (adc_bits - 1) - 1, -(2 ** (adc_bits - 1)))
    G = grad_out.unsqueeze(1).unsqueeze(1).unsqueeze(1).repeat(1, T, nbw, nba, 1, 1) * ctx["binary_mask"]
    G_after = G.clone()
    ge, le = ps.ge(qp + 1e-5), ps.le(qn - 1e-5)
    G[torch.logical_or(ge, le)] = 0
    grad_alpha = None
    if adc_bits in (1, 1.5):
        q = torch.sign(ps) if adc_bits == 1 else torch.round(ps)
        if adc_bits == 1.5:
            q[ge] = qp
            q[le] = qn
        grad_alpha = torch.sum(q * (1.0 / math.sqrt(ps.numel() * qp)) * G_after, dim=(0, 4), keepdim=True)
    gi = torch.empty(B, nbw, nba, P, K)
    gw = torch.empty(B, nbw, nba, K, O)
    for i in range(T):
        lo, hi = i * ctx["arr"], min(K, (i + 1) * ctx["arr"])
        for j in range(nba):
            for kk in range(nbw):
                gi[:, kk, j, :, lo:hi] = torch.matmul(G[:, i, kk, j], w_sl[kk, lo:hi, :].t())
                gw[:, kk, j, lo:hi, :] = torch.matmul(xs[:, j, :, lo:hi].transpose(1, 2), G[:, i, kk, j])
    gw = gw.sum(0).sum(1)
    for i in range(1, nbw):
        gw[i] = gw[i] / (2 ** ctx["w_bs"]) ** i
    gw = gw.mean(0).t().reshape(O, -1, ctx["k"], ctx["k"])
    gi = gi.sum(1)
    for i in range(1, nba):
        gi[:, i] = gi[:, i] / (2 ** ctx["act_bs"]) ** i
    gi = gi.mean(1)
    gx = F.fold(gi.transpose(1, 2), ctx["hw"], ctx["k"], padding=ctx["padding"], stride=ctx["stride"])
    return gx, gw, grad_alpha

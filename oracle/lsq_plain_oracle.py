"""CPU restatement (numpy) of the reference's plain LSQ modules -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and the golden generator) import this; the product path is libcimq
(cimq_part_qlsq.hip) behind cim_quantization_amd.functional.lsq_quantize / qconv2d.  Pinned by
tests/golden/plain_*.npz, which tests/golden/make_golden_plain.py generates from the real
reference modules (models/_modules/lsq.py) in the build container.

Follows, in fp32 with the reference's op order:
  ActLSQ.forward      lsq.py:620-662  x_q = round_pass(clamp(x / a, Qn, Qp)), a = grad_scale(alpha, g)
  Conv2dLSQ.forward   lsq.py:396-436  y = conv2d(x_q, w_q, bias) * a * ws, w_q = round_pass(clamp(w / ws))
  LinearLSQ.forward   lsq.py:598-617  y = linear(x, round_pass(clamp(w / a)) * a, bias)
and torch autograd's backward of those graphs (round_pass / grad_scale: _quan_base.py STE forms).
Reductions (the scale gradients, the conv contractions) are evaluated in float64 -- the
reference's own summation order is torch's, so the tests compare within a tolerance scaled by
the sum of absolute terms, which these functions also return.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def grad_scale_value(alpha, g):
    """(alpha - alpha * g).detach() + alpha * g in fp32 (_quan_base.py grad_scale)."""
    a, g = F32(alpha), F32(g)
    ag = F32(a * g)
    return F32(F32(a - ag) + ag)


def round_pass_value(v):
    """(round(v) - v).detach() + v in fp32 (_quan_base.py round_pass); round half to even."""
    v = np.asarray(v, F32)
    return (np.rint(v).astype(F32) - v).astype(F32) + v


def lsq_forward(x, s, qn, qp, scaled=False):
    """round_pass(clamp(x / s, qn, qp)) [* s] (lsq.py:412, :611, :656)."""
    x = np.asarray(x, F32)
    s = F32(s)
    t = (x / s).astype(F32)
    c = np.clip(t, F32(qn), F32(qp)).astype(F32)
    r = round_pass_value(c)
    return (r * s).astype(F32) if scaled else r


def lsq_backward(x, s, qn, qp, g, scaled=False):
    """autograd of lsq_forward: (grad_x, grad_s, abs_terms_s).  grad_s sums MulBackward's g * r
    (scaled) and DivBackward's -grad_t * ((x / s) / s); float64 sums."""
    x = np.asarray(x, F32)
    g = np.asarray(g, F32)
    s = F32(s)
    t = (x / s).astype(F32)
    r = round_pass_value(np.clip(t, F32(qn), F32(qp)).astype(F32))
    grad_r = (g * s).astype(F32) if scaled else g
    passed = (t >= F32(qn)) & (t <= F32(qp))
    grad_t = np.where(passed, grad_r, F32(0)).astype(F32)
    gx = (grad_t / s).astype(F32)
    div = -(grad_t.astype(np.float64) * (t / s).astype(F32).astype(np.float64))
    mul = (g.astype(np.float64) * r.astype(np.float64)) if scaled else np.zeros(1)
    gs = mul.sum() + div.sum()
    return gx, gs, np.abs(mul).sum() + np.abs(div).sum()


def _unfold(x, KH, KW, stride, padding, dilation):
    """im2col [B, C*KH*KW, Ho*Wo] of NCHW x (float64), zero padding."""
    B, C, H, W = x.shape
    Ho = (H + 2 * padding[0] - dilation[0] * (KH - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * padding[1] - dilation[1] * (KW - 1) - 1) // stride[1] + 1
    xp = np.zeros((B, C, H + 2 * padding[0], W + 2 * padding[1]), np.float64)
    xp[:, :, padding[0]:padding[0] + H, padding[1]:padding[1] + W] = x
    cols = np.empty((B, C, KH, KW, Ho, Wo), np.float64)
    for kh in range(KH):
        for kw in range(KW):
            h0, w0 = kh * dilation[0], kw * dilation[1]
            cols[:, :, kh, kw] = xp[:, :, h0:h0 + stride[0] * (Ho - 1) + 1:stride[0],
                                    w0:w0 + stride[1] * (Wo - 1) + 1:stride[1]]
    return cols.reshape(B, C * KH * KW, Ho * Wo), Ho, Wo


def _fold(cols, shape, KH, KW, stride, padding, dilation, Ho, Wo):
    B, C, H, W = shape
    cols = cols.reshape(B, C, KH, KW, Ho, Wo)
    xp = np.zeros((B, C, H + 2 * padding[0], W + 2 * padding[1]), np.float64)
    for kh in range(KH):
        for kw in range(KW):
            h0, w0 = kh * dilation[0], kw * dilation[1]
            xp[:, :, h0:h0 + stride[0] * (Ho - 1) + 1:stride[0], w0:w0 + stride[1] * (Wo - 1) + 1:stride[1]] += \
                cols[:, :, kh, kw]
    return xp[:, :, padding[0]:padding[0] + H, padding[1]:padding[1] + W]


def qconv_forward(x_q, w_q, a, ws, bias, stride, padding, dilation=(1, 1)):
    """Conv2dLSQ's tail (lsq.py:436): y0 = conv2d(x_q, w_q, bias), y = (y0 * a) * ws.  Integer
    codes: the float64 contraction is exact, then one fp32 rounding (+ bias)."""
    O, C, KH, KW = w_q.shape
    cols, Ho, Wo = _unfold(np.asarray(x_q, np.float64), KH, KW, stride, padding, dilation)
    conv = np.einsum("ok,bkp->bop", np.asarray(w_q, np.float64).reshape(O, -1), cols)
    y0 = conv.astype(F32)
    if bias is not None:
        y0 = (y0 + np.asarray(bias, F32)[None, :, None]).astype(F32)
    y = ((y0 * F32(a)).astype(F32) * F32(ws)).astype(F32)
    B = x_q.shape[0]
    return y.reshape(B, O, Ho, Wo), y0.reshape(B, O, Ho, Wo)


def qconv_backward(x_q, w_q, a, ws, y0, g, stride, padding, dilation=(1, 1)):
    """autograd of y = (conv2d(x_q, w_q, bias) * a) * ws: (grad_x_q, grad_w_q, grad_a, grad_ws,
    grad_bias) and the absolute-term sums of grad_a / grad_ws."""
    g = np.asarray(g, F32)
    y0 = np.asarray(y0, F32)
    a, ws = F32(a), F32(ws)
    y1 = (y0 * a).astype(F32)
    g1 = (g * ws).astype(F32)
    gy0 = (g1 * a).astype(F32)
    d_ws = (g.astype(np.float64) * y1).sum()
    d_a = (g1.astype(np.float64) * y0).sum()
    abs_ws = np.abs(g.astype(np.float64) * y1).sum()
    abs_a = np.abs(g1.astype(np.float64) * y0).sum()
    O, C, KH, KW = w_q.shape
    B = x_q.shape[0]
    cols, Ho, Wo = _unfold(np.asarray(x_q, np.float64), KH, KW, stride, padding, dilation)
    gyf = gy0.reshape(B, O, -1).astype(np.float64)
    gw = np.einsum("bop,bkp->ok", gyf, cols).reshape(O, C, KH, KW)
    gcols = np.einsum("ok,bop->bkp", np.asarray(w_q, np.float64).reshape(O, -1), gyf)
    gx = _fold(gcols, x_q.shape, KH, KW, stride, padding, dilation, Ho, Wo)
    gb = gy0.astype(np.float64).sum(axis=(0, 2, 3))
    return dict(grad_x_q=gx, grad_w_q=gw, grad_a=d_a, grad_ws=d_ws, grad_bias=gb, abs_a=abs_a, abs_ws=abs_ws,
                grad_y0=gy0)


def act_conv_chain(x, alpha_a, nbits_a, signed, weight, alpha_w, nbits_w, bias, stride, padding, g):
    """ActLSQ -> Conv2dLSQ, forward and backward (the chain the golden fixtures record):
    returns y and the gradients of x, alpha_a, weight, alpha_w, bias, with abs-term sums."""
    qn_a, qp_a = (-(2 ** (nbits_a - 1)), 2 ** (nbits_a - 1) - 1) if signed else (0, 2 ** nbits_a - 1)
    qn_w, qp_w = -(2 ** (nbits_w - 1)), 2 ** (nbits_w - 1) - 1
    gs_a = F32(1.0 / np.sqrt(x.size * qp_a))
    gs_w = F32(1.0 / np.sqrt(weight.size * qp_w))
    a = grad_scale_value(alpha_a, gs_a)
    ws = grad_scale_value(alpha_w, gs_w)
    x_q = lsq_forward(x, a, qn_a, qp_a)
    w_q = lsq_forward(weight, ws, qn_w, qp_w)
    y, y0 = qconv_forward(x_q, w_q, a, ws, bias, stride, padding)
    cb = qconv_backward(x_q, w_q, a, ws, y0, g, stride, padding)
    gx, ga_div, abs_ga_div = lsq_backward(x, a, qn_a, qp_a, cb["grad_x_q"].astype(F32))
    gw, gws_div, abs_gws_div = lsq_backward(weight, ws, qn_w, qp_w, cb["grad_w_q"].astype(F32))
    return dict(y=y, grad_x=gx, grad_weight=gw,
                grad_alpha_a=(cb["grad_a"] + ga_div) * float(gs_a), abs_alpha_a=(cb["abs_a"] + abs_ga_div) * float(gs_a),
                grad_alpha_w=(cb["grad_ws"] + gws_div) * float(gs_w),
                abs_alpha_w=(cb["abs_ws"] + abs_gws_div) * float(gs_w),
                grad_bias=cb["grad_bias"], x_q=x_q, w_q=w_q)


def linear_lsq(x, weight, alpha, nbits_w, bias, g):
    """LinearLSQ forward + backward (lsq.py:598-617)."""
    qn, qp = -(2 ** (nbits_w - 1)), 2 ** (nbits_w - 1) - 1
    gs = F32(1.0 / np.sqrt(weight.size * qp))
    a = grad_scale_value(alpha, gs)
    w_q = lsq_forward(weight, a, qn, qp, scaled=True)
    x64 = np.asarray(x, np.float64)
    y = (x64 @ w_q.astype(np.float64).T)
    if bias is not None:
        y = y + np.asarray(bias, np.float64)
    g64 = np.asarray(g, np.float64)
    grad_wq = (g64.reshape(-1, g64.shape[-1]).T @ x64.reshape(-1, x64.shape[-1])).astype(F32)
    gx = g64 @ w_q.astype(np.float64)
    gw, ga, abs_ga = lsq_backward(weight, a, qn, qp, grad_wq, scaled=True)
    return dict(y=y, grad_x=gx, grad_weight=gw, grad_alpha=ga * float(gs), abs_alpha=abs_ga * float(gs),
                grad_bias=None if bias is None else g64.reshape(-1, g64.shape[-1]).sum(0))

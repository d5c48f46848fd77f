"""Module-level CPU oracle: ``Conv2dLSQCiM`` restated on torch-CPU autograd around the
numpy partial-sum Function of ``cim_oracle``.

TEST INFRASTRUCTURE ONLY (see ``cim_oracle`` header).  The LSQ quantisers, the alpha
quantiser and the first-step initialisation are expressed with the same torch-CPU
autograd graph the reference builds (lsq.py:522-588), so the scale gradients
(``alpha_act``, ``alpha_weight``, ``alpha_cim`` through max/min) follow torch's own
backward formulas; the partial-sum Function itself is the numpy restatement.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import cim_oracle as co


def _np(t):
    return None if t is None else t.detach().cpu().numpy()


class OracleCimFunction(torch.autograd.Function):
    """numpy ``get_cim_output_signed`` (lsq.py:89-386) wrapped for autograd; same 17 args."""

    @staticmethod
    def forward(ctx, x_q, w_q, stride, padding, dilation, act_bits, act_bs, w_bits, w_bs,
                adc_bits, arr, binary_mask, alpha_cim, sw, sa, stochastic, signed_act):
        out, c = co.cim_forward(_np(x_q), _np(w_q), stride, padding, dilation, act_bits, act_bs,
                                w_bits, w_bs, adc_bits, arr, _np(binary_mask), _np(alpha_cim),
                                _np(sw), _np(sa), bool(stochastic), _np(signed_act))
        ctx.c = c
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, g):
        gx, gw, ga = co.cim_backward(ctx.c, _np(g))
        ga_t = None if ga is None else torch.from_numpy(np.ascontiguousarray(ga))
        return (torch.from_numpy(gx), torch.from_numpy(gw)) + (None,) * 10 + (ga_t,) + (None,) * 4


class OracleCimShiftFunction(torch.autograd.Function):
    """numpy partial-sum Function with the scale/shift ADC option (cim_oracle.adc_apply beta)."""

    @staticmethod
    def forward(ctx, x_q, w_q, stride, padding, act_bits, act_bs, w_bits, w_bs, adc_bits, arr, binary_mask,
                alpha_q, beta, sw, sa, signed_act):
        out, c = co.cim_forward(_np(x_q), _np(w_q), stride, padding, (1, 1), act_bits, act_bs, w_bits, w_bs,
                                adc_bits, arr, _np(binary_mask), _np(alpha_q), _np(sw), _np(sa), False,
                                _np(signed_act), beta=_np(beta))
        ctx.c = c
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, g):
        gx, gw, ga, gb = co.cim_backward(ctx.c, _np(g))
        t = lambda v: torch.from_numpy(np.ascontiguousarray(v))  # noqa: E731
        return (t(gx), t(gw)) + (None,) * 9 + (t(ga), t(gb)) + (None,) * 3


def _gs(x, s):
    """grad_scale (lsq.py:23-26)."""
    yg = x * s
    return x.detach() - yg.detach() + yg


def _rp(x):
    """round_pass (lsq.py:29-32)."""
    return x.round().detach() - x.detach() + x


class OracleConv2dLSQCiM(torch.nn.Conv2d):
    """Parameters, buffers and forward of ``_Conv2dQCiM``/``Conv2dLSQCiM``
    (_quan_base.py:174-237, lsq.py:511-588), on the CPU."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, nbits_w=8, nbits_a=8, nbits_alpha=8, wbitslice=1,
                 abitslice=1, xbar=64, adcbits=6, stochastic_quant=False, adc_shift=False, **kwargs):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         dilation=dilation, groups=groups, bias=bias)
        self.nbits_w, self.nbits_a, self.nbits_alpha = nbits_w, nbits_a, nbits_alpha
        self.wbitslice, self.abitslice, self.xbar = wbitslice, abitslice, xbar
        self.adcbits, self.stochastic_quant = adcbits, stochastic_quant
        kk = self.kernel_size
        self.num_xbars = int(math.ceil(in_channels * kk[0] * kk[1] / xbar))
        self.num_bit_slice_weight = int(nbits_w / wbitslice)
        self.num_bit_slice_act = int(nbits_a / abitslice)
        self.binary_mask = torch.from_numpy(co.make_binary_mask(
            self.num_bit_slice_weight, self.num_bit_slice_act, wbitslice, abitslice))
        if adcbits in (1, 1.5):
            self.alpha_cim = torch.nn.Parameter(torch.ones(
                1, self.num_xbars, self.num_bit_slice_weight, self.num_bit_slice_act, 1, out_channels))
        else:
            self.alpha_cim = None
        self.alpha_weight = torch.nn.Parameter(torch.ones(1))
        self.alpha_act = torch.nn.Parameter(torch.ones(1))
        self.register_buffer("init_state", torch.zeros(1))
        self.register_buffer("signed_act", torch.zeros(1))
        self.register_buffer("init_state_cim", torch.zeros(1))
        self._state_cache = None  # (parity with the product module; unused here)
        self.adc_shift = bool(adc_shift)
        self.beta_cim = torch.nn.Parameter(torch.zeros_like(self.alpha_cim)) if self.adc_shift else None

    def forward(self, x):
        qn_w, qp_w = co.lsq_weight_params(self.nbits_w)
        _, qp_adc = co.adc_range(self.adcbits)
        first = self.training and self.init_state == 0
        if first and x.min() < -1e-5:
            self.signed_act.data.fill_(1)
        qn_a, qp_a = co.lsq_act_params(self.nbits_a)
        if first:
            self.alpha_act.data.copy_(2 * x.abs().mean() / math.sqrt(qp_a))
            self.alpha_weight.data.copy_(2 * self.weight.abs().mean() / math.sqrt(qp_w))
            self.init_state.fill_(1)
        sa = _gs(self.alpha_act, 1.0 / math.sqrt(x.numel() * qp_a))
        x_q = _rp((x / sa).clamp(qn_a, qp_a)) * sa
        sw = _gs(self.alpha_weight, 1.0 / math.sqrt(self.weight.numel() * qp_w))
        w_q = _rp((self.weight / sw).clamp(qn_w, qp_w)) * sw
        if getattr(self, "debug_retain", False):  # tests: keep the LSQ intermediates' grads
            x_q.retain_grad()
            w_q.retain_grad()
            self.dbg = dict(x=x, x_q=x_q, w_q=w_q, sa=sa, sw=sw, qa=(qn_a, qp_a), qw=(qn_w, qp_w))
        if self.training and self.init_state_cim == 0 and self.alpha_cim is not None:
            a0 = co.alpha_cim_init(_np(x_q), _np(w_q), self.stride, self.padding, self.nbits_a,
                                   self.abitslice, self.nbits_w, self.wbitslice, self.xbar,
                                   _np(sw), _np(sa), self.adcbits)
            self.alpha_cim.data.copy_(torch.from_numpy(a0))
            self.init_state_cim.fill_(1)
        alpha_q = None
        if self.alpha_cim is not None:
            qp_al, qn_al = 2 ** self.nbits_alpha - 1, 1
            a = self.alpha_cim
            scale = (a.max() - a.min()) / (qp_al - qn_al)
            alpha_q = _rp(a / scale).clamp(qn_al, qp_al) * scale
        if self.adcbits == 0:
            return F.conv2d(x_q, w_q, self.bias, self.stride, self.padding, self.dilation)
        if self.adc_shift:
            out = OracleCimShiftFunction.apply(x_q, w_q, self.stride, self.padding, self.nbits_a, self.abitslice,
                                               self.nbits_w, self.wbitslice, self.adcbits, self.xbar,
                                               self.binary_mask, alpha_q, self.beta_cim, sw, sa, self.signed_act)
        else:
            out = OracleCimFunction.apply(x_q, w_q, self.stride, self.padding, self.dilation,
                                          self.nbits_a, self.abitslice, self.nbits_w, self.wbitslice,
                                          self.adcbits, self.xbar, self.binary_mask, alpha_q, sw, sa,
                                          self.stochastic_quant, self.signed_act)
        fx = int((x_q.shape[-1] - self.weight.shape[-1] + 2 * self.padding[0]) / self.stride[0] + 1)
        out = out.transpose(1, 2).view(x_q.shape[0], self.out_channels, fx, fx)
        if self.bias is not None:
            out = out + self.bias
        return out


def alpha_cim_terms(alpha, aa, nbits_alpha=8):
    """Checker helper: per-entry sum of |terms| of grad alpha_cim through the alpha quantiser (lsq.py:566-571).

    alpha_q_e = clamp(round_pass(alpha_e / scale), 1, Qp) * scale with scale = (max - min) / (Qp - 1), so
    d loss / d alpha_f = G_f * pass_f + ([f is the max] - [f is the min]) / (Qp - 1) * sum_e G_e * (r_e - pass_e * v_e)
    (G = d loss / d alpha_q, v = alpha / scale, r its clamped code, pass the clamp mask of rint(v); tied extrema share
    the scale gradient).  ``aa`` is the oracle's fp64 sum of |terms| of G per entry (cim_backward absolute=True), so
    an entry's terms are aa_f * pass_f plus, on the max / min entries, sum_e aa_e * (r_e + pass_e |v_e|) / (Qp - 1):
    the exact first-order error bound of the fp32 sums.  All-equal alpha (scale 0: v infinite or NaN, no entry
    passes) gives every entry the edge form with finite terms."""
    a32 = np.asarray(alpha, np.float32)
    a = a32.astype(np.float64)
    aa = np.broadcast_to(np.asarray(aa, np.float64), a.shape)
    qp = 2 ** nbits_alpha - 1
    # the clamp's pass mask is decided on the ROUNDED value (clamp(round_pass(v), 1, Qp): its input is rint(v)), in
    # fp32 as the module computes it
    sc32 = (a32.max() - a32.min()) / np.float32(qp - 1)
    with np.errstate(all="ignore"):
        v32 = (a32 / sc32).astype(np.float32)
    rv = np.rint(v32).astype(np.float64)
    passed = (rv >= 1) & (rv <= qp)
    vabs = np.where(passed, np.abs(v32.astype(np.float64)), 0.0)
    r = np.nan_to_num(np.clip(rv, 1, qp), nan=float(qp))
    t = aa * passed
    edge = (a == a.max()) | (a == a.min())
    return np.where(edge, aa + (aa * (r + vabs)).sum() / (qp - 1), t)


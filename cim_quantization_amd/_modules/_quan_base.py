"""Quantised-module base classes: the state / kwargs contract of
models/_modules/_quan_base.py (UtkarshSaxena1/CiM_Quantization).

Parameter, buffer and attribute names, shapes and dtypes match the reference so its
checkpoints (state_dict) load unchanged and ``ReplaceModuleTool`` can construct these
classes with the same kwargs.
"""
from __future__ import annotations

import math
from enum import Enum

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

__all__ = ["Qmodes", "_Conv2dQ", "_LinearQ", "_ActQ", "truncation", "get_sparsity_mask",
           "FunStopGradient", "round_pass", "grad_scale", "Qmodes_cim", "_Conv2dQCiM"]


class Qmodes(Enum):
    layer_wise = 1
    kernel_wise = 2


class Qmodes_cim(Enum):
    column_wise = 1
    bit_wise = 2


def grad_scale(x, scale):
    """Forward value x, backward gradient scaled by ``scale`` (_quan_base.py:25-28)."""
    scaled = x * scale
    return (x.detach() - scaled.detach()) + scaled


def round_pass(x):
    """Round in the forward, identity in the backward (_quan_base.py:37-40)."""
    return (x.round().detach() - x.detach()) + x


def get_sparsity_mask(param, sparsity):
    """1 for the entries above the ``sparsity`` quantile of |param| (_quan_base.py:31-34)."""
    k = int(sparsity * param.numel())
    smallest, _ = torch.topk(param.abs().view(-1), k, largest=False, sorted=True)
    return torch.gt(torch.abs(param), smallest.data[-1]).type(param.type())


class FunStopGradient(torch.autograd.Function):
    """Identity whose gradient is multiplied by a 0/1 mask (_quan_base.py:43-54)."""

    @staticmethod
    def forward(ctx, weight, stop_gradient_mask):
        ctx.save_for_backward(stop_gradient_mask)
        return weight

    @staticmethod
    def backward(ctx, grad_outputs):
        (mask,) = ctx.saved_tensors
        return grad_outputs * mask, None


def truncation(fp_data, nbits=8):
    """Power-of-two fixed-point truncation (_quan_base.py:95-103)."""
    il = torch.log2(torch.max(fp_data.max(), fp_data.min().abs())) + 1
    il = math.ceil(il - 1e-5)
    qcode = nbits - il
    scale = 2 ** qcode
    lo, hi = -(2 ** (nbits - 1)), 2 ** (nbits - 1) - 1
    q = torch.clamp(torch.round(scale * fp_data), lo, hi)
    return q / scale, qcode


def get_default_kwargs_q(kwargs_q, layer_type):
    """Fill the defaults of the quantiser kwargs (_quan_base.py:106-137)."""
    defaults = {"nbits": 4}
    if isinstance(layer_type, _Conv2dQCiM):
        defaults["cimmode"] = Qmodes_cim.bit_wise
    if isinstance(layer_type, (_Conv2dQ, _Conv2dQCiM)):
        defaults["mode"] = Qmodes.layer_wise
    for k, v in defaults.items():
        kwargs_q.setdefault(k, v)
    return kwargs_q


class _Conv2dQ(nn.Conv2d):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, **kwargs_q):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         dilation=dilation, groups=groups, bias=bias)
        self.kwargs_q = get_default_kwargs_q(kwargs_q, layer_type=self)
        self.nbits = kwargs_q["nbits"]
        if self.nbits < 0:
            self.register_parameter("alpha", None)
            self.register_parameter("alpha_cim", None)
            return
        self.q_mode = kwargs_q["mode"]
        n = out_channels if self.q_mode == Qmodes.kernel_wise else 1
        self.alpha = Parameter(torch.Tensor(n))
        self.register_buffer("init_state", torch.zeros(1))

    def add_param(self, param_k, param_v):
        self.kwargs_q[param_k] = param_v

    def set_bit(self, nbits):
        self.kwargs_q["nbits"] = nbits

    def extra_repr(self):
        s = super().extra_repr()
        return f"{s}, fake" if self.alpha is None else f"{s}, {self.kwargs_q}"


class _Conv2dQCiM(nn.Conv2d):
    """State of a CiM conv (_quan_base.py:174-237): crossbar count, bit-slice counts, the
    int8 shift-and-add ``binary_mask`` (a plain attribute, wraps for 8-bit layers), the ADC
    scale ``alpha_cim`` [1, T, nbw, nba, 1, O] (ADC 1 / 1.5 bits only), LSQ step sizes and
    the init buffers."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, **kwargs_q):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         dilation=dilation, groups=groups, bias=bias)
        self.kwargs_q = get_default_kwargs_q(kwargs_q, layer_type=self)
        self.nbits_w = kwargs_q["nbits_w"]
        self.nbits_a = kwargs_q["nbits_a"]
        self.nbits_alpha = kwargs_q["nbits_alpha"]
        self.wbitslice = kwargs_q["wbitslice"]
        self.abitslice = kwargs_q["abitslice"]
        self.xbar = kwargs_q["xbar"]
        self.stochastic_quant = kwargs_q["stochastic_quant"]
        self.adcbits = kwargs_q["adcbits"]
        if self.nbits_w < 0:
            self.register_parameter("alpha", None)
            self.register_parameter("alpha_cim", None)
            return
        self.q_mode = kwargs_q["mode"]
        ks = self.kernel_size
        self.num_xbars = int(math.ceil(in_channels * ks[0] * ks[1] / self.xbar))
        self.num_bit_slice_weight = int(self.nbits_w / self.wbitslice)
        self.num_bit_slice_act = int(self.nbits_a / self.abitslice)
        nbw, nba = self.num_bit_slice_weight, self.num_bit_slice_act
        mask = torch.empty(nbw, nba)
        for j in range(nba):
            for k in range(nbw):
                mask[k, j] = float((2 ** self.abitslice) ** j) * float((2 ** self.wbitslice) ** k)
        # float -> int8 keeps the low byte: 2^7 -> -128, >= 2^8 -> 0 (as the reference's cast)
        self.binary_mask = (mask.to(torch.int64) & 0xFF).to(torch.uint8).view(torch.int8).view(
            1, 1, nbw, nba, 1, 1)
        if self.adcbits in (1, 1.5):
            self.alpha_cim = Parameter(torch.ones(1, self.num_xbars, nbw, nba, 1, out_channels),
                                       requires_grad=True)
        else:
            self.alpha_cim = None
        self.alpha_weight = Parameter(torch.ones(1), requires_grad=True)
        self.alpha_act = Parameter(torch.ones(1), requires_grad=True)
        self.register_buffer("init_state", torch.zeros(1))
        self.register_buffer("signed_act", torch.zeros(1))
        self.register_buffer("init_state_cim", torch.zeros(1))

    def add_param(self, param_k, param_v):
        self.kwargs_q[param_k] = param_v

    def set_bit(self, nbits):
        self.kwargs_q["nbits"] = nbits

    def extra_repr(self):
        return f"{super().extra_repr()}, {self.kwargs_q}"


class _LinearQ(nn.Linear):
    def __init__(self, in_features, out_features, bias=True, **kwargs_q):
        super().__init__(in_features=in_features, out_features=out_features, bias=bias)
        self.kwargs_q = get_default_kwargs_q(kwargs_q, layer_type=self)
        self.nbits = kwargs_q["nbits"]
        if self.nbits < 0:
            self.register_parameter("alpha", None)
            return
        self.alpha = Parameter(torch.Tensor(1))
        self.register_buffer("init_state", torch.zeros(1))

    def add_param(self, param_k, param_v):
        self.kwargs_q[param_k] = param_v

    def extra_repr(self):
        s = super().extra_repr()
        return f"{s}, fake" if self.alpha is None else f"{s}, {self.kwargs_q}"


class _ActQ(nn.Module):
    def __init__(self, **kwargs_q):
        super().__init__()
        self.kwargs_q = get_default_kwargs_q(kwargs_q, layer_type=self)
        self.nbits = kwargs_q["nbits"]
        if self.nbits < 0:
            self.register_parameter("alpha", None)
            return
        self.alpha = Parameter(torch.Tensor(1))
        self.register_buffer("init_state", torch.zeros(1))
        self.register_buffer("signed", torch.zeros(1))

    def add_param(self, param_k, param_v):
        self.kwargs_q[param_k] = param_v

    def set_bit(self, nbits):
        self.kwargs_q["nbits"] = nbits

    def extra_repr(self):
        return "fake" if self.alpha is None else f"{self.kwargs_q}"

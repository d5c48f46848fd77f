"""LSQ and CiM quantised modules -- MI355X drop-in for models/_modules/lsq.py.

``Conv2dLSQCiM`` keeps the reference's constructor, parameters, buffers, first-step
initialisation and output layout, and runs the quantised conv on libcimq's HIP kernels:
the activation quantiser is fused into the CiM kernels (x_q is never materialised), the
partial sums are integer MFMA products, the ADC is applied from exact integer thresholds.
``get_cim_output_signed`` is re-exported with the reference's 17-argument signature.

``Conv2dLSQ`` / ``LinearLSQ`` / ``ActLSQ`` (plain LSQ fake-quant, unused by the CiM
example, SURVEY.md section 8f "next") run their quantisers on libcimq and Conv2dLSQ's conv of
integer codes on int8 MFMA (functional.lsq_quantize / qconv2d).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..functional import (alpha_cim_init, cim_conv2d_lsq, cim_conv2d_lsq_shift, cim_module_conv,  # noqa: F401
                          cim_module_shift_conv, get_adcless_cim_output, get_analog_partial_sums_autograd_ver2,
                          get_cim_output_signed, lsq_quantize, module_shift_supported, qconv2d)
from ._quan_base import (_ActQ, _Conv2dQ, _Conv2dQCiM, _LinearQ, Qmodes, grad_scale,  # noqa: F401
                         round_pass)

__all__ = ["Conv2dLSQ", "LinearLSQ", "ActLSQ", "Conv2dLSQCiM"]


def _act_range(nbits):
    return 0, 2 ** nbits - 1


def _weight_range(nbits):
    return -(2 ** (nbits - 1)), 2 ** (nbits - 1) - 1


def _adc_qp(adcbits):
    if adcbits in (1, 1.5):
        return 1
    return 2 ** (adcbits - 1) - 1


class Conv2dLSQCiM(_Conv2dQCiM):
    """CiM-aware LSQ conv (lsq.py:511-588) on MI355X.

    ``adc_shift=True`` (this build's option, off by default so the state_dict matches the
    reference): a learnable per-(tile, w-slice, a-slice, channel) shift ``beta_cim`` next to
    ``alpha_cim``, and the ADC of test/test_backward_cimlayer_scale_shift.py on the rescaled
    partial sum u -- adcbits 1.5: clamp(round((u-beta)/alpha_q), -1, 1)*alpha_q + beta (ver2);
    adcbits 1: sign((u-beta)/alpha_q)*alpha_q + beta (adcless).  beta starts at 0."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, nbits_w=8, nbits_a=8, nbits_alpha=8, wbitslice=1, abitslice=1,
                 xbar=64, adcbits=6, stochastic_quant=False, adc_shift=False, **kwargs):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=padding, dilation=dilation, groups=groups, bias=bias,
                         nbits_w=nbits_w, nbits_a=nbits_a, nbits_alpha=nbits_alpha, wbitslice=wbitslice,
                         abitslice=abitslice, xbar=xbar, adcbits=adcbits, stochastic_quant=stochastic_quant)
        self.adc_shift = bool(adc_shift)
        if self.adc_shift:
            if adcbits not in (1, 1.5) or stochastic_quant:
                raise ValueError("adc_shift needs a deterministic 1- or 1.5-bit ADC (adcbits 1 / 1.5)")
            self.beta_cim = torch.nn.Parameter(torch.zeros_like(self.alpha_cim))
        else:
            self.beta_cim = None
        self._state_cache = None  # host mirror of (init_state, init_state_cim) to avoid a sync per step
        self.fused = True  # steady state through cimq_module_forward/backward (False: torch quantisers)
        # parameter grads added into the existing .grad buffers inside the library (no
        # AccumulateGrad kernels); set by dist.GradBucket.own(), which owns the exchange
        self.accumulate_grads_in_place = False
        self.tail_stream = None  # GradBucket.own(overlap=True): stream of the parameter-gradient epilogue
        # CIMQ_OPT_RECOMPUTE: where the library has a recompute backward for this shape, keep no per-partial-sum
        # state words between forward and backward (33.5 MB less per 16-channel ResNet-20 layer at B = 256) and
        # recompute the partial sums in the backward -- slower on MI355X, so off by default
        self.recompute_psum = False
        self._wprep = None        # functional.prepare_weights: the next forward's weight side, computed ahead
        self._last_x_shape = None

    def _fused_ready(self):
        """True once the steady-state library path applies and an input shape is known
        (prepare_weights needs both)."""
        flags = self._init_flags()
        return (self.fused and flags[0] and (flags[1] or self.alpha_cim is None) and self.adcbits != 0
                and not self.adc_shift and not self.stochastic_quant and self._last_x_shape is not None
                and self.weight.is_cuda)

    def _shift_fused(self, x):
        """Whether libcimq's fused shift path takes input shape x.shape (cached per shape)."""
        key = tuple(x.shape)
        if getattr(self, "_shift_ok", None) is None or self._shift_ok[0] != key:
            self._shift_ok = (key, x.is_cuda and module_shift_supported(
                key, self.weight, self.stride, self.padding, self.dilation, self.nbits_a, self.abitslice,
                self.nbits_w, self.wbitslice, self.adcbits, self.xbar, self.nbits_alpha))
        return self._shift_ok[1]

    def _load_from_state_dict(self, *args, **kwargs):
        self._state_cache = None
        return super()._load_from_state_dict(*args, **kwargs)

    def _init_flags(self):
        key = (self.init_state._version, self.init_state_cim._version)
        if self._state_cache is None or getattr(self, "_state_key", None) != key:
            self._state_cache = [bool(self.init_state.item() != 0), bool(self.init_state_cim.item() != 0)]
            self._state_key = key
        return self._state_cache

    def forward(self, x):
        qn_w, qp_w = _weight_range(self.nbits_w)
        qp_adc = _adc_qp(self.adcbits)
        qn_a, qp_a = _act_range(self.nbits_a)
        flags = self._init_flags()
        if self.training and not flags[0]:
            # lsq.py:532-542: sign detection and LSQ step-size init on the first training step
            if x.min() < -1e-5:
                self.signed_act.data.fill_(1)
            self.alpha_act.data.copy_(2 * x.abs().mean() / math.sqrt(qp_a))
            self.alpha_weight.data.copy_(2 * self.weight.abs().mean() / math.sqrt(qp_w))
            self.init_state.fill_(1)
            flags[0] = True
        if self.binary_mask.device != x.device:
            self.binary_mask = self.binary_mask.to(x.device)
        if (self.fused and self.adc_shift and flags[0] and flags[1] and self._shift_fused(x)):
            # steady state of the shift ADC on libcimq's fused path (quantisers in the library)
            out = cim_module_shift_conv(x, self.weight, self.alpha_act, self.alpha_weight, self.alpha_cim,
                                        self.beta_cim, self.binary_mask, self.signed_act, self.stride, self.padding,
                                        self.dilation, self.nbits_a, self.abitslice, self.nbits_w, self.wbitslice,
                                        self.xbar, self.nbits_alpha)
            return out if self.bias is None else out + self.bias  # lsq.py:583's broadcast
        if (self.fused and flags[0] and (flags[1] or self.alpha_cim is None) and self.adcbits != 0
                and not self.adc_shift):
            # steady state: the three quantisers and the CiM conv in one library call each way (the
            # weight side possibly prepared ahead by prepare_weights; taken once)
            wprep, self._wprep = self._wprep, None
            self._last_x_shape = tuple(x.shape)
            out = cim_module_conv(x, self.weight, self.alpha_act, self.alpha_weight, self.alpha_cim,
                                  self.binary_mask, self.signed_act, self.stride, self.padding, self.dilation,
                                  self.nbits_a, self.abitslice, self.nbits_w, self.wbitslice, self.adcbits,
                                  self.xbar, self.nbits_alpha, self.accumulate_grads_in_place,
                                  bool(self.stochastic_quant),
                                  self.tail_stream if self.accumulate_grads_in_place else None, wprep,
                                  self.recompute_psum)
            if self.bias is not None:
                out = out + self.bias  # broadcasts over the last axis, as lsq.py:583
            return out
        sa = grad_scale(self.alpha_act, 1.0 / math.sqrt(x.numel() * qp_a))            # lsq.py:547-548
        sw = grad_scale(self.alpha_weight, 1.0 / math.sqrt(self.weight.numel() * qp_w))  # lsq.py:553-554
        w_q = round_pass((self.weight / sw).clamp(qn_w, qp_w)) * sw                   # lsq.py:555
        if self.training and not flags[1] and self.alpha_cim is not None:
            with torch.no_grad():                                                      # lsq.py:557-563
                a0 = alpha_cim_init(x, w_q, sa, sw, self.binary_mask, self.signed_act, self.stride,
                                    self.padding, self.nbits_a, self.abitslice, self.nbits_w,
                                    self.wbitslice, self.adcbits, self.xbar, self.num_xbars)
                self.alpha_cim.data.copy_(a0)
                self.init_state_cim.fill_(1)
            flags[1] = True
        alpha_q = None
        if self.alpha_cim is not None:                                                 # lsq.py:566-571
            qp_al, qn_al = 2 ** self.nbits_alpha - 1, 1
            a = self.alpha_cim
            scale = (a.max() - a.min()) / (qp_al - qn_al)
            alpha_q = round_pass(a / scale).clamp(qn_al, qp_al) * scale
        if self.adcbits == 0:                                                          # lsq.py:584-585
            x_q = round_pass((x / sa).clamp(qn_a, qp_a)) * sa
            return F.conv2d(x_q, w_q, self.bias, self.stride, self.padding, self.dilation)
        if self.adc_shift:
            out = cim_conv2d_lsq_shift(x, w_q, sa, sw, alpha_q, self.beta_cim, self.binary_mask, self.signed_act,
                                       self.stride, self.padding, self.dilation, self.nbits_a, self.abitslice,
                                       self.nbits_w, self.wbitslice, self.adcbits, self.xbar)
        else:
            out = cim_conv2d_lsq(x, w_q, sa, sw, alpha_q, self.binary_mask, self.signed_act, self.stride,
                                 self.padding, self.dilation, self.nbits_a, self.abitslice, self.nbits_w,
                                 self.wbitslice, self.adcbits, self.xbar, bool(self.stochastic_quant))
        fold_x = int((x.shape[-1] - self.weight.shape[-1] + 2 * self.padding[0]) / self.stride[0] + 1)
        out = out.transpose(1, 2).view(x.shape[0], self.out_channels, fold_x, fold_x)  # lsq.py:580-581
        if self.bias is not None:
            out = out + self.bias  # broadcasts over the last axis, as lsq.py:583
        return out


class _HostFlags:
    """Host mirror of the init_state (and ActLSQ's signed) buffers for the plain modules.

    The reference tests ``self.init_state == 0`` (and ActLSQ ``self.signed == 1``) on every
    forward (lsq.py:407, :601, :628, :634, :643); on a GPU tensor each test is a device sync that stalls the
    launch queue. The values are read once and cached, keyed by the buffers' version counters: any
    in-place write to them -- load_state_dict, dist.GradBucket.broadcast_from, torch DDP's buffer
    broadcast from rank 0 before every forward (train.py:232 wraps the model in DDP) -- bumps the counter
    and the next forward re-reads them, so a rank follows rank 0's buffers as the reference does.  Writes
    through ``.data`` (which bypass the counter) update the cache alongside.

    Cost under torch DDP with ``broadcast_buffers=True`` (its default): the per-forward buffer broadcast
    bumps the counters on every step, so every module re-reads its flags with a blocking ``.item()`` per
    forward -- the device sync this cache exists to avoid.  The buffers only change in the first
    (initialising) step, so prefer ``dist.GradBucket`` (one exchange per step, broadcast_from(0) after the
    first step) or DDP with ``broadcast_buffers=False`` after that step."""

    _state_cache = None
    _state_key = None

    def _load_from_state_dict(self, *args, **kwargs):
        self._state_cache = None
        return super()._load_from_state_dict(*args, **kwargs)

    def _flags(self):
        sg = getattr(self, "signed", None)
        key = (self.init_state._version, -1 if sg is None else sg._version)
        if self._state_cache is None or self._state_key != key:
            self._state_cache = [bool(self.init_state.item() != 0), sg is not None and bool(sg.item() == 1)]
            self._state_key = key
        return self._state_cache


class Conv2dLSQ(_HostFlags, _Conv2dQ):
    """Plain LSQ conv (lsq.py:389-436); consumes the (x_q, act_scale) tuple of ActLSQ.

    The weight quantiser runs on libcimq (lsq_quantize) and the conv of the two integer-code
    tensors on int8 MFMA (qconv2d) when x_q comes from this package's ActLSQ (codes by
    construction, their range recorded on the tensor); any other x_q -- the reference accepts
    arbitrary tensors in the tuple -- is convolved by torch's fp32 conv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, nbits_w=8, **kwargs):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=padding, dilation=dilation, groups=groups, bias=bias,
                         nbits=nbits_w)

    def forward(self, x):
        if self.alpha is None:
            return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        x_q, act_scale = x
        qn, qp = _weight_range(self.nbits)
        if self.training and not self._flags()[0]:
            self.alpha.data.copy_(2 * self.weight.abs().mean() / math.sqrt(qp))
            self.init_state.fill_(1)
            self._flags()[0] = True
        ws = grad_scale(self.alpha, 1.0 / math.sqrt(self.weight.numel() * qp))
        w_q = lsq_quantize(self.weight, ws, qn, qp)
        code_range = getattr(x_q, "_cimq_code_range", None)
        if code_range is not None and self.groups == 1 and self.nbits <= 8:
            return qconv2d(x_q, act_scale, w_q, ws, self.bias, self.stride, self.padding, self.dilation,
                           code_range)
        y = F.conv2d(x_q, w_q, self.bias, self.stride, self.padding, self.dilation, self.groups)
        return y * act_scale * ws


class LinearLSQ(_HostFlags, _LinearQ):
    """Plain LSQ linear (lsq.py:591-617): the weight quantiser on libcimq, the fp32 linear of the
    unquantised input by torch's GEMM (the reference quantises only the weight here)."""

    def __init__(self, in_features, out_features, bias=True, nbits_w=4, **kwargs):
        super().__init__(in_features=in_features, out_features=out_features, bias=bias, nbits=nbits_w)

    def forward(self, x):
        if self.alpha is None:
            return F.linear(x, self.weight, self.bias)
        qn, qp = _weight_range(self.nbits)
        if self.training and not self._flags()[0]:
            self.alpha.data.copy_(2 * self.weight.abs().mean() / math.sqrt(qp))
            self.init_state.fill_(1)
            self._flags()[0] = True
        a = grad_scale(self.alpha, 1.0 / math.sqrt(self.weight.numel() * qp))
        return F.linear(x, lsq_quantize(self.weight, a, qn, qp, scaled=True), self.bias)


class ActLSQ(_HostFlags, _ActQ):
    """LSQ activation quantiser (lsq.py:620-662): returns (integer codes, step size); the codes
    come from libcimq and carry their range for Conv2dLSQ's int8 conv."""

    def __init__(self, nbits_a=4, **kwargs):
        super().__init__(nbits=nbits_a)

    def _range(self):
        if self._flags()[1]:
            return -(2 ** (self.nbits - 1)), 2 ** (self.nbits - 1) - 1
        return 0, 2 ** self.nbits - 1

    def forward(self, x):
        if self.alpha is None:
            return x
        if self.training and not self._flags()[0]:
            if x.min() < -1e-5:
                self.signed.data.fill_(1)
                self._flags()[1] = True
            _, qp = self._range()
            self.alpha.data.copy_(2 * x.abs().mean() / math.sqrt(qp))
            self.init_state.fill_(1)
            self._flags()[0] = True
        qn, qp = self._range()
        a = grad_scale(self.alpha, 1.0 / math.sqrt(x.numel() * qp))
        x_q = lsq_quantize(x, a, qn, qp)
        if -128 <= qn and qp <= 255 and (qn >= 0 or qp <= 127):
            x_q._cimq_code_range = (int(qn), int(qp))
        return x_q, a

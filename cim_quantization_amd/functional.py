"""Autograd Functions backed by libcimq (HIP, gfx950).

``get_cim_output_signed``  drop-in for the reference Function of the same name
                           (models/_modules/lsq.py:89-386): same 17 positional args,
                           same [B, P, O] output, same 17-tuple of grads.
``cim_conv2d_lsq``         the fused path used by ``Conv2dLSQCiM``: the activation LSQ
                           quantiser (lsq.py:547-549) runs inside the CiM kernels, so x_q
                           is never materialised; grads flow to x and to the step size sa.
``get_analog_partial_sums_autograd_ver2`` / ``get_adcless_cim_output``
                           drop-ins for the scale + shift ADC Functions of
                           test/test_backward_cimlayer_scale_shift.py (:336-546 / :113-334):
                           same 14 positional args, grads for x, w, alpha_cim, beta_cim.
``cim_conv2d_lsq_shift``   the scale + shift ADC as a Conv2dLSQCiM option (adc_shift=True).

Device-only: CPU tensors raise (there is no CPU fallback in the product path).
"""
from __future__ import annotations

import contextlib
import ctypes
import math

import torch

from . import _lib


def _require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("cim_quantization_amd runs on ROCm devices only (got a CPU tensor); "
                               "the CPU restatement lives in oracle/ and is test infrastructure")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def stochastic_seed() -> int:
    """Philox key of one stochastic-ADC call, drawn from torch's default CPU generator: the
    draws are reproducible under ``torch.manual_seed`` (the reference draws torch.cuda
    uniform_ noise, lsq.py:215-216) and no device synchronisation is needed."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def _f32(t, device):
    t = t if torch.is_tensor(t) else torch.tensor(t)
    return t.detach().to(device=device, dtype=torch.float32).contiguous()


def _geometry(x, w, stride, padding, dilation):
    stride = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
    padding = tuple(padding) if isinstance(padding, (tuple, list)) else (padding, padding)
    dilation = tuple(dilation) if isinstance(dilation, (tuple, list)) else (dilation, dilation)
    if tuple(dilation) != (1, 1):
        # lsq.py:141 unfolds without dilation while lsq.py:382 folds with it; only 1 is consistent
        raise NotImplementedError("CiM conv supports dilation 1 only (as the reference's unfold)")
    B, C, H, W = x.shape
    O, Cw, KH, KW = w.shape
    if Cw != C:
        raise ValueError(f"weight in_channels {Cw} != input channels {C} (groups are not supported)")
    return B, C, H, W, O, KH, KW, stride, padding


class get_cim_output_signed(torch.autograd.Function):
    """HIP implementation of ``get_cim_output_signed`` (lsq.py:89-386)."""

    @staticmethod
    def forward(ctx, x, w, conv_stride, conv_padding, conv_dilation, act_bits, act_bit_slice,
                weight_bits, weight_bit_slice, adc_bits, arr, binary_mask, alpha_cim,
                weight_scaling_factor, act_scaling_factor, stochastic, signed_act):
        if stochastic:
            assert adc_bits == 1.5  # lsq.py:136-137
        _require_device(x)
        dev = x.device
        B, C, H, W, O, KH, KW, st, pd = _geometry(x, w, conv_stride, conv_padding, conv_dilation)
        desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, arr, weight_bits, act_bits,
                              weight_bit_slice, act_bit_slice, adc_bits, _lib.CIMQ_INPUT_XQ,
                              adc_variant=_lib.CIMQ_ADC_STOCHASTIC if stochastic else _lib.CIMQ_ADC_LIBRARY,
                              seed=stochastic_seed() if stochastic else 0)
        sizes = _lib.query_sizes(desc)
        xq = x.detach().to(torch.float32).contiguous()
        wq = w.detach().to(torch.float32).contiguous()
        sa = _f32(act_scaling_factor, dev).reshape(-1)[:1].contiguous()
        sw = _f32(weight_scaling_factor, dev).reshape(-1)[:1].contiguous()
        bm = binary_mask.detach().to(device=dev, dtype=torch.int8).contiguous()
        sg = _f32(signed_act, dev).reshape(-1)[:1].contiguous()
        al = None if alpha_cim is None else alpha_cim.detach().to(device=dev, dtype=torch.float32).contiguous()
        Ho = (H + 2 * pd[0] - KH) // st[0] + 1
        Wo = (W + 2 * pd[1] - KW) // st[1] + 1
        out = torch.empty(B, Ho * Wo, O, device=dev, dtype=torch.float32)
        cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        _lib.check(lib.cimq_forward(desc, xq.data_ptr(), wq.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                                    None if al is None else al.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                    out.data_ptr(), cbuf.data_ptr(), None, _stream()), "cimq_forward")
        ctx.desc, ctx.sizes = desc, sizes
        ctx.bufs = (xq, sa, sw, al, bm, sg, cbuf)
        ctx.save_for_backward(x, w)  # autograd's version check: in-place edits before backward raise
        ctx.wshape, ctx.xshape = wq.shape, xq.shape
        ctx.has_alpha = alpha_cim is not None
        return out

    @staticmethod
    def backward(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018 -- raises if x / w changed in place since the forward
        xq, sa, sw, al, bm, sg, cbuf = ctx.bufs
        dev = xq.device
        g = grad_output.detach().to(torch.float32).contiguous()
        gx = torch.empty(ctx.xshape, device=dev, dtype=torch.float32)
        gw = torch.empty(ctx.wshape, device=dev, dtype=torch.float32)
        ga = torch.empty_like(al) if (ctx.has_alpha and al is not None) else None
        ws = torch.empty(max(ctx.sizes.bwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        _lib.check(lib.cimq_backward(ctx.desc, g.data_ptr(), xq.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                                     None if al is None else al.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                     cbuf.data_ptr(), gx.data_ptr(), gw.data_ptr(),
                                     None if ga is None else ga.data_ptr(), None, ws.data_ptr(),
                                     _stream()), "cimq_backward")
        return (gx, gw) + (None,) * 10 + (ga,) + (None,) * 4


class _CimConv2dLSQ(torch.autograd.Function):
    """Fused LSQ-activation-quantiser + CiM conv (lsq.py:547-549 followed by lsq.py:578)."""

    @staticmethod
    def forward(ctx, x, w_q, sa, sw, alpha_q, binary_mask, signed_act, stride, padding, dilation,
                nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, stochastic=False):
        _require_device(x)
        dev = x.device
        B, C, H, W, O, KH, KW, st, pd = _geometry(x, w_q, stride, padding, dilation)
        qp_a = float(2 ** nbits_a - 1)
        desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, xbar, nbits_w, nbits_a, wbitslice,
                              abitslice, adcbits, _lib.CIMQ_INPUT_RAW_LSQ, qp_a,
                              _lib.CIMQ_ADC_STOCHASTIC if stochastic else _lib.CIMQ_ADC_LIBRARY,
                              stochastic_seed() if stochastic else 0)
        sizes = _lib.query_sizes(desc)
        xc = x.detach().to(torch.float32).contiguous()
        wq = w_q.detach().to(torch.float32).contiguous()
        sa_ = sa.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        sw_ = sw.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        al = None if alpha_q is None else alpha_q.detach().to(torch.float32).contiguous()
        bm = binary_mask.to(device=dev, dtype=torch.int8).contiguous()
        sg = signed_act.detach().to(device=dev, dtype=torch.float32).reshape(-1)[:1].contiguous()
        Ho = (H + 2 * pd[0] - KH) // st[0] + 1
        Wo = (W + 2 * pd[1] - KW) // st[1] + 1
        out = torch.empty(B, Ho * Wo, O, device=dev, dtype=torch.float32)
        cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        _lib.check(lib.cimq_forward(desc, xc.data_ptr(), wq.data_ptr(), sa_.data_ptr(), sw_.data_ptr(),
                                    None if al is None else al.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                    out.data_ptr(), cbuf.data_ptr(), None, _stream()), "cimq_forward")
        ctx.desc, ctx.sizes = desc, sizes
        ctx.bufs = (xc, sa_, sw_, al, bm, sg, cbuf)
        ctx.save_for_backward(x, w_q)
        ctx.wshape = wq.shape
        ctx.has_alpha = alpha_q is not None
        return out

    @staticmethod
    def backward(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018 -- version check of x / w_q
        xc, sa, sw, al, bm, sg, cbuf = ctx.bufs
        dev = xc.device
        g = grad_output.detach().to(torch.float32).contiguous()
        gx = torch.empty_like(xc)
        gw = torch.empty(ctx.wshape, device=dev, dtype=torch.float32)
        gsa = torch.empty(1, device=dev, dtype=torch.float32)
        ga = torch.empty_like(al) if (ctx.has_alpha and al is not None) else None
        ws = torch.empty(max(ctx.sizes.bwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        _lib.check(lib.cimq_backward(ctx.desc, g.data_ptr(), xc.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                                     None if al is None else al.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                     cbuf.data_ptr(), gx.data_ptr(), gw.data_ptr(),
                                     None if ga is None else ga.data_ptr(), gsa.data_ptr(), ws.data_ptr(),
                                     _stream()), "cimq_backward")
        return (gx, gw, gsa, None, ga) + (None,) * 12


def cim_conv2d_lsq(x, w_q, sa, sw, alpha_q, binary_mask, signed_act, stride, padding, dilation,
                   nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, stochastic=False):
    """out[B, P, O] of the fused act-LSQ + CiM conv; differentiable in x, w_q, sa, alpha_q.
    ``stochastic``: the stochastic 1.5-bit ADC of lsq.py:205-221 in the forward."""
    return _CimConv2dLSQ.apply(x, w_q, sa, sw, alpha_q, binary_mask, signed_act, stride, padding,
                               dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, stochastic)


# ---------------------------------------------------------------------------------------------
# scale + shift ADC (test/test_backward_cimlayer_scale_shift.py)
# ---------------------------------------------------------------------------------------------
def _mask_int8(binary_mask, dev):
    bm = binary_mask.detach().to(device=dev)
    b8 = bm.to(torch.int8)
    if not torch.equal(b8.to(bm.dtype), bm):
        raise ValueError("binary_mask values must be int8 integers (as _Conv2dQCiM builds them)")
    return b8.contiguous()


def _shift_forward(ctx, x, w, sa, sw, alpha, beta, binary_mask, signed_act, stride, padding, dilation,
                   act_bits, act_bs, w_bits, w_bs, adc_bits, arr, variant, input_kind, qp_a):
    _require_device(x)
    dev = x.device
    B, C, H, W, O, KH, KW, st, pd = _geometry(x, w, stride, padding, dilation)
    desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, arr, w_bits, act_bits, w_bs, act_bs, adc_bits,
                          input_kind, qp_a, variant)
    sizes = _lib.query_sizes(desc)
    xc = x.detach().to(torch.float32).contiguous()
    wc = w.detach().to(torch.float32).contiguous()
    sa_ = _f32(sa, dev).reshape(-1)[:1].contiguous()
    sw_ = _f32(sw, dev).reshape(-1)[:1].contiguous()
    al = _f32(alpha, dev)
    be = _f32(beta, dev)
    T = num_xbars(C, (KH, KW), arr)
    nbw, nba = int(w_bits / w_bs), int(act_bits / act_bs)
    if al.numel() != T * nbw * nba * O or be.numel() != T * nbw * nba * O:
        al = al.expand(1, T, nbw, nba, 1, O).contiguous()
        be = be.expand(1, T, nbw, nba, 1, O).contiguous()
    bm = _mask_int8(binary_mask, dev)
    sg = _f32(signed_act, dev).reshape(-1)[:1].contiguous()
    Ho = (H + 2 * pd[0] - KH) // st[0] + 1
    Wo = (W + 2 * pd[1] - KW) // st[1] + 1
    out = torch.empty(B, Ho * Wo, O, device=dev, dtype=torch.float32)
    cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
    lib = _lib.load()
    _lib.check(lib.cimq_shift_forward(desc, xc.data_ptr(), wc.data_ptr(), sa_.data_ptr(), sw_.data_ptr(),
                                      al.data_ptr(), be.data_ptr(), bm.data_ptr(), sg.data_ptr(), out.data_ptr(),
                                      cbuf.data_ptr(), None, _stream()), "cimq_shift_forward")
    ctx.desc, ctx.sizes = desc, sizes
    ctx.bufs = (xc, sa_, sw_, al, be, bm, sg, cbuf)
    ctx.shapes = (wc.shape, alpha.shape if torch.is_tensor(alpha) else al.shape,
                  beta.shape if torch.is_tensor(beta) else be.shape)
    return out


def _shift_backward(ctx, grad_output):
    xc, sa, sw, al, be, bm, sg, cbuf = ctx.bufs
    dev = xc.device
    wshape, ashape, bshape = ctx.shapes
    g = grad_output.detach().to(torch.float32).contiguous()
    gx = torch.empty_like(xc)
    gw = torch.empty(wshape, device=dev, dtype=torch.float32)
    ga = torch.empty_like(al)
    gb = torch.empty_like(be)
    gsa = torch.empty(1, device=dev, dtype=torch.float32)
    ws = torch.empty(max(ctx.sizes.bwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
    lib = _lib.load()
    _lib.check(lib.cimq_shift_backward(ctx.desc, g.data_ptr(), xc.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                                       al.data_ptr(), be.data_ptr(), bm.data_ptr(), sg.data_ptr(), cbuf.data_ptr(),
                                       gx.data_ptr(), gw.data_ptr(), ga.data_ptr(), gb.data_ptr(), gsa.data_ptr(),
                                       ws.data_ptr(), _stream()), "cimq_shift_backward")
    # full [1, T, nbw, nba, 1, O]: autograd sums them down to a broadcast alpha / beta's own shape
    return gx, gw, ga, gb, gsa


class _ShiftTestFunction:
    """Shared body of the 14-argument scale + shift Functions of test_backward_cimlayer_scale_
    shift.py on integer inputs x_int / w_int (no LSQ scales): sa = sw = 1 on the device."""

    @staticmethod
    def _fwd(ctx, variant, x_int, w_int, conv_stride, conv_padding, conv_dilation, act_bits, act_bit_slice,
             weight_bits, weight_bit_slice, adc_bits, arr, binary_mask, alpha_cim, beta_cim):
        if int(weight_bits / weight_bit_slice) != int(act_bits / act_bit_slice):
            # the reference divides the act-slice grads with the weight-slice count as loop
            # bound (scale_shift.py:534): only nbw == nba is well defined there
            raise ValueError("the scale/shift Functions need as many weight as activation bit slices")
        one = torch.ones(1, device=x_int.device, dtype=torch.float32)
        zero = torch.zeros(1, device=x_int.device, dtype=torch.float32)
        ctx.save_for_backward(x_int, w_int)
        return _shift_forward(ctx, x_int, w_int, one, one, alpha_cim, beta_cim, binary_mask, zero, conv_stride,
                              conv_padding, conv_dilation, act_bits, act_bit_slice, weight_bits, weight_bit_slice,
                              adc_bits, arr, variant, _lib.CIMQ_INPUT_XQ, 0.0)

    @staticmethod
    def _bwd(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018 -- version check of x_int / w_int
        gx, gw, ga, gb, _ = _shift_backward(ctx, grad_output)
        return (gx, gw) + (None,) * 10 + (ga, gb)


class get_analog_partial_sums_autograd_ver2(torch.autograd.Function):
    """Scale + shift ADC ``clamp(round((ps-beta)/alpha))*alpha + beta`` on int8-stored partial
    sums (test_backward_cimlayer_scale_shift.py:336-546): same 14 positional args, grads at 0, 1,
    12 (alpha_cim) and 13 (beta_cim)."""

    @staticmethod
    def forward(ctx, x_int, w_int, conv_stride, conv_padding, conv_dilation, act_bits, act_bit_slice,
                weight_bits, weight_bit_slice, adc_bits, arr, binary_mask, alpha_cim, beta_cim):
        v = _lib.CIMQ_ADC_SHIFT_ROUND | _lib.CIMQ_ADC_F_PS_INT8 | _lib.CIMQ_ADC_F_SHIFT_RANGE
        return _ShiftTestFunction._fwd(ctx, v, x_int, w_int, conv_stride, conv_padding, conv_dilation, act_bits,
                                       act_bit_slice, weight_bits, weight_bit_slice, adc_bits, arr, binary_mask,
                                       alpha_cim, beta_cim)

    @staticmethod
    def backward(ctx, grad_output):
        return _ShiftTestFunction._bwd(ctx, grad_output)


class get_adcless_cim_output(torch.autograd.Function):
    """Scale + shift sign ADC ``sign((ps-beta)/alpha)*alpha + beta`` (test_backward_cimlayer_scale_
    shift.py:113-334): same 14 positional args, grads at 0, 1, 12 and 13."""

    @staticmethod
    def forward(ctx, x_int, w_int, conv_stride, conv_padding, conv_dilation, act_bits, act_bit_slice,
                weight_bits, weight_bit_slice, adc_bits, arr, binary_mask, alpha_cim, beta_cim):
        if adc_bits != 1:
            raise ValueError("get_adcless_cim_output is a 1-bit (sign) ADC")
        v = _lib.CIMQ_ADC_SHIFT_SIGN | _lib.CIMQ_ADC_F_SHIFT_RANGE
        return _ShiftTestFunction._fwd(ctx, v, x_int, w_int, conv_stride, conv_padding, conv_dilation, act_bits,
                                       act_bit_slice, weight_bits, weight_bit_slice, adc_bits, arr, binary_mask,
                                       alpha_cim, beta_cim)

    @staticmethod
    def backward(ctx, grad_output):
        return _ShiftTestFunction._bwd(ctx, grad_output)


class _CimConv2dLSQShift(torch.autograd.Function):
    """Conv2dLSQCiM(adc_shift=True): fused act-LSQ + CiM conv whose ADC is the scale + shift one
    applied to the library's rescaled partial sum u = fp16(ps)*sw*sa (lsq.py:195)."""

    @staticmethod
    def forward(ctx, x, w_q, sa, sw, alpha_q, beta, binary_mask, signed_act, stride, padding, dilation,
                nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar):
        variant = _lib.CIMQ_ADC_SHIFT_SIGN if adcbits == 1 else _lib.CIMQ_ADC_SHIFT_ROUND
        ctx.save_for_backward(x, w_q)
        return _shift_forward(ctx, x, w_q, sa, sw, alpha_q, beta, binary_mask, signed_act, stride, padding,
                              dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, variant,
                              _lib.CIMQ_INPUT_RAW_LSQ, float(2 ** nbits_a - 1))

    @staticmethod
    def backward(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018
        gx, gw, ga, gb, gsa = _shift_backward(ctx, grad_output)
        return (gx, gw, gsa, None, ga, gb) + (None,) * 11


def cim_conv2d_lsq_shift(x, w_q, sa, sw, alpha_q, beta, binary_mask, signed_act, stride, padding, dilation,
                         nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar):
    """out[B, P, O] of the fused act-LSQ + scale/shift-ADC CiM conv; differentiable in x, w_q, sa,
    alpha_q and beta.  adcbits 1.5: clamp(round((u-beta)/alpha), -1, 1)*alpha + beta (ver2 on u);
    adcbits 1: sign((u-beta)/alpha)*alpha + beta (adcless on u)."""
    if adcbits not in (1, 1.5):
        raise ValueError("the scale/shift ADC option needs adcbits 1 or 1.5")
    return _CimConv2dLSQShift.apply(x, w_q, sa, sw, alpha_q, beta, binary_mask, signed_act, stride, padding,
                                    dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar)


class _ChainState:
    """The chained module backward of one device (cimq_module_backward_chain): the epilogues the
    calls left, the tensors each reads / writes (kept alive until it has been issued), the stream
    of the chain, and whether the end-of-backward flush is queued or a chained_epilogues() scope
    owns the flush."""

    def __init__(self):
        self.pending = _lib.Pending()
        self.keep = []
        self.stream = None
        self.queued = False
        self.scopes = 0

    def add(self, bufs):
        # a call that issued the earlier epilogues itself (a full list) leaves only its own
        if _lib.load().cimq_pending_jobs(self.pending) <= 1:
            self.keep = []
        self.keep.append(bufs)

    def flush(self):
        if self.keep:
            _lib.check(_lib.load().cimq_pending_flush(self.pending, self.stream), "cimq_pending_flush")
        self.keep = []
        self.queued = False


_CHAINS = {}
CHAIN_EPILOGUES = True  # tests switch it off to compare against the unchained backward


def _chain(dev):
    return _CHAINS.setdefault(dev.index if dev.index is not None else torch.cuda.current_device(), _ChainState())


@contextlib.contextmanager
def chained_epilogues(device=None):
    """Chain the parameter-gradient epilogues of Conv2dLSQCiM backwards across separate
    ``backward()`` calls made inside this scope (e.g. one per layer, as bench.py does): every
    layer's epilogue is held back and all are launched together, packed, when the scope ends.  Without a scope, a single backward pass chains its layers and flushes
    at its end (a queued autograd callback).  Applies to the in-place accumulating backward
    (GradBucket-owned layers); read the gradients only after the scope."""
    ch = _chain(torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device))
    ch.scopes += 1
    try:
        yield
    finally:
        ch.scopes -= 1
        if ch.scopes == 0:
            ch.flush()


class WeightPrep:
    """The weight side of one Conv2dLSQCiM forward, computed ahead by ``prepare_weights``
    (cimq_module_prepare): the buffer, the descriptors it was made for and the parameter
    versions it saw.  A forward takes it once (``take``) if all three still match."""

    __slots__ = ("buf", "key", "versions")

    def __init__(self, buf, key, versions):
        self.buf, self.key, self.versions = buf, key, versions


def _prep_key(desc, lsq, x_shape):
    return (bytes(desc), lsq.qn_w, lsq.qp_w, lsq.gscale_a, lsq.gscale_w, lsq.nbits_alpha, tuple(x_shape))


def _versions(*ts):
    """Staleness key of a prepared weight side: each tensor's version counter and storage
    address.  An edit through ``p.data`` bumps neither; after one, call prepare_weights again
    (or torch.autograd.graph.increment_version(p)) before the next forward."""
    return tuple(-1 if t is None else (t._version, t.data_ptr()) for t in ts)


def _module_descs(x_shape, weight, stride, padding, dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits,
                  xbar, nbits_alpha, has_alpha, stochastic, recompute=False):
    B, C, H, W = x_shape
    O, _, KH, KW = weight.shape
    st = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
    pd = tuple(padding) if isinstance(padding, (tuple, list)) else (padding, padding)
    qp_a = float(2 ** nbits_a - 1)
    qn_w, qp_w = -(2 ** (nbits_w - 1)), 2 ** (nbits_w - 1) - 1
    desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, xbar, nbits_w, nbits_a, wbitslice,
                          abitslice, adcbits, _lib.CIMQ_INPUT_RAW_LSQ, qp_a,
                          _lib.CIMQ_ADC_STOCHASTIC if stochastic else _lib.CIMQ_ADC_LIBRARY,
                          stochastic_seed() if stochastic else 0,
                          _lib.CIMQ_OPT_RECOMPUTE if recompute else 0)
    lsq = _lib.make_lsq_desc(qn_w, qp_w, 1.0 / math.sqrt(B * C * H * W * qp_a),
                             1.0 / math.sqrt(weight.numel() * qp_w), nbits_alpha if has_alpha else 0)
    return desc, lsq


def prepare_weights(modules, stream=None):
    """Run the weight side of the next forward of every fused Conv2dLSQCiM in ``modules`` (the
    weight and alpha_cim quantisers into the CiM operands and ADC thresholds, lsq.py:552-571) in
    one library call, ahead of the forwards: each layer's forward then only quantises its
    activation.  Call it after the parameters are final for the step (after the optimizer step,
    before the forward pass); a forward whose parameters or input shape changed since, or that
    finds no prepared state, does the whole prologue itself, as without this call.  Layers still
    in their first (initialising) step, stochastic-ADC layers and non-fused paths are skipped."""
    items, keep, taken = [], [], []
    dev = None
    for m in modules:
        if not getattr(m, "_fused_ready", None) or not m._fused_ready():
            continue
        shape = m._last_x_shape
        has_alpha = m.alpha_cim is not None
        desc, lsq = _module_descs(shape, m.weight, m.stride, m.padding, m.dilation, m.nbits_a, m.abitslice,
                                  m.nbits_w, m.wbitslice, m.adcbits, m.xbar, m.nbits_alpha, has_alpha, False,
                                  bool(getattr(m, "recompute_psum", False)))
        sizes = _lib.query_sizes(desc)
        dev = m.weight.device
        buf = torch.empty(max(sizes.wprep_bytes, 1), device=dev, dtype=torch.uint8)
        bm = m.binary_mask.to(device=dev, dtype=torch.int8).contiguous()
        ps = (m.weight, m.alpha_act, m.alpha_weight, m.alpha_cim)
        for t in ps:
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
                raise ValueError("prepare_weights: parameters must be contiguous fp32")
        it = _lib.PrepareItem()
        it.desc = ctypes.pointer(desc)
        it.lsq = ctypes.pointer(lsq)
        it.weight = m.weight.data_ptr()
        it.alpha_act = m.alpha_act.data_ptr()
        it.alpha_weight = m.alpha_weight.data_ptr()
        it.alpha_cim = m.alpha_cim.data_ptr() if has_alpha else None
        it.binary_mask = bm.data_ptr()
        it.wprep = buf.data_ptr()
        items.append(it)
        keep.append((desc, lsq, bm))
        taken.append((m, WeightPrep(buf, _prep_key(desc, lsq, shape), _versions(*ps, m.binary_mask))))
    if not items:
        return 0
    arr = (_lib.PrepareItem * len(items))(*items)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.load().cimq_module_prepare(len(items), arr, s), "cimq_module_prepare")
    for m, wp in taken:
        m._wprep = wp
    return len(items)


class _CimModuleConv(torch.autograd.Function):
    """A whole Conv2dLSQCiM layer after its first-step init (lsq.py:544-581): the activation,
    weight and alpha_cim quantisers run inside libcimq on the raw parameters (no torch ops,
    no materialised x_q / w_q / alpha_q tensors); returns the NCHW output.

    With ``accumulate`` set, the backward adds the parameter gradients straight into the
    parameters' existing ``.grad`` buffers inside the library (what torch's AccumulateGrad
    would do, without its four extra add kernels) and returns None for them.  It does so only
    when all four ``.grad`` buffers exist as contiguous fp32 device tensors; otherwise the
    gradients are returned as usual.  Parameter hooks (e.g. DistributedDataParallel's) do not
    fire for in-place accumulated gradients, so this is for callers that own the gradient
    exchange, like ``dist.GradBucket``.  ``tail_stream`` (accumulate mode only): the parameter-
    gradient epilogue runs there, off the grad_x chain, ordered after this backward by an event;
    the bucket joins that stream before it reads the gradients (GradBucket.join)."""

    @staticmethod
    def forward(ctx, x, weight, alpha_act, alpha_weight, alpha_cim, binary_mask, signed_act, stride, padding,
                dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, nbits_alpha, accumulate=False,
                stochastic=False, tail_stream=None, wprep=None, recompute=False):
        _require_device(x)
        dev = x.device
        B, C, H, W, O, KH, KW, st, pd = _geometry(x, weight, stride, padding, dilation)
        desc, lsq = _module_descs(tuple(x.shape), weight, st, pd, dilation, nbits_a, abitslice, nbits_w, wbitslice,
                                  adcbits, xbar, nbits_alpha, alpha_cim is not None, stochastic, recompute)
        # a prepared weight side (prepare_weights) if it was made for exactly this call
        ctx.wprep_buf = None
        if (wprep is not None and not stochastic and wprep.key == _prep_key(desc, lsq, x.shape)
                and wprep.versions == _versions(weight, alpha_act, alpha_weight, alpha_cim, binary_mask)):
            lsq.wprep = wprep.buf.data_ptr()
            ctx.wprep_buf = wprep.buf
        sizes = _lib.query_sizes(desc)
        xc = x.detach().to(torch.float32).contiguous()
        wc = weight.detach().to(torch.float32).contiguous()
        aa = alpha_act.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        aw = alpha_weight.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        ac = None if alpha_cim is None else alpha_cim.detach().to(torch.float32).contiguous()
        bm = binary_mask.to(device=dev, dtype=torch.int8).contiguous()
        sg = signed_act.detach().to(device=dev, dtype=torch.float32).reshape(-1)[:1].contiguous()
        Ho = (H + 2 * pd[0] - KH) // st[0] + 1
        Wo = (W + 2 * pd[1] - KW) // st[1] + 1
        out = torch.empty(B, O, Ho, Wo, device=dev, dtype=torch.float32)
        # the module ctx: no per-partial-sum state words where the backward recomputes them (ABI 13)
        cbuf = torch.empty(max(sizes.module_ctx_bytes, 1), device=dev, dtype=torch.uint8)
        ws = torch.empty(max(sizes.fwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        _lib.check(lib.cimq_module_forward(desc, lsq, xc.data_ptr(), wc.data_ptr(), aa.data_ptr(), aw.data_ptr(),
                                           None if ac is None else ac.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                           out.data_ptr(), cbuf.data_ptr(), ws.data_ptr(), _stream()),
                   "cimq_module_forward")
        ctx.desc, ctx.lsq, ctx.sizes = desc, lsq, sizes
        ctx.bufs = (xc, wc, aa, aw, ac, bm, sg, cbuf)
        ctx.module_path = True  # a cimq_module_forward ctx (debug_state_codes)
        # the backward reads x and the raw parameters again (act-LSQ / weight-LSQ STE); saving
        # them lets autograd's version counters catch an in-place change in between
        ctx.save_for_backward(x, weight, alpha_act, alpha_weight, alpha_cim)
        ctx.params = (weight, alpha_act, alpha_weight, alpha_cim) if accumulate else None
        ctx.tail_stream = tail_stream if accumulate else None
        return out

    @staticmethod
    def _grad_targets(ctx):
        """The parameters' .grad buffers when the backward may accumulate into them."""
        if ctx.params is None:
            return None
        grads = []
        for p in ctx.params:
            if p is None:
                grads.append(None)
                continue
            g = p.grad
            if (g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.device != p.device
                    or g.shape != p.shape):
                return None
            grads.append(g)
        return grads

    @staticmethod
    def backward(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018 -- version check of x and the parameters
        xc, wc, aa, aw, ac, bm, sg, cbuf = ctx.bufs
        dev = xc.device
        g = grad_output.detach().to(torch.float32).contiguous()
        gx = torch.empty_like(xc)
        targets = _CimModuleConv._grad_targets(ctx)
        lsq = ctx.lsq
        side = ctx.tail_stream if targets is not None else None
        if targets is not None:
            gw, gaa, gaw, gac = targets
            lsq = _lib.make_lsq_desc(lsq.qn_w, lsq.qp_w, lsq.gscale_a, lsq.gscale_w, lsq.nbits_alpha,
                                     _lib.CIMQ_LSQ_ACCUMULATE_GRADS | (_lib.CIMQ_LSQ_DEFER_GW if side else 0),
                                     lsq.wprep)
        else:
            gw = torch.empty_like(wc)
            gaa = torch.empty(1, device=dev, dtype=torch.float32)
            gaw = torch.empty(1, device=dev, dtype=torch.float32)
            gac = None if ac is None else torch.empty_like(ac)
        ws = torch.empty(max(ctx.sizes.bwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        lib = _lib.load()
        if targets is not None and side is None and CHAIN_EPILOGUES:
            # chained: this layer's epilogue waits in the pending list; the flush launches all of
            # them packed into a few launches
            ch = _chain(dev)
            stream = _stream()
            if ch.keep and ch.stream != stream:
                ch.flush()
            if ch.scopes == 0 and not ch.queued:
                torch.autograd.Variable._execution_engine.queue_callback(ch.flush)
                ch.queued = True
            ch.stream = stream
            _lib.check(lib.cimq_module_backward_chain(ctx.desc, lsq, g.data_ptr(), xc.data_ptr(), wc.data_ptr(),
                                                      aa.data_ptr(), aw.data_ptr(),
                                                      None if ac is None else ac.data_ptr(), bm.data_ptr(),
                                                      sg.data_ptr(), cbuf.data_ptr(), gx.data_ptr(), gw.data_ptr(),
                                                      gaa.data_ptr(), gaw.data_ptr(),
                                                      None if gac is None else gac.data_ptr(), ws.data_ptr(),
                                                      ch.pending, stream), "cimq_module_backward_chain")
            ch.add((ws, cbuf, wc, ac, gw, gaa, gaw, gac, ctx.wprep_buf))
            return (gx,) + (None,) * 21
        _lib.check(lib.cimq_module_backward(ctx.desc, lsq, g.data_ptr(), xc.data_ptr(), wc.data_ptr(),
                                            aa.data_ptr(), aw.data_ptr(), None if ac is None else ac.data_ptr(),
                                            bm.data_ptr(), sg.data_ptr(), cbuf.data_ptr(), gx.data_ptr(),
                                            gw.data_ptr(), gaa.data_ptr(), gaw.data_ptr(),
                                            None if gac is None else gac.data_ptr(), ws.data_ptr(), _stream()),
                   "cimq_module_backward")
        if side is not None:
            # the parameter-gradient half (the grad_w kernel of the v7 layers, then the epilogue) on
            # the bucket's stream: the next layer's backward does not wait for it; grad_out / ws /
            # ctx stay alive until that stream is done with them
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                _lib.check(lib.cimq_module_backward_params(ctx.desc, lsq, g.data_ptr(), wc.data_ptr(),
                                                           None if ac is None else ac.data_ptr(), cbuf.data_ptr(),
                                                           gw.data_ptr(), gaa.data_ptr(), gaw.data_ptr(),
                                                           None if gac is None else gac.data_ptr(), ws.data_ptr(),
                                                           side.cuda_stream), "cimq_module_backward_params")
            for t in (g, ws, cbuf, wc) + ((ac,) if ac is not None else ()) + \
                    ((ctx.wprep_buf,) if ctx.wprep_buf is not None else ()):
                t.record_stream(side)
        if targets is not None:
            return (gx,) + (None,) * 21
        return (gx, gw, gaa, gaw, gac) + (None,) * 17


def cim_module_conv(x, weight, alpha_act, alpha_weight, alpha_cim, binary_mask, signed_act, stride, padding,
                    dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar, nbits_alpha,
                    accumulate=False, stochastic=False, tail_stream=None, wprep=None, recompute=False):
    """NCHW output of a Conv2dLSQCiM layer (quantisers fused); differentiable in x, weight and
    the three step-size parameters (alpha_act and alpha_weight are 1-element tensors).
    ``accumulate`` / ``tail_stream``: see _CimModuleConv; ``stochastic``: the stochastic 1.5-bit ADC;
    ``wprep``: a WeightPrep from prepare_weights (used only if it matches this call); ``recompute``:
    CIMQ_OPT_RECOMPUTE (no state words in the ctx where a recompute backward exists; slower)."""
    return _CimModuleConv.apply(x, weight, alpha_act, alpha_weight, alpha_cim, binary_mask, signed_act, stride,
                                padding, dilation, nbits_a, abitslice, nbits_w, wbitslice, adcbits, xbar,
                                nbits_alpha, accumulate, stochastic, tail_stream, wprep, recompute)


def _shift_module_descs(x_shape, weight, stride, padding, dilation, nbits_a, abitslice, nbits_w, wbitslice, xbar,
                        nbits_alpha):
    desc, lsq = _module_descs(tuple(x_shape), weight, stride, padding, dilation, nbits_a, abitslice, nbits_w,
                              wbitslice, 1.5, xbar, nbits_alpha, True, False)
    desc.adc_variant = _lib.CIMQ_ADC_SHIFT_ROUND
    return desc, lsq


def module_shift_supported(x_shape, weight, stride, padding, dilation, nbits_a, abitslice, nbits_w, wbitslice,
                           adcbits, xbar, nbits_alpha):
    """Whether cim_module_shift_conv takes this Conv2dLSQCiM(adc_shift=True) layer (libcimq's fused
    shift path: adc 1.5, 2 or 3 equal slices, a fast-path conv shape); else the module quantises in
    torch and calls the unfused shift entry points."""
    if adcbits != 1.5 or len(x_shape) != 4:
        return False
    dl = tuple(dilation) if isinstance(dilation, (tuple, list)) else (dilation, dilation)
    if dl != (1, 1):
        return False
    desc, _ = _shift_module_descs(x_shape, weight, stride, padding, dilation, nbits_a, abitslice, nbits_w, wbitslice,
                                  xbar, nbits_alpha)
    return bool(_lib.load().cimq_module_shift_supported(desc))


class _CimModuleShiftConv(torch.autograd.Function):
    """Conv2dLSQCiM(adc_shift=True) after its first-step init: as _CimModuleConv (activation, weight and
    alpha_cim quantisers inside libcimq), with the scale + shift ADC of test_backward_cimlayer_scale_
    shift.py:336-546 on the rescaled partial sum; differentiable in x, weight, alpha_act, alpha_weight,
    alpha_cim and beta_cim.  NCHW output."""

    @staticmethod
    def forward(ctx, x, weight, alpha_act, alpha_weight, alpha_cim, beta_cim, binary_mask, signed_act, stride,
                padding, dilation, nbits_a, abitslice, nbits_w, wbitslice, xbar, nbits_alpha):
        _require_device(x)
        dev = x.device
        B, C, H, W, O, KH, KW, st, pd = _geometry(x, weight, stride, padding, dilation)
        desc, lsq = _shift_module_descs(tuple(x.shape), weight, st, pd, dilation, nbits_a, abitslice, nbits_w,
                                        wbitslice, xbar, nbits_alpha)
        sizes = _lib.query_sizes(desc)
        xc = x.detach().to(torch.float32).contiguous()
        wc = weight.detach().to(torch.float32).contiguous()
        aa = alpha_act.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        aw = alpha_weight.detach().to(torch.float32).reshape(-1)[:1].contiguous()
        ac = alpha_cim.detach().to(torch.float32).contiguous()
        bc = beta_cim.detach().to(torch.float32).contiguous()
        bm = binary_mask.to(device=dev, dtype=torch.int8).contiguous()
        sg = signed_act.detach().to(device=dev, dtype=torch.float32).reshape(-1)[:1].contiguous()
        Ho = (H + 2 * pd[0] - KH) // st[0] + 1
        Wo = (W + 2 * pd[1] - KW) // st[1] + 1
        out = torch.empty(B, O, Ho, Wo, device=dev, dtype=torch.float32)
        cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
        ws = torch.empty(max(sizes.fwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        _lib.check(_lib.load().cimq_module_shift_forward(desc, lsq, xc.data_ptr(), wc.data_ptr(), aa.data_ptr(),
                                                         aw.data_ptr(), ac.data_ptr(), bc.data_ptr(), bm.data_ptr(),
                                                         sg.data_ptr(), out.data_ptr(), cbuf.data_ptr(),
                                                         ws.data_ptr(), _stream()), "cimq_module_shift_forward")
        ctx.desc, ctx.lsq, ctx.sizes = desc, lsq, sizes
        ctx.bufs = (xc, wc, aa, aw, ac, bc, bm, sg, cbuf)
        ctx.save_for_backward(x, weight, alpha_act, alpha_weight, alpha_cim, beta_cim)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        ctx.saved_tensors  # noqa: B018 -- version check of x and the parameters
        xc, wc, aa, aw, ac, bc, bm, sg, cbuf = ctx.bufs
        dev = xc.device
        g = grad_output.detach().to(torch.float32).contiguous()
        gx = torch.empty_like(xc)
        gw = torch.empty_like(wc)
        gaa = torch.empty(1, device=dev, dtype=torch.float32)
        gaw = torch.empty(1, device=dev, dtype=torch.float32)
        gac = torch.empty_like(ac)
        gbc = torch.empty_like(bc)
        ws = torch.empty(max(ctx.sizes.bwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
        _lib.check(_lib.load().cimq_module_shift_backward(
            ctx.desc, ctx.lsq, g.data_ptr(), xc.data_ptr(), wc.data_ptr(), aa.data_ptr(), aw.data_ptr(), ac.data_ptr(),
            bc.data_ptr(), bm.data_ptr(), sg.data_ptr(), cbuf.data_ptr(), gx.data_ptr(), gw.data_ptr(), gaa.data_ptr(),
            gaw.data_ptr(), gac.data_ptr(), gbc.data_ptr(), ws.data_ptr(), _stream()), "cimq_module_shift_backward")
        return (gx, gw, gaa, gaw, gac, gbc) + (None,) * 11


def cim_module_shift_conv(x, weight, alpha_act, alpha_weight, alpha_cim, beta_cim, binary_mask, signed_act, stride,
                          padding, dilation, nbits_a, abitslice, nbits_w, wbitslice, xbar, nbits_alpha):
    """NCHW output of a Conv2dLSQCiM(adc_shift=True, adcbits=1.5) layer with its quantisers fused
    (module_shift_supported must hold)."""
    return _CimModuleShiftConv.apply(x, weight, alpha_act, alpha_weight, alpha_cim, beta_cim, binary_mask,
                                     signed_act, stride, padding, dilation, nbits_a, abitslice, nbits_w, wbitslice,
                                     xbar, nbits_alpha)


def alpha_cim_init(x, w_q, sa, sw, binary_mask, signed_act, stride, padding, nbits_a, abitslice,
                   nbits_w, wbitslice, adcbits, xbar, num_xbars):
    """First-step alpha_cim initialisation on the device (lsq.py:557-563, 35-87)."""
    _require_device(x)
    dev = x.device
    B, C, H, W, O, KH, KW, st, pd = _geometry(x, w_q, stride, padding, (1, 1))
    desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, xbar, nbits_w, nbits_a, wbitslice, abitslice,
                          adcbits, _lib.CIMQ_INPUT_RAW_LSQ, float(2 ** nbits_a - 1))
    sizes = _lib.query_sizes(desc)
    nbw, nba = int(nbits_w / wbitslice), int(nbits_a / abitslice)
    out = torch.empty(1, num_xbars, nbw, nba, 1, O, device=dev, dtype=torch.float32)
    cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
    ws = torch.empty(max(sizes.fwd_workspace_bytes, 1), device=dev, dtype=torch.uint8)
    xc = x.detach().to(torch.float32).contiguous()
    wq = w_q.detach().to(torch.float32).contiguous()
    sa_ = sa.detach().reshape(-1)[:1].contiguous()
    sw_ = sw.detach().reshape(-1)[:1].contiguous()
    bm = binary_mask.to(device=dev, dtype=torch.int8).contiguous()
    sg = signed_act.detach().to(device=dev, dtype=torch.float32).reshape(-1)[:1].contiguous()
    lib = _lib.load()
    _lib.check(lib.cimq_alpha_init(desc, xc.data_ptr(), wq.data_ptr(), sa_.data_ptr(), sw_.data_ptr(),
                                   bm.data_ptr(), sg.data_ptr(), out.data_ptr(), cbuf.data_ptr(),
                                   ws.data_ptr(), _stream()), "cimq_alpha_init")
    return out


def debug_partial_sums(x_q, w_q, conv_stride, conv_padding, act_bits, act_bit_slice, weight_bits,
                       weight_bit_slice, adc_bits, arr, binary_mask, alpha_cim, weight_scaling_factor,
                       act_scaling_factor, signed_act, stochastic=False, seed=None):
    """Forward on the device that also returns the integer partial sums [B,T,nbw,nba,P,O]
    (int32) and the ADC outputs (fp32) -- the reference's ctx.ps_int / adc_out
    (lsq.py:169-230).  Parity-test hook; ``stochastic`` (with an optional Philox ``seed``)
    draws the stochastic ADC of lsq.py:205-221."""
    _require_device(x_q)
    dev = x_q.device
    B, C, H, W, O, KH, KW, st, pd = _geometry(x_q, w_q, conv_stride, conv_padding, (1, 1))
    desc = _lib.make_desc(B, C, H, W, O, KH, KW, st, pd, arr, weight_bits, act_bits, weight_bit_slice,
                          act_bit_slice, adc_bits, _lib.CIMQ_INPUT_XQ,
                          adc_variant=_lib.CIMQ_ADC_STOCHASTIC if stochastic else _lib.CIMQ_ADC_LIBRARY,
                          seed=(stochastic_seed() if seed is None else seed) if stochastic else 0)
    sizes = _lib.query_sizes(desc)
    nbw, nba = int(weight_bits / weight_bit_slice), int(act_bits / act_bit_slice)
    T = int(math.ceil(C * KH * KW / arr))
    Ho = (H + 2 * pd[0] - KH) // st[0] + 1
    Wo = (W + 2 * pd[1] - KW) // st[1] + 1
    out = torch.empty(B, Ho * Wo, O, device=dev, dtype=torch.float32)
    ps = torch.zeros(B, T, nbw, nba, Ho * Wo, O, device=dev, dtype=torch.int32)
    adc = torch.zeros(B, T, nbw, nba, Ho * Wo, O, device=dev, dtype=torch.float32)
    cbuf = torch.empty(max(sizes.ctx_bytes, 1), device=dev, dtype=torch.uint8)
    xq = x_q.detach().float().contiguous()
    wq = w_q.detach().float().contiguous()
    sa = _f32(act_scaling_factor, dev).reshape(-1)[:1].contiguous()
    sw = _f32(weight_scaling_factor, dev).reshape(-1)[:1].contiguous()
    bm = binary_mask.to(device=dev, dtype=torch.int8).contiguous()
    sg = _f32(signed_act, dev).reshape(-1)[:1].contiguous()
    al = None if alpha_cim is None else _f32(alpha_cim, dev)
    lib = _lib.load()
    _lib.check(lib.cimq_debug_partial_sums(desc, xq.data_ptr(), wq.data_ptr(), sa.data_ptr(), sw.data_ptr(),
                                           None if al is None else al.data_ptr(), bm.data_ptr(), sg.data_ptr(),
                                           out.data_ptr(), ps.data_ptr(), adc.data_ptr(), cbuf.data_ptr(),
                                           _stream()), "cimq_debug_partial_sums")
    return out, ps, adc


def debug_state_codes(out):
    """ADC codes (int8) and STE-pass bits (uint8) [B, T, nbw, nba, P, O] of every partial sum that
    the production forward (cim_fwd_v3_kernel, v7 path) recorded for ``out`` -- the output of
    get_cim_output_signed / cim_conv2d_lsq / cim_module_conv whose backward has not run yet.
    Parity-test hook (cimq_debug_state_codes)."""
    ctx = out.grad_fn
    while ctx is not None and not hasattr(ctx, "desc"):  # through views (the module's NCHW reshape)
        ctx = ctx.next_functions[0][0] if ctx.next_functions else None
    if ctx is None:
        raise RuntimeError("no libcimq forward context behind this tensor")
    d = ctx.desc
    cbuf = ctx.bufs[-1]
    nbw, nba = int(d.bits_w / d.bs_w), int(d.bits_a / d.bs_a)
    T = num_xbars(d.in_channels, (d.kernel_h, d.kernel_w), d.xbar)
    Ho = (d.in_h + 2 * d.pad_h - d.kernel_h) // d.stride_h + 1
    Wo = (d.in_w + 2 * d.pad_w - d.kernel_w) // d.stride_w + 1
    shape = (d.batch, T, nbw, nba, Ho * Wo, d.out_channels)
    code = torch.empty(shape, device=cbuf.device, dtype=torch.int8)
    passed = torch.empty(shape, device=cbuf.device, dtype=torch.uint8)
    if getattr(ctx, "module_path", False) and _lib.module_route(d)[1] == _lib.CIMQ_ROUTE_R6:
        # a module layer whose backward recomputes the partial sums: its forward left no state words, so the
        # codes come from the recomputing backward's own code path (cimq_debug_recompute_codes)
        xc, sg = ctx.bufs[0], ctx.bufs[6]
        st = torch.empty(T * d.batch * Ho * Wo * d.out_channels * 4, device=cbuf.device, dtype=torch.uint8)
        _lib.check(_lib.load().cimq_debug_recompute_codes(d, xc.data_ptr(), sg.data_ptr(), cbuf.data_ptr(),
                                                          st.data_ptr(), code.data_ptr(), passed.data_ptr(),
                                                          _stream()), "cimq_debug_recompute_codes")
        return code, passed
    _lib.check(_lib.load().cimq_debug_state_codes(d, cbuf.data_ptr(), code.data_ptr(), passed.data_ptr(), _stream()),
               "cimq_debug_state_codes")
    return code, passed


def logical_macs(B, C, H, W, O, KH, KW, stride, padding) -> int:
    """ptflops convention B*Ho*Wo*O*C*KH*KW (utils/ptflops/flops_counter.py:314-318)."""
    Ho = (H + 2 * padding[0] - KH) // stride[0] + 1
    Wo = (W + 2 * padding[1] - KW) // stride[1] + 1
    return B * Ho * Wo * O * C * KH * KW


def num_xbars(in_channels, kernel_size, xbar) -> int:
    return int(math.ceil(in_channels * kernel_size[0] * kernel_size[1] / xbar))


# =============================================================================================
# plain LSQ modules (lsq.py:389-436 Conv2dLSQ, :591-617 LinearLSQ, :620-662 ActLSQ)
# =============================================================================================
_LSQ_WS = {}  # cimq_lsq_quantize_workspace_bytes per element count


class _LsqQuantize(torch.autograd.Function):
    """out = round_pass(clamp(x / s, qn, qp)) [* s] with s the grad-scaled step size (a [1]
    tensor: grad_scale(alpha, g) evaluated by torch, so its graph back to alpha stays torch's).
    Backward: grad_x and d loss / d s from libcimq (cimq_lsq_quantize_backward)."""

    @staticmethod
    def forward(ctx, x, s, qn, qp, scaled):
        _require_device(x, s)
        xc = x.detach().float().contiguous()
        sc = s.detach().float().reshape(-1)[:1].contiguous()
        out = torch.empty_like(xc)
        _lib.check(_lib.load().cimq_lsq_quantize_forward(xc.data_ptr(), xc.numel(), sc.data_ptr(), float(qn),
                                                         float(qp), 1 if scaled else 0, out.data_ptr(), _stream()),
                   "cimq_lsq_quantize_forward")
        ctx.save_for_backward(xc, sc)
        ctx.q = (float(qn), float(qp), 1 if scaled else 0)
        ctx.s_shape = s.shape
        return out

    @staticmethod
    def backward(ctx, g):
        xc, sc = ctx.saved_tensors
        qn, qp, scaled = ctx.q
        lib = _lib.load()
        gc = g.float().contiguous()
        gx = torch.empty_like(xc)
        gs = torch.empty(1, device=xc.device, dtype=torch.float32)
        n = xc.numel()
        nb = _LSQ_WS.get(n)
        if nb is None:
            nb = _LSQ_WS[n] = max(lib.cimq_lsq_quantize_workspace_bytes(n), 4)
        ws = torch.empty(nb, device=xc.device, dtype=torch.uint8)
        _lib.check(lib.cimq_lsq_quantize_backward(xc.data_ptr(), xc.numel(), sc.data_ptr(), qn, qp, scaled,
                                                  gc.data_ptr(), gx.data_ptr(), gs.data_ptr(), ws.data_ptr(),
                                                  _stream()), "cimq_lsq_quantize_backward")
        return gx, gs.reshape(ctx.s_shape), None, None, None


def lsq_quantize(x, s, qn, qp, scaled=False):
    """LSQ fake-quantiser on libcimq: round_pass(clamp(x / s, qn, qp)) [* s] (lsq.py:412,611,656)."""
    return _LsqQuantize.apply(x, s, qn, qp, scaled)


_QCONV_PLANS = {}


def _qconv_plan(*key):
    """descriptor and workspace sizes of one conv shape, built once (host time per call)"""
    p = _QCONV_PLANS.get(key)
    if p is None:
        B, C, H, W, O, KH, KW, stride, padding, dilation, code_range, has_bias = key
        desc = _lib.make_qconv_desc(B, C, H, W, O, KH, KW, stride, padding, dilation, 1, code_range[0],
                                    code_range[1], has_bias)
        p = (desc,) + tuple(_lib.qconv_sizes(desc))
        _QCONV_PLANS[key] = p
    return p


class _QConv2d(torch.autograd.Function):
    """Conv2dLSQ's quantised conv (lsq.py:436): conv2d(x_q, w_q, bias) * act_scale * w_scale with
    integer-code operands, forward on int8 MFMA (cimq_qconv_forward).  Backward: the scale
    products and grad_y0 on libcimq (cimq_qconv_backward_scales), the conv's input / weight
    gradients of grad_y0 as plain fp32 convolutions (torch.nn.grad: the library conv)."""

    @staticmethod
    def forward(ctx, x_q, act_scale, w_q, w_scale, bias, stride, padding, dilation, code_range):
        _require_device(x_q, act_scale, w_q, w_scale, bias)
        xc = x_q.detach().float().contiguous()
        wc = w_q.detach().float().contiguous()
        a = act_scale.detach().float().reshape(-1)[:1].contiguous()
        s = w_scale.detach().float().reshape(-1)[:1].contiguous()
        bc = None if bias is None else bias.detach().float().contiguous()
        B, C, H, W = xc.shape
        O, _, KH, KW = wc.shape
        desc, fws, bws = _qconv_plan(B, C, H, W, O, KH, KW, stride, padding, dilation, code_range, bc is not None)
        Ho = (H + 2 * padding[0] - dilation[0] * (KH - 1) - 1) // stride[0] + 1
        Wo = (W + 2 * padding[1] - dilation[1] * (KW - 1) - 1) // stride[1] + 1
        y = torch.empty(B, O, Ho, Wo, device=xc.device, dtype=torch.float32)
        y0 = torch.empty_like(y)
        ws = torch.empty(max(fws, 16), device=xc.device, dtype=torch.uint8)
        _lib.check(_lib.load().cimq_qconv_forward(desc, xc.data_ptr(), wc.data_ptr(), a.data_ptr(), s.data_ptr(),
                                                  None if bc is None else bc.data_ptr(), y.data_ptr(), y0.data_ptr(),
                                                  ws.data_ptr(), _stream()), "cimq_qconv_forward")
        ctx.save_for_backward(xc, wc, a, s, y0)
        ctx.desc, ctx.bws = desc, bws
        ctx.conv = (tuple(stride), tuple(padding), tuple(dilation))
        ctx.shapes = (act_scale.shape, w_scale.shape, bias is not None)
        return y

    @staticmethod
    def backward(ctx, g):
        xc, wc, a, s, y0 = ctx.saved_tensors
        stride, padding, dilation = ctx.conv
        gc = g.float().contiguous()
        gy0 = torch.empty_like(y0)
        scales = torch.empty(2, device=y0.device, dtype=torch.float32)
        ws = torch.empty(max(ctx.bws, 16), device=y0.device, dtype=torch.uint8)
        _lib.check(_lib.load().cimq_qconv_backward_scales(ctx.desc, gc.data_ptr(), y0.data_ptr(), a.data_ptr(),
                                                          s.data_ptr(), gy0.data_ptr(), scales.data_ptr(),
                                                          ws.data_ptr(), _stream()), "cimq_qconv_backward_scales")
        a_shape, s_shape, has_bias = ctx.shapes
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.nn.grad.conv2d_input(xc.shape, wc, gy0, stride, padding, dilation, 1)
        if ctx.needs_input_grad[2]:
            gw = torch.nn.grad.conv2d_weight(xc, wc.shape, gy0, stride, padding, dilation, 1)
        gb = gy0.sum(dim=(0, 2, 3)) if has_bias else None
        return gx, scales[1:2].reshape(a_shape), gw, scales[0:1].reshape(s_shape), gb, None, None, None, None


def qconv2d(x_q, act_scale, w_q, w_scale, bias=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1),
            code_range=(-128, 127)):
    """conv2d(x_q, w_q, bias) * act_scale * w_scale on int8 MFMA; x_q / w_q hold integer codes,
    x_q's within ``code_range`` (ActLSQ's [Qn, Qp]; [0, 255] runs as two 4-bit halves)."""
    pair = lambda v: tuple(v) if isinstance(v, (tuple, list)) else (int(v), int(v))  # noqa: E731
    return _QConv2d.apply(x_q, act_scale, w_q, w_scale, bias, pair(stride), pair(padding), pair(dilation),
                          tuple(int(c) for c in code_range))

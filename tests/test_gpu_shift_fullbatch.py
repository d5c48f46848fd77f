"""GPU parity of BASELINE cfg4 (ResNet-56 w2a2 xbar 64) on the module path at full batch: the scale +
shift ADC (Conv2dLSQCiM(adc_shift=True), the per-tile partial-sum scale/shift of
test/test_backward_cimlayer_scale_shift.py:336-546 as a module option), alpha only (the reference
module, lsq.py:511-588), and the layers outside the shift fast path.

* ResNet-56 w2a2 xbar 64 at B = 256, every stage geometry and both stride-2 transitions: out, grad_x,
  grad_w, grad_alpha_cim, grad_beta and both step-size gradients against the module oracle on the
  whole batch (the batch-summed gradients included), elementwise, plus run-to-run bit identity.
* ResNet-56's first conv, forced to w8a8 by ReplaceModuleTool (utils/wrapper/replace_module.py:83-95):
  3 -> 16 @ 32, signed input, xbar 64 (K = 27, T = 1, 64 slice pairs, the int8-wrapped binary_mask),
  at B = 2 and B = 256.  Since round 4 it runs the shift fast path's w8a8 form (cim_fwd_v3_kernel<8,1,8,1>
  with plane state, the v7 backward pair and shift_stats8_kernel; test_abi_host.py asserts the routing);
  a w8a8 shape that fast path refuses (C = 8, K = 72) keeps the general recompute kernels under test.
  Deterministic (fixed-order reductions, no atomics).
* alpha only (adc_shift=False) at B = 256: the 32x32 stage, a stride-2 transition and the 8x8 stage.
* Shift layers the fast path refuses for other reasons: 128 output channels (more than four 16-channel
  blocks) and a batch-1 8x8 image (M % 128 != 0).

Bars (north_star 1e-5): out within 1e-6 and grad_x / grad_w / grad_beta within 1e-5 of
max(|ref|, sum of |terms|) element by element (the oracle's fp64 re-run on |operands|); grad_alpha_cim
elementwise 1e-5 of its terms (conftest.alpha_cim_terms: for the max / min entries of alpha_cim, which
collect the alpha quantiser's scale gradient from every element, the exact terms of that sum too); the
step sizes within 1e-5 of their sum of |terms|.
"""
import math

import numpy as np
import pytest
import torch

from conftest import alpha_cim_report, alpha_cim_terms, rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co

pytestmark = pytest.mark.gpu


def _kw(bits, xbar=64, shift=True):
    return dict(nbits_w=bits, nbits_a=bits, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=xbar, adcbits=1.5,
                stochastic_quant=False, adc_shift=shift)


def _capture_oracle_ctx(monkeypatch):
    box = {}
    real = co.cim_forward

    def rec(*a, **k):
        k["return_debug"] = True
        out, c = real(*a, **k)
        box["c"] = c
        return out, c
    monkeypatch.setattr(cmo.co, "cim_forward", rec)
    return box


def _scalar_terms(x, g_xq, s, qn, qp, gscale):
    x, g = x.astype(np.float64), g_xq.astype(np.float64)
    y = x / float(s)
    r = np.rint(np.clip(y, qn, qp))
    inside = (y >= qn) & (y <= qp)
    return gscale * (np.abs(g * r).sum() + np.abs(np.where(inside, g * float(s), 0) * y / float(s)).sum())


def _build(dev, C, O, H, s, bits, B, seed, signed, shift=True):
    """The MI355X module and the oracle module with identical weights and step sizes; alpha_cim from
    the reference's data-driven init (lsq.py:557-563) on a few images, spread so codes vary; beta a
    fraction of alpha of either sign."""
    import cim_quantization_amd._modules as my_nn
    rng = np.random.default_rng(seed)
    m = my_nn.Conv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **_kw(bits, shift=shift)).to(dev)
    om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **_kw(bits, shift=shift))
    om.debug_retain = True
    w = (rng.standard_normal((O, C, 3, 3)) * math.sqrt(2.0 / (9 * C))).astype(np.float32)
    x = rng.standard_normal((B, C, H, H)).astype(np.float32)
    if not signed:
        x = np.maximum(x, 0)
    qp_a, (qn_w, qp_w) = 2 ** bits - 1, co.lsq_weight_params(bits)
    aa = np.float32(2 * np.abs(x).mean() / math.sqrt(qp_a))
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(qp_w))
    sa0 = co.grad_scale_value(np.array([aa], np.float32), 1.0 / math.sqrt(x.size * qp_a))
    sw0 = co.grad_scale_value(np.array([aw], np.float32), 1.0 / math.sqrt(w.size * qp_w))
    xq0, _ = co.lsq_quantize(x[:2], sa0, 0, qp_a)
    wq0, _ = co.lsq_quantize(w, sw0, qn_w, qp_w)
    ac = co.alpha_cim_init(xq0, wq0, (s, s), (1, 1), bits, 1, bits, 1, 64, sw0, sa0, 1.5)
    ac = (ac * (0.6 + 0.8 * rng.random(ac.shape))).astype(np.float32)
    bc = (ac * (rng.random(ac.shape) - 0.5)).astype(np.float32)
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
            mod.alpha_act.fill_(float(aa))
            mod.alpha_weight.fill_(float(aw))
            mod.alpha_cim.copy_(torch.from_numpy(ac))
            if shift:
                mod.beta_cim.copy_(torch.from_numpy(bc))
            mod.init_state.fill_(1)
            mod.init_state_cim.fill_(1)
            mod.signed_act.fill_(1 if signed else 0)
        mod._state_cache = None
        mod.train()
    ho = (H + 2 - 3) // s + 1
    g = (rng.standard_normal((B, O, ho, ho)) / math.sqrt(B * O * ho * ho)).astype(np.float32)
    return m, om, x, w, g, qp_a, qn_w, qp_w


def _run(m, x, g, dev):
    for p in m.parameters():
        p.grad = None
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g).to(dev))
    torch.cuda.synchronize()
    return dict(out=out.detach().clone(), gx=xt.grad.clone(), gw=m.weight.grad.clone(), ga=m.alpha_cim.grad.clone(),
                gb=m.beta_cim.grad.clone() if m.beta_cim is not None else torch.zeros(1, device=dev),
                gaa=m.alpha_act.grad.clone(), gaw=m.alpha_weight.grad.clone())


def _check(dev, monkeypatch, C, O, H, s, bits, B, seed, signed, repeat=True, shift=True):
    m, om, x, w, g, qp_a, qn_w, qp_w = _build(dev, C, O, H, s, bits, B, seed, signed, shift)
    r1 = _run(m, x, g, dev)
    if repeat:
        r2 = _run(m, x, g, dev)
        for k in r1:
            assert torch.equal(r1[k], r2[k]), f"{k}: not bit-identical run to run"
    box = _capture_oracle_ctx(monkeypatch)
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))
    c = box["c"]
    ho = g.shape[-1]
    g_bpo = np.ascontiguousarray(g.reshape(B, O, ho * ho).transpose(0, 2, 1))
    terms = co.cim_backward(c, g_bpo, absolute=True)
    ax, aw, aa = terms[:3]
    bm = np.abs(om.binary_mask.numpy().astype(np.float64))
    out_terms = (np.abs(c.adc.astype(np.float64)) * bm).sum(axis=(1, 2, 3)).transpose(0, 2, 1).reshape(B, O, ho, ho)
    np_ = lambda t: t.detach().cpu().numpy()  # noqa: E731
    assert rel_err(np_(r1["out"]), np_(oout), out_terms) < 1e-6, "out"
    assert rel_err(np_(r1["gx"]), np_(ox.grad), ax) < 1e-5, "grad_x"
    assert rel_err(np_(r1["gw"]), np_(om.weight.grad), aw.reshape(om.weight.shape)) < 1e-5, "grad_w"
    if shift:
        assert rel_err(np_(r1["gb"]), np_(om.beta_cim.grad), terms[3].reshape(om.beta_cim.shape)) < 1e-5, "grad_beta"
    ga, gr = np_(r1["ga"]), np_(om.alpha_cim.grad)
    # every entry, the max / min ones included: those also collect the alpha quantiser's scale gradient
    # (lsq.py:566-571), a sum over every entry whose exact |terms| alpha_cim_terms adds
    assert rel_err(ga, gr, alpha_cim_terms(np_(om.alpha_cim), aa)) < 1e-5, \
        "grad_alpha_cim: " + alpha_cim_report(ga, gr, np_(om.alpha_cim), aa)
    d = om.dbg
    t_act = _scalar_terms(x, np_(d["x_q"].grad), d["sa"].item(), 0, qp_a, 1.0 / math.sqrt(x.size * qp_a))
    t_w = _scalar_terms(w, np_(d["w_q"].grad), d["sw"].item(), qn_w, qp_w, 1.0 / math.sqrt(w.size * qp_w))
    assert abs(r1["gaa"].item() - om.alpha_act.grad.item()) <= 1e-5 * t_act, "grad_alpha_act"
    assert abs(r1["gaw"].item() - om.alpha_weight.grad.item()) <= 1e-5 * t_w, "grad_alpha_weight"
    # the check must bite: partial sums inside and outside the STE interval, codes of either sign
    with np.errstate(all="ignore"):
        be = c.beta.astype(np.float64) if c.beta is not None else 0.0
        v = (c.u.astype(np.float64) - be) / c.alpha.astype(np.float64)
    assert (np.abs(v) >= 1 + 1e-5).mean() > 0.01 and (np.abs(v) < 1).mean() > 0.01
    assert (np.rint(v) > 0).any() and (np.rint(v) < 0).any()
    return m


RESNET56_SHAPES = [(16, 16, 32, 1), (32, 32, 16, 1), (64, 64, 8, 1), (16, 32, 32, 2), (32, 64, 16, 2)]


@pytest.mark.parametrize("C,O,H,s", RESNET56_SHAPES)
def test_resnet56_shift_fullbatch_vs_oracle(cuda_device, monkeypatch, C, O, H, s):
    """B = 256, w2a2, xbar 64: every gradient on the whole batch (the shift fast path: thresholds with
    beta folded in, the v7 backward, the statistics kernel)."""
    _check(cuda_device, monkeypatch, C, O, H, s, 2, 256, 9100 + C + O + H + s, signed=False)


@pytest.mark.parametrize("B", [2, 256])
def test_resnet56_conv1_w8a8_shift_vs_oracle(cuda_device, monkeypatch, B):
    """ResNet-56's first conv under the scale/shift ADC: w8a8 (replace_module.py:83-95), signed input,
    3 -> 16 @ 32, xbar 64 -- the shift fast path's w8a8 form (v3<8,1,8,1> + v7 + shift_stats8_kernel),
    bit-identical run to run."""
    _check(cuda_device, monkeypatch, 3, 16, 32, 1, 8, B, 9200 + B, signed=True)


def test_w8a8_shift_general_kernels_vs_oracle(cuda_device, monkeypatch):
    """A w8a8 signed shift layer the fast path refuses (C = 8 -> K = 72 > xbar 64: two tiles; test_abi_host
    shows cimq_module_shift_supported returns 0 for it): the general recompute kernels at w8a8 with signed
    input and the int8-wrapped mask, against the module oracle on the whole batch."""
    _check(cuda_device, monkeypatch, 8, 16, 16, 1, 8, 8, 9250, signed=True)


@pytest.mark.parametrize("C,O,H,s,B", [(16, 128, 8, 1, 2), (16, 16, 8, 1, 1), (32, 32, 8, 2, 1)])
def test_shift_off_fast_path_vs_oracle(cuda_device, monkeypatch, C, O, H, s, B):
    """Shift layers outside the fast path's plan (O = 128: eight 16-channel blocks; batch 1 at 8x8:
    M % 128 != 0): the general backward, with grad_beta, the shift ADC's grad_alpha and the act-LSQ
    backward applied once."""
    _check(cuda_device, monkeypatch, C, O, H, s, 2, B, 9300 + C + O + H + B, signed=False)


@pytest.mark.parametrize("C,O,H,s", [(16, 16, 32, 1), (16, 32, 32, 2), (64, 64, 8, 1)])
def test_resnet56_alpha_only_fullbatch_vs_oracle(cuda_device, monkeypatch, C, O, H, s):
    """BASELINE cfg4 without the shift option: Conv2dLSQCiM w2a2 xbar 64, alpha only (lsq.py:511-588),
    on the module path at ResNet-56's 32x32 geometry (and a stride-2 transition and an 8x8 stage),
    B = 256: out, grad_x, grad_w, grad_alpha_cim and both step sizes against the module oracle on the
    whole batch, elementwise, plus run-to-run bit identity."""
    _check(cuda_device, monkeypatch, C, O, H, s, 2, 256, 9400 + C + O + H + s, signed=False, shift=False)

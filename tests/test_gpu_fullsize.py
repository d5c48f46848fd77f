"""GPU parity at the benchmarked sizes, through the module path the bench runs.

* ResNet-20 (BASELINE cfg2): every distinct CiM conv shape of the network -- the w8a8 first conv,
  the 16/32/64-channel stages and both stride-2 transitions -- as ``Conv2dLSQCiM`` at batch 256
  (fused LSQ quantisers, ``cimq_module_forward/backward``, the kernels bench.py times), against
  the module oracle on the FULL batch: out, grad_x, grad_w, grad_alpha_cim, grad_alpha_act,
  grad_alpha_weight.  The ADC codes and STE-pass bits that the production forward
  (cim_fwd5_kernel; cim_fwd_v3_kernel on the first conv) wrote into its state words are decoded and
  compared with the oracle's, element by element, on sampled images.  ``layer1_recompute`` runs the
  16-channel layer with CIMQ_OPT_RECOMPUTE (no state words; cim_bwd_r6_kernel recomputes the partial
  sums): the codes / pass bits there are the ones the recomputing backward derives, through its
  debug instantiation (cimq_debug_recompute_codes).
* QuantLinear 1024->1024 w4a4, 128-row tiles (BASELINE cfg5, ``Conv2dLSQCiM`` with k = 1, SURVEY
  section 0): the module at batch 4096 against the oracle on 64 sampled rows (out, grad_x), every
  integer partial sum and ADC output bit-exact, and all gradients against the module oracle on a
  256-row batch at the full layer shape.

Tolerances (north_star "1e-5 relative", elementwise): out within 1e-6 and grad_x / grad_w within
1e-5 of max(|ref|, sum of |terms|) element by element (the oracle's fp64 re-run of the Function's
contractions on |operands|); grad_alpha_cim elementwise 1e-5 of its terms except the max / min
entries, which also collect the alpha quantiser's scale gradient from every element (normwise
there); the step-size grads 1e-5 of their sum of |terms|.
"""
import math

import numpy as np
import pytest
import torch

from conftest import alpha_cim_report, alpha_cim_terms, rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co

pytestmark = pytest.mark.gpu

# (name, C, O, H, stride, bits): the six distinct CiM conv shapes of ResNet-20 (bench.py RESNET20)
RESNET20_SHAPES = [
    ("conv1_w8a8", 3, 16, 32, 1, 8),
    ("layer1", 16, 16, 32, 1, 3),
    ("layer2.0.conv1_s2", 16, 32, 32, 2, 3),
    ("layer2", 32, 32, 16, 1, 3),
    ("layer3.0.conv1_s2", 32, 64, 16, 2, 3),
    ("layer3", 64, 64, 8, 1, 3),
    ("layer1_recompute", 16, 16, 32, 1, 3),  # CIMQ_OPT_RECOMPUTE: cim_bwd_r6_kernel
]


def _kw(bits, xbar=128, adc=1.5):
    return dict(nbits_w=bits, nbits_a=bits, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=xbar, adcbits=adc,
                signed_xbar=True, stochastic_quant=False)


def _close(mine, ref, tol, what):
    mine = mine.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(mine) else np.asarray(mine, np.float64)
    ref = ref.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(ref) else np.asarray(ref, np.float64)
    assert mine.shape == ref.shape, (what, mine.shape, ref.shape)
    err = np.abs(mine - ref).max()
    assert err <= tol * (np.abs(ref).max() + 1e-30), (what, err, np.abs(ref).max())


def _capture_oracle_ctx(monkeypatch):
    """Keep the module oracle's Function context (with the ADC outputs) for the absolute-term re-run."""
    box = {}
    real = co.cim_forward

    def rec(*a, **k):
        k["return_debug"] = True
        out, c = real(*a, **k)
        box["c"] = c
        return out, c
    monkeypatch.setattr(cmo.co, "cim_forward", rec)
    return box


def _check_elementwise(c, bm, g_nchw, out, oout, xt, ox, m, om):
    """out / grad_x / grad_w / grad_alpha_cim of the module against the oracle module, elementwise."""
    B, O = g_nchw.shape[:2]
    g_bpo = np.ascontiguousarray(g_nchw.reshape(B, O, -1).transpose(0, 2, 1))
    ax, aw, aa = co.cim_backward(c, g_bpo, absolute=True)
    np_ = lambda t: t.detach().cpu().numpy()  # noqa: E731
    out_terms = (np.abs(c.adc.astype(np.float64)) * np.abs(bm.astype(np.float64))).sum(axis=(1, 2, 3))
    out_terms = out_terms.transpose(0, 2, 1).reshape(np_(oout).shape)
    assert rel_err(np_(out), np_(oout), out_terms) < 1e-6, "out"
    assert rel_err(np_(xt.grad), np_(ox.grad), ax.reshape(np_(ox.grad).shape)) < 1e-5, "grad_x"
    assert rel_err(np_(m.weight.grad), np_(om.weight.grad), aw.reshape(np_(om.weight.grad).shape)) < 1e-5, "grad_w"
    ga, gr = np_(m.alpha_cim.grad), np_(om.alpha_cim.grad)
    # every entry; the max / min ones with the exact terms of the alpha quantiser's scale gradient
    assert rel_err(ga, gr, alpha_cim_terms(np_(om.alpha_cim), aa)) < 1e-5, \
        "grad_alpha_cim: " + alpha_cim_report(ga, gr, np_(om.alpha_cim), aa)


def _lsq_scalar_terms(x, g_xq, s, qn, qp, gscale):
    """sum of |terms| of d loss / d alpha through the LSQ quantiser (lsq.py:547-555)."""
    x = x.astype(np.float64)
    g = g_xq.astype(np.float64)
    y = x / float(s)
    r = np.rint(np.clip(y, qn, qp))
    inside = (y >= qn) & (y <= qp)
    return gscale * (np.abs(g * r).sum() + np.abs(np.where(inside, g * float(s), 0) * y / float(s)).sum())


def _pin(mods, aa, aw, ac):
    for m in mods:
        with torch.no_grad():
            m.alpha_act.fill_(float(aa))
            m.alpha_weight.fill_(float(aw))
            if m.alpha_cim is not None:
                m.alpha_cim.copy_(torch.from_numpy(ac))
            m.init_state.fill_(1)
            m.init_state_cim.fill_(1)
            m.signed_act.fill_(0)
        m._state_cache = None
        m.train()


def _oracle_codes(xq, wq, st, pd, bits, xbar, alpha_q, sw, sa, signed):
    """ADC code and STE-pass bit of every partial sum (lsq.py:195-230, 257-313), from the oracle."""
    _, c = co.cim_forward(xq, wq, st, pd, (1, 1), bits, 1, bits, 1, 1.5, xbar, co.make_binary_mask(bits, bits, 1, 1),
                          alpha_q, sw, sa, False, np.array([signed], np.float32))
    u = ((c.ps16.astype(np.float32) * sw).astype(np.float32) * sa).astype(np.float32)
    with np.errstate(all="ignore"):
        v = (u / alpha_q).astype(np.float32)
    code = np.clip(np.rint(v), -1, 1).astype(np.int8)
    passed = ~((v >= np.float32(1 + 1e-5)) | (v <= np.float32(-1 - 1e-5)))
    return code, passed.astype(np.uint8)


@pytest.mark.parametrize("shape", RESNET20_SHAPES, ids=[s[0] for s in RESNET20_SHAPES])
def test_resnet20_layer_module_fullbatch(cuda_device, monkeypatch, shape):
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd import functional as F
    name, C, O, H, s, bits = shape
    B = 256
    rng = np.random.default_rng(sum(map(ord, name)))
    torch.manual_seed(0)
    m = my_nn.Conv2dLSQCiM(C, O, 3, s, 1, bias=False, **_kw(bits)).to(cuda_device)
    m.recompute_psum = name.endswith("_recompute")
    om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **_kw(bits))
    om.debug_retain = True
    w = (rng.standard_normal((O, C, 3, 3)) * math.sqrt(2.0 / (9 * C))).astype(np.float32)
    x = rng.standard_normal((B, C, H, H)).astype(np.float32)
    signed = bits == 8  # the first conv sees the normalised image (signed_act = 1)
    if not signed:
        x = np.maximum(x, 0)
    ho = (H + 2 - 3) // s + 1
    g = (rng.standard_normal((B, O, ho, ho)) / math.sqrt(B * O * ho * ho)).astype(np.float32)
    qp_a, (qn_w, qp_w) = 2 ** bits - 1, co.lsq_weight_params(bits)
    aa = np.float32(2 * np.abs(x).mean() / math.sqrt(qp_a))  # lsq.py:539-542
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(qp_w))
    # a data-driven alpha_cim (lsq.py:557-563 on four images), spread so the codes vary
    sa0 = co.grad_scale_value(np.array([aa], np.float32), 1.0 / math.sqrt(x.size * qp_a))
    sw0 = co.grad_scale_value(np.array([aw], np.float32), 1.0 / math.sqrt(w.size * qp_w))
    xq0, _ = co.lsq_quantize(x[:4], sa0, 0, qp_a)
    wq0, _ = co.lsq_quantize(w, sw0, qn_w, qp_w)
    ac = co.alpha_cim_init(xq0, wq0, (s, s), (1, 1), bits, 1, bits, 1, 128, sw0, sa0, 1.5)
    ac = (ac * (0.7 + 0.6 * rng.random(ac.shape))).astype(np.float32)
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
    _pin((m, om), aa, aw, ac)
    if signed:
        for mod in (m, om):
            mod.signed_act.fill_(1)

    xt = torch.from_numpy(x).to(cuda_device).requires_grad_(True)
    out = m(xt)
    # what cim_fwd5_kernel recorded, before the backward (with the recompute option, what the recomputing
    # backward derives; the w8a8 first conv records nothing: its backward recomputes the partial sums,
    # cimq_c1.hip; its integer decisions are checked below on the debug forward instead)
    code, passed = (None, None) if signed else F.debug_state_codes(out)
    out.backward(torch.from_numpy(g).to(cuda_device))
    torch.cuda.synchronize()

    box = _capture_oracle_ctx(monkeypatch)
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))

    _check_elementwise(box["c"], om.binary_mask.numpy(), g, out, oout, xt, ox, m, om)
    d = om.dbg
    t_act = _lsq_scalar_terms(x, d["x_q"].grad.numpy(), d["sa"].item(), 0, qp_a, 1.0 / math.sqrt(x.size * qp_a))
    t_w = _lsq_scalar_terms(w, d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w, 1.0 / math.sqrt(w.size * qp_w))
    assert abs(m.alpha_act.grad.item() - om.alpha_act.grad.item()) <= 1e-5 * t_act
    assert abs(m.alpha_weight.grad.item() - om.alpha_weight.grad.item()) <= 1e-5 * t_w

    # the production forward's integer decisions, element by element, on 8 images
    sel = [0, 37, 85, 128, 170, 200, 231, B - 1]
    a = om.alpha_cim.detach().numpy()
    alpha_q = co.alpha_quantize(a, 8)
    sw_np, sa_np = d["sw"].detach().numpy().reshape(1), d["sa"].detach().numpy().reshape(1)
    oc, op = _oracle_codes(d["x_q"].detach().numpy()[sel], d["w_q"].detach().numpy(), (s, s), (1, 1), bits, 128,
                           alpha_q, sw_np, sa_np, float(signed))
    if code is None:
        # every integer partial sum of the sampled images on the debug forward, bit-exact, and the codes
        # / pass bits the recomputing backward derives from them by the same thresholds
        dv = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda_device)  # noqa: E731
        bm = co.make_binary_mask(bits, bits, 1, 1)
        _, ps, adc = F.debug_partial_sums(dv(d["x_q"].detach().numpy()[sel]), dv(d["w_q"].detach().numpy()), (s, s),
                                          (1, 1), bits, 1, bits, 1, 1.5, 128, dv(bm), dv(alpha_q), dv(sw_np), dv(sa_np),
                                          dv(np.array([1.0], np.float32)))
        _, c_ref = co.cim_forward(d["x_q"].detach().numpy()[sel], d["w_q"].detach().numpy(), (s, s), (1, 1), (1, 1),
                                  bits, 1, bits, 1, 1.5, 128, bm, alpha_q, sw_np, sa_np, False,
                                  np.array([1.0], np.float32), return_debug=True)
        assert np.array_equal(ps.cpu().numpy(), np.rint(c_ref.ps16.astype(np.float64)).astype(np.int32))
        assert np.array_equal(adc.cpu().numpy(), c_ref.adc)
        return
    mc, mp = code.cpu().numpy()[sel], passed.cpu().numpy()[sel]
    # slice pairs whose binary_mask entry is 0 (the int8 wrap of the w8a8 layer, j + k >= 8) touch
    # neither the output nor any gradient; the forward skips them and records code 0 / pass 0
    live = (co.make_binary_mask(bits, bits, 1, 1) != 0).reshape(1, 1, bits, bits, 1, 1)
    live = np.broadcast_to(live, mc.shape)
    assert np.array_equal(mc[live], oc[live]), f"ADC codes differ at {np.argwhere((mc != oc) & live)[:5].tolist()}"
    assert np.array_equal(mp[live], op[live]), f"STE pass bits differ at {np.argwhere((mp != op) & live)[:5].tolist()}"
    assert not mc[~live].any() and not mp[~live].any()
    assert (oc != 0).mean() > 0.05 and (oc == 0).mean() > 0.05, "codes must vary for the check to bite"


def test_cfg5_quantlinear_1024_w4a4_xbar128(cuda_device, monkeypatch):
    """BASELINE cfg5: QuantLinear 1024->1024 w4a4, 128-row tiles (T = 8, 16 slice pairs), batch 4096,
    as Conv2dLSQCiM(1024, 1024, k=1) on [B, 1024, 1, 1]."""
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd import functional as F
    rng = np.random.default_rng(55)
    C = O = 1024
    bits, xbar = 4, 128
    qp_a, (qn_w, qp_w) = 2 ** bits - 1, co.lsq_weight_params(bits)
    w = (rng.standard_normal((O, C, 1, 1)) * math.sqrt(2.0 / C)).astype(np.float32)

    def make(B):
        x = np.maximum(rng.standard_normal((B, C, 1, 1)), 0).astype(np.float32)
        g = (rng.standard_normal((B, O, 1, 1)) / math.sqrt(B * O)).astype(np.float32)
        return x, g

    aa = np.float32(2 * 0.4 / math.sqrt(qp_a))
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(qp_w))
    x4k, g4k = make(4096)
    sa0 = co.grad_scale_value(np.array([aa], np.float32), 1.0 / math.sqrt(x4k.size * qp_a))
    sw0 = co.grad_scale_value(np.array([aw], np.float32), 1.0 / math.sqrt(w.size * qp_w))
    xq0, _ = co.lsq_quantize(x4k[:16], sa0, 0, qp_a)
    wq0, _ = co.lsq_quantize(w, sw0, qn_w, qp_w)
    ac = co.alpha_cim_init(xq0, wq0, (1, 1), (0, 0), bits, 1, bits, 1, xbar, sw0, sa0, 1.5)
    ac = (ac * (0.7 + 0.6 * rng.random(ac.shape))).astype(np.float32)

    m = my_nn.Conv2dLSQCiM(C, O, 1, 1, 0, bias=False, **_kw(bits, xbar)).to(cuda_device)
    with torch.no_grad():
        m.weight.copy_(torch.from_numpy(w))
    _pin((m,), aa, aw, ac)

    # batch 4096: out and grad_x on 64 sampled rows against the Function oracle (same step sizes:
    # grad_scale's value depends on numel(x), lsq.py:547)
    xt = torch.from_numpy(x4k).to(cuda_device).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g4k).to(cuda_device))
    torch.cuda.synchronize()
    sel = rng.choice(4096, 64, replace=False)
    xq, _ = co.lsq_quantize(x4k[sel], sa0, 0, qp_a)
    wq, _ = co.lsq_quantize(w, sw0, qn_w, qp_w)
    alpha_q = co.alpha_quantize(ac, 8)
    bm = co.make_binary_mask(bits, bits, 1, 1)
    o_ref, c = co.cim_forward(xq, wq, (1, 1), (0, 0), (1, 1), bits, 1, bits, 1, 1.5, xbar, bm, alpha_q, sw0, sa0,
                              False, np.zeros(1, np.float32), return_debug=True)
    gxq, _, _ = co.cim_backward(c, g4k[sel].reshape(64, 1, O))
    axq, _, _ = co.cim_backward(c, g4k[sel].reshape(64, 1, O), absolute=True)
    y = (x4k[sel] / sa0).astype(np.float32)
    inside = (y >= 0) & (y <= qp_a)
    gx_ref = np.where(inside, ((gxq * sa0).astype(np.float32) / sa0).astype(np.float32), 0)  # lsq.py:549 STE
    out_terms = (np.abs(c.adc.astype(np.float64)) * np.abs(bm.astype(np.float64))).sum(axis=(1, 2, 3))
    assert rel_err(out.detach()[sel].reshape(64, O).cpu().numpy(), o_ref.reshape(64, O),
                   out_terms.reshape(64, O)) < 1e-6, "out (B=4096 rows)"
    assert rel_err(xt.grad[sel].cpu().numpy(), gx_ref, axq.reshape(gx_ref.shape)) < 1e-5, "grad_x (B=4096 rows)"
    # every integer partial sum and ADC output of those rows, bit-exact (the general kernel that
    # runs this 1x1 layer, lsq.py:166-230)
    sa_t = torch.from_numpy(sa0).to(cuda_device)
    sw_t = torch.from_numpy(sw0).to(cuda_device)
    _, ps, adc = F.debug_partial_sums(torch.from_numpy(xq).to(cuda_device), torch.from_numpy(wq).to(cuda_device),
                                      (1, 1), (0, 0), bits, 1, bits, 1, 1.5, xbar, torch.from_numpy(bm).to(cuda_device),
                                      torch.from_numpy(alpha_q).to(cuda_device), sw_t, sa_t,
                                      torch.zeros(1, device=cuda_device))
    assert np.array_equal(ps.cpu().numpy(), np.rint(c.ps16.astype(np.float64)).astype(np.int32))
    assert np.array_equal(adc.cpu().numpy(), c.adc)

    # batch 256: every gradient against the module oracle (full layer shape, full batch)
    x256, g256 = make(256)
    om = cmo.OracleConv2dLSQCiM(C, O, (1, 1), (1, 1), (0, 0), (1, 1), bias=False, **_kw(bits, xbar))
    om.debug_retain = True
    with torch.no_grad():
        om.weight.copy_(torch.from_numpy(w))
    _pin((m, om), aa, aw, ac)
    m.zero_grad()
    xt = torch.from_numpy(x256).to(cuda_device).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g256).to(cuda_device))
    box = _capture_oracle_ctx(monkeypatch)
    ox = torch.from_numpy(x256).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g256))
    _check_elementwise(box["c"], om.binary_mask.numpy(), g256, out, oout, xt, ox, m, om)
    d = om.dbg
    t_act = _lsq_scalar_terms(x256, d["x_q"].grad.numpy(), d["sa"].item(), 0, qp_a, 1.0 / math.sqrt(x256.size * qp_a))
    t_w = _lsq_scalar_terms(w, d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w, 1.0 / math.sqrt(w.size * qp_w))
    assert abs(m.alpha_act.grad.item() - om.alpha_act.grad.item()) <= 1e-5 * t_act
    assert abs(m.alpha_weight.grad.item() - om.alpha_weight.grad.item()) <= 1e-5 * t_w

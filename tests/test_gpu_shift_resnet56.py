"""GPU parity of BASELINE cfg4 at its own layer shapes: Conv2dLSQCiM(adc_shift=True) -- the
per-tile partial-sum scale + shift ADC of test/test_backward_cimlayer_scale_shift.py:336-546 as a
module option -- for ResNet-56 w2a2 xbar 64, adc 1.5, at every stage geometry (16->16 @32,
32->32 @16, 64->64 @8) and both stride-2 transitions (16->32 @32, 32->64 @16).

Bars (elementwise): out within 1e-6 of max(|ref|, sum |terms|); grad_x, grad_w and
grad_beta within 1e-5 of max(|ref|, sum |terms|) (the oracle's fp64 re-run on |operands|);
grad_alpha_cim normwise 1e-5 (its max/min scale terms gather every element's gradient); the two
step-size gradients within 1e-5 of their sum of |terms|.  Plus one B = 256 run per stage: images 0
and B-1 against the oracle on the module's own quantised operands, forward determinism and linearity in
grad_out for the batch-summed gradients; these shapes run the fast path (threshold ADC with beta
folded into the integer thresholds, v7 backward, cimq_part_shift.hip statistics), bit-identical run
to run.
"""
import math

import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co

pytestmark = pytest.mark.gpu

KW = dict(nbits_w=2, nbits_a=2, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=64, adcbits=1.5,
          stochastic_quant=False, adc_shift=True)
SHAPES = [(16, 16, 32, 1), (32, 32, 16, 1), (64, 64, 8, 1), (16, 32, 32, 2), (32, 64, 16, 2)]


def _pair(dev, C, O, s, rng, x):
    """The MI355X module and the CPU oracle module with identical parameters and step sizes."""
    import cim_quantization_amd._modules as my_nn
    m = my_nn.Conv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **KW).to(dev)
    om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **KW)
    om.debug_retain = True
    w = (rng.standard_normal((O, C, 3, 3)) * math.sqrt(2.0 / (9 * C))).astype(np.float32)
    aa = np.float32(2 * np.abs(x).mean() / math.sqrt(3))
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(1))
    shp = tuple(m.alpha_cim.shape)
    ac = (rng.random(shp) * 2 + 0.5).astype(np.float32) * aa * aw * 4
    bc = ((rng.random(shp) - 0.5) * 2).astype(np.float32) * aa * aw * 4
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
            mod.alpha_act.fill_(float(aa))
            mod.alpha_weight.fill_(float(aw))
            mod.alpha_cim.copy_(torch.from_numpy(ac))
            mod.beta_cim.copy_(torch.from_numpy(bc))
            mod.init_state.fill_(1)
            mod.init_state_cim.fill_(1)
        mod._state_cache = None
        mod.train()
    return m, om


def _capture_oracle_ctx(monkeypatch):
    """Keep the oracle Function's forward context (for the absolute-term re-run)."""
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
    """sum of |terms| of d loss / d alpha through grad_scale(alpha) (lsq.py:547-555)."""
    x, g = x.astype(np.float64), g_xq.astype(np.float64)
    y = x / float(s)
    r = np.rint(np.clip(y, qn, qp))
    inside = (y >= qn) & (y <= qp)
    return gscale * (np.abs(g * r).sum() + np.abs(np.where(inside, g * float(s), 0) * y / float(s)).sum())


@pytest.mark.parametrize("C,O,H,s", SHAPES)
def test_resnet56_shift_module_vs_oracle(cuda_device, monkeypatch, C, O, H, s):
    dev = cuda_device
    rng = np.random.default_rng(5600 + C + O + H + s)
    B = 2
    x = np.maximum(rng.standard_normal((B, C, H, H)), 0).astype(np.float32)
    m, om = _pair(dev, C, O, s, rng, x)
    box = _capture_oracle_ctx(monkeypatch)
    ho = (H + 2 - 3) // s + 1
    g = rng.standard_normal((B, O, ho, ho)).astype(np.float32)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g).to(dev))
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))
    c = box["c"]
    g_bpo = np.ascontiguousarray(g.reshape(B, O, ho * ho).transpose(0, 2, 1))
    ax, aw, _, ab = co.cim_backward(c, g_bpo, absolute=True)
    bm = np.abs(om.binary_mask.numpy().astype(np.float64))
    out_terms = (np.abs(c.adc.astype(np.float64)) * bm).sum(axis=(1, 2, 3))  # [B, P, O]
    out_terms = out_terms.transpose(0, 2, 1).reshape(B, O, ho, ho)
    np_ = lambda t: t.detach().cpu().numpy()  # noqa: E731
    assert rel_err(np_(out), np_(oout), out_terms) < 1e-6
    assert rel_err(np_(xt.grad), np_(ox.grad), ax) < 1e-5
    assert rel_err(np_(m.weight.grad), np_(om.weight.grad), aw.reshape(om.weight.shape)) < 1e-5
    assert rel_err(np_(m.beta_cim.grad), np_(om.beta_cim.grad), ab.reshape(om.beta_cim.shape)) < 1e-5
    ga, gr = np_(m.alpha_cim.grad), np_(om.alpha_cim.grad)
    assert np.abs(ga - gr).max() <= 1e-5 * np.abs(gr).max()
    d = om.dbg
    t_act = _scalar_terms(x, np_(d["x_q"].grad), d["sa"].item(), *d["qa"], 1.0 / math.sqrt(x.size * d["qa"][1]))
    t_w = _scalar_terms(np_(om.weight), np_(d["w_q"].grad), d["sw"].item(), *d["qw"],
                        1.0 / math.sqrt(om.weight.numel() * d["qw"][1]))
    assert abs(m.alpha_act.grad.item() - om.alpha_act.grad.item()) <= 1e-5 * t_act
    assert abs(m.alpha_weight.grad.item() - om.alpha_weight.grad.item()) <= 1e-5 * t_w


def _gs(a, n, qp):
    """grad_scale's forward value (lsq.py:23-26) in fp32, as the module evaluates it."""
    s = torch.tensor(1.0 / math.sqrt(n * qp), dtype=torch.float32)
    yg = a * s
    return (a - yg) + yg


@pytest.mark.parametrize("C,O,H", [(16, 16, 32), (32, 32, 16), (64, 64, 8)])
def test_resnet56_shift_fullbatch_sampled(cuda_device, C, O, H):
    """B = 256: images 0 and B-1 (forward, grad_x) against the oracle on the module's own quantised
    operands; the batch sums (grad_w, grad_alpha_cim, grad_beta) deterministic and linear in grad_out."""
    dev = cuda_device
    rng = np.random.default_rng(5700 + C)
    B = 256
    x = np.maximum(rng.standard_normal((B, C, H, H)), 0).astype(np.float32)
    m, _ = _pair(dev, C, O, 1, rng, x[:2])
    g1 = (rng.standard_normal((B, O, H, H)) / math.sqrt(B * O * H * H)).astype(np.float32)
    g2 = (rng.standard_normal((B, O, H, H)) / math.sqrt(B * O * H * H)).astype(np.float32)

    def run(gn):
        for p in m.parameters():
            p.grad = None
        xt = torch.from_numpy(x).to(dev).requires_grad_(True)
        out = m(xt)
        out.backward(torch.from_numpy(gn).to(dev))
        torch.cuda.synchronize()
        return out.detach(), xt.grad, m.weight.grad.clone(), m.alpha_cim.grad.clone(), m.beta_cim.grad.clone()

    o1, gx1, gw1, ga1, gb1 = run(g1)
    o1b, gx1b, gw1b, ga1b, gb1b = run(g1)
    assert torch.equal(o1, o1b), "forward run-to-run determinism"
    # the fast path (v7 backward + shift statistics) sums in a fixed order: bit-identical run to run
    for a_, b_ in ((gx1, gx1b), (gw1, gw1b), (ga1, ga1b), (gb1, gb1b)):
        assert torch.equal(a_, b_), "backward run-to-run determinism"
    _, _, gw2, ga2, gb2 = run(g2)
    _, _, gws, gas, gbs = run((g1 + g2).astype(np.float32))
    for a_, b_ in ((gw1 + gw2, gws), (ga1 + ga2, gas), (gb1 + gb2, gbs)):
        assert (a_ - b_).abs().max() <= 1e-5 * b_.abs().max()
    # the oracle on images 0 and B-1 with the module's step sizes (their grad_scale factors see B)
    qn_w, qp_w = co.lsq_weight_params(2)
    sa = _gs(m.alpha_act.detach().cpu(), x.size, 3.0)
    sw = _gs(m.alpha_weight.detach().cpu(), m.weight.numel(), float(qp_w))
    sel = [0, B - 1]
    xs = torch.from_numpy(x[sel])
    x_q = (torch.round((xs / sa).clamp(0, 3)) * sa).numpy()
    w = m.weight.detach().cpu()
    w_q = (torch.round((w / sw).clamp(qn_w, qp_w)) * sw).numpy()
    a = m.alpha_cim.detach().cpu()
    scale = (a.max() - a.min()) / 254.0
    alpha_q = (torch.round(a / scale).clamp(1, 255) * scale).numpy()
    bm = co.make_binary_mask(2, 2, 1, 1)
    out_o, c = co.cim_forward(x_q, w_q, (1, 1), (1, 1), (1, 1), 2, 1, 2, 1, 1.5, 64, bm, alpha_q, sw.numpy(),
                              sa.numpy(), False, np.zeros(1, np.float32), return_debug=True,
                              beta=m.beta_cim.detach().cpu().numpy())
    gsel = np.ascontiguousarray(g1[sel].reshape(2, O, H * H).transpose(0, 2, 1))
    gxq, _, _, _ = co.cim_backward(c, gsel)
    ax, _, _, _ = co.cim_backward(c, gsel, absolute=True)
    out_terms = (np.abs(c.adc.astype(np.float64)) * np.abs(bm)).sum(axis=(1, 2, 3)).transpose(0, 2, 1)
    mine = o1.cpu().numpy()[sel].reshape(2, O, H * H)
    assert rel_err(mine, out_o.transpose(0, 2, 1), out_terms) < 1e-6
    y = xs / sa
    inside = ((y >= 0) & (y <= 3)).numpy()
    assert rel_err(gx1.cpu().numpy()[sel], np.where(inside, gxq, 0), ax) < 1e-5

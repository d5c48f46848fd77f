"""GPU parity: libcimq (HIP, gfx950) against the reference's golden vectors and the oracle.

Bars:
  * integer steps bit-exact: every partial sum equals round(reference ps), every ADC output
    equals the reference ADC applied to it (same fp32 ops), NaN patterns included;
  * float reductions (out, grad_x, grad_w, grad_alpha, LSQ scale grads) within 1e-5 of
    max(|ref|, sum of |terms|) -- out within 1e-6.
"""
import math

import numpy as np
import pytest
import torch

from conftest import function_cases, golden_manifest, load_golden, module_cases, rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co

pytestmark = pytest.mark.gpu


def _fn():
    from cim_quantization_amd import functional as F
    return F


def _dev(a, dev, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t.requires_grad_(True) if grad else t


def run_hip_function(dev, cfg, inp, backward=True):
    F = _fn()
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    x = _dev(inp["x_q"], dev, True)
    w = _dev(inp["w_q"], dev, True)
    a = None if inp.get("alpha_q") is None else _dev(inp["alpha_q"], dev, True)
    args = (x, w, st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"], cfg["adc"], cfg["xbar"],
            _dev(inp["binary_mask"], dev), a, _dev(inp["sw"], dev), _dev(inp["sa"], dev), False,
            _dev(inp["signed_act"], dev))
    out = F.get_cim_output_signed.apply(*args)
    res = {"out": out.detach().cpu().numpy()}
    if backward:
        out.backward(_dev(inp["grad"], dev))
        res["grad_x"] = x.grad.cpu().numpy()
        res["grad_w"] = w.grad.cpu().numpy()
        if a is not None:
            res["grad_alpha"] = a.grad.cpu().numpy()
    _, ps, adc = F.debug_partial_sums(x.detach(), w.detach(), st, pd, cfg["ab"], cfg["abs"], cfg["wb"],
                                      cfg["wbs"], cfg["adc"], cfg["xbar"], _dev(inp["binary_mask"], dev),
                                      None if a is None else a.detach(), _dev(inp["sw"], dev),
                                      _dev(inp["sa"], dev), _dev(inp["signed_act"], dev))
    res["ps"] = ps.cpu().numpy()
    res["adc"] = adc.cpu().numpy()
    return res


def _golden_inputs(z):
    return dict(x_q=z["in_x_q"], w_q=z["in_w_q"], sa=z["in_sa"], sw=z["in_sw"],
                alpha_q=z.get("in_alpha_q"), grad=z["in_grad"], binary_mask=z["in_binary_mask"],
                signed_act=z["in_signed_act"])


def _check_integer_steps(cfg, inp, res, ref_ps16):
    """ps == round(reference ps) exactly; ADC output == reference ADC of that ps."""
    ps_ref = np.rint(ref_ps16.astype(np.float64)).astype(np.int64)
    assert np.array_equal(res["ps"].astype(np.int64), ps_ref), "integer partial sums differ"
    _, adc_ref = co.adc_apply(ps_ref.astype(np.float16), cfg["adc"], inp.get("alpha_q"), inp["sw"], inp["sa"])
    mine = res["adc"]
    same = (mine == adc_ref) | (np.isnan(mine) & np.isnan(adc_ref))
    assert same.all(), f"ADC outputs differ at {np.argwhere(~same)[:5].tolist()}"
    # and the reference's own ADC (on its fp16 ps) agrees wherever its ps had no fp32 residue
    _, adc_ref16 = co.adc_apply(ref_ps16, cfg["adc"], inp.get("alpha_q"), inp["sw"], inp["sa"])
    exact = ref_ps16.astype(np.float64) == ps_ref
    assert ((mine == adc_ref16) | np.isnan(adc_ref16) | ~exact).all()


@pytest.mark.parametrize("name", function_cases())
def test_function_vs_golden(cuda_device, name):
    cfg = golden_manifest()[name]["cfg"]
    z = load_golden(name)
    inp = _golden_inputs(z)
    res = run_hip_function(cuda_device, cfg, inp)
    _check_integer_steps(cfg, inp, res, z["ref_ps16"])
    if cfg.get("alpha_equal"):
        assert np.isnan(res["out"]).all()
        return
    assert rel_err(res["out"], z["ref_out"], z["ref_abs_out"]) < 1e-6
    assert rel_err(res["grad_x"], z["ref_grad_x"], z["ref_abs_grad_x"]) < 1e-5
    assert rel_err(res["grad_w"], z["ref_grad_w"], z["ref_abs_grad_w"]) < 1e-5
    if "ref_grad_alpha" in z:
        assert rel_err(res["grad_alpha"], z["ref_grad_alpha"], z["ref_abs_grad_alpha"]) < 1e-5


# ------------------------------------------------------------------------------------------
# random configurations against the oracle (run on the host CPU)
# ------------------------------------------------------------------------------------------
RANDOM_CASES = [
    # cfg1 of BASELINE.json: 16->16, 32x32, k3, B=4, w3a3, xbar 64, adc 4 and 1.5
    dict(B=4, C=16, O=16, H=32, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=64, adc=4, signed=0),
    dict(B=4, C=16, O=16, H=32, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=64, adc=1.5, signed=0),
    dict(B=2, C=24, O=40, H=9, k=3, s=2, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=32, adc=1.5, signed=0),
    dict(B=2, C=32, O=16, H=7, k=3, s=1, p=1, wb=4, ab=4, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=2, C=3, O=16, H=12, k=3, s=1, p=1, wb=8, ab=8, wbs=1, abs=1, xbar=128, adc=1.5, signed=1),
    dict(B=2, C=16, O=16, H=6, k=3, s=1, p=0, wb=4, ab=4, wbs=2, abs=2, xbar=64, adc=1, signed=0),
    dict(B=3, C=64, O=64, H=8, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=64, C=128, O=96, H=1, k=1, s=1, p=0, wb=4, ab=4, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    # v7 backward (compact state words, grad_x v8, grad_w v7): every stage / fold variant
    dict(B=2, C=64, O=64, H=8, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=2, C=32, O=64, H=16, k=3, s=2, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=2, C=16, O=32, H=32, k=3, s=2, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=2, C=32, O=32, H=16, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=2, C=16, O=16, H=16, k=3, s=1, p=1, wb=2, ab=2, wbs=1, abs=1, xbar=64, adc=1.5, signed=0),
    dict(B=2, C=32, O=16, H=16, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=64, adc=4, signed=0),
    # w8a8 on the v7 backward (64 slice pairs: plane state words): the first conv, a 2-tile case
    dict(B=2, C=3, O=16, H=32, k=3, s=1, p=1, wb=8, ab=8, wbs=1, abs=1, xbar=128, adc=1.5, signed=1),
    dict(B=2, C=3, O=16, H=16, k=3, s=2, p=1, wb=8, ab=8, wbs=1, abs=1, xbar=128, adc=1.5, signed=1),
    dict(B=2, C=16, O=16, H=16, k=3, s=1, p=1, wb=8, ab=8, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    # the dense GEMM path (1x1 kernels on 1x1 images, cimq_part_dense.hip): 16 / 4 / 9 slice pairs, a
    # partial last tile, signed activations
    dict(B=128, C=256, O=128, H=1, k=1, s=1, p=0, wb=4, ab=4, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=128, C=192, O=64, H=1, k=1, s=1, p=0, wb=2, ab=2, wbs=1, abs=1, xbar=64, adc=1.5, signed=0),
    dict(B=256, C=80, O=64, H=1, k=1, s=1, p=0, wb=3, ab=3, wbs=1, abs=1, xbar=64, adc=1.5, signed=1),
    # sign ADC: sign(ps) at ps = 0 follows the reference's fp32 residues (slice artifacts,
    # summation order), so this case uses power-of-two scales: x_int, w_int exact
    dict(B=2, C=16, O=16, H=16, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1, signed=0, sa=0.125,
         sw=0.0625),
]


def _random_inputs(cfg, seed):
    rng = np.random.default_rng(seed)
    B, C, O, H, k = cfg["B"], cfg["C"], cfg["O"], cfg["H"], cfg["k"]
    qp_a = 2 ** cfg["ab"] - 1
    qn_w, qp_w = co.lsq_weight_params(cfg["wb"])
    sa = np.array([cfg.get("sa", rng.uniform(0.05, 0.4))], np.float32)
    sw = np.array([cfg.get("sw", rng.uniform(0.01, 0.3))], np.float32)
    r = rng.integers(0, qp_a + 1, size=(B, C, H, H)).astype(np.float32)
    r[rng.random(r.shape) < 0.35] = 0
    x_q = (r * sa).astype(np.float32)
    w_q = (rng.integers(qn_w, qp_w + 1, size=(O, C, k, k)).astype(np.float32) * sw).astype(np.float32)
    nbw, nba = cfg["wb"] // cfg["wbs"], cfg["ab"] // cfg["abs"]
    T = math.ceil(C * k * k / cfg["xbar"])
    alpha_q = None
    if cfg["adc"] in (1, 1.5):
        a = (rng.random((1, T, nbw, nba, 1, O)) * 4 + 0.2).astype(np.float32) * np.float32(sw[0] * sa[0])
        alpha_q = co.alpha_quantize(a, 8)
    ho = co.out_size(H, k, cfg["p"], cfg["s"])
    g = rng.standard_normal((B, ho * ho, O)).astype(np.float32)
    return dict(x_q=x_q, w_q=w_q, sa=sa, sw=sw, alpha_q=alpha_q, grad=g,
                binary_mask=co.make_binary_mask(nbw, nba, cfg["wbs"], cfg["abs"]),
                signed_act=np.array([float(cfg["signed"])], np.float32))


@pytest.mark.parametrize("idx", range(len(RANDOM_CASES)))
def test_function_vs_oracle_random(cuda_device, idx):
    cfg = RANDOM_CASES[idx]
    inp = _random_inputs(cfg, 7000 + idx)
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    out, c = co.cim_forward(inp["x_q"], inp["w_q"], st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"],
                            cfg["adc"], cfg["xbar"], inp["binary_mask"], inp["alpha_q"], inp["sw"], inp["sa"],
                            False, inp["signed_act"], return_debug=True)
    gx, gw, ga = co.cim_backward(c, inp["grad"])
    ax, aw, aa = co.cim_backward(c, inp["grad"], absolute=True)
    res = run_hip_function(cuda_device, cfg, inp)
    _check_integer_steps(cfg, inp, res, c.ps16)
    out_terms = np.sum(np.abs(c.adc.astype(np.float64) * inp["binary_mask"]), axis=(1, 2, 3))
    assert rel_err(res["out"], out, out_terms) < 1e-6
    assert rel_err(res["grad_x"], gx, ax) < 1e-5
    assert rel_err(res["grad_w"], gw, aw) < 1e-5
    if ga is not None:
        assert rel_err(res["grad_alpha"], ga, aa) < 1e-5


# ------------------------------------------------------------------------------------------
# module level: Conv2dLSQCiM (fused LSQ + CiM, first-step init) against the golden runs
# ------------------------------------------------------------------------------------------
def _module_kwargs(cfg):
    return dict(nbits_w=cfg["wb"], nbits_a=cfg["ab"], nbits_alpha=8, wbitslice=1, abitslice=1,
                xbar=cfg["xbar"], adcbits=cfg["adc"], signed_xbar=True, stochastic_quant=False)


def _lsq_scalar_terms(x, g_xq, s, qn, qp, gscale):
    """sum of |terms| of d loss/d alpha through grad_scale(alpha)*... (lsq.py:547-555)."""
    x = x.astype(np.float64)
    g = g_xq.astype(np.float64)
    s = float(s)
    y = x / s
    r = np.rint(np.clip(y, qn, qp))
    inside = (y >= qn) & (y <= qp)
    return gscale * (np.abs(g * r).sum() + np.abs(np.where(inside, g * s, 0) * y / s).sum())


def _set_state_from_golden(m, z, p):
    """Pin the module's scalar state to the reference's after-step values.  The reference's
    backward is discontinuous in the last bit of sa (int8 truncation of x_q/sa at
    lsq.py:99, the clamp boundary at lsq.py:549), and a device-side mean differs from the
    CPU mean by an ulp, so step comparisons run on identical scalars."""
    with torch.no_grad():
        m.alpha_act.copy_(torch.from_numpy(z[p + "alpha_act"]))
        m.alpha_weight.copy_(torch.from_numpy(z[p + "alpha_weight"]))
        m.signed_act.copy_(torch.from_numpy(z[p + "signed_act"]))
        m.init_state.fill_(1)
        if m.alpha_cim is not None:
            m.alpha_cim.copy_(torch.from_numpy(z[p + "alpha_cim"]))
            m.init_state_cim.fill_(1)
    m._state_cache = None


@pytest.mark.parametrize("name", module_cases())
def test_module_init_vs_golden(cuda_device, name):
    """First training step initialisation (lsq.py:532-542, 557-563) on the device."""
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd import functional as F
    cfg = golden_manifest()[name]["cfg"]
    z = load_golden(name)
    st, pd = cfg["s"], cfg["p"]
    m = my_nn.Conv2dLSQCiM(cfg["C"], cfg["O"], (cfg["k"], cfg["k"]), (st, st), (pd, pd), (1, 1), groups=1,
                           bias=cfg["bias"], **_module_kwargs(cfg)).to(cuda_device)
    with torch.no_grad():
        m.weight.copy_(torch.from_numpy(z["in_weight"]))
    m.train()
    x = torch.from_numpy(z["in_x0"]).to(cuda_device)
    m(x)
    assert abs(m.alpha_act.item() - z["ref_s0_alpha_act"][0]) <= 1e-6 * abs(z["ref_s0_alpha_act"][0])
    assert abs(m.alpha_weight.item() - z["ref_s0_alpha_weight"][0]) <= 1e-6 * abs(z["ref_s0_alpha_weight"][0])
    assert m.signed_act.item() == z["ref_s0_signed_act"][0]
    if m.alpha_cim is None:
        return
    # alpha_cim init on the reference's exact step sizes
    qn_w, qp_w = co.lsq_weight_params(cfg["wb"])
    qp_a = 2 ** cfg["ab"] - 1
    aa = torch.from_numpy(z["ref_s0_alpha_act"]).to(cuda_device)
    aw = torch.from_numpy(z["ref_s0_alpha_weight"]).to(cuda_device)
    sa = my_nn.grad_scale(aa, 1.0 / math.sqrt(x.numel() * qp_a))
    sw = my_nn.grad_scale(aw, 1.0 / math.sqrt(m.weight.numel() * qp_w))
    w_q = my_nn.round_pass((m.weight.detach() / sw).clamp(qn_w, qp_w)) * sw
    a0 = F.alpha_cim_init(x, w_q, sa, sw, m.binary_mask, m.signed_act, m.stride, m.padding, m.nbits_a,
                          m.abitslice, m.nbits_w, m.wbitslice, m.adcbits, m.xbar, m.num_xbars)
    assert rel_err(a0.cpu().numpy(), z["ref_s0_alpha_cim"]) < 1e-5


def _capture_oracle_ctx(monkeypatch):
    """Keep the oracle module's Function context (the ADC outputs, the saved operands) for the
    absolute-term re-run that scales the elementwise bars."""
    box = {}
    real = co.cim_forward

    def rec(*a, **k):
        k["return_debug"] = True
        out, c = real(*a, **k)
        box["c"] = c
        return out, c
    monkeypatch.setattr(cmo.co, "cim_forward", rec)
    return box


@pytest.mark.parametrize("name", module_cases())
def test_module_steps_vs_golden(cuda_device, monkeypatch, name):
    """Two module steps against the reference's golden runs, element by element: out within 1e-6 and
    grad_x / grad_w / grad_alpha_cim within 1e-5 of max(|ref|, sum of |terms|) (the oracle's fp64
    re-run of the Function's contractions on |operands|; alpha_cim's max / min entries, which collect
    the alpha quantiser's scale gradient from every element, normwise), the step sizes within 1e-5
    of their sum of |terms|."""
    import cim_quantization_amd._modules as my_nn
    cfg = golden_manifest()[name]["cfg"]
    z = load_golden(name)
    st, pd = cfg["s"], cfg["p"]
    m = my_nn.Conv2dLSQCiM(cfg["C"], cfg["O"], (cfg["k"], cfg["k"]), (st, st), (pd, pd), (1, 1), groups=1,
                           bias=cfg["bias"], **_module_kwargs(cfg)).to(cuda_device)
    om = cmo.OracleConv2dLSQCiM(cfg["C"], cfg["O"], (cfg["k"], cfg["k"]), (st, st), (pd, pd), (1, 1), groups=1,
                                bias=cfg["bias"], **_module_kwargs(cfg))
    om.debug_retain = True
    with torch.no_grad():
        m.weight.copy_(torch.from_numpy(z["in_weight"]))
        om.weight.copy_(torch.from_numpy(z["in_weight"]))
    m.train()
    om.train()
    for step in range(2):
        p = f"ref_s{step}_"
        _set_state_from_golden(m, z, p)
        _set_state_from_golden(om, z, p)
        xin = z[f"in_x{step}"]
        x = torch.from_numpy(xin.copy()).to(cuda_device).requires_grad_(True)
        out = m(x)
        out.backward(torch.from_numpy(z[f"in_g{step}"]).to(cuda_device))
        box = _capture_oracle_ctx(monkeypatch)
        ox = torch.from_numpy(xin.copy()).requires_grad_(True)
        om(ox).backward(torch.from_numpy(z[f"in_g{step}"]))
        c = box["c"]
        B, O = z[p + "out"].shape[:2]
        g_bpo = np.ascontiguousarray(z[f"in_g{step}"].reshape(B, O, -1).transpose(0, 2, 1))
        ab = co.cim_backward(c, g_bpo, absolute=True)
        ax, aw, aa = ab[0], ab[1], ab[2]
        bmask = np.abs(om.binary_mask.numpy().astype(np.float64))
        out_terms = (np.abs(c.adc.astype(np.float64)) * bmask).sum(axis=(1, 2, 3)).transpose(0, 2, 1)
        out_terms = out_terms.reshape(z[p + "out"].shape)
        assert rel_err(out.detach().cpu().numpy(), z[p + "out"], out_terms) < 1e-6, "out"
        assert rel_err(x.grad.cpu().numpy(), z[p + "grad_x"], ax.reshape(xin.shape)) < 1e-5, "grad_x"
        assert rel_err(m.weight.grad.cpu().numpy(), z[p + "grad_weight"], aw.reshape(z[p + "grad_weight"].shape)) \
            < 1e-5, "grad_weight"
        if m.alpha_cim is not None:
            ga, gr = m.alpha_cim.grad.cpu().numpy(), z[p + "grad_alpha_cim"]
            a = om.alpha_cim.detach().numpy()
            inner = (a != a.max()) & (a != a.min())
            aab = np.broadcast_to(aa, gr.shape)
            assert rel_err(ga[inner], gr[inner], aab[inner]) < 1e-5, "grad_alpha_cim"
            assert np.abs(ga - gr).max() <= 1e-5 * np.abs(gr).max(), "grad_alpha_cim (max / min entries)"
        d = om.dbg
        qn_a, qp_a = d["qa"]
        qn_w, qp_w = d["qw"]
        ga = 1.0 / math.sqrt(xin.size * qp_a)
        gw_ = 1.0 / math.sqrt(z["in_weight"].size * qp_w)
        t_act = _lsq_scalar_terms(xin, d["x_q"].grad.numpy(), d["sa"].item(), qn_a, qp_a, ga)
        t_w = _lsq_scalar_terms(om.weight.detach().numpy(), d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w, gw_)
        assert abs(m.alpha_act.grad.item() - z[p + "grad_alpha_act"][0]) <= 1e-5 * t_act
        assert abs(m.alpha_weight.grad.item() - z[p + "grad_alpha_weight"][0]) <= 1e-5 * t_w
        for mod in (m, om):
            for prm in mod.parameters():
                prm.grad = None


# ------------------------------------------------------------------------------------------
# full ResNet-20 sizes (B = 256): size-independent properties + sampled images vs oracle
# ------------------------------------------------------------------------------------------
FULL = [
    dict(B=256, C=16, O=16, H=32, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=256, C=32, O=64, H=16, k=3, s=2, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
    dict(B=256, C=64, O=64, H=8, k=3, s=1, p=1, wb=3, ab=3, wbs=1, abs=1, xbar=128, adc=1.5, signed=0),
]


@pytest.mark.parametrize("idx", range(len(FULL)))
def test_fullsize_sampled_images_and_properties(cuda_device, idx):
    F = _fn()
    cfg = FULL[idx]
    inp = _random_inputs(cfg, 9100 + idx)
    dev = cuda_device
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])

    def run(g_np):
        x = _dev(inp["x_q"], dev, True)
        w = _dev(inp["w_q"], dev, True)
        a = _dev(inp["alpha_q"], dev, True)
        out = F.get_cim_output_signed.apply(x, w, st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"],
                                            cfg["adc"], cfg["xbar"], _dev(inp["binary_mask"], dev), a,
                                            _dev(inp["sw"], dev), _dev(inp["sa"], dev), False,
                                            _dev(inp["signed_act"], dev))
        out.backward(_dev(g_np, dev))
        return out.detach(), x.grad, w.grad, a.grad

    o1, gx1, gw1, ga1 = run(inp["grad"])
    o2, _, _, _ = run(inp["grad"])
    assert torch.equal(o1, o2), "forward must be deterministic"
    # linearity of the backward in grad_out (masks depend only on the forward)
    rng = np.random.default_rng(5)
    g2 = rng.standard_normal(inp["grad"].shape).astype(np.float32)
    _, gxa, gwa, gaa = run(g2)
    _, gxs, gws, gas = run((inp["grad"] + g2).astype(np.float32))
    for a_, b_ in ((gx1 + gxa, gxs), (gw1 + gwa, gws), (ga1 + gaa, gas)):
        assert (a_ - b_).abs().max() <= 1e-5 * b_.abs().max()
    # images 0 and B-1 against the oracle (forward and grad_x are per-image)
    sel = [0, cfg["B"] - 1]
    xs = inp["x_q"][sel]
    out_o, c = co.cim_forward(xs, inp["w_q"], st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"],
                              cfg["adc"], cfg["xbar"], inp["binary_mask"], inp["alpha_q"], inp["sw"], inp["sa"],
                              False, inp["signed_act"], return_debug=True)
    gx_o, _, _ = co.cim_backward(c, inp["grad"][sel])
    ax, _, _ = co.cim_backward(c, inp["grad"][sel], absolute=True)
    out_terms = np.sum(np.abs(c.adc.astype(np.float64) * inp["binary_mask"]), axis=(1, 2, 3))
    assert rel_err(o1.cpu().numpy()[sel], out_o, out_terms) < 1e-6
    assert rel_err(gx1.cpu().numpy()[sel], gx_o, ax) < 1e-5
    _, ps, adc = F.debug_partial_sums(_dev(xs, dev), _dev(inp["w_q"], dev), st, pd, cfg["ab"], cfg["abs"],
                                      cfg["wb"], cfg["wbs"], cfg["adc"], cfg["xbar"], _dev(inp["binary_mask"], dev),
                                      _dev(inp["alpha_q"], dev), _dev(inp["sw"], dev), _dev(inp["sa"], dev),
                                      _dev(inp["signed_act"], dev))
    assert np.array_equal(ps.cpu().numpy().astype(np.int64), np.rint(c.ps16.astype(np.float64)).astype(np.int64))

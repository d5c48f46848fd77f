"""GPU parity of the ADC variants: the scale + shift ADC (test/test_backward_cimlayer_scale_shift.py
Functions, the Conv2dLSQCiM(adc_shift=True) option) and the stochastic 1.5-bit ADC (lsq.py:205-221).

Bars: the reference's golden vectors and the oracle, out within 1e-6 and gradients within 1e-5 of
max(|ref|, sum of |terms|); exact equality where every value is an integer (the reference
scripts' own configurations); the stochastic ADC statistically (exact code distribution) and its
backward equal to the deterministic one (lsq.py:244-386 never sees the draws).
"""
import math

import numpy as np
import pytest
import torch

from conftest import load_golden, rel_err, shift_manifest
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co
from oracle import cim_shift_oracle as so

pytestmark = pytest.mark.gpu


def _F():
    from cim_quantization_amd import functional as F
    return F


def _dev(a, dev, grad=False):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t.requires_grad_(True) if grad else t


def _run_shift(dev, fn, cfg, x, w, alpha, beta, bm, grad):
    xt, wt = _dev(x, dev, True), _dev(w, dev, True)
    at, bt = _dev(alpha, dev, True), _dev(beta, dev, True)
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    out = fn.apply(xt, wt, st, pd, (1, 1), cfg["ab"], 1, cfg["wb"], 1, cfg["adc"], cfg["xbar"], _dev(bm, dev), at, bt)
    out.backward(_dev(grad, dev))
    torch.cuda.synchronize()
    return dict(out=out.detach().cpu().numpy(), grad_x=xt.grad.cpu().numpy(), grad_w=wt.grad.cpu().numpy(),
                grad_alpha=at.grad.cpu().numpy(), grad_beta=bt.grad.cpu().numpy())


@pytest.mark.parametrize("name", sorted(shift_manifest()))
def test_shift_function_vs_golden(cuda_device, name):
    F = _F()
    cfg = shift_manifest()[name]["cfg"]
    z = load_golden(name)
    fn = F.get_adcless_cim_output if cfg["fn"] == "adcless" else F.get_analog_partial_sums_autograd_ver2
    beta = z["in_beta"] if "in_beta" in z else np.zeros((1,) + z["in_alpha"].shape[1:2] + (cfg["wb"], cfg["ab"], 1,
                                                                                            cfg["O"]), np.float32)
    res = _run_shift(cuda_device, fn, cfg, z["in_x"], z["in_w"], z["in_alpha"], beta, z["in_binary_mask"],
                     z["in_grad"])
    assert rel_err(res["out"], z["ref_out"], z["ref_abs_out"]) < 1e-6
    assert rel_err(res["grad_x"], z["ref_grad_x"], z["ref_abs_grad_x"]) < 1e-5
    assert rel_err(res["grad_w"], z["ref_grad_w"], z["ref_abs_grad_w"]) < 1e-5
    assert rel_err(res["grad_alpha"], z["ref_grad_alpha"], z["ref_abs_grad_alpha"]) < 1e-5
    if "ref_grad_beta" in z:
        assert rel_err(res["grad_beta"], z["ref_grad_beta"], z["ref_abs_grad_beta"]) < 1e-5
    if cfg["alpha"] in ("int13", "ones_tile") and cfg["beta"] in ("int14", None):
        # integer alpha / beta: every output is an integer sum, identical in any order
        assert np.array_equal(res["out"], z["ref_out"])


def test_reference_backward_cimlayer_config_exact(cuda_device):
    """test_backward_cimlayer.py:398-461 on the device: B=1, C=16, O=32, 32x32, k3 s2 p1, w3a3,
    xbar 64, adc 4, alpha_cim = 1, grad = 1 -- the script checks its manual Function against
    autograd by exact equality; the MI355X Function (ver2 with beta = 0: round-then-clamp equals
    the script's clamp-then-round at integer bounds) equals both exactly on out and grad_alpha,
    and to the last ulp on grad_x / grad_w (their 1/3 slice means round in summation order)."""
    F = _F()
    cfg = shift_manifest()["bk_adc4_ref_cfg"]["cfg"]
    z = load_golden("bk_adc4_ref_cfg")
    T = z["in_alpha"].shape[1]
    beta = np.zeros((1, T, cfg["wb"], cfg["ab"], 1, cfg["O"]), np.float32)
    res = _run_shift(cuda_device, F.get_analog_partial_sums_autograd_ver2, cfg, z["in_x"], z["in_w"], z["in_alpha"],
                     beta, z["in_binary_mask"], z["in_grad"])
    for k in ("out", "grad_alpha"):  # integer sums: identical in any order
        assert np.array_equal(res[k], z["ref_" + k]), k
        assert np.array_equal(res[k], z["auto_" + k]), k
    for k in ("grad_x", "grad_w"):  # the slice recombination divides by nba / nbw = 3: last-ulp order effects
        assert rel_err(res[k], z["ref_" + k]) < 1e-6, k
        assert rel_err(res[k], z["auto_" + k]) < 1e-6, k


def test_reference_scale_shift_config_criteria(cuda_device):
    """test_backward_cimlayer_scale_shift.py:700-767 on the device, with the script's own
    acceptance criteria against its autograd twin (|dx|, |dw| < 0.05; |dalpha|, |dbeta| < 5e-4)."""
    F = _F()
    cfg = shift_manifest()["ss_ver2_ref_cfg"]["cfg"]
    z = load_golden("ss_ver2_ref_cfg")
    res = _run_shift(cuda_device, F.get_analog_partial_sums_autograd_ver2, cfg, z["in_x"], z["in_w"], z["in_alpha"],
                     z["in_beta"], z["in_binary_mask"], z["in_grad"])
    assert np.mean(res["out"] == z["auto_out"]) == 1.0
    assert np.mean(np.abs(res["grad_x"] - z["auto_grad_x"]) < 0.05) == 1.0
    assert np.mean(np.abs(res["grad_w"] - z["auto_grad_w"]) < 0.05) == 1.0
    assert np.mean(np.abs(res["grad_alpha"] - z["auto_grad_alpha"]) < 0.0005) == 1.0
    assert np.mean(np.abs(res["grad_beta"] - z["auto_grad_beta"]) < 0.0005) == 1.0


# ResNet-56 w2a2 xbar 64 shapes (BASELINE cfg4: T = 3, 5, 9) and both variants, against the oracle
SHIFT_RANDOM = [
    dict(fn="ver2", B=2, C=16, O=16, H=8, k=3, s=1, p=1, wb=2, ab=2, xbar=64, adc=1),
    dict(fn="ver2", B=2, C=32, O=32, H=8, k=3, s=1, p=1, wb=2, ab=2, xbar=64, adc=2),
    dict(fn="ver2", B=2, C=64, O=64, H=8, k=3, s=2, p=1, wb=2, ab=2, xbar=64, adc=1),
    dict(fn="adcless", B=2, C=32, O=16, H=8, k=3, s=2, p=1, wb=2, ab=2, xbar=64, adc=1),
    dict(fn="adcless", B=2, C=64, O=64, H=6, k=3, s=1, p=1, wb=3, ab=3, xbar=64, adc=1),
]


@pytest.mark.parametrize("idx", range(len(SHIFT_RANDOM)))
def test_shift_function_vs_oracle_random(cuda_device, idx):
    F = _F()
    cfg = SHIFT_RANDOM[idx]
    rng = np.random.default_rng(8100 + idx)
    B, C, O, H, k = cfg["B"], cfg["C"], cfg["O"], cfg["H"], cfg["k"]
    T = math.ceil(C * k * k / cfg["xbar"])
    x = rng.integers(0, 2 ** cfg["ab"], (B, C, H, H)).astype(np.float32)
    w = rng.integers(-(2 ** (cfg["wb"] - 1)), 2 ** (cfg["wb"] - 1), (O, C, k, k)).astype(np.float32)
    shp = (1, T, cfg["wb"], cfg["ab"], 1, O)
    a = (rng.random(shp) * 3 + 0.5).astype(np.float32)
    b = (rng.random(shp) * 4 - 2).astype(np.float32)
    bm = co.make_binary_mask(cfg["wb"], cfg["ab"], 1, 1).astype(np.float32)
    ho = co.out_size(H, k, cfg["p"], cfg["s"])
    g = rng.standard_normal((B, ho * ho, O)).astype(np.float32)
    variant = so.VARIANT_SIGN if cfg["fn"] == "adcless" else so.VARIANT_ROUND
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    out, c = so.shift_forward(x, w, st, pd, cfg["ab"], 1, cfg["wb"], 1, cfg["adc"], cfg["xbar"], bm, a, b, variant)
    gx, gw, ga, gb = so.shift_backward(c, g)
    ax, aw, aa, ab = so.shift_backward(c, g, absolute=True)
    fn = F.get_adcless_cim_output if cfg["fn"] == "adcless" else F.get_analog_partial_sums_autograd_ver2
    res = _run_shift(cuda_device, fn, cfg, x, w, a, b, bm, g)
    out_terms = (np.abs(c.code.astype(np.float64) * a + b) * np.abs(bm)).sum(axis=(1, 2, 3))
    assert rel_err(res["out"], out, out_terms) < 1e-6
    assert rel_err(res["grad_x"], gx, ax) < 1e-5
    assert rel_err(res["grad_w"], gw, aw) < 1e-5
    assert rel_err(res["grad_alpha"], ga, aa) < 1e-5
    assert rel_err(res["grad_beta"], gb, ab) < 1e-5


# ------------------------------------------------------------------------------------------------
# Conv2dLSQCiM(adc_shift=True): the module option against the oracle module (same scalar state)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("adc,wb,C,H,s", [(1.5, 2, 16, 8, 1), (1.5, 2, 32, 8, 2), (1, 3, 16, 8, 1)])
def test_module_adc_shift_vs_oracle(cuda_device, adc, wb, C, H, s):
    import cim_quantization_amd._modules as my_nn
    rng = np.random.default_rng(int(adc * 10) + wb + C)
    O, B = 16, 2
    kw = dict(nbits_w=wb, nbits_a=wb, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=64, adcbits=adc,
              stochastic_quant=False, adc_shift=True)
    m = my_nn.Conv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **kw).to(cuda_device)
    om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, **kw)
    w = (rng.standard_normal((O, C, 3, 3)) * math.sqrt(2.0 / (9 * C))).astype(np.float32)
    x = np.maximum(rng.standard_normal((B, C, H, H)), 0).astype(np.float32)
    qp_a, qp_w = 2 ** wb - 1, 2 ** (wb - 1) - 1
    aa = np.float32(2 * np.abs(x).mean() / math.sqrt(qp_a))
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(qp_w))
    shp = tuple(m.alpha_cim.shape)
    ac = (rng.random(shp) * 2 + 0.5).astype(np.float32) * aa * aw * 3
    bc = ((rng.random(shp) - 0.5) * 2).astype(np.float32) * aa * aw * 3
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
    ho = (H + 2 - 3) // s + 1
    g = rng.standard_normal((B, O, ho, ho)).astype(np.float32)
    xt = torch.from_numpy(x).to(cuda_device).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g).to(cuda_device))
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))

    def close(mine, ref, tol):
        mine, ref = mine.detach().cpu().numpy().astype(np.float64), ref.detach().numpy().astype(np.float64)
        assert np.abs(mine - ref).max() <= tol * (np.abs(ref).max() + 1e-30), (np.abs(mine - ref).max(),
                                                                              np.abs(ref).max())

    close(out, oout, 1e-5)
    close(xt.grad, ox.grad, 1e-5)
    close(m.weight.grad, om.weight.grad, 1e-5)
    close(m.alpha_cim.grad, om.alpha_cim.grad, 1e-5)
    close(m.beta_cim.grad, om.beta_cim.grad, 1e-5)
    close(m.alpha_act.grad, om.alpha_act.grad, 1e-4)
    close(m.alpha_weight.grad, om.alpha_weight.grad, 1e-4)


# ------------------------------------------------------------------------------------------------
# stochastic 1.5-bit ADC (lsq.py:205-221)
# ------------------------------------------------------------------------------------------------
def _stoch_inputs(seed):
    rng = np.random.default_rng(seed)
    B, C, O, H = 2, 16, 16, 7  # P = 49: the general kernels for both the stochastic and the plain ADC
    sa, sw = np.array([0.05], np.float32), np.array([0.1], np.float32)
    x_q = (rng.integers(0, 8, (B, C, H, H)).astype(np.float32) * sa).astype(np.float32)
    w_q = (rng.integers(-4, 4, (O, C, 3, 3)).astype(np.float32) * sw).astype(np.float32)
    a = (0.02 * (1 + 0.5 * rng.random((1, 3, 3, 3, 1, O)))).astype(np.float32)
    alpha_q = co.alpha_quantize(a, 8)
    g = rng.standard_normal((B, H * H, O)).astype(np.float32)
    return dict(x_q=x_q, w_q=w_q, sa=sa, sw=sw, alpha_q=alpha_q, g=g, bm=co.make_binary_mask(3, 3, 1, 1))


def test_stochastic_adc_distribution(cuda_device):
    """Per-partial-sum codes of the stochastic ADC against their exact distribution: the counts of
    +1 / -1 codes within 6 sigma of the expectation, overall and per partial-sum value."""
    F = _F()
    dev = cuda_device
    inp = _stoch_inputs(11)
    st, pd = (1, 1), (1, 1)
    _, c = co.cim_forward(inp["x_q"], inp["w_q"], st, pd, (1, 1), 3, 1, 3, 1, 1.5, 64, inp["bm"], inp["alpha_q"],
                          inp["sw"], inp["sa"], False, np.zeros(1, np.float32), return_debug=True)
    alpha_full = np.broadcast_to(inp["alpha_q"], c.u.shape)
    p_plus, p_minus = co.stochastic_code_probs(c.u, alpha_full)
    nz = ((p_plus > 1e-9) & (p_plus < 1 - 1e-9)).sum()
    assert nz > 2000, "the configuration must exercise the random regime"
    tot_p = np.zeros(3)
    exp_p = np.zeros(3)
    var_p = np.zeros(3)
    for rep in range(4):
        _, ps, adc = F.debug_partial_sums(_dev(inp["x_q"], dev), _dev(inp["w_q"], dev), st, pd, 3, 1, 3, 1, 1.5, 64,
                                          _dev(inp["bm"], dev), _dev(inp["alpha_q"], dev), _dev(inp["sw"], dev),
                                          _dev(inp["sa"], dev), torch.zeros(1, device=dev), stochastic=True,
                                          seed=1234567 + 7919 * rep)
        assert np.array_equal(ps.cpu().numpy(), np.rint(c.ps16.astype(np.float64)).astype(np.int32))
        code = np.rint(adc.cpu().numpy() / alpha_full)
        assert np.isin(code, (-1, 0, 1)).all()
        n_plus, n_minus = (code == 1).sum(), (code == -1).sum()
        tot_p += (n_plus, n_minus, 0)
        exp_p += (p_plus.sum(), p_minus.sum(), 0)
        var_p += ((p_plus * (1 - p_plus)).sum(), (p_minus * (1 - p_minus)).sum(), 0)
        # saturated elements are deterministic
        sure = (p_plus > 1 - 1e-12)
        assert (code[sure] == 1).all()
        sure = (p_minus > 1 - 1e-12)
        assert (code[sure] == -1).all()
        # per partial-sum value (the probabilities depend on ps and alpha only)
        ps_i = np.rint(c.ps16.astype(np.float64)).astype(np.int64)
        for v in (-2, 0, 2, 4, 6):
            sel = ps_i == v
            if sel.sum() < 200:
                continue
            e, s = p_plus[sel].sum(), math.sqrt((p_plus[sel] * (1 - p_plus[sel])).sum()) + 1.0
            assert abs((code[sel] == 1).sum() - e) <= 6 * s, (v, (code[sel] == 1).sum(), e, s)
    for i in range(2):
        assert abs(tot_p[i] - exp_p[i]) <= 6 * math.sqrt(var_p[i]) + 1.0, (i, tot_p[i], exp_p[i], var_p[i])


def test_stochastic_seeded_and_backward_deterministic(cuda_device):
    """Same seed -> same draws; the backward of a stochastic forward equals the deterministic one
    (lsq.py:244-386 reads ctx.ps_int, not the stochastic ADC output)."""
    F = _F()
    dev = cuda_device
    inp = _stoch_inputs(12)
    st, pd = (1, 1), (1, 1)

    def dbg(seed):
        return F.debug_partial_sums(_dev(inp["x_q"], dev), _dev(inp["w_q"], dev), st, pd, 3, 1, 3, 1, 1.5, 64,
                                    _dev(inp["bm"], dev), _dev(inp["alpha_q"], dev), _dev(inp["sw"], dev),
                                    _dev(inp["sa"], dev), torch.zeros(1, device=dev), stochastic=True, seed=seed)[2]
    assert torch.equal(dbg(99), dbg(99))
    assert not torch.equal(dbg(99), dbg(100))

    def run(stochastic):
        torch.manual_seed(5)
        x, w, a = _dev(inp["x_q"], dev, True), _dev(inp["w_q"], dev, True), _dev(inp["alpha_q"], dev, True)
        out = F.get_cim_output_signed.apply(x, w, st, pd, (1, 1), 3, 1, 3, 1, 1.5, 64, _dev(inp["bm"], dev), a,
                                            _dev(inp["sw"], dev), _dev(inp["sa"], dev), stochastic,
                                            torch.zeros(1, device=dev))
        out.backward(_dev(inp["g"], dev))
        return out.detach(), x.grad, w.grad, a.grad

    o_s, gx_s, gw_s, ga_s = run(True)
    o_d, gx_d, gw_d, ga_d = run(False)
    assert torch.isfinite(o_s).all()
    # same masks and codes (they come from the partial sums only); the general kernels sum in a
    # fixed order (no atomics), so the two backwards are bit-identical
    for a_, b_ in ((gx_s, gx_d), (gw_s, gw_d), (ga_s, ga_d)):
        assert torch.equal(a_, b_)
    o_s2 = run(True)[0]
    assert torch.equal(o_s, o_s2), "torch.manual_seed must make the stochastic forward reproducible"


def test_stochastic_module_runs(cuda_device):
    """Conv2dLSQCiM(stochastic_quant=True): first (init) step and a fused steady-state step."""
    import cim_quantization_amd._modules as my_nn
    torch.manual_seed(3)
    m = my_nn.Conv2dLSQCiM(16, 16, 3, 1, 1, bias=False, nbits_w=3, nbits_a=3, xbar=64, adcbits=1.5,
                           stochastic_quant=True).to(cuda_device).train()
    for _ in range(2):
        x = torch.randn(2, 16, 8, 8, device=cuda_device).relu().requires_grad_(True)
        out = m(x)
        out.backward(torch.randn_like(out))
        assert torch.isfinite(out).all() and torch.isfinite(x.grad).all()
        assert torch.isfinite(m.alpha_cim.grad).all()
        m.zero_grad()

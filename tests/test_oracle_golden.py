"""CPU: the numpy oracle reproduces the reference's golden vectors (tests/golden, generated
from the real reference by tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from conftest import function_cases, load_golden, module_cases, golden_manifest, rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co


def _fn_args(cfg, z):
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    alpha = z.get("in_alpha_q")
    return (z["in_x_q"], z["in_w_q"], st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"],
            cfg["adc"], cfg["xbar"], z["in_binary_mask"], alpha, z["in_sw"], z["in_sa"], False,
            z["in_signed_act"])


@pytest.mark.parametrize("name", function_cases())
def test_oracle_function_matches_reference(name):
    cfg = golden_manifest()[name]["cfg"]
    z = load_golden(name)
    out, c = co.cim_forward(*_fn_args(cfg, z))
    # integer context: bit-exact
    assert np.array_equal(c.x_int8, z["ref_ctx_x_int8"])
    assert np.array_equal(c.w_sliced8, z["ref_ctx_w_sliced8"])
    ref_ps = z["ref_ps16"].astype(np.float64)
    assert np.array_equal(np.rint(c.ps16.astype(np.float64)), np.rint(ref_ps))
    # fp16 partial sums: equal except near-zero fp32 residues of the non-integer slices
    assert np.abs(c.ps16.astype(np.float64) - ref_ps).max() < 1e-3
    if cfg.get("alpha_equal"):
        assert np.isnan(out).all() and np.isnan(z["ref_out"]).all()
        return
    assert rel_err(out, z["ref_out"], z["ref_abs_out"]) < 1e-6
    gx, gw, ga = co.cim_backward(c, z["in_grad"])
    assert rel_err(gx, z["ref_grad_x"], z["ref_abs_grad_x"]) < 1e-5
    assert rel_err(gw, z["ref_grad_w"], z["ref_abs_grad_w"]) < 1e-5
    if "ref_grad_alpha" in z:
        assert rel_err(ga, z["ref_grad_alpha"], z["ref_abs_grad_alpha"]) < 1e-5


def _module_kwargs(cfg):
    return dict(nbits_w=cfg["wb"], nbits_a=cfg["ab"], nbits_alpha=8, wbitslice=1, abitslice=1,
                xbar=cfg["xbar"], adcbits=cfg["adc"], signed_xbar=True, stochastic_quant=False)


@pytest.mark.parametrize("name", module_cases())
def test_oracle_module_matches_reference(name):
    cfg = golden_manifest()[name]["cfg"]
    z = load_golden(name)
    st, pd = cfg["s"], cfg["p"]
    m = cmo.OracleConv2dLSQCiM(cfg["C"], cfg["O"], (cfg["k"], cfg["k"]), (st, st), (pd, pd), (1, 1),
                               groups=1, bias=cfg["bias"], **_module_kwargs(cfg))
    with torch.no_grad():
        m.weight.copy_(torch.from_numpy(z["in_weight"]))
    m.train()
    for step in range(2):
        x = torch.from_numpy(z[f"in_x{step}"].copy()).requires_grad_(True)
        out = m(x)
        out.backward(torch.from_numpy(z[f"in_g{step}"]))
        p = f"ref_s{step}_"
        scale = lambda k: np.abs(z[p + k]).max()  # noqa: E731
        assert np.abs(out.detach().numpy() - z[p + "out"]).max() <= 1e-5 * scale("out")
        assert np.abs(x.grad.numpy() - z[p + "grad_x"]).max() <= 1e-5 * scale("grad_x") + 1e-12
        assert np.abs(m.weight.grad.numpy() - z[p + "grad_weight"]).max() <= 1e-5 * scale("grad_weight")
        assert np.array_equal(m.signed_act.numpy(), z[p + "signed_act"])
        if m.alpha_cim is not None:
            assert np.abs(m.alpha_cim.grad.numpy() - z[p + "grad_alpha_cim"]).max() <= \
                1e-5 * scale("grad_alpha_cim")
        for prm in m.parameters():
            prm.grad = None
        with torch.no_grad():
            m.alpha_act.mul_(1.07)
            m.alpha_weight.mul_(0.93)
            if m.alpha_cim is not None:
                m.alpha_cim.mul_(torch.linspace(0.8, 1.2, m.alpha_cim.numel()).view_as(m.alpha_cim))


def test_binary_mask_wraps_like_reference():
    # 8-bit layers: entries with j+k = 7 become -128, j+k >= 8 become 0 (_quan_base.py:207-214)
    m = co.make_binary_mask(8, 8, 1, 1).reshape(8, 8)
    for k in range(8):
        for j in range(8):
            e = j + k
            want = (1 << e) if e < 7 else (-128 if e == 7 else 0)
            assert m[k, j] == want


def test_xq_roundtrip_artifact_slices():
    # fl(fl(6*s)/s) < 6 for s=0.08475284: slicing gives [2-eps, 0, 1], not [0, 1, 1]
    s = np.float32(0.08475284)
    xi = (np.float32(6) * s).astype(np.float32) / s
    assert xi < 6
    sl = co.slicing_act(np.array([xi], np.float32), 3, 1)[:, 0]
    assert np.rint(sl).tolist() == [2.0, 0.0, 1.0]
    assert co.to_int8(np.array([xi]))[0] == 5

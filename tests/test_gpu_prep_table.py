"""GPU parity of the module path's activation prep on inputs that sit on the quantiser's edges.

The prep tabulates the slice words of every LSQ code r = rint(clamp(x/sa, 0, Qp)) once per
block (cimq_kernels.hip, act_lut_build) and looks each element up by its code.  These inputs
put x/sa exactly on the rint ties (k + 0.5 with a power-of-two step size, so the division is
exact), just inside and outside the clamp range, on -0.0 and on large magnitudes, and the layer
is checked against the module oracle (lsq.py:522-588): out, every gradient, and the ADC codes
and STE-pass bits the production forward recorded.  Tolerances as test_gpu_fullsize.py.
"""
import math

import numpy as np
import pytest
import torch

from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co
from test_gpu_fullsize import _close, _kw, _lsq_scalar_terms, _oracle_codes, _pin

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("aa", [0.25, 0.3])
def test_prep_table_edges(cuda_device, aa):
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd import functional as F
    B, C, O, H, bits = 8, 16, 16, 16, 3
    rng = np.random.default_rng(7)
    torch.manual_seed(0)
    m = my_nn.Conv2dLSQCiM(C, O, 3, 1, 1, bias=False, **_kw(bits)).to(cuda_device)
    om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (1, 1), (1, 1), (1, 1), bias=False, **_kw(bits))
    om.debug_retain = True
    aa = np.float32(aa)
    qp_a, (qn_w, qp_w) = 2 ** bits - 1, co.lsq_weight_params(bits)
    edges = np.array([(k + 0.5) * aa for k in range(-2, 10)] + [k * aa for k in range(-1, 10)] +
                     [np.nextafter(np.float32(7.5 * aa), np.float32(0)), np.nextafter(np.float32(0.5 * aa), np.float32(1)),
                      -0.0, 0.0, 1e6, -1e6, 3.4e38, 1e-30], np.float32)
    x = edges[rng.integers(0, edges.size, (B, C, H, H))]
    x = np.where(rng.random(x.shape) < 0.3, np.abs(rng.standard_normal(x.shape)).astype(np.float32) * aa * 4, x)
    x = x.astype(np.float32)
    w = (rng.standard_normal((O, C, 3, 3)) * math.sqrt(2.0 / (9 * C))).astype(np.float32)
    g = (rng.standard_normal((B, O, H, H)) / math.sqrt(B * O * H * H)).astype(np.float32)
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(qp_w))
    sa0 = co.grad_scale_value(np.array([aa], np.float32), 1.0 / math.sqrt(x.size * qp_a))
    sw0 = co.grad_scale_value(np.array([aw], np.float32), 1.0 / math.sqrt(w.size * qp_w))
    xq0, _ = co.lsq_quantize(x[:4], sa0, 0, qp_a)
    wq0, _ = co.lsq_quantize(w, sw0, qn_w, qp_w)
    ac = co.alpha_cim_init(xq0, wq0, (1, 1), (1, 1), bits, 1, bits, 1, 128, sw0, sa0, 1.5)
    ac = (ac * (0.7 + 0.6 * rng.random(ac.shape))).astype(np.float32)
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
    _pin((m, om), aa, aw, ac)

    xt = torch.from_numpy(x).to(cuda_device).requires_grad_(True)
    out = m(xt)
    code, passed = F.debug_state_codes(out)
    out.backward(torch.from_numpy(g).to(cuda_device))
    torch.cuda.synchronize()
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))

    _close(out, oout, 1e-5, "out")
    _close(xt.grad, ox.grad, 1e-5, "grad_x")
    _close(m.weight.grad, om.weight.grad, 1e-5, "grad_weight")
    _close(m.alpha_cim.grad, om.alpha_cim.grad, 1e-5, "grad_alpha_cim")
    d = om.dbg
    t_act = _lsq_scalar_terms(x, d["x_q"].grad.numpy(), d["sa"].item(), 0, qp_a, 1.0 / math.sqrt(x.size * qp_a))
    t_w = _lsq_scalar_terms(w, d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w, 1.0 / math.sqrt(w.size * qp_w))
    # x = 3.4e38 overflows x / sa to inf: the reference's act step-size gradient is then
    # (inf-related) NaN, and so must this one be
    ma, oa = m.alpha_act.grad.item(), om.alpha_act.grad.item()
    assert (math.isnan(ma) and math.isnan(oa)) or abs(ma - oa) <= 1e-5 * t_act, (ma, oa)
    assert abs(m.alpha_weight.grad.item() - om.alpha_weight.grad.item()) <= 1e-5 * t_w

    alpha_q = co.alpha_quantize(om.alpha_cim.detach().numpy(), 8)
    oc, op = _oracle_codes(d["x_q"].detach().numpy(), d["w_q"].detach().numpy(), (1, 1), (1, 1), bits, 128, alpha_q,
                           d["sw"].detach().numpy().reshape(1), d["sa"].detach().numpy().reshape(1), 0.0)
    assert np.array_equal(code.cpu().numpy(), oc)
    assert np.array_equal(passed.cpu().numpy(), op)

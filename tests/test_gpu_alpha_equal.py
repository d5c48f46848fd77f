"""The all-equal alpha_cim quirk at module level (lsq.py:566-573): max == min gives scale = 0, so
alpha_q = clamp(round_pass(alpha / 0), 1, 2^b - 1) * 0 is NaN (inf - inf inside round_pass) and the
ADC divides by it.  The fused module prologue (prep_module_kernel: alpha_cim's quantiser inside the
threshold search) must set the literal-ADC flag and reproduce the reference's NaNs -- through the
general / v3 kernels for a 3x3 conv and through the dense path's literal kernel for a 1x1 layer --
and the backward must give the module oracle's gradients: the same NaN pattern, the finite entries
within 1e-5 of the oracle's largest finite magnitude.
"""
import math

import numpy as np
import pytest
import torch

from oracle import cim_module_oracle as cmo

pytestmark = pytest.mark.gpu

CASES = [
    # (B, C, O, H, k, bits, xbar): a 3x3 conv and a dense 1x1 layer (cimq_part_dense.hip)
    (2, 16, 16, 8, 3, 3, 64),
    (128, 128, 64, 1, 1, 2, 64),
]


def _same(mine, ref, what):
    mine = mine.detach().cpu().numpy().astype(np.float64)
    ref = ref.detach().cpu().numpy().astype(np.float64)
    nm, nr = np.isnan(mine), np.isnan(ref)
    assert np.array_equal(nm, nr), f"{what}: NaN pattern ({nm.sum()} vs {nr.sum()} NaNs)"
    fin = ~nr
    if fin.any():
        scale = max(np.abs(ref[fin]).max(), 1e-30)
        assert np.abs(mine[fin] - ref[fin]).max() <= 1e-5 * scale, what


@pytest.mark.parametrize("B,C,O,H,k,bits,xbar", CASES)
def test_module_all_equal_alpha(cuda_device, B, C, O, H, k, bits, xbar):
    import cim_quantization_amd._modules as my_nn
    rng = np.random.default_rng(566 + C)
    p = k // 2
    kw = dict(nbits_w=bits, nbits_a=bits, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=xbar, adcbits=1.5,
              stochastic_quant=False)
    m = my_nn.Conv2dLSQCiM(C, O, k, 1, p, bias=False, **kw).to(cuda_device)
    om = cmo.OracleConv2dLSQCiM(C, O, (k, k), (1, 1), (p, p), (1, 1), bias=False, **kw)
    w = (rng.standard_normal((O, C, k, k)) * math.sqrt(2.0 / (C * k * k))).astype(np.float32)
    x = np.maximum(rng.standard_normal((B, C, H, H)), 0).astype(np.float32)
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
            mod.alpha_act.fill_(0.3)
            mod.alpha_weight.fill_(float(2 * np.abs(w).mean() / math.sqrt(2 ** (bits - 1) - 1)))
            mod.alpha_cim.fill_(0.05)  # every entry equal: scale = 0
            mod.init_state.fill_(1)
            mod.init_state_cim.fill_(1)
        mod.train()
    g = rng.standard_normal((B, O, H, H)).astype(np.float32)
    xt = torch.from_numpy(x).to(cuda_device).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g).to(cuda_device))
    torch.cuda.synchronize()
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))
    assert torch.isnan(oout).all(), "the oracle's forward is NaN throughout (lsq.py:566-573)"
    _same(out, oout, "out")
    _same(xt.grad, ox.grad, "grad_x")
    _same(m.weight.grad, om.weight.grad, "grad_w")
    _same(m.alpha_cim.grad, om.alpha_cim.grad, "grad_alpha_cim")
    _same(m.alpha_act.grad, om.alpha_act.grad, "grad_alpha_act")
    _same(m.alpha_weight.grad, om.alpha_weight.grad, "grad_alpha_weight")

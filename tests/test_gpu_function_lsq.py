"""GPU: the fused-LSQ Function path (functional.cim_conv2d_lsq: the raw activation, its LSQ quantiser inside the
library, lsq.py:547-549 followed by lsq.py:578) on the w3a3 stride-1 shapes whose backward runs the round-5
kernels (cim_bwd_gx5_kernel / cim_bwd_gw5_kernel: 16 -> 16 at 32 x 32, 32 -> 32 at 16 x 16).  This is the
path Conv2dLSQCiM takes on its first (initialising) training step and with ``fused = False``; its prologue
(prep_all) must build every operand those kernels read.  Against the oracle on the same quantised operands:
out within 1e-6 and grad_x / grad_w / grad_alpha within 1e-5 of max(|ref|, sum of |terms|) elementwise."""
import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import cim_oracle as co

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C,H", [(16, 32), (32, 16)])
def test_function_lsq_vs_oracle_gx5_gw5_shapes(cuda_device, C, H):
    from cim_quantization_amd import functional as F
    rng = np.random.default_rng(C * 7 + H)
    B, O, bits, xbar = 8, C, 3, 128
    qp_a = 2 ** bits - 1
    qn_w, qp_w = co.lsq_weight_params(bits)
    x = np.maximum(rng.standard_normal((B, C, H, H)), 0).astype(np.float32)
    sa = np.array([0.2], np.float32)
    sw = np.array([0.05], np.float32)
    w_q = (rng.integers(qn_w, qp_w + 1, size=(O, C, 3, 3)).astype(np.float32) * sw).astype(np.float32)
    T = -(-9 * C // xbar)
    a = (rng.random((1, T, bits, bits, 1, O)) * 4 + 0.2).astype(np.float32) * np.float32(sw[0] * sa[0])
    alpha_q = co.alpha_quantize(a, 8)
    bm = co.make_binary_mask(bits, bits, 1, 1)
    g = rng.standard_normal((B, H * H, O)).astype(np.float32)

    x_q, _ = co.lsq_quantize(x, sa, 0, qp_a)
    out_ref, c = co.cim_forward(x_q, w_q, (1, 1), (1, 1), (1, 1), bits, 1, bits, 1, 1.5, xbar, bm, alpha_q, sw, sa,
                                False, np.zeros(1, np.float32), return_debug=True)
    gxq, gw_ref, ga_ref = co.cim_backward(c, g)
    axq, aw, aa = co.cim_backward(c, g, absolute=True)
    y = (x / sa).astype(np.float32)
    inside = (y >= 0) & (y <= qp_a)
    gx_ref = np.where(inside, ((gxq * sa).astype(np.float32) / sa).astype(np.float32), 0)  # lsq.py:549 STE

    dv = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(cuda_device)  # noqa: E731
    xt = dv(x).requires_grad_(True)
    wt = dv(w_q).requires_grad_(True)
    at = dv(alpha_q).requires_grad_(True)
    out = F.cim_conv2d_lsq(xt, wt, dv(sa), dv(sw), at, dv(bm), dv(np.zeros(1, np.float32)), (1, 1), (1, 1), (1, 1),
                           bits, 1, bits, 1, 1.5, xbar)
    out.backward(dv(g))
    torch.cuda.synchronize()
    np_ = lambda t: t.detach().cpu().numpy()  # noqa: E731
    out_terms = np.sum(np.abs(c.adc.astype(np.float64) * bm), axis=(1, 2, 3))
    assert rel_err(np_(out), out_ref, out_terms) < 1e-6, "out"
    assert np.isfinite(np_(xt.grad)).all() and np.isfinite(np_(wt.grad)).all(), "non-finite gradients"
    assert rel_err(np_(xt.grad), gx_ref, axq.reshape(gx_ref.shape)) < 1e-5, "grad_x"
    assert rel_err(np_(wt.grad), gw_ref, aw) < 1e-5, "grad_w"
    assert rel_err(np_(at.grad), ga_ref, aa) < 1e-5, "grad_alpha"

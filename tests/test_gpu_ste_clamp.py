"""Port of test/test_backward_cim.py:57-84: the straight-through gradient of a clamped per-tile
partial sum.

The reference script builds per-tile partial sums ``out_temp[i] = layer_in[:, tile i] @ weight[tile i]``
of random integer operands (activations in [0, 2^3 - 2], weights in [-4, 2]), clamps each to a band,
sums the tiles, back-propagates ones, and checks ``layer_in.grad`` against ``(g * in_band) @ weight^T``
built by hand.  Here the same computation runs through the library Function
(``get_cim_output_signed`` with one slice pair, ``wbitslice = nbits_w`` and ``abitslice = nbits_a``,
and a multi-level ADC whose band is [Qn, Qp] = [-2^(b-1), 2^(b-1) - 1], lsq.py:125-131 and :310-313)
on unit step sizes, and every quantity is rebuilt independently in numpy from the integer operands:

* the per-tile partial sums (``debug_partial_sums``) equal ``x[:, tile] @ w[:, tile]^T`` exactly;
* ``out`` equals the sum over the tiles of ``clip(ps, Qn, Qp)`` exactly;
* ``grad_x`` and ``grad_w`` equal ``(g * in_band) @ W`` and ``x^T @ (g * in_band)`` summed over the
  tiles: exactly for g = ones (integer sums, as the reference prints ``1.``), within 1e-6 of the
  sum of |terms| for a random g.

The library's band keeps the gradient at its edges (``ps >= Qp + 1e-5`` / ``ps <= Qn - 1e-5`` are
the clamped ones, lsq.py:310-311), where the script's hand-made mask (``ge(clamp_x)``,
``le(-clamp_x)``) drops it; the test follows the library.
"""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu

BITS = 3


def _run(dev, x, w, g, xbar, adc):
    from cim_quantization_amd import functional as F
    B, C = x.shape[:2]
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    wt = torch.from_numpy(w).to(dev).requires_grad_(True)
    one = torch.ones(1, device=dev)
    bm = torch.ones((1, 1, 1, 1, 1, 1), dtype=torch.float32, device=dev)
    zero = torch.zeros(1, device=dev)
    args = (xt, wt, (1, 1), (0, 0), (1, 1), BITS, BITS, BITS, BITS, adc, xbar, bm, None, one, one, False, zero)
    out = F.get_cim_output_signed.apply(*args)
    out.backward(torch.from_numpy(g).to(dev))
    _, ps, _ = F.debug_partial_sums(xt.detach(), wt.detach(), (1, 1), (0, 0), BITS, BITS, BITS, BITS, adc, xbar, bm,
                                    None, one, one, zero)
    torch.cuda.synchronize()
    return out.detach().cpu().numpy(), xt.grad.cpu().numpy(), wt.grad.cpu().numpy(), ps.cpu().numpy()


@pytest.mark.parametrize("gkind", ["ones", "randn"])
@pytest.mark.parametrize("xbar,adc,zfrac", [(64, 8, 0.4), (128, 8, 0.6)])
def test_clamped_tile_sum_ste(cuda_device, gkind, xbar, adc, zfrac):
    rng = np.random.default_rng(84 + xbar + adc)
    B, C, O = 512, 256, 128
    x = rng.integers(0, 2 ** BITS - 1, (B, C)).astype(np.float32)  # torch.randint(0, 2^3 - 1)
    x[rng.random(x.shape) < zfrac] = 0                              # about 60 % / 30 % of the tile sums in band
    w = rng.integers(-(2 ** (BITS - 1)), 2 ** (BITS - 1) - 1, (O, C)).astype(np.float32)
    g = np.ones((B, O), np.float32) if gkind == "ones" else rng.standard_normal((B, O)).astype(np.float32)
    qn, qp = -(2 ** (adc - 1)), 2 ** (adc - 1) - 1
    out, gx, gw, ps = _run(cuda_device, x.reshape(B, C, 1, 1), w.reshape(O, C, 1, 1), g.reshape(B, 1, O), xbar,
                           adc)
    T = C // xbar
    x64, w64, g64 = x.astype(np.float64), w.astype(np.float64), g.astype(np.float64)
    exp_out = np.zeros((B, O))
    exp_gx = np.zeros((B, C))
    exp_gw = np.zeros((O, C))
    abs_gx = np.zeros((B, C))
    abs_gw = np.zeros((O, C))
    band = []
    for i in range(T):
        sl = slice(i * xbar, (i + 1) * xbar)
        p = x64[:, sl] @ w64[:, sl].T                                          # out_temp[i]
        assert np.array_equal(ps[:, i, 0, 0, 0, :], p), "per-tile partial sums"
        exp_out += np.clip(p, qn, qp)                                          # clamp, then sum over tiles
        inb = (p >= qn) & (p <= qp)
        band.append(inb.mean())
        gm = np.where(inb, g64, 0.0)                                           # grad_temp with the clamp mask
        exp_gx[:, sl] = gm @ w64[:, sl]
        exp_gw[:, sl] = gm.T @ x64[:, sl]
        abs_gx[:, sl] = np.abs(gm) @ np.abs(w64[:, sl])
        abs_gw[:, sl] = np.abs(gm).T @ np.abs(x64[:, sl])
    assert 0.05 < np.mean(band) < 0.95, f"band fraction {np.mean(band):.3f}: the test needs both clamped and passed sums"
    assert np.array_equal(out.reshape(B, O).astype(np.float64), exp_out), "out = sum of clamped tile sums"
    gx, gw = gx.reshape(B, C).astype(np.float64), gw.reshape(O, C).astype(np.float64)
    if gkind == "ones":
        assert np.array_equal(gx, exp_gx), "grad_x (layer_in.grad)"
        assert np.array_equal(gw, exp_gw), "grad_w"
    else:
        assert rel_err(gx, exp_gx, abs_gx) < 1e-6, "grad_x (layer_in.grad)"
        assert rel_err(gw, exp_gw, abs_gw) < 1e-6, "grad_w"

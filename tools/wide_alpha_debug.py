"""A dense Conv2dLSQCiM whose alpha_cim is wider than the one-block epilogue (T*nbw*nba*O > 8192)
against the module oracle: prints the worst elementwise errors of every gradient.
    python tools/wide_alpha_debug.py            (CIMQ_LIB_PATH=<variant .so> to try a build)"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import cim_module_oracle as cmo  # noqa: E402


def main():
    import cim_quantization_amd._modules as my_nn
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(3)
    B, C, O, bits, xbar = 128, 384, 256, 4, 128
    kw = dict(nbits_w=bits, nbits_a=bits, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=xbar, adcbits=1.5,
              stochastic_quant=False)
    m = my_nn.Conv2dLSQCiM(C, O, 1, 1, 0, bias=False, **kw).to(dev)
    om = cmo.OracleConv2dLSQCiM(C, O, (1, 1), (1, 1), (0, 0), (1, 1), bias=False, **kw)
    w = (rng.standard_normal((O, C, 1, 1)) * math.sqrt(2.0 / C)).astype(np.float32)
    x = np.maximum(rng.standard_normal((B, C, 1, 1)), 0).astype(np.float32)
    g = (rng.standard_normal((B, O, 1, 1)) / math.sqrt(B * O)).astype(np.float32)
    aa = np.float32(2 * 0.4 / math.sqrt(15))
    aw = np.float32(2 * np.abs(w).mean() / math.sqrt(7))
    shp = tuple(m.alpha_cim.shape)
    ac = ((rng.random(shp) * 2 + 0.5) * aa * aw * 4).astype(np.float32)
    for mod in (m, om):
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(w))
            mod.alpha_act.fill_(float(aa))
            mod.alpha_weight.fill_(float(aw))
            mod.alpha_cim.copy_(torch.from_numpy(ac))
            mod.init_state.fill_(1)
            mod.init_state_cim.fill_(1)
        mod.train()
    print("nalpha", m.alpha_cim.numel(), flush=True)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    out = m(xt)
    out.backward(torch.from_numpy(g).to(dev))
    torch.cuda.synchronize()
    ox = torch.from_numpy(x).requires_grad_(True)
    oout = om(ox)
    oout.backward(torch.from_numpy(g))
    for name, a, b in (("out", out, oout), ("grad_x", xt.grad, ox.grad), ("grad_w", m.weight.grad, om.weight.grad),
                       ("grad_alpha_cim", m.alpha_cim.grad, om.alpha_cim.grad),
                       ("grad_alpha_act", m.alpha_act.grad, om.alpha_act.grad),
                       ("grad_alpha_w", m.alpha_weight.grad, om.alpha_weight.grad)):
        a = a.detach().cpu().numpy().astype(np.float64).ravel()
        b = b.detach().numpy().astype(np.float64).ravel()
        d = np.abs(a - b)
        k = int(d.argmax())
        print(f"{name:15s} max|d| {d.max():.3e} at {k} mine {a[k]:.6e} ref {b[k]:.6e} max|ref| {np.abs(b).max():.3e}",
              flush=True)


if __name__ == "__main__":
    main()

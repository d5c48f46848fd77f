"""The ctx format word: where cim_fwd5_kernel stores one activation code byte per ctx element for
cim_bwd_gw5_kernel (ctx_codes, the 16 / 32-channel w3a3 stride-1 module layers), it also writes kCodesMagic at
the code table's entry 300 (csrc/cimq_kernels_v3.hip), and gw5 checks it.  A ctx whose format word is not the
magic -- a forward and backward planned differently -- must give NaN parameter gradients, not gradients read
from words taken as codes."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MAGIC = np.array([0xC0DE5EED], dtype=np.uint32).view(np.int32)[0]


def _layer(dev):
    import cim_quantization_amd._modules as my_nn
    torch.manual_seed(3)
    m = my_nn.Conv2dLSQCiM(16, 16, 3, 1, 1, bias=False, nbits_w=3, nbits_a=3, nbits_alpha=8, wbitslice=1, abitslice=1,
                           xbar=128, adcbits=1.5).to(dev)
    with torch.no_grad():
        m.alpha_act.fill_(0.4)
        m.alpha_weight.fill_(2 * float(m.weight.abs().mean()) / math.sqrt(3))
        m.alpha_cim.copy_(torch.rand(m.alpha_cim.shape, generator=torch.Generator().manual_seed(5)) + 0.5)
        m.alpha_cim.mul_(0.2)
        m.init_state.fill_(1)
        m.init_state_cim.fill_(1)
        m.signed_act.fill_(0)
    m._state_cache = None
    return m.train()


@pytest.mark.parametrize("corrupt", [False, True])
def test_gw5_refuses_a_ctx_of_the_other_format(cuda_device, corrupt):
    m = _layer(cuda_device)
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.randn(8, 16, 32, 32, generator=g).relu().to(cuda_device)
    gy = (torch.randn(8, 16, 32, 32, generator=g) / 512.0).to(cuda_device)
    out = m(x)
    cbuf = out.grad_fn.bufs[7]  # the module ctx (functional._CimModuleConv.forward)
    words = cbuf[: cbuf.numel() // 4 * 4].view(torch.int32)
    hits = (words == int(MAGIC)).nonzero().flatten()
    assert hits.numel() == 1, hits  # exactly one format word, written by the forward
    if corrupt:
        words[hits[0]] = 0
    out.backward(gy)
    torch.cuda.synchronize()
    gw = m.weight.grad
    if corrupt:
        # (weights outside the LSQ clamp range pass no gradient: 0 there, NaN everywhere else)
        assert torch.isnan(gw).float().mean() > 0.5, "grad_w from a ctx of the wrong format must be NaN"
        assert torch.isnan(m.alpha_cim.grad).any()
    else:
        assert torch.isfinite(gw).all() and gw.abs().max() > 0

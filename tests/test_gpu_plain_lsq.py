"""GPU: the plain LSQ modules (ActLSQ -> Conv2dLSQ, LinearLSQ; lsq.py:389-436, :591-662) on
libcimq -- the quantiser kernels and Conv2dLSQ's int8-MFMA conv -- against the golden vectors
from the reference modules and against the numpy oracle at larger shapes."""
import numpy as np
import pytest
import torch

from conftest import load_golden, normwise_err, plain_manifest
from oracle import lsq_plain_oracle as po

pytestmark = pytest.mark.gpu


def _conv_modules(cfg, z, dev):
    from cim_quantization_amd._modules.lsq import ActLSQ, Conv2dLSQ
    act = ActLSQ(nbits_a=cfg["na"]).to(dev)
    conv = Conv2dLSQ(z["in_x"].shape[1], z["in_weight"].shape[0], cfg["k"], stride=cfg["s"], padding=cfg["p"],
                     bias=cfg["bias"], nbits_w=cfg["nw"]).to(dev)
    with torch.no_grad():
        act.alpha.copy_(torch.from_numpy(z["in_alpha_a"]))
        act.signed.copy_(torch.from_numpy(z["in_signed"]))
        act.init_state.fill_(1)
        conv.weight.copy_(torch.from_numpy(z["in_weight"]))
        conv.alpha.copy_(torch.from_numpy(z["in_alpha_w"]))
        conv.init_state.fill_(1)
        if cfg["bias"]:
            conv.bias.copy_(torch.from_numpy(z["in_bias"]))
    return act.train(), conv.train()


@pytest.mark.parametrize("name", sorted(k for k, v in plain_manifest().items() if v["kind"] == "conv"))
def test_act_conv_vs_reference(cuda_device, name):
    cfg = plain_manifest()[name]["cfg"]
    z = load_golden(name)
    act, conv = _conv_modules(cfg, z, cuda_device)
    x = torch.from_numpy(z["in_x"]).to(cuda_device).requires_grad_(True)
    x_q, a = act(x)
    assert getattr(x_q, "_cimq_code_range", None) is not None
    y = conv((x_q, a))
    assert "QConv2d" in type(y.grad_fn).__name__  # the int8-MFMA conv ran, not torch's conv
    y.backward(torch.from_numpy(z["in_grad"]).to(cuda_device))
    np.testing.assert_array_equal(y.detach().cpu().numpy(), z["ref_y"])  # exact integer conv, same fp32 scaling
    assert normwise_err(x.grad.cpu().numpy(), z["ref_grad_x"]) < 1e-5
    assert normwise_err(conv.weight.grad.cpu().numpy(), z["ref_grad_weight"]) < 1e-5
    assert abs(act.alpha.grad.item() - float(z["ref_grad_alpha_a"][0])) <= 1e-5 * float(z["ref_abs_alpha_a"])
    assert abs(conv.alpha.grad.item() - float(z["ref_grad_alpha_w"][0])) <= 1e-5 * float(z["ref_abs_alpha_w"])
    if cfg["bias"]:
        assert normwise_err(conv.bias.grad.cpu().numpy(), z["ref_grad_bias"]) < 1e-5


@pytest.mark.parametrize("name", sorted(k for k, v in plain_manifest().items() if v["kind"] == "linear"))
def test_linear_vs_reference(cuda_device, name):
    from cim_quantization_amd._modules.lsq import LinearLSQ
    cfg = plain_manifest()[name]["cfg"]
    z = load_golden(name)
    lin = LinearLSQ(cfg["IN"], cfg["OUT"], bias=cfg["bias"], nbits_w=cfg["nw"]).to(cuda_device)
    with torch.no_grad():
        lin.weight.copy_(torch.from_numpy(z["in_weight"]))
        lin.alpha.copy_(torch.from_numpy(z["in_alpha_w"]))
        lin.init_state.fill_(1)
        if cfg["bias"]:
            lin.bias.copy_(torch.from_numpy(z["in_bias"]))
    x = torch.from_numpy(z["in_x"]).to(cuda_device).requires_grad_(True)
    y = lin.train()(x)
    y.backward(torch.from_numpy(z["in_grad"]).to(cuda_device))
    assert normwise_err(y.detach().cpu().numpy(), z["ref_y"]) < 1e-6
    assert normwise_err(x.grad.cpu().numpy(), z["ref_grad_x"]) < 1e-5
    assert normwise_err(lin.weight.grad.cpu().numpy(), z["ref_grad_weight"]) < 1e-5
    assert abs(lin.alpha.grad.item() - float(z["ref_grad_alpha_w"][0])) <= 1e-5 * float(z["ref_abs_alpha_w"])


@pytest.mark.parametrize("B,C,O,H,k,s,na,nw,signed", [
    (32, 64, 64, 16, 3, 1, 4, 4, False),   # a ResNet-56 stage-3 shape, 4-bit
    (16, 16, 32, 32, 3, 2, 8, 3, False),   # unsigned 8-bit codes: the two-MFMA split
    (16, 3, 16, 32, 3, 1, 8, 8, True),     # signed first layer
    (64, 128, 96, 8, 1, 1, 3, 4, False),   # 1x1
])
def test_act_conv_vs_oracle_larger(cuda_device, B, C, O, H, k, s, na, nw, signed):
    from cim_quantization_amd._modules.lsq import ActLSQ, Conv2dLSQ
    g = torch.Generator().manual_seed(B * 1000 + C)
    x = torch.randn(B, C, H, H, generator=g)
    if not signed:
        x = x.clamp_min(0)
    w = torch.randn(O, C, k, k, generator=g) * 0.1
    gout = None
    act = ActLSQ(nbits_a=na).to(cuda_device).train()
    conv = Conv2dLSQ(C, O, k, stride=s, padding=k // 2, bias=False, nbits_w=nw).to(cuda_device).train()
    with torch.no_grad():
        conv.weight.copy_(w)
    xd = x.to(cuda_device).requires_grad_(True)
    y = conv(act(xd))  # first step: the alphas initialise from the data (lsq.py:404-408, :641-650)
    gout = torch.randn(y.shape, generator=g)
    y.backward(gout.to(cuda_device))
    o = po.act_conv_chain(x.numpy(), act.alpha.item(), na, bool(act.signed.item()), w.numpy(), conv.alpha.item(), nw,
                          None, (s, s), (k // 2, k // 2), gout.numpy())
    np.testing.assert_array_equal(y.detach().cpu().numpy(), o["y"])
    assert normwise_err(xd.grad.cpu().numpy(), o["grad_x"]) < 1e-5
    assert normwise_err(conv.weight.grad.cpu().numpy(), o["grad_weight"]) < 1e-5
    assert abs(act.alpha.grad.item() - o["grad_alpha_a"]) <= 1e-5 * o["abs_alpha_a"]
    assert abs(conv.alpha.grad.item() - o["grad_alpha_w"]) <= 1e-5 * o["abs_alpha_w"]


def test_quantiser_ties_and_clamp(cuda_device):
    """round half to even at exact .5 codes, both clamp ends, NaN propagation, a ragged length"""
    from cim_quantization_amd.functional import lsq_quantize
    s = 0.25
    codes = np.arange(-9, 9, dtype=np.float32) + 0.5
    x = np.concatenate([codes * s, np.array([np.nan, 1e9, -1e9, 0.0, 0.1], np.float32)]).astype(np.float32)
    st = torch.tensor([s], device=cuda_device)
    for scaled in (False, True):
        out = lsq_quantize(torch.from_numpy(x).to(cuda_device), st, -4, 3, scaled=scaled).cpu().numpy()
        np.testing.assert_array_equal(out, po.lsq_forward(x, s, -4, 3, scaled=scaled))


def test_plain_modules_with_flat_params(cuda_device):
    """Parameters inside dist.FlatSGD's flat buffer sit at arbitrary 4-byte offsets (a 432-element
    conv weight plus a 1-element alpha put the next weight at byte 1732), and so does a batch
    slice of a flat activation buffer: the quantiser takes them element-wise, same results."""
    import copy

    from cim_quantization_amd._modules.lsq import ActLSQ, Conv2dLSQ, LinearLSQ
    from cim_quantization_amd.dist import FlatSGD, GradBucket
    dev = cuda_device
    torch.manual_seed(3)
    mods = [ActLSQ(nbits_a=4), Conv2dLSQ(3, 16, 3, padding=1, bias=False, nbits_w=4), LinearLSQ(576, 10, nbits_w=4)]
    refs = copy.deepcopy(mods)
    mods = [m.to(dev).train() for m in mods]
    refs = [m.to(dev).train() for m in refs]
    bucket = GradBucket([p for m in mods for p in m.parameters()])
    opt = FlatSGD(bucket, lr=0.05, momentum=0.9)
    assert mods[2].weight.data_ptr() % 16 != 0  # the case the 16-byte-only quantiser refused
    buf = torch.randn(1 + 4 * 3 * 6 * 6, device=dev).relu()
    x = buf[1:].view(4, 3, 6, 6)  # misaligned activation
    xr = x.clone()
    g = torch.randn(4, 10, device=dev)
    for step in range(2):
        bucket.zero()
        for m in refs:
            for p in m.parameters():
                p.grad = None
        y = mods[2](mods[1](mods[0](x)).flatten(1))
        yr = refs[2](refs[1](refs[0](xr)).flatten(1))
        assert torch.equal(y, yr)
        y.backward(g)
        yr.backward(g)
        bucket.exchange()
        for m, r in zip(mods, refs):
            for (n, p), pr in zip(m.named_parameters(), r.parameters()):
                assert torch.equal(p.grad, pr.grad), n
        opt.step()
        with torch.no_grad():  # the same SGD step on the reference copies
            for m, r in zip(mods, refs):
                for p, pr in zip(m.parameters(), r.parameters()):
                    pr.copy_(p)

"""GPU: the chained module backward (cimq_module_backward_chain): each layer's parameter-gradient
epilogue is held in the pending list and the flush launches them all, packed two launches per up
to 20 layers.  The gradients must match the unchained backward: grad_x bit for bit (same
kernels), the parameter gradients to fp32 summation order (the packed launch sums each slab in
float4 rows of 256 outputs per block, a layer's own launch one output per lane, 64 per block)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (C, O, H, stride, bits): w8a8 first conv, w3a3 stride 1 / 2, a 16x16 layer, and a 12x12 one
# (non-power-of-two width: the general backward, so the chain flushes before it)
def _close(a, b):
    """elementwise within the reordering of fp32 sums: 1e-5 relative, plus 1e-6 of the largest"""
    tol = 1e-5 * b.abs() + 1e-6 * b.abs().max()
    assert ((a - b).abs() <= tol).all(), ((a - b).abs() - tol).max().item()


SPECS = [(3, 16, 32, 1, 8), (16, 16, 32, 1, 3), (16, 32, 32, 2, 3), (32, 32, 16, 1, 3), (32, 32, 12, 1, 3),
         (32, 64, 16, 2, 3), (64, 64, 8, 1, 3)]


def _stack(dev, seed=5, overlap=False):
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd.dist import GradBucket
    torch.manual_seed(seed)
    layers = []
    for c, o, h, s, nb in SPECS:
        m = my_nn.Conv2dLSQCiM(c, o, 3, s, 1, bias=False, nbits_w=nb, nbits_a=nb, nbits_alpha=8, xbar=128,
                               adcbits=1.5)
        torch.nn.init.kaiming_normal_(m.weight)
        layers.append(m.to(dev).train())
    bucket = GradBucket([p for m in layers for p in m.parameters()])
    bucket.own(layers, overlap=overlap)
    return layers, bucket


def _data(dev, B=8, seed=9):
    g = torch.Generator().manual_seed(seed)
    xs, gs = [], []
    for c, o, h, s, nb in SPECS:
        x = torch.randn(B, c, h, h, generator=g)
        xs.append((x if nb == 8 else x.relu()).to(dev))
        ho = (h + 2 - 3) // s + 1
        gs.append((torch.randn(B, o, ho, ho, generator=g) / (B * o * ho * ho) ** 0.5).to(dev))
    return xs, gs


def _step(layers, bucket, xs, gs, chained_scope):
    from cim_quantization_amd.functional import chained_epilogues
    grads_x = []
    bucket.zero()
    scope = chained_epilogues() if chained_scope else torch.enable_grad()
    with scope:
        for m, x, g in zip(layers, xs, gs):
            xr = x.detach().requires_grad_(True)
            m(xr).backward(g)
            grads_x.append(xr.grad)
    bucket.join()
    torch.cuda.synchronize()
    return grads_x, bucket.flat.detach().clone()


def test_chained_equals_unchained_per_layer_backwards(cuda_device):
    import cim_quantization_amd.functional as F
    la, ba = _stack(cuda_device)
    lb, bb = _stack(cuda_device)
    xs, gs = _data(cuda_device)
    for layers, bucket in ((la, ba), (lb, bb)):  # first step: the alpha initialisation (torch path)
        _step(layers, bucket, xs, gs, False)
    xs2, gs2 = _data(cuda_device, seed=10)
    F.CHAIN_EPILOGUES = False
    try:
        gx_ref, flat_ref = _step(lb, bb, xs2, gs2, False)
    finally:
        F.CHAIN_EPILOGUES = True
    gx_ch, flat_ch = _step(la, ba, xs2, gs2, True)
    for i, (a, b) in enumerate(zip(gx_ch, gx_ref)):
        assert torch.equal(a, b), i  # same kernels, fixed-order sums
    _close(flat_ch, flat_ref)
    assert torch.isfinite(flat_ch).all()


def _deep(dev, n, shared):
    """n chained applications of small 16x16 layers (one shared layer if ``shared``)"""
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd.dist import GradBucket
    torch.manual_seed(3)
    ms = []
    for i in range(1 if shared else n):
        m = my_nn.Conv2dLSQCiM(16, 16, 3, 1, 1, bias=False, nbits_w=3, nbits_a=3, nbits_alpha=8, xbar=128,
                               adcbits=1.5)
        torch.nn.init.kaiming_normal_(m.weight)
        ms.append(m.to(dev).train())
    bucket = GradBucket([p for m in ms for p in m.parameters()])
    bucket.own(ms)
    return [ms[0]] * n if shared else ms, bucket


@pytest.mark.parametrize("n,shared", [(35, False), (4, True)])
def test_chain_packs_and_capacity(cuda_device, n, shared):
    """35 layers: a list full at 32 issued by the 33rd call (tail packs of 20 and 12), then 3 at the flush;
    one layer run 4 times: each call issues the pending epilogue that writes the same gradients.
    grad_x bit for bit against the unchained backward, the parameter gradients to summation order."""
    import cim_quantization_amd.functional as F
    g = torch.Generator().manual_seed(4)
    xs = [torch.randn(2, 16, 8, 8, generator=g).relu().to(cuda_device) for _ in range(n)]
    gs = [(torch.randn(2, 16, 8, 8, generator=g) / 32.0).to(cuda_device) for _ in range(n)]
    runs = []
    for chained in (False, True):
        layers, bucket = _deep(cuda_device, n, shared)
        _step(layers, bucket, xs, gs, False)  # initialising step
        F.CHAIN_EPILOGUES = chained
        try:
            gx, flat = _step(layers, bucket, xs, gs, chained)
        finally:
            F.CHAIN_EPILOGUES = True
        runs.append((gx, flat))
    for a, b in zip(runs[0][0], runs[1][0]):
        assert torch.equal(a, b)
    _close(runs[1][1], runs[0][1])
    assert F._chain(torch.device(cuda_device)).keep == []


def test_chain_inside_one_backward_pass(cuda_device):
    """one backward() through a sequential stack: the end-of-backward callback flushes"""
    import cim_quantization_amd.functional as F
    la, ba = _stack(cuda_device)
    lb, bb = _stack(cuda_device)
    specs = [(16, 16, 32, 1, 3), (16, 16, 32, 1, 3), (16, 16, 32, 1, 3)]
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd.dist import GradBucket
    nets = []
    for seed in (1, 1):
        torch.manual_seed(seed)
        ms = [my_nn.Conv2dLSQCiM(c, o, 3, s, 1, bias=False, nbits_w=nb, nbits_a=nb, xbar=128, adcbits=1.5)
              .to(cuda_device).train() for c, o, h, s, nb in specs]
        bk = GradBucket([p for m in ms for p in m.parameters()])
        bk.own(ms)
        nets.append((torch.nn.Sequential(ms[0], torch.nn.ReLU(), ms[1], torch.nn.ReLU(), ms[2]), bk))
    x = torch.randn(8, 16, 32, 32, device=cuda_device).relu()
    for net, bk in nets:  # initialising step
        bk.zero()
        net(x).square().mean().backward()
    outs = []
    for i, (net, bk) in enumerate(nets):
        bk.zero()
        F.CHAIN_EPILOGUES = i == 0
        try:
            net(x).square().mean().backward()
        finally:
            F.CHAIN_EPILOGUES = True
        torch.cuda.synchronize()
        outs.append(bk.flat.detach().clone())
    _close(outs[0], outs[1])


def test_overlapped_param_half_equals_single_stream(cuda_device):
    """GradBucket.own(overlap=True): the grad_w kernel of the v7 layers (CIMQ_LSQ_DEFER_GW) and every
    layer's epilogue run on the bucket's second stream (cimq_module_backward_params).  Same kernels,
    same inputs as the unchained single-stream backward: every gradient bit for bit."""
    import cim_quantization_amd.functional as F
    la, ba = _stack(cuda_device, overlap=True)
    lb, bb = _stack(cuda_device)
    xs, gs = _data(cuda_device)
    for layers, bucket in ((la, ba), (lb, bb)):
        _step(layers, bucket, xs, gs, False)
    xs2, gs2 = _data(cuda_device, seed=10)
    F.CHAIN_EPILOGUES = False
    try:
        gx_ref, flat_ref = _step(lb, bb, xs2, gs2, False)
    finally:
        F.CHAIN_EPILOGUES = True
    gx_ov, flat_ov = _step(la, ba, xs2, gs2, True)
    for i, (a, b) in enumerate(zip(gx_ov, gx_ref)):
        assert torch.equal(a, b), i
    assert torch.equal(flat_ov, flat_ref)
    assert torch.isfinite(flat_ov).all()


def test_chain_with_wide_alpha_dense_layers(cuda_device):
    """Two QuantLinear-shaped layers (BASELINE cfg5's 1024 -> 1024 w4a4, xbar 128, the dense path) in
    one chain: alpha_cim has T * nbw * nba * O = 131072 elements, so their packed epilogues take the
    wide tail (one output per thread) and the multi-block finish (module_finish_wide_block per job)."""
    import cim_quantization_amd._modules as my_nn
    import cim_quantization_amd.functional as F
    from cim_quantization_amd.dist import GradBucket
    g = torch.Generator().manual_seed(8)
    xs = [torch.randn(256, 1024, 1, 1, generator=g).relu().to(cuda_device) for _ in range(2)]
    gs = [(torch.randn(256, 1024, 1, 1, generator=g) / 512.0).to(cuda_device) for _ in range(2)]
    runs = []
    for chained in (False, True):
        torch.manual_seed(4)
        ms = []
        for _ in range(2):
            m = my_nn.Conv2dLSQCiM(1024, 1024, 1, 1, 0, bias=False, nbits_w=4, nbits_a=4, nbits_alpha=8, xbar=128,
                                   adcbits=1.5)
            torch.nn.init.kaiming_normal_(m.weight)
            ms.append(m.to(cuda_device).train())
        bucket = GradBucket([p for m in ms for p in m.parameters()])
        bucket.own(ms)
        _step(ms, bucket, xs, gs, False)  # initialising step
        F.CHAIN_EPILOGUES = chained
        try:
            gx, flat = _step(ms, bucket, xs, gs, chained)
        finally:
            F.CHAIN_EPILOGUES = True
        assert ms[0].alpha_cim.numel() == 8 * 4 * 4 * 1024
        runs.append((gx, flat))
    for a, b in zip(runs[0][0], runs[1][0]):
        assert torch.equal(a, b)
    _close(runs[1][1], runs[0][1])
    assert torch.isfinite(runs[1][1]).all()

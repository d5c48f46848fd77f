"""GPU: the prepared weight side (cimq_module_prepare via functional.prepare_weights): one launch
computes the weight / alpha_cim quantisers' operands and ADC thresholds of many layers ahead of
their forwards, which then only quantise the activation.  Outputs and every gradient must equal the
unprepared path bit for bit (same kernels, same per-element op sequences), over several SGD steps;
a prepared state is used only by the forward it was made for (same parameters, same input shape)."""
import pytest
import torch

from test_gpu_chain import SPECS, _data

pytestmark = pytest.mark.gpu


def _stack(dev, seed=5):
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
    bucket.own(layers)
    opt = torch.optim.SGD([p for m in layers for p in m.parameters()], lr=0.05, momentum=0.9)
    return layers, bucket, opt


def _step(layers, bucket, opt, xs, gs, prepare):
    from cim_quantization_amd.functional import chained_epilogues, prepare_weights
    n = prepare_weights(layers) if prepare else 0
    outs, gxs = [], []
    bucket.zero()
    with chained_epilogues():
        for m, x, g in zip(layers, xs, gs):
            xr = x.detach().requires_grad_(True)
            y = m(xr)
            y.backward(g)
            outs.append(y.detach())
            gxs.append(xr.grad)
    torch.cuda.synchronize()
    flat = bucket.flat.detach().clone()
    opt.step()
    return n, outs, gxs, flat


def test_prepared_equals_unprepared_over_steps(cuda_device):
    la, ba, oa = _stack(cuda_device)
    lb, bb, ob = _stack(cuda_device)
    xs, gs = _data(cuda_device)
    for L, B, O in ((la, ba, oa), (lb, bb, ob)):
        _step(L, B, O, xs, gs, False)  # the initialising step (torch path): nothing to prepare
        _step(L, B, O, xs, gs, False)  # the first library step records the input shapes
    for it in range(3):
        xs2, gs2 = _data(cuda_device, seed=20 + it)
        n, out_p, gx_p, flat_p = _step(la, ba, oa, xs2, gs2, True)
        _, out_r, gx_r, flat_r = _step(lb, bb, ob, xs2, gs2, False)
        assert n == len(SPECS)
        for i in range(len(SPECS)):
            assert torch.equal(out_p[i], out_r[i]), (it, i)
            assert torch.equal(gx_p[i], gx_r[i]), (it, i)  # every backward is fixed-order
        err = (flat_p - flat_r).abs().max().item()
        assert err <= 1e-6 * flat_r.abs().max().item(), (it, err)
        for pa, pb in zip([p for m in la for p in m.parameters()], [p for m in lb for p in m.parameters()]):
            assert (pa - pb).abs().max().item() <= 1e-6 * max(pb.abs().max().item(), 1e-30)


def test_stale_prepared_state_is_not_used(cuda_device):
    """A prepared state made before a parameter change (or for another input shape) is ignored:
    the forward recomputes the weight side itself."""
    from cim_quantization_amd.functional import prepare_weights
    la, ba, oa = _stack(cuda_device)
    xs, gs = _data(cuda_device)
    _step(la, ba, oa, xs, gs, False)
    _step(la, ba, oa, xs, gs, False)  # records the input shapes
    m, x = la[1], xs[1]
    with torch.no_grad():
        ref = m(x).clone()
        assert prepare_weights([m]) == 1
        m.weight.mul_(0.5)  # after prepare: the state is stale
        out = m(x)
        m.weight.mul_(2.0)
        ref2 = m(x)
        assert torch.equal(ref, ref2)
        assert not torch.equal(out, ref)  # computed from the halved weight, not the prepared one
        assert prepare_weights([m]) == 1
        out_small = m(x[:4])  # another batch size: not the prepared shape
        assert torch.equal(out_small, m(x[:4]))
        assert m._wprep is None  # taken (and discarded) by the first forward

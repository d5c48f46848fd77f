"""CPU: dist.FlatSGD (the bench's optimizer on the flat parameter / gradient buffers) takes the
same steps as torch.optim.SGD with momentum and per-group weight decay (examples/__init__.py:
184-188), and bumps the parameters' version counters as an in-place update does."""
import torch

from cim_quantization_amd.dist import FlatSGD, GradBucket


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(16, 3, 3, 3), (1,), (1,), (2, 3, 1, 16), (8, 16, 3, 3), (1,), (1,)]
    return [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in shapes]


def test_flat_sgd_matches_torch_sgd():
    pa, pb = _params(0), _params(0)
    decay = [i not in (1, 2, 3, 5, 6) for i in range(len(pa))]  # "alpha_*" entries without decay
    ref = torch.optim.SGD([{"params": [p for p, d in zip(pb, decay) if d], "weight_decay": 1e-4},
                           {"params": [p for p, d in zip(pb, decay) if not d], "weight_decay": 0.0}],
                          lr=0.01, momentum=0.9)
    bucket = GradBucket(pa)
    opt = FlatSGD(bucket, lr=0.01, momentum=0.9, weight_decay=[1e-4 if d else 0.0 for d in decay])
    gen = torch.Generator().manual_seed(3)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=gen) for p in pa]
        bucket.zero()
        for p, g in zip(pa, grads):
            p.grad.copy_(g)
        for p, g in zip(pb, grads):
            p.grad = g.clone()
        v0 = [p._version for p in pa]
        opt.step()
        ref.step()
        for a, b in zip(pa, pb):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), step
        assert all(p._version > v for p, v in zip(pa, v0))
    # the parameters are views of the optimizer's flat buffer
    assert pa[0].data_ptr() == opt.flat.data_ptr()

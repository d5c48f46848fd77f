"""GPU: dist.FlatSGD's one-launch update (cimq_flat_sgd) takes torch.optim.SGD's steps (momentum,
per-group weight decay; examples/__init__.py:184-188) on an odd element count (the n % 4 tail),
and zeroes the bucket's gradients in the same launch when asked."""
import pytest
import torch

from cim_quantization_amd.dist import FlatSGD, GradBucket

pytestmark = pytest.mark.gpu


def test_flat_sgd_gpu_matches_torch_sgd(cuda_device):
    g0 = torch.Generator().manual_seed(0)
    shapes = [(16, 3, 3, 3), (1,), (1,), (2, 3, 1, 16), (8, 16, 3, 3), (1,), (3,)]  # 1686 elements
    init = [torch.randn(*s, generator=g0) for s in shapes]
    pa = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    pb = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    decay = [i not in (1, 2, 3, 5, 6) for i in range(len(pa))]
    ref = torch.optim.SGD([{"params": [p for p, d in zip(pb, decay) if d], "weight_decay": 1e-4},
                           {"params": [p for p, d in zip(pb, decay) if not d], "weight_decay": 0.0}],
                          lr=0.01, momentum=0.9)
    bucket = GradBucket(pa)
    opt = FlatSGD(bucket, lr=0.01, momentum=0.9, weight_decay=[1e-4 if d else 0.0 for d in decay])
    assert opt.flat.numel() % 4 != 0
    gen = torch.Generator().manual_seed(3)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=gen).to(cuda_device) for p in pa]
        bucket.zero()
        for p, g in zip(pa, grads):
            p.grad.copy_(g)
        for p, g in zip(pb, grads):
            p.grad = g.clone()
        v0 = [p._version for p in pa]
        opt.step(zero_grad=step % 2 == 1)
        ref.step()
        torch.cuda.synchronize()
        for a, b in zip(pa, pb):
            # torch's kernels may contract a multiply-add; cimq_flat_sgd rounds each operation
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), step
        assert all(p._version > v for p, v in zip(pa, v0))
        if step % 2 == 1:
            assert torch.count_nonzero(bucket.flat) == 0
        else:
            assert torch.equal(bucket.flat, torch.cat([g.reshape(-1) for g in grads]))

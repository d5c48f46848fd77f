"""Data-parallel gradient exchange for the CiM layers.

Samples are independent through the CiM conv, so the path shards by batch: one process per
GPU, and one all-reduce per step of every gradient.  The gradients of all parameters live
in ONE flat fp32 bucket (1.17 MB for ResNet-20): autograd accumulates straight into it
(each ``p.grad`` is a view), and the exchange is a single ``all_reduce`` + scale, which on
ROCm runs on RCCL over xGMI (backend ``"nccl"``).  Gradients keep the reference's
local-batch semantics (its DDP run averages per-GPU gradients the same way).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradBucket:
    """One flat gradient buffer over ``params``; ``exchange()`` averages it across ranks."""

    def __init__(self, params, device=None):
        self.params = [p for p in params]
        n = sum(p.numel() for p in self.params)
        dev = device if device is not None else self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.nbytes = n * 4

    def own(self, modules):
        """Let the CiM layers among ``modules`` add their parameter gradients into this bucket
        inside libcimq (no per-parameter AccumulateGrad kernels).  Only for parameters whose
        gradients the bucket exchanges itself: parameter hooks do not see those gradients."""
        mine = {id(p) for p in self.params}
        for m in modules:
            if hasattr(m, "accumulate_grads_in_place"):
                if all(id(p) in mine for p in m.parameters()):
                    m.accumulate_grads_in_place = True
        return self

    def exchange(self, group=None):
        """Average the bucket over the ranks of ``group`` (no-op for a single process)."""
        if dist.is_available() and dist.is_initialized():
            world = dist.get_world_size(group)
            if world > 1:
                dist.all_reduce(self.flat, group=group)
                self.flat.mul_(1.0 / world)

    def zero(self):
        self.flat.zero_()

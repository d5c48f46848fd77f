"""Data-parallel training state for the CiM layers.

Samples are independent through the CiM conv, so the path shards by batch: one process per
GPU, one all-reduce per step of every gradient.  The gradients of all parameters live in ONE
flat fp32 bucket (1.17 MB for ResNet-20): autograd accumulates straight into it (each
``p.grad`` is a view), and the exchange is a single ``all_reduce`` + scale, which on ROCm
runs on RCCL over xGMI (backend ``"nccl"``).  Gradients keep the reference's local-batch
semantics (its DDP run averages per-GPU gradients the same way: ``ga``, the grad_scale
factors and ``ps.numel()`` of lsq.py:323,547,553 see the local batch).

What the reference's DDP wrapper does besides the all-reduce (examples/__init__.py:693-731),
and how this module covers it:

* construction-time broadcast of rank 0's parameters and buffers -> ``broadcast_from(0)``;
* the first training step initialises ``alpha_act`` / ``alpha_weight`` / ``alpha_cim`` and
  ``signed_act`` from each rank's OWN batch (lsq.py:532-563), after DDP's broadcast, so the
  reference's ranks keep different step sizes for the whole run.  Decision (DESIGN.md section
  5): call ``broadcast_from(0)`` again right after that first step's backward, before the
  optimizer step -- every rank then continues from rank 0's initialised step sizes and the
  replicas stay identical.  The first step's own gradients are the local ones, as in the
  reference.
* DDP's per-forward buffer broadcast only re-sends ``init_state`` / ``signed_act`` /
  ``init_state_cim``, which the post-init broadcast already made identical.

Callers zero the bucket with ``zero()``.  ``optimizer.zero_grad()`` (set_to_none=True since
torch 2.0) detaches ``p.grad`` from the bucket; ``exchange()`` detects that (by data pointer)
and copies such gradients back into their slot before reducing, so a misused bucket costs a
copy but never silently exchanges stale values.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


def _world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


class GradBucket:
    """One flat gradient buffer over ``params``; ``exchange()`` averages it across ranks."""

    def __init__(self, params, device=None):
        self.params = [p for p in params]
        n = sum(p.numel() for p in self.params)
        dev = device if device is not None else self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.nbytes = n * 4
        self.reattached = 0  # gradients found detached from the bucket (diagnostic)
        self.side = None  # stream of the overlapped parameter-gradient epilogues (own(overlap=True))
        self._works, self._sent = [], 0  # segments already in flight (exchange_segment)
        self._attach()

    def _attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def own(self, modules, overlap=False):
        """Let the CiM layers among ``modules`` add their parameter gradients into this bucket
        inside libcimq (no per-parameter AccumulateGrad kernels).  Only for parameters whose
        gradients the bucket exchanges itself: parameter hooks do not see those gradients.

        ``overlap``: the layers run their parameter-gradient half -- the grad_w kernel where it is
        one of its own (CIMQ_LSQ_DEFER_GW), then the epilogue (slab reductions, quantiser backward,
        step-size gradients) -- on the bucket's own stream, off the grad_x chain: the backward of
        the previous layer proceeds meanwhile.  ``join()`` (called by ``exchange()``) orders the
        current stream after it; read the gradients only after that."""
        mine = {id(p) for p in self.params}
        if overlap and self.side is None and self.flat.is_cuda:
            self.side = torch.cuda.Stream(self.flat.device)
        for m in modules:
            if hasattr(m, "accumulate_grads_in_place"):
                if all(id(p) in mine for p in m.parameters()):
                    m.accumulate_grads_in_place = True
                    if overlap:
                        m.tail_stream = self.side
        return self

    def join(self):
        """Order the current stream after the parameter-gradient work on the bucket's stream."""
        if self.side is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.side)

    def sync_views(self):
        """Make every ``p.grad`` the bucket view again, copying gradients that autograd put in
        fresh tensors (after ``zero_grad(set_to_none=True)`` or a reassigned ``.grad``)."""
        for p, v in zip(self.params, self.views):
            g = p.grad
            if g is not None and g.data_ptr() == v.data_ptr() and g.shape == v.shape:
                continue
            self.reattached += 1
            if g is None:
                v.zero_()
            else:
                v.copy_(g.detach().reshape(v.shape))
            p.grad = v

    def exchange_segment(self, hi, group=None):
        """Start summing ``flat[sent:hi]`` over the ranks of ``group`` without waiting for it: the
        gradients of the layers whose backward (and epilogue) has finished, while the backward of
        the next layers runs.  Segments go out in bucket order, each from where the last one ended;
        ``exchange()`` sends the rest, waits for all of them and averages.  On RCCL the collective
        runs on the process group's stream, ordered after the work already on the current stream,
        so the next segment's kernels overlap it.  Each element is reduced by one collective whatever
        the segmentation: with two ranks the sum is bit-identical to the single-bucket exchange
        (fp32 addition commutes); with more, the ring's order of additions can differ in the last
        bit.  No-op for a single process."""
        if _world(group) <= 1 or hi <= self._sent:
            return
        self.join()
        self.sync_views()
        self._works.append(dist.all_reduce(self.flat[self._sent:hi], group=group, async_op=True))
        self._sent = hi

    def exchange(self, group=None):
        """Average the bucket over the ranks of ``group`` (no-op for a single process): the part no
        ``exchange_segment`` sent, then the wait for every segment, then one scale."""
        self.join()
        self.sync_views()
        world = _world(group)
        if world > 1:
            if self._sent < self.flat.numel():
                dist.all_reduce(self.flat[self._sent:], group=group)
            for w in self._works:
                w.wait()
            self._works, self._sent = [], 0
            self.flat.mul_(1.0 / world)

    def zero(self):
        self.join()
        self.flat.zero_()
        self._attach()

    def broadcast_from(self, src=0, modules=(), group=None):
        """Copy rank ``src``'s parameters (and the buffers of ``modules``) to every rank: the
        DDP construction-time broadcast, and the post-initialisation re-sync of the
        data-dependent step sizes (module docstring).  One coalesced collective per dtype."""
        if _world(group) <= 1:
            return
        seen, tensors = set(), []
        for t in list(self.params) + [b for m in modules for b in m.buffers()]:
            if id(t) not in seen:
                seen.add(id(t))
                tensors.append(t)
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault((t.dtype, t.device), []).append(t)
        with torch.no_grad():
            for ts in by_dtype.values():
                flat = _flatten_dense_tensors([t.detach() for t in ts])
                dist.broadcast(flat, src, group=group)
                for t, v in zip(ts, _unflatten_dense_tensors(flat, ts)):
                    t.copy_(v)
        for m in modules:
            if hasattr(m, "_state_cache"):
                m._state_cache = None  # init flags may have changed with the buffers


class FlatSGD:
    """``torch.optim.SGD`` (momentum, per-parameter weight decay, no dampening / Nesterov) over
    the parameters of a GradBucket, on flat buffers.

    The parameters move into one flat fp32 tensor laid out like the bucket's gradients (each
    ``p.data`` becomes a view of it), so one step is one libcimq launch over every parameter on
    the GPU (``cimq_flat_sgd``; four torch elementwise ops on the CPU) instead of torch's
    per-tensor-list foreach kernels (seven launches, 57 us per ResNet-20 step).  Per element it is
    torch's SGD step:

        d = g + wd * p;   buf = d (first step) or momentum * buf + d;   p = p - lr * buf

    (the reference's optimizer, examples/__init__.py:184-188, with alpha_* out of weight decay).
    Each step bumps the parameters' autograd version counters, as torch's in-place update of
    the parameters would (functional.prepare_weights relies on them)."""

    def __init__(self, bucket, lr, momentum=0.9, weight_decay=None):
        """``weight_decay``: one float per parameter of ``bucket.params`` (0 for no decay)."""
        self.bucket, self.lr, self.momentum = bucket, float(lr), float(momentum)
        params = bucket.params
        wds = [0.0] * len(params) if weight_decay is None else [float(w) for w in weight_decay]
        if len(wds) != len(params):
            raise ValueError("one weight decay per parameter")
        self.flat = torch.empty_like(bucket.flat)
        self.wd = torch.empty_like(bucket.flat)
        off = 0
        with torch.no_grad():
            for p, w in zip(params, wds):
                k = p.numel()
                if p.dtype != torch.float32 or p.device != self.flat.device:
                    raise ValueError("FlatSGD takes fp32 parameters on the bucket's device")
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                self.wd[off:off + k].fill_(w)
                off += k
        self.params = params
        self.buf = torch.zeros_like(self.flat)
        self.started = False

    @torch.no_grad()
    def step(self, zero_grad=False):
        """One update from the bucket's gradients.  Every parameter takes part (a parameter that
        got no gradient this step updates from a zero gradient -- momentum and weight decay still
        apply -- where torch.optim.SGD would skip it; the CiM training step gives every parameter
        a gradient).  Gradients autograd left outside the bucket are copied in first.  On the GPU
        the update is one libcimq launch (cimq_flat_sgd; torch's elementwise ops took four);
        ``zero_grad`` also zeroes the bucket's gradients in it."""
        self.bucket.join()
        self.bucket.sync_views()
        if self.flat.is_cuda:
            from . import _lib
            _lib.check(_lib.load().cimq_flat_sgd(self.flat.numel(), self.flat.data_ptr(), self.bucket.flat.data_ptr(),
                                                 self.buf.data_ptr(), self.wd.data_ptr(), self.lr, self.momentum,
                                                 0 if self.started else 1, 1 if zero_grad else 0,
                                                 torch.cuda.current_stream(self.flat.device).cuda_stream),
                       "cimq_flat_sgd")
            self.started = True
        else:
            d = torch.addcmul(self.bucket.flat, self.wd, self.flat)  # g + wd * p
            if self.started:
                self.buf.mul_(self.momentum).add_(d)
            else:
                self.buf.copy_(d)
                self.started = True
            self.flat.add_(self.buf, alpha=-self.lr)
            if zero_grad:
                self.bucket.flat.zero_()
        torch.autograd.graph.increment_version(self.params)

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
        self.bounds = [0]  # parameter boundaries in the bucket: segments start and end on them
        for p in self.params:
            self.bounds.append(self.bounds[-1] + p.numel())
        self.reattached = 0  # gradients found detached from the bucket (diagnostic)
        self.side = None  # stream of the overlapped parameter-gradient epilogues (own(overlap=True))
        self._works, self._ranges, self._sent = [], [], 0  # segments in flight; end of the forward run
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

    def _in(self, i, ranges):
        lo, hi = self.bounds[i], self.bounds[i + 1]
        return any(a <= lo and hi <= b for a, b in ranges)

    def sync_views(self, lo=0, hi=None):
        """Make every ``p.grad`` whose slot lies in ``flat[lo:hi]`` the bucket view again, copying
        gradients that autograd put in fresh tensors (after ``zero_grad(set_to_none=True)`` or a
        reassigned ``.grad``).  Never touches a slot whose segment is still being reduced."""
        hi = self.flat.numel() if hi is None else hi
        for i, (p, v) in enumerate(zip(self.params, self.views)):
            if not (lo <= self.bounds[i] and self.bounds[i + 1] <= hi) or self._in(i, self._ranges):
                continue
            g = p.grad
            if g is not None and g.data_ptr() == v.data_ptr() and g.shape == v.shape:
                continue
            self.reattached += 1
            if g is None:
                v.zero_()
            else:
                v.copy_(g.detach().reshape(v.shape))
            p.grad = v

    def span(self, params):
        """``(lo, hi)``: the bucket range holding the gradients of ``params`` (contiguous in the
        bucket, e.g. one layer's parameters), for ``exchange_range``."""
        ids = {id(p) for p in params}
        idx = [i for i, p in enumerate(self.params) if id(p) in ids]
        if not idx or idx != list(range(idx[0], idx[-1] + 1)):
            raise ValueError("span: the parameters are not one contiguous run of the bucket")
        return self.bounds[idx[0]], self.bounds[idx[-1] + 1]

    def exchange_range(self, lo, hi, group=None):
        """Start summing ``flat[lo:hi]`` over the ranks of ``group`` without waiting for it: the
        gradients of layers whose backward (and epilogue) has FINISHED, while the backward of the
        other layers runs.  Ranges may go out in any order -- bucket order (``exchange_segment``),
        or reverse order as a network's backward finishes its last layers first -- but must start
        and end on parameter boundaries and must not overlap a range already in flight (ValueError).
        The caller guarantees completion: every gradient in the range is written (on the current
        stream, or on the bucket's side stream, which is joined first) and nothing writes it again
        before ``exchange()``; the bucket itself never touches a range in flight.  ``exchange()``
        sends what no range covered, waits for every range and averages.  On RCCL the collective
        runs on the process group's stream, ordered after the work already on the current stream,
        so later kernels overlap it.  Each element is reduced by one collective whatever the
        segmentation: with two ranks the sum is bit-identical to the single-bucket exchange (fp32
        addition commutes); with more, the ring's order of additions can differ in the last bit.
        No-op for a single process."""
        if _world(group) <= 1 or hi <= lo:
            return
        if lo not in self.bounds or hi not in self.bounds:
            raise ValueError(f"exchange_range({lo}, {hi}): not on parameter boundaries")
        if any(lo < b and a < hi for a, b in self._ranges):
            raise ValueError(f"exchange_range({lo}, {hi}) overlaps a range already in flight")
        self.join()
        self.sync_views(lo, hi)
        self._works.append(dist.all_reduce(self.flat[lo:hi], group=group, async_op=True))
        self._ranges.append((lo, hi))

    def exchange_segment(self, hi, group=None):
        """``exchange_range`` from where the last bucket-order segment ended (0 first) to ``hi``:
        for backward passes that finish layers in parameter order (bench.Trainer runs each layer's
        fwd+bwd in turn).  A segment already sent is a no-op."""
        if _world(group) <= 1 or hi <= self._sent:
            return
        self.exchange_range(self._sent, hi, group)
        self._sent = hi

    def _wait_pending(self):
        for w in self._works:
            w.wait()
        had = bool(self._works)
        self._works, self._ranges, self._sent = [], [], 0
        return had

    def exchange(self, group=None):
        """Average the bucket over the ranks of ``group`` (no-op for a single process): the parts no
        ``exchange_range`` sent, then the wait for every range, then one scale.  A gradient found
        detached from a slot that already went out raises: the range sent a stale value."""
        self.join()
        for i, (p, v) in enumerate(zip(self.params, self.views)):
            if self._in(i, self._ranges) and p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                self._wait_pending()
                raise RuntimeError("exchange: a gradient was detached from a bucket range already sent")
        self.sync_views()  # the slots outside the ranges in flight
        world = _world(group)
        if world > 1:
            lo = 0
            for a, b in sorted(self._ranges) + [(self.flat.numel(), self.flat.numel())]:
                if a > lo:
                    dist.all_reduce(self.flat[lo:a], group=group)
                lo = max(lo, b)
            self._wait_pending()
            self.flat.mul_(1.0 / world)

    def zero(self):
        self.join()
        self._wait_pending()  # a reduction still in flight would write after the zeroing
        self.flat.zero_()
        self._attach()

    def broadcast_from(self, src=0, modules=(), group=None):
        """Copy rank ``src``'s parameters (and the buffers of ``modules``) to every rank: the
        DDP construction-time broadcast, and the post-initialisation re-sync of the
        data-dependent step sizes (module docstring).  One coalesced collective per dtype."""
        if _world(group) <= 1:
            return
        self._wait_pending()
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
        if self.bucket._wait_pending():
            raise RuntimeError("FlatSGD.step: exchange segments in flight; call bucket.exchange() first")
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

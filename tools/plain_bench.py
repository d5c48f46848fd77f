#!/usr/bin/env python
"""Time the plain LSQ chain ActLSQ -> Conv2dLSQ (lsq.py:389-436, :620-662), forward + backward,
on libcimq (quantiser kernels + int8-MFMA conv) against the same graph written with torch ops
(the reference's formulas on the GPU: F.conv2d in fp32), for a few ResNet shapes.

    python tools/plain_bench.py          (GPU)
"""
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cim_quantization_amd._modules._quan_base import grad_scale, round_pass  # noqa: E402
from cim_quantization_amd._modules.lsq import ActLSQ, Conv2dLSQ  # noqa: E402


def torch_chain(x, act, conv):
    qp = 2 ** act.nbits - 1
    a = grad_scale(act.alpha, 1.0 / math.sqrt(x.numel() * qp))
    x_q = round_pass((x / a).clamp(0, qp))
    qn_w, qp_w = -(2 ** (conv.nbits - 1)), 2 ** (conv.nbits - 1) - 1
    ws = grad_scale(conv.alpha, 1.0 / math.sqrt(conv.weight.numel() * qp_w))
    w_q = round_pass((conv.weight / ws).clamp(qn_w, qp_w))
    return F.conv2d(x_q, w_q, None, conv.stride, conv.padding) * a * ws


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda:0")
    for (B, C, O, H, s, na, nw) in [(256, 16, 16, 32, 1, 4, 4), (256, 32, 32, 16, 1, 4, 4), (256, 64, 64, 8, 1, 4, 4),
                                    (256, 16, 32, 32, 2, 8, 8)]:
        torch.manual_seed(0)
        x = torch.randn(B, C, H, H, device=dev).clamp_min(0)
        act = ActLSQ(nbits_a=na).to(dev).train()
        conv = Conv2dLSQ(C, O, 3, stride=s, padding=1, bias=False, nbits_w=nw).to(dev).train()
        g = torch.randn_like(conv(act(x)))  # also the first-step alpha init

        def ours():
            xr = x.detach().requires_grad_(True)
            conv(act(xr)).backward(g)

        def ref():
            xr = x.detach().requires_grad_(True)
            torch_chain(xr, act, conv).backward(g)

        t_ours, t_ref = timed(ours), timed(ref)
        print(f"B{B} {C}->{O} {H}x{H} s{s} a{na}w{nw}: libcimq {t_ours:.3f} ms  torch ops {t_ref:.3f} ms "
              f"({t_ref / t_ours:.2f}x)", flush=True)


if __name__ == "__main__":
    main()

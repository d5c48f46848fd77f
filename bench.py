#!/usr/bin/env python
"""Benchmark: ResNet-20 w3a3 CiM conv layers, batch 256 per GPU, on MI355X.

One step = forward + backward of all 19 CiM convolutions of a CIFAR ResNet-20
(BASELINE.json configs[1]; the first conv is w8a8 as ReplaceModuleTool forces it,
replace_module.py:83-95), xbar 128, 1.5-bit ADC, followed by the data-parallel gradient
exchange (one flat RCCL all-reduce bucket, N > 1) and an SGD update of the weights and
step sizes.  Inputs / grads are synthetic tensors of the layer shapes (no dataset);
weights are kaiming-normal (resnet.py:43-45).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line (metric / value / roofline / cpu_baseline ...).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# (name, in_channels, out_channels, input H=W, stride, bits)
RESNET20 = [("conv1", 3, 16, 32, 1, 8)]
RESNET20 += [(f"layer1.{b}.conv{c}", 16, 16, 32, 1, 3) for b in range(3) for c in (1, 2)]
RESNET20 += [("layer2.0.conv1", 16, 32, 32, 2, 3), ("layer2.0.conv2", 32, 32, 16, 1, 3)]
RESNET20 += [(f"layer2.{b}.conv{c}", 32, 32, 16, 1, 3) for b in (1, 2) for c in (1, 2)]
RESNET20 += [("layer3.0.conv1", 32, 64, 16, 2, 3), ("layer3.0.conv2", 64, 64, 8, 1, 3)]
RESNET20 += [(f"layer3.{b}.conv{c}", 64, 64, 8, 1, 3) for b in (1, 2) for c in (1, 2)]
XBAR, ADC = 128, 1.5
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md); the backward runs bf16 x3
PEAK_I8_TOPS = 5000.0      # dense int8 MFMA: the forward's bit-sliced partial sums
PEAK_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9  # 256 CUs x 4 SIMD-32 x 2.4 GHz (a wave64 VALU op issues over 2 cycles)
# grad_w + the parameter-gradient epilogue on a second stream (CIMQ_BENCH_OVERLAP=0: one stream,
# the epilogues of all layers packed into a few launches at the end of the backward)
OVERLAP = os.environ.get("CIMQ_BENCH_OVERLAP", "0") == "1"
# CIMQ_BENCH_RECOMPUTE=1: the layers run with Conv2dLSQCiM.recompute_psum (CIMQ_OPT_RECOMPUTE)
RECOMPUTE = os.environ.get("CIMQ_BENCH_RECOMPUTE", "0") == "1"
TRAFFIC_JSON = os.environ.get("CIMQ_TRAFFIC_JSON", os.path.join(REPO, "profiles", "r06_final", "pmc_traffic.json"))
# the kernel families the roofline is reported for (libcimq profiler ids) and their rocprof symbol
# prefixes (the keys of pmc_traffic.json); every launch of a family is timed, all its instantiations
FAMILIES = {"fwd_v7": ("cimq::cim_fwd_v3_kernel<", "cimq::cim_fwd5_kernel"),
            "bwd_fused": ("cimq::cim_bwd_fused_kernel<", "cimq::cim_bwd_gxw5_kernel"),
            "gx_v8": ("cimq::cim_bwd_gx_v8_kernel<", "cimq::cim_bwd_gx5_kernel"), "gw_v7": ("cimq::cim_bwd_gw_v7_kernel<", "cimq::cim_bwd_gw5_kernel")}


def out_hw(h, s):
    return (h + 2 - 3) // s + 1


def macs_per_sample():
    return sum(out_hw(h, s) ** 2 * o * c * 9 for _, c, o, h, s, _ in RESNET20)


def build(device, batch, seed=0, data_seed=None):
    """The 19 layers (weights from ``seed``: identical on every rank) and one synthetic batch
    of activations / output grads per layer (from ``data_seed``: each rank its own shard)."""
    import cim_quantization_amd._modules as my_nn
    torch.manual_seed(seed)
    layers, xs, gs = [], [], []
    gen = torch.Generator().manual_seed(seed + 1 if data_seed is None else data_seed)
    for name, c, o, h, s, nb in RESNET20:
        m = my_nn.Conv2dLSQCiM(c, o, 3, s, 1, bias=False, nbits_w=nb, nbits_a=nb, nbits_alpha=8, wbitslice=1,
                               abitslice=1, xbar=XBAR, adcbits=ADC, signed_xbar=True, stochastic_quant=False)
        torch.nn.init.kaiming_normal_(m.weight)
        m.recompute_psum = RECOMPUTE
        layers.append(m.to(device).train())
        x = torch.randn(batch, c, h, h, generator=gen)
        if name != "conv1":
            x = x.relu()  # every later conv sees a post-ReLU (BN+ReLU) activation
        ho = out_hw(h, s)
        gy = torch.randn(batch, o, ho, ho, generator=gen) / math.sqrt(batch * o * ho * ho)
        xs.append(x.to(device))
        gs.append(gy.to(device))
    return layers, xs, gs


class Trainer:
    """fwd+bwd over the CiM layers, flat-bucket gradient all-reduce, SGD (examples/__init__.py:184-188:
    alpha_* excluded from weight decay)."""

    def __init__(self, layers, world, segments=None):
        from cim_quantization_amd.dist import GradBucket
        self.layers, self.world = layers, world
        # the step in segments of consecutive layers (world > 1: three): at the end of a segment its
        # layers' parameter-gradient epilogues are flushed and their slice of the bucket goes out
        # (GradBucket.exchange_segment) while the next segment computes; one segment at world 1
        nseg = (3 if world > 1 else 1) if segments is None else segments
        nseg = max(1, min(nseg, len(layers)))
        cut = [round(i * len(layers) / nseg) for i in range(nseg + 1)]
        self.segments = [(cut[i], cut[i + 1]) for i in range(nseg)]
        offs = [0]
        for m in layers:
            offs.append(offs[-1] + sum(p.numel() for p in m.parameters()))
        self.seg_hi = [offs[b] for _, b in self.segments]  # bucket end of each segment's gradients
        self.bucket = GradBucket([p for m in layers for p in m.parameters()])  # one all-reduce per step
        # the layers add their grads straight into the bucket; with OVERLAP their parameter-gradient
        # half (grad_w + epilogue) runs on the bucket's second stream (GradBucket.own(overlap=True))
        self.bucket.own(layers, overlap=OVERLAP)
        # DDP's construction-time broadcast; the step sizes are re-sent once more after the
        # first (initialising) step -- cim_quantization_amd/dist.py, DESIGN.md section 5
        self.bucket.broadcast_from(0, layers)
        self.synced_init = False
        self.flat = self.bucket.flat
        # SGD with momentum, weight decay 1e-4 except alpha_* (examples/__init__.py:184-188), on the
        # flat parameter / gradient buffers (dist.FlatSGD: one cimq_flat_sgd launch that also zeroes
        # the gradients; torch's foreach SGD took 7 launches, 57 us per step, its fused SGD 77 us)
        from cim_quantization_amd.dist import FlatSGD
        wd = [0.0 if nm.startswith("alpha") else 1e-4 for m in layers for nm, _ in m.named_parameters()]
        self.opt = FlatSGD(self.bucket, lr=0.01, momentum=0.9, weight_decay=wd)
        self.bucket_mb = self.bucket.nbytes / 1e6

    def compute_segment(self, k, xs, gs):
        """fwd + bwd of segment ``k``'s layers; gradients accumulate into the flat bucket.  Each
        layer's parameter-gradient epilogue is held back (the chained module backward,
        functional.chained_epilogues) and the segment's run packed at the scope's end."""
        from cim_quantization_amd.functional import chained_epilogues, prepare_weights
        if k == 0:
            # the weight side of all 19 prologues in one launch, ahead of the forwards
            prepare_weights(self.layers)
        a, b = self.segments[k]
        with chained_epilogues():
            for m, x, gy in zip(self.layers[a:b], xs[a:b], gs[a:b]):
                m(x).backward(gy)
        self.bucket.join()  # the parameter-gradient epilogues are part of the step

    def compute(self, xs, gs, exchange=False):
        """Every segment; ``exchange``: send each finished segment's gradients on (world > 1)."""
        for k in range(len(self.segments)):
            self.compute_segment(k, xs, gs)
            if exchange:
                self.bucket.exchange_segment(self.seg_hi[k])

    def finish(self):
        """gradient exchange (one RCCL all-reduce of the bucket) + SGD update."""
        self.bucket.exchange()
        self.opt.step(zero_grad=True)  # the update and the gradients' zeroing in one launch

    def step(self, xs, gs):
        self.compute(xs, gs, exchange=self.synced_init)
        if not self.synced_init:
            self.bucket.broadcast_from(0, self.layers)  # rank 0's initialised alpha_* / signed_act
            self.synced_init = True
        self.finish()

    def forward_only(self, xs):
        with torch.no_grad():
            for m, x in zip(self.layers, xs):
                m(x)

    def capture(self, xs, gs):
        """Record fwd+bwd of all layers as HIP graphs, one per segment: a step is then one graph
        launch per segment (each followed by its gradients' exchange at world > 1) plus the
        update, instead of ~50 host-side kernel launches per layer."""
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.compute(xs, gs)  # allocator / autograd warm-up on the capture stream
            self.flat.zero_()
        torch.cuda.current_stream().wait_stream(side)
        self.graphs = []
        for k in range(len(self.segments)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.compute_segment(k, xs, gs)
            self.graphs.append(g)

    def step_graph(self, xs, gs):
        for k, g in enumerate(self.graphs):
            g.replay()
            self.bucket.exchange_segment(self.seg_hi[k])
        self.finish()

    def capture_forward(self, xs):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.forward_only(xs)
        torch.cuda.current_stream().wait_stream(side)
        self.fgraph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.fgraph):
            self.forward_only(xs)


def timed(trainer, xs, gs, steps, dev, world, graph):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        if graph:
            trainer.step_graph(xs, gs)
        else:
            trainer.step(xs, gs)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def timed_forward(trainer, xs, steps, dev, world, graph):
    """The metric's own quantized-MAC/s (logical MAC / forward time): the
    forward of the 19 convs only, bracketed like the step timing."""
    if graph:
        trainer.capture_forward(xs)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        if graph:
            trainer.fgraph.replay()
        else:
            trainer.forward_only(xs)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def live_pairs(nb):
    """slice pairs with a nonzero int8 binary_mask entry (2^(j+k) wraps to 0 at >= 2^8, _quan_base.py:207-214)."""
    return sum(1 for k in range(nb) for j in range(nb) if j + k <= 7)


def step_context(batch, world, ms_step, ms_fwd):
    """SURVEY 8(d) / BASELINE.md rates of the 19 layers: bit-sliced MAC/s of the forward (logical MAC x the
    live slice pairs, the products the crossbar model computes), algorithmic HBM GB/s of fwd+bwd (per layer
    12 B per input element + 8 B per output element: the forward reads x and writes y, the backward reads
    grad_y and x and writes grad_x -- 961.5 MB per step at B = 256) and the step's own roofs: HBM on those
    bytes, MFMA on the forward's int8 bit-slice products plus the backward's fp32-accurate contraction as
    three bf16 products."""
    bs_mac = 0.0
    byts = 0.0
    t_i8 = t_bf = 0.0
    for _, c, o, h, s, nb in RESNET20:
        ho = out_hw(h, s)
        mac = batch * ho * ho * o * c * 9
        bs_mac += mac * live_pairs(nb)
        nx, ny = batch * c * h * h, batch * o * ho * ho
        byts += 12.0 * nx + 8.0 * ny
        t_i8 += 2.0 * mac * live_pairs(nb) / (PEAK_I8_TOPS * 1e12)
        t_bf += 3.0 * 2.0 * mac * (nb + nb) / (PEAK_BF16_TFLOPS * 1e12)
    t_hbm = byts / (PEAK_HBM_GBS * 1e9)
    return {"bit_sliced_mac_per_s_fwd": bs_mac * world / (ms_fwd * 1e-3),
            "algorithmic_hbm_gb_per_s_fwd_bwd": byts * world / (ms_step * 1e-3) / 1e9,
            "algorithmic_bytes_per_step_per_gpu": byts,
            "step_roofline": {"t_hbm_us": t_hbm * 1e6, "t_mfma_us": (t_i8 + t_bf) * 1e6,
                              "t_mfma_fwd_i8_us": t_i8 * 1e6, "t_mfma_bwd_bf16x3_us": t_bf * 1e6,
                              "frac_hbm": t_hbm / (ms_step * 1e-3), "frac_mfma": (t_i8 + t_bf) / (ms_step * 1e-3)}}


def family_roofline(kt, family, steps):
    """Roofline of one kernel family from its per-launch HIP-event times (cimq_profile_read): each launch
    is bounded by t_roof = max(t_HBM, t_MFMA) of its own algorithmic bytes and MFMA operations (int8 at
    5 POP/s forward, bf16 at 2.5 PFLOP/s backward); frac = sum t_roof / sum t_measured over the family.
    achieved = frac x the peak of the roof that binds most of the family's t_roof."""
    peak_m = PEAK_I8_TOPS if family == "fwd_v7" else PEAK_BF16_TFLOPS
    pl = kt.per_launch
    tm = sum(ms for ms, _, _, _ in pl) * 1e-3
    roof_h = roof_m = 0.0
    classes = {}
    for ms, byts, _, mops in pl:
        th, tmf = byts / (PEAK_HBM_GBS * 1e9), mops / (peak_m * 1e12)
        if th >= tmf:
            roof_h += th
        else:
            roof_m += tmf
        c = classes.setdefault((round(byts), round(mops)), [0, 0.0, th, tmf])
        c[0] += 1
        c[1] += ms * 1e-3
    frac = (roof_h + roof_m) / tm
    bound = "hbm" if roof_h >= roof_m else "mfma"
    peak = PEAK_HBM_GBS if bound == "hbm" else peak_m
    unit = "GB/s" if bound == "hbm" else ("TOP/s" if family == "fwd_v7" else "TFLOP/s")
    inst = [{"launches": n, "algo_bytes": b, "mfma_ops": m, "t_hbm_us": th * 1e6, "t_mfma_us": tmf * 1e6,
             "avg_launch_us": t / n * 1e6, "frac": max(th, tmf) / (t / n)}
            for (b, m), (n, t, th, tmf) in sorted(classes.items(), key=lambda kv: -kv[1][1])]
    return {"bound": bound, "achieved": frac * peak, "peak": peak, "unit": unit, "frac": frac,
            "family_us_per_step": tm / steps * 1e6, "t_roof_us_per_step": (roof_h + roof_m) / steps * 1e6,
            "launches": len(pl), "instances": inst,
            "method": "frac = sum_i max(t_hbm_i, t_mfma_i) / sum_i t_i over every launch i of the family "
                      "(HIP events on the launch stream); achieved = frac x peak of the binding roof"}


def measured_peaks(dev):
    """Attainable peaks on this box, beside the spec peaks the roofline uses: a 4 GiB device copy
    (read + write bytes / time) and a 8192^3 bf16 torch.matmul (hipBLASLt)."""
    res = {}
    n = 1 << 30
    a = torch.empty(n, device=dev, dtype=torch.float32)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    res["hbm_copy_gb_per_s"] = 10 * 2 * 4.0 * n / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    m = 8192
    x = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
    y = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
    torch.matmul(x, y)
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(10):
        torch.matmul(x, y)
    e1.record()
    torch.cuda.synchronize(dev)
    res["bf16_matmul_tflop_per_s"] = 10 * 2.0 * m ** 3 / (e0.elapsed_time(e1) * 1e-3) / 1e12
    res["spec"] = {"hbm_gb_per_s": PEAK_HBM_GBS, "bf16_tflop_per_s": PEAK_BF16_TFLOPS, "i8_top_per_s": PEAK_I8_TOPS}
    return res


def source_sha():
    """sha256 of the kernel sources: ties a committed PMC traffic file to the kernels it measured."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(REPO, "cim_quantization_amd", "csrc", "*")))
    for f in files + [os.path.join(REPO, "include", "cimq.h")]:
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def measured_pmc(family):
    """Launch-weighted HBM bytes (2 FETCH_SIZE + WRITE_SIZE) and VALU instructions per launch of a kernel
    family from the committed PMC passes (tools/pmc_traffic.py), or None with the reason when those
    passes measured other kernel sources."""
    if not os.path.exists(TRAFFIC_JSON):
        return None, None, "no PMC file"
    tj = json.load(open(TRAFFIC_JSON))
    meta = tj.pop("_meta", {})
    src = os.path.relpath(TRAFFIC_JSON, REPO)
    if meta.get("source_sha") != source_sha():
        return None, None, f"{src} measured other kernel sources"
    hits = [v for k, v in tj.items() if k.startswith(FAMILIES[family])]
    if not hits:
        return None, None, "family absent from the PMC file"
    n = sum(v.get("dispatches", 1) for v in hits)
    traffic = sum(v["traffic_bytes"] * v.get("dispatches", 1) for v in hits) / n
    valu = None
    if all(v.get("valu_insts") is not None for v in hits):
        valu = sum(v["valu_insts"] * v.get("dispatches", 1) for v in hits) / n
    return traffic, valu, src


def layer_breakdown(trainer, xs, gs, dev):
    """Per-layer fwd+bwd ms from events on the compute stream (one untimed pass)."""
    res = []
    for m, x, gy, spec in zip(trainer.layers, xs, gs, RESNET20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        m(x).backward(gy)
        trainer.bucket.join()  # include the layer's parameter-gradient epilogue
        e1.record()
        res.append((spec[0], e0, e1))
    torch.cuda.synchronize(dev)
    trainer.flat.zero_()
    return {n: round(a.elapsed_time(b), 4) for n, a, b in res}


def cpu_baseline(batch_cpu: int, threads: int):
    """The op-faithful torch-CPU port of the reference's Function (oracle/cim_torch_port.py: the
    lsq.py:92-386 op sequence, bit-identical to the reference and 0.95-0.98x its time in the
    build container, tools/cpu_port_ratio.py) timed on this box's host cores: forward + backward
    of all 19 ResNet-20 CiM convs at ``batch_cpu`` (default: the full batch 256)."""
    import numpy as np

    from oracle import cim_oracle as co
    from oracle import cim_torch_port as tp
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    t = 0.0
    for name, c, o, h, s, nb in RESNET20:
        sa = torch.tensor([0.11])
        sw = torch.tensor([0.07])
        qn_w, qp_w = co.lsq_weight_params(nb)
        x_q = torch.from_numpy(rng.integers(0, 2 ** nb, (batch_cpu, c, h, h)).astype(np.float32)) * sa
        w_q = torch.from_numpy(rng.integers(qn_w, qp_w + 1, (o, c, 3, 3)).astype(np.float32)) * sw
        T = math.ceil(c * 9 / XBAR)
        a = torch.from_numpy(co.alpha_quantize(((rng.random((1, T, nb, nb, 1, o)) * 3 + 0.1) * 0.11 * 0.07)
                                               .astype(np.float32), 8))
        bm = torch.from_numpy(co.make_binary_mask(nb, nb, 1, 1))
        ho = out_hw(h, s)
        g = torch.from_numpy(rng.standard_normal((batch_cpu, ho * ho, o)).astype(np.float32))
        t0 = time.perf_counter()
        out, ctx = tp.cim_forward(x_q, w_q, (s, s), (1, 1), nb, 1, nb, 1, ADC, XBAR, bm, a, sw, sa,
                                  signed_act=(name == "conv1"))
        tp.cim_backward(ctx, g)
        t += time.perf_counter() - t0
    macs = macs_per_sample() * batch_cpu
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return dict(value=macs / t, unit="MAC/s", cores=threads, kind="port", seconds=t, cpu=cpu,
                sample=f"op-faithful torch-CPU port of get_cim_output_signed (oracle/cim_torch_port.py), fwd+bwd "
                       f"of the 19 ResNet-20 CiM convs at batch {batch_cpu}, {threads} threads, {t:.2f} s",
                reference_in_container={"resnet20_b256_fwd_bwd_s": 27.99, "threads": 8,
                                        "source": "SURVEY.md section 6 (whole model incl. BN/FC, 8 Xeon cores)",
                                        "port_over_reference_time": [0.952, 0.981],
                                        "ratio_source": "tools/cpu_port_ratio.py, layer1 / layer3 at B=256"})


def bench_cfg5(dev, steps, warmup):
    """BASELINE cfg5: QuantLinear 1024->1024 w4a4, 128-row tiles, batch 4096, as Conv2dLSQCiM(k=1)
     through the module path (the dense GEMM kernels, cimq_part_dense.hip): fwd+bwd
    ms per step, forward MAC/s, and the roofline of each of its three kernels (HIP events around
    every launch; bound = the larger of the HBM time of the algorithmic bytes and the MFMA time of
    the products as issued: int8 bit-slice products forward, three bf16 products per fp32-accurate
    backward MAC)."""
    import cim_quantization_amd._modules as my_nn
    from cim_quantization_amd import _lib
    torch.manual_seed(7)
    B, C, O, nb = 4096, 1024, 1024, 4
    m = my_nn.Conv2dLSQCiM(C, O, 1, 1, 0, bias=False, nbits_w=nb, nbits_a=nb, nbits_alpha=8, wbitslice=1,
                           abitslice=1, xbar=128, adcbits=1.5).to(dev).train()
    x = torch.randn(B, C, 1, 1, device=dev).relu()
    gy = torch.randn(B, O, 1, 1, device=dev) / 2048.0
    for _ in range(max(1, warmup)):
        m(x).backward(gy)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        m(x).backward(gy)
    torch.cuda.synchronize(dev)
    fb = (time.perf_counter() - t0) / steps
    with torch.no_grad():
        t0 = time.perf_counter()
        for _ in range(steps):
            m(x)
        torch.cuda.synchronize(dev)
    fw = (time.perf_counter() - t0) / steps
    macs = B * O * C
    roofs = {}
    for kname, ops_per_mac, peak, unit in (("fwd", 2.0 * nb * nb, PEAK_I8_TOPS, "TOP/s"),
                                           ("bwd_gx", 3.0 * 2 * nb, PEAK_BF16_TFLOPS, "TFLOP/s"),
                                           ("bwd_gw", 3.0 * 2 * nb, PEAK_BF16_TFLOPS, "TFLOP/s")):
        with _lib.KernelTimer(kname, max_launches=steps + 4) as kt:
            for _ in range(steps):
                m(x).backward(gy)
            torch.cuda.synchronize(dev)
        n = max(kt.launches, 1)
        avg = kt.total_ms / n * 1e-3
        byts = kt.algo_bytes / n
        t_hbm = byts / (PEAK_HBM_GBS * 1e9)
        ops = macs * ops_per_mac
        t_mfma = ops / (peak * 1e12)
        r = ({"bound": "hbm", "achieved": byts / avg / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s"} if t_hbm >= t_mfma
             else {"bound": "mfma", "achieved": ops / avg / 1e12, "peak": peak, "unit": unit})
        r.update(frac=r["achieved"] / r["peak"], avg_launch_us=avg * 1e6, t_hbm_us=t_hbm * 1e6, t_mfma_us=t_mfma * 1e6)
        roofs[kname] = r
    dom = max(roofs, key=lambda k: roofs[k]["avg_launch_us"])
    return {"workload": "quantlinear_1024x1024_w4a4_xbar128_b4096", "ms_fwd_bwd": fb * 1e3, "ms_fwd": fw * 1e3,
            "fwd_mac_per_s": macs / fw, "fwd_bwd_mac_per_s": macs / fb, "launch": "eager",
            "roofline": dict(roofs[dom], kernel=dom, traffic=None), "kernel_roofs": roofs,
            "reference_cpu_container_ms": {"fwd": 2420.0, "fwd_bwd": 45940.0}}


def resnet56_convs():
    """(name, in, out, H, stride, bits) of ResNet-56's 55 CiM convs (models/cifar10/resnet.py, 9 blocks
    per stage; the first conv forced to w8a8 by ReplaceModuleTool)."""
    convs = [("conv1", 3, 16, 32, 1, 8)]
    for st, (cin, cout, h) in enumerate(((16, 16, 32), (16, 32, 32), (32, 64, 16))):
        for b in range(9):
            s = 2 if (st > 0 and b == 0) else 1
            c_in = cin if b == 0 else cout
            h_in = h if b == 0 else (h // 2 if st > 0 else h)
            convs.append((f"layer{st + 1}.{b}.conv1", c_in, cout, h_in, s, 2))
            convs.append((f"layer{st + 1}.{b}.conv2", cout, cout, out_hw(h_in, s), 1, 2))
    return convs


def bench_layers(dev, specs, batch, xbar, adc, steps, warmup, adc_shift=False, ref=None):
    """fwd+bwd and fwd-only wall time of a stack of Conv2dLSQCiM layers (eager launches; the
    first-step alpha init runs in the warm-up), logical MAC/s as SURVEY 8(d) defines it."""
    import cim_quantization_amd._modules as my_nn
    torch.manual_seed(11)
    torch.cuda.synchronize(dev)
    mem0 = torch.cuda.memory_allocated(dev)  # what earlier configs still hold
    torch.cuda.reset_peak_memory_stats(dev)
    layers, xs, gs, macs = [], [], [], 0
    for name, c, o, h, s, nb in specs:
        m = my_nn.Conv2dLSQCiM(c, o, 3, s, 1, bias=False, nbits_w=nb, nbits_a=nb, nbits_alpha=8, wbitslice=1,
                               abitslice=1, xbar=xbar, adcbits=adc, adc_shift=adc_shift)
        torch.nn.init.kaiming_normal_(m.weight)
        layers.append(m.to(dev).train())
        x = torch.randn(batch, c, h, h, device=dev)
        xs.append(x if name == "conv1" else x.relu())
        ho = out_hw(h, s)
        gs.append(torch.randn(batch, o, ho, ho, device=dev) / math.sqrt(batch * o * ho * ho))
        macs += batch * ho * ho * o * c * 9

    def fb():
        for m, x, g in zip(layers, xs, gs):
            m(x).backward(g)

    for _ in range(max(1, warmup)):
        fb()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fb()
    torch.cuda.synchronize(dev)
    t_fb = (time.perf_counter() - t0) / steps
    peak_mb = (torch.cuda.max_memory_allocated(dev) - mem0) / 2 ** 20
    with torch.no_grad():
        t0 = time.perf_counter()
        for _ in range(steps):
            for m, x in zip(layers, xs):
                m(x)
        torch.cuda.synchronize(dev)
    t_f = (time.perf_counter() - t0) / steps
    out = {"ms_fwd_bwd": t_fb * 1e3, "ms_fwd": t_f * 1e3, "fwd_mac_per_s": macs / t_f, "launch": "eager",
           "layers": len(specs), "batch": batch,
           "peak_mem_mb": round(peak_mb, 1)}  # device memory this stack's inputs, parameters and fwd+bwd peaked at
    # the same fwd+bwd replayed as one HIP graph: device time without the host's per-launch cost
    # (eager timings of these many-small-launch stacks move with the box's host load)
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fb()
        torch.cuda.current_stream().wait_stream(side)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            fb()
        gr.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            gr.replay()
        torch.cuda.synchronize(dev)
        out["ms_fwd_bwd_graph"] = (time.perf_counter() - t0) / steps * 1e3
        del gr
    except Exception as e:  # noqa: BLE001 -- reported, the eager numbers stand
        out["graph_error"] = f"{type(e).__name__}: {e}"[:200]
    if ref is not None:
        out["reference_cpu_container_ms"] = ref
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--cpu-batch", type=int, default=256)
    ap.add_argument("--no-cfg5", action="store_true", help="skip the BASELINE cfg5 (QuantLinear) extra line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured HBM-copy / bf16-GEMM peaks")
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel from the host each step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # "nccl" is RCCL on ROCm (one GPU per rank); CIMQ_DIST_BACKEND=gloo runs the same branch with
        # several ranks on one GPU (tests/test_gpu_dist.py)
        dist.init_process_group(os.environ.get("CIMQ_DIST_BACKEND", "nccl"), rank=rank, world_size=world)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)

    from cim_quantization_amd import _lib
    _lib.load()  # fail loudly if the HIP library is missing

    torch.cuda.reset_peak_memory_stats(dev)
    layers, xs, gs = build(dev, args.batch, seed=1234, data_seed=1235 + 1000 * rank)
    tr = Trainer(layers, world)
    for _ in range(max(1, args.warmup)):  # the first step runs the LSQ / alpha_cim init (lsq.py:532-563)
        tr.step(xs, gs)
    torch.cuda.synchronize(dev)

    # per-role kernel ms of one untimed step (all variants), and the dominant kernel family
    per_kernel = {}
    for kname in ("fwd", "bwd_gx", "bwd_gw", "prep_act") + tuple(FAMILIES):
        with _lib.KernelTimer(kname) as kt:
            tr.step(xs, gs)
        per_kernel[kname] = kt.total_ms
    dominant = max(FAMILIES, key=per_kernel.get)

    graph = not args.no_graph
    if graph:
        tr.flat.zero_()
        tr.capture(xs, gs)
        elapsed = timed(tr, xs, gs, args.steps, dev, world, True)
        # HIP events recorded inside a graph cannot be timed on ROCm 7: the dominant family's
        # launches are timed over the same number of host-launched steps right after (same
        # inputs, same kernels; only the launch path differs)
        with _lib.KernelTimer(dominant, max_launches=len(RESNET20) * args.steps + 8) as kt:
            for _ in range(args.steps):
                tr.step(xs, gs)
            torch.cuda.synchronize(dev)
    else:
        with _lib.KernelTimer(dominant, max_launches=len(RESNET20) * args.steps + 8) as kt:
            elapsed = timed(tr, xs, gs, args.steps, dev, world, False)
    fwd_elapsed = timed_forward(tr, xs, args.steps, dev, world, graph)
    t = torch.tensor([elapsed, fwd_elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, fwd_elapsed = t.tolist()
    # device memory of the whole training step (inputs, parameters, bucket, ctx / workspaces, the graph's pool)
    peak_mb = torch.cuda.max_memory_allocated(dev) / 2 ** 20
    breakdown = layer_breakdown(tr, xs, gs, dev)

    ms_per_step = elapsed / args.steps * 1e3
    macs_step = macs_per_sample() * args.batch * world
    value = macs_step / (elapsed / args.steps)
    roof = family_roofline(kt, dominant, args.steps)
    nl = max(kt.launches, 1)
    traffic, valu, pmc_source = measured_pmc(dominant)
    roof["traffic"] = traffic
    # VALU issue roof: the family's VALU instructions (PMC SQ_INSTS_VALU per launch) at one wave64
    # instruction per 2 cycles per SIMD on every SIMD of the chip, against its measured time
    if valu is not None:
        t_valu = valu * 64.0 / PEAK_VALU_LANE_OPS
        roof["valu"] = {"insts_per_launch": valu, "t_valu_us": t_valu * 1e6,
                        "frac": t_valu / (kt.total_ms / nl * 1e-3), "peak_lane_ops_per_s": PEAK_VALU_LANE_OPS}
    else:
        roof["valu"] = None
    result = {
        "metric": "quantized-MAC/s + fwd+bwd ms per ResNet-20 w3a3 CiM layer, batch 256",
        "value": value,
        "unit": "MAC/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "ms_per_layer_fwd_bwd": ms_per_step / len(RESNET20),
        "value_semantics": "logical MAC (B*P*O*K, flops_counter.py:314-318) of the 19 convs per fwd+bwd+SGD "
                           "step / step time; the forward-only rate SURVEY 8(d) defines is fwd_only.value",
        "fwd_only": {"value": macs_step / (fwd_elapsed / args.steps), "unit": "MAC/s",
                     "ms_per_forward": fwd_elapsed / args.steps * 1e3},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "i8+f32",
        "data": "synthetic (random-init weights, randn / relu(randn) activations of the layer shapes)",
        "config": {"workload": "resnet20_w3a3_all_19_cim_convs_fwd_bwd_sgd", "global_batch": args.batch * world,
                   "per_gpu_batch": args.batch, "xbar": XBAR, "adc_bits": ADC, "first_layer": "w8a8",
                   "parallelism": f"dp{world}", "grad_bucket_mb": round(tr.bucket_mb, 3), "exchange_segments": len(tr.segments),
                   "launch": "hip_graph" if graph else "eager", "recompute_psum": RECOMPUTE},
        "roofline": dict(roof, kernel=_lib.KERNEL_SYMBOLS[_lib.KERNEL_IDS[dominant]] + " (every instantiation the "
                         "19 layers launch)", avg_launch_us=kt.total_ms / nl * 1e3, pmc_source=pmc_source),
        "peak_mem_mb": round(peak_mb, 1),
        "kernel_ms_per_step": {k: round(v, 4) for k, v in per_kernel.items()},
        "layer_fwd_bwd_ms": breakdown,
        "rates": step_context(args.batch, world, ms_per_step, fwd_elapsed / args.steps * 1e3),
    }
    if world == 1 and not args.no_peaks:
        result["peaks_measured"] = measured_peaks(dev)
    if world == 1 and not args.no_cfg5:
        ex = {"cfg5": bench_cfg5(dev, args.steps, args.warmup)}
        one = [("layer", 16, 16, 32, 1, 3)]
        # BASELINE.md's in-container reference times (8 Xeon cores) beside each extra config
        ex["cfg1_adc4"] = dict(workload="conv3x3_16x16_32x32_w3a3_xbar64_adc4_b4",
                               **bench_layers(dev, one, 4, 64, 4, args.steps, args.warmup,
                                              ref={"fwd": 5.2, "fwd_bwd": 15.8}))
        ex["cfg1_adc1.5"] = dict(workload="conv3x3_16x16_32x32_w3a3_xbar64_adc1.5_b4",
                                 **bench_layers(dev, one, 4, 64, 1.5, args.steps, args.warmup,
                                                ref={"fwd": 6.9, "fwd_bwd": 24.1}))
        r56 = resnet56_convs()
        ex["cfg4_alpha"] = dict(workload="resnet56_w2a2_xbar64_adc1.5_b256_55convs_alpha_only",
                                **bench_layers(dev, r56, 256, 64, 1.5, 3, 1, ref={"fwd": 16890.0, "fwd_bwd": 50010.0}))
        ex["cfg4_shift"] = dict(workload="resnet56_w2a2_xbar64_adc1.5_b256_55convs_alpha_beta_shift",
                                **bench_layers(dev, r56, 256, 64, 1.5, 2, 1, adc_shift=True))
        result["extra_configs"] = ex
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_batch, min(16, os.cpu_count() or 1))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

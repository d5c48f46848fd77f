"""The HIP path under two ranks (BASELINE cfg3's data parallelism, examples/__init__.py:693-731):
two processes share the one GPU, torch.distributed on gloo over device tensors.

* bench.Trainer's real step -- prepare_weights, the chained module epilogues, GradBucket.own,
  broadcast_from and FlatSGD -- on three ResNet-20 layer shapes (the w8a8 first conv, a 16-channel
  32x32 and a 64-channel 8x8 layer) at batch 64 per rank: each rank's local bucket matches the CPU
  module oracle run on the same state and data (every element within 1e-5 of max(|ref|, its sum of
  |terms|): grad_w from the oracle's absolute re-run, grad_alpha_cim through conftest.alpha_cim_terms;
  the two scalar step sizes within 1e-5 of their sum of |terms|), the exchanged bucket is the mean of
  the two ranks' buckets and of the two ranks' oracle gradients (elementwise, 1e-5 of the mean of the
  ranks' |terms|), and after
  three steps every parameter is bit-identical across the ranks;
* bench.py's own world > 1 branch, launched by torch.distributed.run with the gloo backend.

The ranks are child processes; this (parent) process never touches the GPU -- no HIP call, not even
torch.cuda.is_available() -- so that starting them is safe on the GPU box.  The file name sorts it
ahead of the other GPU tests, which do initialise the GPU in the pytest process.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu_present():
    if torch.cuda.device_count() == 0:  # counts devices without initialising the runtime
        pytest.skip("no ROCm device")

LAYERS = [("conv1", 3, 16, 32, 1, 8), ("layer1.0.conv1", 16, 16, 32, 1, 3), ("layer3.1.conv1", 64, 64, 8, 1, 3)]
BATCH = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _lsq_terms(v, g_q, s, qn, qp, gscale):
    """sum of |terms| of d loss / d alpha through the LSQ quantiser (lsq.py:547-555)."""
    import numpy as np
    v, g_q = v.astype(np.float64), g_q.astype(np.float64)
    y = v / float(s)
    r = np.rint(np.clip(y, qn, qp))
    inside = (y >= qn) & (y <= qp)
    return gscale * (np.abs(g_q * r).sum() + np.abs(np.where(inside, g_q * float(s), 0) * y / float(s)).sum())


def _oracle_grads(layers, xs, gs):
    """Local gradients of the CPU module oracle from each layer's current state, by parameter name, and
    the sums of |terms| of the two step-size gradients."""
    import math

    import numpy as np

    from conftest import alpha_cim_terms
    from oracle import cim_module_oracle as cmo
    from oracle import cim_oracle as co
    res = []
    for (name, c, o, h, s, nb), m, x, g in zip(LAYERS, layers, xs, gs):
        om = cmo.OracleConv2dLSQCiM(c, o, 3, s, 1, bias=False, nbits_w=nb, nbits_a=nb, nbits_alpha=8, wbitslice=1,
                                    abitslice=1, xbar=128, adcbits=1.5)
        om.debug_retain = True
        om.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=False)
        om.train()
        xc = x.detach().cpu()
        box = {}
        real = co.cim_forward

        def rec(*a, **k):
            k["return_debug"] = True
            out, c = real(*a, **k)
            box["c"] = c
            return out, c
        cmo.co.cim_forward = rec
        try:
            om(xc).backward(g.detach().cpu())
        finally:
            cmo.co.cim_forward = real
        gb = g.detach().cpu().numpy()
        g_bpo = np.ascontiguousarray(gb.reshape(gb.shape[0], o, -1).transpose(0, 2, 1))
        _, aw, aa = co.cim_backward(box["c"], g_bpo, absolute=True)
        d = om.dbg
        (qn_a, qp_a), (qn_w, qp_w) = d["qa"], d["qw"]
        w = om.weight.detach().numpy()
        terms = {"alpha_act": _lsq_terms(xc.numpy(), d["x_q"].grad.numpy(), d["sa"].item(), qn_a, qp_a,
                                         1.0 / math.sqrt(xc.numel() * qp_a)),
                 "alpha_weight": _lsq_terms(w, d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w,
                                            1.0 / math.sqrt(w.size * qp_w))}
        # elementwise sums of |terms| of the tensor gradients: grad_w (the STE passes d loss / d w_q), and
        # grad_alpha_cim through the alpha quantiser (conftest.alpha_cim_terms)
        terms["weight"] = torch.from_numpy(aw.reshape(w.shape))
        terms["alpha_cim"] = torch.from_numpy(alpha_cim_terms(om.alpha_cim.detach().numpy(), aa))
        res.append(({n: p.grad.detach().clone() for n, p in om.named_parameters()}, terms))
    return res


def _trainer_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, REPO)
        import bench
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        bench.RESNET20[:] = LAYERS
        layers, xs, gs = bench.build(dev, BATCH, seed=1234, data_seed=1235 + 1000 * rank)
        tr = bench.Trainer(layers, world)
        tr.step(xs, gs)  # first step: the data-dependent step sizes, then rank 0's re-broadcast
        torch.cuda.synchronize()
        # step 2 by hand: local bucket -> oracle; exchanged bucket -> mean of the ranks' oracles
        ref = _oracle_grads(layers, xs, gs)
        tr.compute(xs, gs)
        torch.cuda.synchronize()
        errs = []
        for m, (r, tt) in zip(layers, ref):
            for n, p in m.named_parameters():
                d = (p.grad.detach().cpu().double() - r[n].double()).abs()
                # elementwise 1e-5 of max(|ref|, sum of |terms|); the two scalar step sizes (sums over the
                # whole batch): 1e-5 of their terms
                if p.numel() == 1:
                    errs.append((n, d.max().item() / tt[n]))
                else:
                    scale = torch.maximum(r[n].double().abs(), tt[n].double().reshape(r[n].shape))
                    errs.append((n, (d / (scale + 1e-30)).max().item()))
        ref_flat = torch.cat([r[n].reshape(-1) for m, (r, _) in zip(layers, ref) for n, _ in m.named_parameters()])
        # per parameter of the flat bucket: the scalar's sum of |terms| (else 0), for the exchanged check
        t_flat = torch.cat([torch.full((p.numel(),), float(tt[n]), dtype=torch.float64) if p.numel() == 1
                            else tt[n].reshape(-1).double() for m, (_, tt) in zip(layers, ref)
                            for n, p in m.named_parameters()])
        t_all = [torch.zeros_like(t_flat) for _ in range(world)]
        dist.all_gather(t_all, t_flat)
        t_mean = sum(t_all) / world
        gathered = [torch.zeros_like(ref_flat) for _ in range(world)]
        dist.all_gather(gathered, ref_flat)
        mean_ref = sum(gathered) / world
        abs_ref = sum(t.abs() for t in gathered) / world  # the mean's terms
        local = tr.flat.detach().cpu().clone()
        locs = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(locs, local)
        tr.bucket.exchange()
        exch = tr.flat.detach().cpu()
        # the exchange itself: (sum of the ranks' buckets) / world, to fp32 rounding
        mean_loc = sum(locs) / world
        allreduce_err = (exch - mean_loc).abs().max().item() / (mean_loc.abs().max().item() + 1e-30)
        off, exch_err = 0, 0.0
        for m in layers:
            for _, p in m.named_parameters():
                k = p.numel()
                seg, rs, ra = exch[off:off + k].double(), mean_ref[off:off + k].double(), abs_ref[off:off + k]
                # elementwise: the mean of the ranks' |terms| (and of their |ref|)
                scale = torch.maximum(ra.double(), t_mean[off:off + k]) + 1e-30
                exch_err = max(exch_err, ((seg - rs).abs() / scale).max().item())
                off += k
        tr.opt.step()
        tr.flat.zero_()
        tr.step(xs, gs)  # step 3
        torch.cuda.synchronize()
        params = tr.opt.flat.detach().cpu()
        allp = [torch.zeros_like(params) for _ in range(world)]
        dist.all_gather(allp, params)
        out[rank] = dict(local_err=max(e for _, e in errs), worst=max(errs, key=lambda t: t[1])[0],
                         exch_err=exch_err, allreduce_err=allreduce_err, params_equal=all(torch.equal(allp[0], a) for a in allp[1:]),
                         finite=bool(torch.isfinite(params).all()))
    finally:
        dist.destroy_process_group()


def test_trainer_step_world2_gloo_on_device(gpu_present):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_trainer_worker, args=(2, port, out), nprocs=2, join=True)
    res = dict(out)
    for rank in (0, 1):
        r = res[rank]
        assert r["finite"]
        assert r["local_err"] < 1e-5, r
        assert r["exch_err"] < 1e-5, r
        assert r["allreduce_err"] < 1e-6, r
        assert r["params_equal"], r


def test_bench_world2_branch_gloo(gpu_present):
    """bench.py's world > 1 branch (barriers, max-over-ranks timing, the bucket all-reduce), two
    ranks on the one GPU with the gloo backend (RCCL needs a GPU per rank)."""
    env = dict(os.environ, CIMQ_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--batch", "16", "--no-cfg5", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    r = json.loads(line[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 32
    assert r["value"] > 0 and r["ms_per_step"] > 0

"""World-size-2 data-parallel exchange on gloo (CPU): the flat gradient bucket that bench.py
all-reduces over RCCL on MI355X (cim_quantization_amd/dist.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cim_quantization_amd.dist import GradBucket
        torch.manual_seed(0)  # same initial parameters on every rank
        w = torch.nn.Parameter(torch.randn(16, 3, 3, 3))
        a = torch.nn.Parameter(torch.tensor([0.5]))
        bucket = GradBucket([w, a])
        opt = torch.optim.SGD([w, a], lr=0.1, momentum=0.9)
        for step in range(3):
            g = torch.Generator().manual_seed(100 * step + rank)  # different data per rank
            x = torch.randn(8, 3, 3, 3, generator=g)
            loss = ((x * w.sum(0, keepdim=True)).sum() * a).square()
            loss.backward()
            local = bucket.flat.clone()
            bucket.exchange()
            gathered = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(gathered, local)
            assert torch.allclose(bucket.flat, torch.stack(gathered).mean(0), rtol=1e-6, atol=1e-7)
            opt.step()
            bucket.zero()
        params = torch.cat([w.detach().reshape(-1), a.detach().reshape(-1)])
        allp = [torch.zeros_like(params) for _ in range(world)]
        dist.all_gather(allp, params)
        out[rank] = float((allp[0] - allp[1]).abs().max())
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bucket_exchange_world2_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    # every rank applied the same averaged gradients: parameters stay identical
    assert out[0] == 0.0 and out[1] == 0.0

"""GPU parity of the exact composition bench.py times: the 19 ResNet-20 CiM
layers at batch 256 in ``bench.Trainer`` -- the weight side of all layers prepared in one launch
(``prepare_weights``), the chained parameter-gradient epilogues, gradients accumulated in place into
the flat ``GradBucket`` -- captured in three segment graphs (as at world > 1) and replayed.  The bucket's gradients of the w8a8
first conv, a 16-channel layer, the first stride-2 transition and a 64-channel layer are compared with
the module oracle (oracle/cim_module_oracle.py, lsq.py:511-588) run on the same inputs and parameters,
elementwise against the sum of |terms| like tests/test_gpu_fullsize.py.
"""
import numpy as np
import pytest
import torch

from conftest import alpha_cim_report, alpha_cim_terms, rel_err
from oracle import cim_module_oracle as cmo
from oracle import cim_oracle as co
from test_gpu_fullsize import _capture_oracle_ctx, _lsq_scalar_terms

pytestmark = pytest.mark.gpu

CHECKED = ("conv1", "layer1.0.conv1", "layer2.0.conv1", "layer3.1.conv1")


def test_bench_graph_composition_vs_oracle(cuda_device, monkeypatch):
    import math

    import bench
    names = [r[0] for r in bench.RESNET20]
    layers, xs, gs = bench.build(cuda_device, 256)
    # three segments, as bench.py runs at world > 1: three graphs, each ending in its own flush of the
    # packed epilogues (the exchange between them is a no-op in one process)
    tr = bench.Trainer(layers, 1, segments=3)
    tr.compute(xs, gs)  # the first (initialising) step, eager, as bench.py's warm-up
    tr.flat.zero_()
    tr.capture(xs, gs)
    tr.flat.zero_()
    for g in tr.graphs:
        g.replay()
    torch.cuda.synchronize()
    grads = {n: [p.grad.detach().cpu().numpy().copy() for p in m.parameters()] for n, m in zip(names, layers)}

    for name in CHECKED:
        li = names.index(name)
        _, C, O, H, s, bits = bench.RESNET20[li]
        m = layers[li]
        om = cmo.OracleConv2dLSQCiM(C, O, (3, 3), (s, s), (1, 1), (1, 1), bias=False, nbits_w=bits, nbits_a=bits,
                                    nbits_alpha=8, wbitslice=1, abitslice=1, xbar=bench.XBAR, adcbits=bench.ADC)
        om.debug_retain = True
        with torch.no_grad():
            for pn in ("weight", "alpha_act", "alpha_weight", "alpha_cim"):
                getattr(om, pn).copy_(getattr(m, pn).detach().cpu())
            om.signed_act.copy_(m.signed_act.cpu())
            om.init_state.fill_(1)
            om.init_state_cim.fill_(1)
        box = _capture_oracle_ctx(monkeypatch)
        x = xs[li].cpu()
        g = gs[li].cpu()
        ox = x.clone().requires_grad_(True)
        om(ox).backward(g)
        c = box["c"]
        B = g.shape[0]
        g_bpo = np.ascontiguousarray(g.numpy().reshape(B, O, -1).transpose(0, 2, 1))
        _, aw, aa = co.cim_backward(c, g_bpo, absolute=True)

        mine = dict(zip([pn for pn, _ in m.named_parameters()], grads[name]))
        gw_ref = om.weight.grad.numpy()
        assert rel_err(mine["weight"], gw_ref, aw.reshape(gw_ref.shape)) < 1e-5, (name, "grad_w")
        ga, gr = mine["alpha_cim"], om.alpha_cim.grad.numpy()
        # every entry; the max / min ones with the exact terms of the alpha quantiser's scale gradient
        assert rel_err(ga, gr, alpha_cim_terms(om.alpha_cim.detach().numpy(), aa)) < 1e-5, \
            (name, "grad_alpha_cim", alpha_cim_report(ga, gr, om.alpha_cim.detach().numpy(), aa))
        d = om.dbg
        qn_a, qp_a = co.lsq_act_params(bits)  # unsigned even for the signed first layer (lsq.py:537-538)
        qn_w, qp_w = co.lsq_weight_params(bits)
        t_act = _lsq_scalar_terms(x.numpy(), d["x_q"].grad.numpy(), d["sa"].item(), qn_a, qp_a,
                                  1.0 / math.sqrt(x.numel() * qp_a))
        t_w = _lsq_scalar_terms(m.weight.detach().cpu().numpy(), d["w_q"].grad.numpy(), d["sw"].item(), qn_w, qp_w,
                                1.0 / math.sqrt(m.weight.numel() * qp_w))
        assert abs(float(np.asarray(mine["alpha_act"]).reshape(-1)[0]) - om.alpha_act.grad.item()) <= 1e-5 * t_act, \
            (name, "alpha_act")
        assert abs(float(np.asarray(mine["alpha_weight"]).reshape(-1)[0]) - om.alpha_weight.grad.item()) <= 1e-5 * t_w, \
            (name, "alpha_weight")
        assert (c.adc != 0).mean() > 0.05, (name, "codes must vary for the check to bite")

"""INTEGRATION.md's reference-side binding (the stub a maintainer would add as
models/_modules/cimq_binding.py, replacing get_cim_output_signed.apply at lsq.py:578) executed
as written.

CPU: the stub loads libcimq.so, its ABI constant equals include/cimq.h's CIMQ_ABI_VERSION and
its struct mirrors match the header's layouts (so an ABI bump without a doc update fails here).
GPU: one forward + backward through the stub's CimqFunction against the oracle.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, rel_err

import cim_quantization_amd._lib as L
from cim_quantization_amd import build as cimq_build


def stub_source():
    txt = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"```python\n(# models/_modules/cimq_binding\.py.*?)```", txt, re.S)
    assert m, "INTEGRATION.md lost its cimq_binding.py block"
    return m.group(1)


def header_abi():
    txt = open(os.path.join(REPO, "include", "cimq.h")).read()
    return int(re.search(r"#define\s+CIMQ_ABI_VERSION\s+(\d+)", txt).group(1))


def exec_stub():
    cimq_build.build(verbose=False)
    os.environ["CIMQ_LIB"] = L.LIB_PATH
    ns = {"__name__": "cimq_binding"}
    exec(compile(stub_source(), "INTEGRATION.md:cimq_binding.py", "exec"), ns)
    return ns


def test_stub_matches_header():
    ns = exec_stub()
    assert ns["CIMQ_ABI_VERSION"] == header_abi() == L.ABI_VERSION
    for mine, ref in ((ns["_Desc"], L.ConvDesc), (ns["_Sizes"], L.Sizes)):
        # L's mirrors are checked against gcc's offsetof on include/cimq.h (test_abi_host.py)
        assert ctypes.sizeof(mine) == ctypes.sizeof(ref)
        assert [getattr(mine, f).offset for f, _ in mine._fields_] == [getattr(ref, f).offset for f, _ in ref._fields_]
    # every call the stub binds exists with the header's arity
    from test_abi_host import header_arities
    ar = header_arities()
    for sym in ("cimq_forward", "cimq_backward", "cimq_query_sizes"):
        assert len(getattr(ns["_lib"], sym).argtypes) == ar[sym], sym


@pytest.mark.gpu
def test_stub_forward_backward_vs_oracle(cuda_device):
    import torch

    from oracle import cim_oracle as co
    ns = exec_stub()
    rng = np.random.default_rng(31)
    B, C, O, H = 2, 16, 16, 16
    sa = np.array([0.08475284], np.float32)
    sw = np.array([0.29980746], np.float32)
    x_q = (rng.integers(0, 8, (B, C, H, H)).astype(np.float32) * sa).astype(np.float32)
    w_q = (rng.integers(-4, 4, (O, C, 3, 3)).astype(np.float32) * sw).astype(np.float32)
    a = (rng.random((1, 2, 3, 3, 1, O)).astype(np.float32) * 3 + 0.1) * np.float32(sa[0] * sw[0])
    alpha_q = co.alpha_quantize(a.astype(np.float32), 8)
    bm = co.make_binary_mask(3, 3, 1, 1)
    g = rng.standard_normal((B, H * H, O)).astype(np.float32)
    sgn = np.zeros(1, np.float32)
    out_o, c = co.cim_forward(x_q, w_q, (1, 1), (1, 1), (1, 1), 3, 1, 3, 1, 1.5, 128, bm, alpha_q, sw, sa, False,
                              sgn, return_debug=True)
    gx_o, gw_o, ga_o = co.cim_backward(c, g)
    ax, aw, aa = co.cim_backward(c, g, absolute=True)

    dev = cuda_device
    t = lambda v, grad=False: torch.from_numpy(np.ascontiguousarray(v)).to(dev).requires_grad_(grad)  # noqa: E731
    x, w, al = t(x_q, True), t(w_q, True), t(alpha_q, True)
    out = ns["CimqFunction"].apply(x, w, (1, 1), (1, 1), (1, 1), 3, 1, 3, 1, 1.5, 128, t(bm), al, t(sw), t(sa),
                                   False, t(sgn))
    out.backward(t(g))
    torch.cuda.synchronize()
    out_terms = np.sum(np.abs(c.adc.astype(np.float64) * bm), axis=(1, 2, 3))
    assert rel_err(out.detach().cpu().numpy(), out_o, out_terms) < 1e-6
    assert rel_err(x.grad.cpu().numpy(), gx_o, ax) < 1e-5
    assert rel_err(w.grad.cpu().numpy(), gw_o, aw) < 1e-5
    assert rel_err(al.grad.cpu().numpy(), ga_o, aa) < 1e-5

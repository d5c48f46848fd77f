import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and libcimq.so")


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def function_cases():
    return sorted(k for k, v in golden_manifest().items() if v["kind"] == "function")


def module_cases():
    return sorted(k for k, v in golden_manifest().items() if v["kind"] == "module")


def rel_err(mine, ref, terms=None):
    """max |mine-ref| / (|ref| + sum|terms|), NaNs must coincide."""
    mine = np.asarray(mine, np.float64)
    ref = np.asarray(ref, np.float64)
    assert mine.shape == ref.shape, (mine.shape, ref.shape)
    nm, nr = np.isnan(mine), np.isnan(ref)
    assert np.array_equal(nm, nr), "NaN pattern differs"
    scale = np.abs(ref)
    if terms is not None:
        scale = np.maximum(scale, np.asarray(terms, np.float64))
    d = np.abs(mine - ref)[~nr]
    s = (scale + 1e-30)[~nr]
    return float((d / s).max()) if d.size else 0.0


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")


def shift_manifest():
    with open(os.path.join(GOLDEN, "manifest_shift.json")) as f:
        return json.load(f)


def plain_manifest():
    with open(os.path.join(GOLDEN, "manifest_plain.json")) as f:
        return json.load(f)


def alpha_cim_terms(alpha, aa, nbits_alpha=8):
    """oracle.cim_module_oracle.alpha_cim_terms (shared with __graft_entry__.smoke)."""
    from oracle.cim_module_oracle import alpha_cim_terms as t
    return t(alpha, aa, nbits_alpha)


def alpha_cim_report(ga, gr, alpha, aa, nbits_alpha=8):
    """the worst entry of rel_err(ga, gr, alpha_cim_terms(alpha, aa)): index, max / min flag, values and terms
    (the assertion message of the grad_alpha_cim checks)"""
    t = alpha_cim_terms(alpha, aa, nbits_alpha)
    ga, gr, a = (np.asarray(v, np.float64).reshape(-1) for v in (ga, gr, alpha))
    t = t.reshape(-1)
    aa = np.broadcast_to(np.asarray(aa, np.float64), np.shape(alpha)).reshape(-1)
    r = np.abs(ga - gr) / (np.maximum(np.abs(gr), t) + 1e-30)
    i = int(np.nanargmax(r))
    kind = "max" if a[i] == a.max() else "min" if a[i] == a.min() else "inner"
    return (f"worst entry {i} ({kind}, {int((a == a[i]).sum())} tied): mine {ga[i]:.9g} ref {gr[i]:.9g} "
            f"terms {t[i]:.6g} aa {aa[i]:.6g} rel {r[i]:.3g}; entries over 1e-5: {int((r > 1e-5).sum())}/{r.size}")


def normwise_err(mine, ref):
    """max |mine - ref| / max |ref| (gradients of contractions, which cancel elementwise)."""
    mine = np.asarray(mine, np.float64)
    ref = np.asarray(ref, np.float64)
    assert mine.shape == ref.shape, (mine.shape, ref.shape)
    return float(np.abs(mine - ref).max() / (np.abs(ref).max() + 1e-30))

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
    """Per-entry sum of |terms| of grad alpha_cim through the alpha quantiser (lsq.py:566-571).

    alpha_q_e = clamp(round_pass(alpha_e / scale), 1, Qp) * scale with scale = (max - min) / (Qp - 1), so
    d loss / d alpha_f = G_f * pass_f + [f is the max] - [f is the min]) / (Qp - 1) * sum_e G_e * (r_e - pass_e * v_e)
    (G = d loss / d alpha_q, v = alpha / scale, r its clamped code, pass the clamp mask of rint(v); tied extrema share the
    scale gradient).  ``aa`` is the oracle's fp64 sum of |terms| of G per entry (cim_backward absolute=True),
    so an entry's terms are aa_f * pass_f plus, on the max / min entries, sum_e aa_e * (r_e + pass_e |v_e|) /
    (Qp - 1): the exact first-order error bound of the fp32 sums, with no magnitude of the result mixed in."""
    a32 = np.asarray(alpha, np.float32)
    a = a32.astype(np.float64)
    aa = np.broadcast_to(np.asarray(aa, np.float64), a.shape)
    qp = 2 ** nbits_alpha - 1
    # the clamp's pass mask is decided on the ROUNDED value (clamp(round_pass(v), 1, Qp): its input is
    # rint(v)), in fp32 as the module computes it
    sc32 = (a32.max() - a32.min()) / np.float32(qp - 1)
    with np.errstate(all="ignore"):
        v32 = (a32 / sc32).astype(np.float32)
    rv = np.rint(v32).astype(np.float64)
    passed = (rv >= 1) & (rv <= qp)
    v = v32.astype(np.float64)
    r = np.clip(rv, 1, qp)
    t = aa * passed
    edge = (a == a.max()) | (a == a.min())
    t = np.where(edge, aa + (aa * (r + passed * np.abs(v))).sum() / (qp - 1), t)
    return t


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

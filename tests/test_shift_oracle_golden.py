"""CPU: the scale/shift oracle (oracle/cim_shift_oracle.py) against the golden vectors that
tests/golden/make_golden_shift.py generated from the reference's own test Functions
(test/test_backward_cimlayer_scale_shift.py, test/test_backward_cimlayer.py), and the
reference scripts' own acceptance criteria on those vectors."""
import math

import numpy as np
import pytest

from conftest import load_golden, rel_err, shift_manifest
from oracle import cim_shift_oracle as so


def _run_oracle(cfg, z):
    variant = so.VARIANT_SIGN if cfg["fn"] == "adcless" else so.VARIANT_ROUND
    T = math.ceil(cfg["C"] * cfg["k"] ** 2 / cfg["xbar"])
    shp = (1, T, cfg["wb"], cfg["ab"], 1, cfg["O"])
    a = np.broadcast_to(z["in_alpha"], shp).astype(np.float32)
    b = z["in_beta"] if "in_beta" in z else np.zeros(shp, np.float32)
    st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
    out, c = so.shift_forward(z["in_x"], z["in_w"], st, pd, cfg["ab"], 1, cfg["wb"], 1, cfg["adc"], cfg["xbar"],
                              z["in_binary_mask"], a, b, variant)
    gx, gw, ga, gb = so.shift_backward(c, z["in_grad"])
    if z["ref_grad_alpha"].shape != ga.shape:
        ga = ga.sum(axis=(2, 3), keepdims=True)
    return out, gx, gw, ga, gb


@pytest.mark.parametrize("name", sorted(shift_manifest()))
def test_shift_oracle_vs_reference(name):
    cfg = shift_manifest()[name]["cfg"]
    z = load_golden(name)
    out, gx, gw, ga, gb = _run_oracle(cfg, z)
    assert rel_err(out, z["ref_out"], z["ref_abs_out"]) < 1e-6
    assert rel_err(gx, z["ref_grad_x"], z["ref_abs_grad_x"]) < 1e-5
    assert rel_err(gw, z["ref_grad_w"], z["ref_abs_grad_w"]) < 1e-5
    assert rel_err(ga, z["ref_grad_alpha"], z["ref_abs_grad_alpha"]) < 1e-5
    if "ref_grad_beta" in z:
        assert rel_err(gb, z["ref_grad_beta"], z["ref_abs_grad_beta"]) < 1e-5


def test_reference_scripts_own_criteria():
    """The checks the reference scripts print (scale_shift.py:763-767, test_backward_cimlayer.py:
    458-461) hold on the recorded vectors: manual Function == autograd twin."""
    z = load_golden("ss_ver2_ref_cfg")
    assert np.mean(z["ref_out"] == z["auto_out"]) == 1.0
    assert np.mean(np.abs(z["ref_grad_x"] - z["auto_grad_x"]) < 0.05) == 1.0
    assert np.mean(np.abs(z["ref_grad_w"] - z["auto_grad_w"]) < 0.05) == 1.0
    assert np.mean(np.abs(z["ref_grad_alpha"] - z["auto_grad_alpha"]) < 0.0005) == 1.0
    assert np.mean(np.abs(z["ref_grad_beta"] - z["auto_grad_beta"]) < 0.0005) == 1.0
    z = load_golden("bk_adc4_ref_cfg")
    for k in ("out", "grad_x", "grad_w", "grad_alpha"):
        assert np.array_equal(z["ref_" + k], z["auto_" + k]), k

"""CPU: the plain-LSQ oracle (oracle/lsq_plain_oracle.py) against the golden vectors that
tests/golden/make_golden_plain.py generated from the reference's ActLSQ -> Conv2dLSQ and
LinearLSQ modules (models/_modules/lsq.py:389-436, :591-662)."""
import numpy as np
import pytest

from conftest import load_golden, normwise_err, plain_manifest
from oracle import lsq_plain_oracle as po


def run_oracle(name):
    m = plain_manifest()[name]
    cfg, z = m["cfg"], load_golden(name)
    if m["kind"] == "conv":
        return z, po.act_conv_chain(z["in_x"], z["in_alpha_a"][0], cfg["na"], bool(z["in_signed"][0]), z["in_weight"],
                                    z["in_alpha_w"][0], cfg["nw"], z.get("in_bias"), (cfg["s"],) * 2, (cfg["p"],) * 2,
                                    z["in_grad"])
    return z, po.linear_lsq(z["in_x"], z["in_weight"], z["in_alpha_w"][0], cfg["nw"], z.get("in_bias"), z["in_grad"])


@pytest.mark.parametrize("name", sorted(plain_manifest()))
def test_plain_oracle_vs_reference(name):
    z, o = run_oracle(name)
    if name.startswith("plain_conv"):
        np.testing.assert_array_equal(o["y"].astype(np.float32), z["ref_y"])  # integer conv, same fp32 scaling
        ga = float(o["grad_alpha_a"])
        assert abs(ga - float(z["ref_grad_alpha_a"][0])) <= 1e-5 * float(z["ref_abs_alpha_a"])
        gaw = float(o["grad_alpha_w"])
    else:
        assert normwise_err(o["y"], z["ref_y"]) < 1e-6
        gaw = float(o["grad_alpha"])
    assert normwise_err(o["grad_x"], z["ref_grad_x"]) < 1e-5
    assert normwise_err(o["grad_weight"], z["ref_grad_weight"]) < 1e-5
    assert abs(gaw - float(z["ref_grad_alpha_w"][0])) <= 1e-5 * float(z["ref_abs_alpha_w"])
    if "ref_grad_bias" in z:
        assert normwise_err(o["grad_bias"], z["ref_grad_bias"]) < 1e-5


def test_lsq_quantiser_values():
    """round half to even after the clamp; scaled output multiplies the code back."""
    x = np.array([-3.0, -0.75, 0.25, 0.75, 1.25, 9.0], np.float32)
    np.testing.assert_array_equal(po.lsq_forward(x, 0.5, -4, 3), [-4.0, -2.0, 0.0, 2.0, 2.0, 3.0])
    np.testing.assert_array_equal(po.lsq_forward(x, 0.5, -4, 3, scaled=True), [-2.0, -1.0, 0.0, 1.0, 1.0, 1.5])

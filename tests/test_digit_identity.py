"""The activation-prep kernel's branch-free digit formula (act_words in
cim_quantization_amd/csrc/cimq_kernels.hip) against the oracle's slicing chain.

The reference slices x_int = x_q / sa (lsq.py:466-509) by floor / remainder on fp32 values;
x_int is not always an integer (fl(fl(r*sa)/sa) != r for some r, sa: the "6 - eps" slice
artifacts).  The kernel computes, for m = x_int (unsigned) or |x_int| (signed, digits
negated for x_int < 0), F = floor(m), fr = m - F:

    digit 0 = min(rint((F mod 2^b) + fr), 127),   digit j = (F >> b*j) mod 2^b,

and the forward word holds clamp_i8(digit).  This test pins that identity on the CPU
(numpy restatement of the formula vs oracle/cim_oracle.py) for integer, near-integer and
quantiser-produced x_int, both signednesses, slice widths 1 and 2.
"""
import numpy as np
import pytest

from oracle import cim_oracle as co

F32 = np.float32


def clamp_i8(v):
    return np.clip(np.rint(np.asarray(v, F32)), -127, 127).astype(np.int32)


def kernel_digits(xi, bits, bs, signed):
    n = bits // bs
    mask = (1 << bs) - 1
    xi = np.asarray(xi, F32)
    m = np.abs(xi) if signed else xi
    F = np.floor(m).astype(F32)
    Fi = F.astype(np.int64)
    fr = (m - F).astype(F32)
    out = []
    for j in range(n):
        if j == 0:
            d = np.minimum(np.rint(((Fi & mask).astype(F32) + fr).astype(F32)), 127).astype(np.int64)
        else:
            d = (Fi >> (bs * j)) & mask
        if signed:
            d = np.where(xi < 0, -d, d)
        out.append(d)
    return np.stack(out).astype(np.int32)


def sample_x_int(rng, signed):
    k = rng.integers(-300 if signed else 0, 300, size=4000).astype(F32)
    ulp = np.spacing(np.abs(k).astype(F32) + F32(1)).astype(F32)
    near = np.concatenate([k + s * ulp for s in (-3, -2, -1, 1, 2, 3)]).astype(F32)
    r = rng.integers(-255 if signed else 0, 256, size=20000).astype(F32)
    sa = rng.uniform(0.01, 0.5, size=r.shape).astype(F32)
    quant = ((r * sa).astype(F32) / sa).astype(F32)  # x_int as lsq.py:97 computes it
    rand = rng.uniform(-300 if signed else 0, 300, size=4000).astype(F32)
    return np.concatenate([k, near, quant, rand]).astype(F32)


@pytest.mark.parametrize("signed", [False, True])
@pytest.mark.parametrize("bits,bs", [(3, 1), (4, 1), (8, 1), (4, 2), (8, 2)])
def test_digit_formula_matches_oracle_slicing(signed, bits, bs):
    rng = np.random.default_rng(1000 + bits * 10 + bs + (5 if signed else 0))
    xi = sample_x_int(rng, signed)
    if signed:
        ref = co.slicing_signed(xi, bits, bs)
    else:
        ref = co.slicing_act(xi, bits, bs)
    want = clamp_i8(ref)
    got = kernel_digits(xi, bits, bs, signed)
    bad = np.argwhere(want != got)
    assert bad.size == 0, f"x_int={xi[bad[0][1]]!r} digit {bad[0][0]}: oracle {want[tuple(bad[0])]} kernel {got[tuple(bad[0])]}"
    # the near-integer samples do produce fractional x_int (the artifact path is exercised)
    assert np.any(xi != np.rint(xi))

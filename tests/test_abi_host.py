"""CPU: libcimq.so loads, exports every symbol include/cimq.h declares, and validates
descriptors on the host (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

import cim_quantization_amd._lib as L
from cim_quantization_amd import build as cimq_build


@pytest.fixture(scope="module")
def lib():
    cimq_build.build(verbose=False)  # no-op when up to date (hipcc cross-compiles, no GPU needed)
    return L.load()


def header_symbols():
    with open(os.path.join(REPO, "include", "cimq.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(cimq_\w+)\s*\(", txt, re.M)))


def test_header_and_binding_agree():
    assert header_symbols() == sorted(L.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(L.LIB_PATH)
    for sym in header_symbols():
        assert hasattr(raw, sym), sym
    assert lib.cimq_abi_version() == L.ABI_VERSION


def test_library_is_gfx950_code_object():
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _desc(**kw):
    base = dict(B=256, C=16, H=32, W=32, O=16, KH=3, KW=3, stride=(1, 1), padding=(1, 1), xbar=128,
                bits_w=3, bits_a=3, bs_w=1, bs_a=1, adc_bits=1.5)
    base.update(kw)
    return L.make_desc(**base)


def test_query_sizes_resnet20_s1(lib):
    s = L.query_sizes(_desc())
    # ctx holds the packed forward slice word and the backward slice word (4 bytes each for
    # nba <= 4) per input element, a 2-byte state word per partial-sum (tile, w-slice, pixel,
    # channel), plus small weight/param tables
    nin = 256 * 16 * 32 * 32
    nst = 2 * 3 * (256 * 32 * 32) * 16 * 2  # T=2 tiles, nbw=3, M pixels, O=16, uint16
    assert 8 * nin + nst <= s.ctx_bytes < 8 * nin + nst + (1 << 20)
    assert s.bwd_workspace_bytes > 0


@pytest.mark.parametrize("kw,code", [
    (dict(xbar=100), 2), (dict(xbar=256), 2), (dict(adc_bits=0.7), 1), (dict(bits_w=0), 1),
    (dict(B=0), 1), (dict(bits_a=9, bs_a=1), 2), (dict(bs_w=6, bits_w=6), 2),
])
def test_query_sizes_rejects(lib, kw, code):
    d = _desc(**kw)
    s = L.Sizes()
    rc = lib.cimq_query_sizes(ctypes.byref(d), ctypes.byref(s))
    assert rc == code
    assert lib.cimq_last_error().decode()


@pytest.mark.parametrize("adc", [0, 1, 1.5, 4, 6])
def test_query_sizes_accepts_adc_modes(lib, adc):
    L.query_sizes(_desc(adc_bits=adc))


def test_forward_rejects_null_pointers(lib):
    d = _desc()
    rc = lib.cimq_forward(ctypes.byref(d), None, None, None, None, None, None, None, None, None, None, None)
    assert rc == 1


def header_arities():
    with open(os.path.join(REPO, "include", "cimq.h")) as f:
        txt = f.read()
    out = {}
    for m in re.finditer(r"^\s*(?:int|size_t|const char\*)\s+(cimq_\w+)\s*\(([^)]*)\)\s*;", txt, re.M | re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else len(params.split(","))
    return out


def test_ctypes_arity_matches_header(lib):
    ar = header_arities()
    assert set(ar) == set(L.EXPORTED_SYMBOLS)
    for sym, n in ar.items():
        assert len(getattr(lib, sym).argtypes) == n, sym


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors have the header's sizes and field offsets (gcc on include/cimq.h)."""
    import subprocess
    mirrors = {"cimq_conv_desc": L.ConvDesc, "cimq_lsq_desc": L.LsqDesc, "cimq_sizes": L.Sizes,
               "cimq_prepare_item": L.PrepareItem, "cimq_qconv_desc": L.QConvDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "cimq.h"', 'int main(void) {']
    for cname, cls in mirrors.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ['  return 0;', '}']
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, got):
        cname, fname, v = line.split()
        cls = mirrors[cname]
        want = ctypes.sizeof(cls) if fname == "size" else getattr(cls, fname).offset
        assert int(v) == want, line


def test_module_prepare_validates_items(lib):
    d = _desc(input_kind=L.CIMQ_INPUT_RAW_LSQ, lsq_qp=7.0)
    q = L.make_lsq_desc(-4, 3, 1e-3, 1e-3, 8)
    it = L.PrepareItem()
    it.desc, it.lsq = ctypes.pointer(d), ctypes.pointer(q)
    arr = (L.PrepareItem * 1)(it)
    assert lib.cimq_module_prepare(1, arr, None) == 1  # null parameter pointers
    assert "null" in lib.cimq_last_error().decode()
    assert lib.cimq_module_prepare(-1, None, None) == 1
    assert lib.cimq_module_prepare(0, None, None) == 0
    assert L.query_sizes(d).wprep_bytes > 0


@pytest.mark.parametrize("C,O,H,s", [(16, 16, 32, 1), (32, 32, 16, 1), (64, 64, 8, 1), (16, 32, 32, 2),
                                     (32, 64, 16, 2)])
def test_module_shift_supported_resnet56_shapes(lib, C, O, H, s):
    """cfg4's Conv2dLSQCiM(adc_shift=True) layers (w2a2 xbar 64, adc 1.5) and, since round 4, its w8a8
    first conv (the plane-state backward + shift_stats8_kernel) take the fused shift path; the test
    scripts' variants (int8 ps buffer, shift range), the sign ADC and non-RAW input do not (host plan
    only, no GPU call)."""
    kw = dict(B=256, C=C, H=H, W=H, O=O, stride=(s, s), xbar=64, bits_w=2, bits_a=2,
              input_kind=L.CIMQ_INPUT_RAW_LSQ, lsq_qp=3.0)
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_SHIFT_ROUND, **kw)) == 1
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_LIBRARY, **kw)) == 0
    scripts = L.CIMQ_ADC_SHIFT_ROUND | L.CIMQ_ADC_F_PS_INT8 | L.CIMQ_ADC_F_SHIFT_RANGE
    assert lib.cimq_module_shift_supported(_desc(adc_variant=scripts, **kw)) == 0
    kw1 = dict(kw, adc_bits=1.0)
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_SHIFT_SIGN, **kw1)) == 0
    kw8 = dict(kw, C=3, O=16, H=32, W=32, stride=(1, 1), bits_w=8, bits_a=8, lsq_qp=255.0)
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_SHIFT_ROUND, **kw8)) == 1
    kw8w = dict(kw8, C=8)  # K = 72 > 64: two K-steps, off the w8a8 statistics kernel
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_SHIFT_ROUND, **kw8w)) == 0
    kwx = dict(kw, input_kind=L.CIMQ_INPUT_XQ)
    assert lib.cimq_module_shift_supported(_desc(adc_variant=L.CIMQ_ADC_SHIFT_ROUND, **kwx)) == 0


def test_pending_host_logic(lib):
    """cimq_pending (ABI 11): a zeroed one holds no epilogue and flushes to nothing (no HIP call);
    one that was never zeroed is refused by every entry point that takes it."""
    p = L.Pending()
    assert ctypes.sizeof(p) == 16384
    assert lib.cimq_pending_jobs(p) == 0
    assert lib.cimq_pending_flush(p, None) == 0
    assert lib.cimq_pending_jobs(p) == 0
    p.opaque[0] = 0x1234  # not the library's magic
    assert lib.cimq_pending_flush(p, None) == L.CIMQ_EINVAL
    assert b"not initialised" in lib.cimq_last_error()
    assert lib.cimq_pending_jobs(p) == 0
    assert lib.cimq_pending_flush(None, None) == L.CIMQ_EINVAL


def test_module_route_resnet20(lib):
    """cimq_module_route (ABI 12; CIMQ_ROUTE_R6 since ABI 13, under CIMQ_OPT_RECOMPUTE since ABI 14): which kernels
    the module entry points run for each ResNet-20 layer of the benchmark (bench.RESNET20, xbar 128, adc 1.5,
    B = 256) -- the round-5 kernels where their plans apply, the round-4 ones elsewhere, and
    with the recompute option the round-6 recompute backward on the 16-channel stride-1 layers.  A host query: no
    device work."""
    import ctypes

    import bench
    want = {
        "conv1": ("v3", "c1", "c1"),
        "layer1.0.conv1": ("fwd5", "gx5", "gw5"),
        "layer2.0.conv1": ("fwd5", "v7", "gw5"),  # stride 2: gx_v8, and gw5 at stride 2
        "layer2.0.conv2": ("fwd5", "gx5", "gw5"),
        "layer3.0.conv1": ("fwd5", "v7", "gw5"),  # stride 2: fwd5 with two output blocks per workgroup (its larger LDS budget)
        "layer3.0.conv2": ("fwd5", "fused", "fused"),
    }
    got, rec = {}, {}
    for name, c, o, h, s, nb in bench.RESNET20:
        for opt, out in ((0, got), (L.CIMQ_OPT_RECOMPUTE, rec)):
            d = _desc(C=c, O=o, H=h, W=h, stride=(s, s), bits_w=nb, bits_a=nb, input_kind=L.CIMQ_INPUT_RAW_LSQ,
                      lsq_qp=float(2 ** nb - 1), options=opt)
            r = (ctypes.c_int * 3)()
            assert lib.cimq_module_route(ctypes.byref(d), r) == 0, lib.cimq_last_error()
            out[name] = tuple(L.ROUTE_NAMES[v] for v in r)
    for name, w in want.items():
        assert got[name] == w, (name, got[name])
    # every 3-bit stride-1 layer takes all three round-5 kernels by default; with the recompute option the
    # 16-channel ones recompute their partial sums in the backward and the others are unchanged
    for name, c, o, h, s, nb in bench.RESNET20:
        if nb == 3 and s == 1 and c in (16, 32):
            assert got[name] == ("fwd5", "gx5", "gw5"), (name, got[name])
        want_rec = ("fwd5", "r6", "r6") if (nb == 3 and s == 1 and c == 16) else got[name]
        assert rec[name] == want_rec, (name, rec[name])
    d = _desc(options=2)
    assert lib.cimq_module_route(ctypes.byref(d), (ctypes.c_int * 3)()) == L.CIMQ_EINVAL  # unknown option bit


def test_module_ctx_without_state_words(lib):
    """ABI 13/14: with CIMQ_OPT_RECOMPUTE the module entry points' ctx (cimq_sizes.module_ctx_bytes) holds no
    per-partial-sum state words where their backward recomputes the partial sums -- 33.5 MB less per 16-channel
    ResNet-20 layer at B = 256 -- and is the Function path's ctx elsewhere and without the option."""
    import ctypes
    for (c, h, s, nb, recompute) in [(16, 32, 1, 3, True), (32, 16, 1, 3, False), (16, 32, 2, 3, False),
                                      (3, 32, 1, 8, False)]:
        for opt in (0, L.CIMQ_OPT_RECOMPUTE):
            d = _desc(B=256, C=c, O=16 if c == 3 else c * s, H=h, W=h, stride=(s, s), bits_w=nb, bits_a=nb,
                      input_kind=L.CIMQ_INPUT_RAW_LSQ, lsq_qp=float(2 ** nb - 1), options=opt)
            sz = L.Sizes()
            assert lib.cimq_query_sizes(ctypes.byref(d), ctypes.byref(sz)) == 0, lib.cimq_last_error()
            if recompute and opt:
                assert sz.ctx_bytes - sz.module_ctx_bytes >= 2 * 256 * 32 * 32 * 16 * 4  # T * M * O * 4 bytes
            else:
                assert sz.module_ctx_bytes == sz.ctx_bytes

"""ctypes binding of libcimq.so (the C ABI declared in include/cimq.h).

The shared library is built in-tree (``python -m cim_quantization_amd.build`` or
``__graft_entry__.build()``) and loaded from this package directory.  There is no
fallback: if the library is missing or was built for another ABI, every compute entry
point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CIMQ_LIB_PATH") or os.path.join(_HERE, "libcimq.so")
ABI_VERSION = 14

CIMQ_EINVAL = 1  # include/cimq.h error codes
CIMQ_EUNSUPPORTED = 2
CIMQ_EHIP = 3
CIMQ_INPUT_XQ = 0
CIMQ_INPUT_RAW_LSQ = 1
# cimq_module_route codes (include/cimq.h CIMQ_ROUTE_*)
ROUTE_NAMES = {0: "general", 1: "v3", 2: "fwd5", 3: "v7", 4: "fused", 5: "c1", 6: "gx5", 7: "gw5", 8: "dense", 9: "r6"}
CIMQ_ROUTE_R6 = 9
CIMQ_LSQ_ACCUMULATE_GRADS = 1
CIMQ_LSQ_SKIP_TAIL = 2
CIMQ_LSQ_DEFER_GW = 4
# cimq_conv_desc.adc_variant (include/cimq.h)
CIMQ_ADC_LIBRARY = 0
CIMQ_ADC_STOCHASTIC = 1
CIMQ_ADC_SHIFT_ROUND = 2
CIMQ_ADC_SHIFT_SIGN = 3
CIMQ_ADC_F_PS_INT8 = 0x100
CIMQ_ADC_F_SHIFT_RANGE = 0x200
CIMQ_OPT_RECOMPUTE = 1  # cimq_conv_desc.options (ABI 14)

# every symbol include/cimq.h declares
EXPORTED_SYMBOLS = (
    "cimq_abi_version",
    "cimq_last_error",
    "cimq_query_sizes",
    "cimq_forward",
    "cimq_backward",
    "cimq_module_forward",
    "cimq_module_backward",
    "cimq_module_backward_tail",
    "cimq_module_backward_params",
    "cimq_module_backward_chain",
    "cimq_pending_flush",
    "cimq_pending_jobs",
    "cimq_module_prepare",
    "cimq_module_shift_supported",
    "cimq_module_route",
    "cimq_module_shift_forward",
    "cimq_module_shift_backward",
    "cimq_alpha_init",
    "cimq_shift_forward",
    "cimq_shift_backward",
    "cimq_debug_partial_sums",
    "cimq_debug_state_codes",
    "cimq_debug_recompute_codes",
    "cimq_lsq_quantize_forward",
    "cimq_lsq_quantize_workspace_bytes",
    "cimq_lsq_quantize_backward",
    "cimq_qconv_sizes",
    "cimq_qconv_forward",
    "cimq_qconv_backward_scales",
    "cimq_profile_start",
    "cimq_profile_stop",
    "cimq_profile_read",
    "cimq_flat_sgd",
)

KERNEL_IDS = {"fwd": 1, "bwd_gx": 2, "bwd_gw": 3, "prep_act": 4, "fwd_v7": 5, "gx_v8": 6, "gw_v7": 7, "bwd_fused": 8}
# ids 1-4 time every launch of a role (all kernel variants); 5-7 only the v7-path kernels, one
# rocprof symbol family each (the <NBW, NBA, ...> instantiation the workload uses)
KERNEL_SYMBOLS = {1: "cim_fwd_*", 2: "cim_bwd_gx_*", 3: "cim_bwd_gw_*", 4: "prep_act_kernel",
                  5: "cim_fwd_v3_kernel<*, *, *, *> + cim_fwd5_kernel", 6: "cim_bwd_gx_v8_kernel<*, *, *, *, *, *> + cim_bwd_gx5_kernel",
                  7: "cim_bwd_gw_v7_kernel<*, *, *> + cim_bwd_gw5_kernel", 8: "cim_bwd_fused_kernel<*, *, *> + cim_bwd_gxw5_kernel<*, *, *> (grad_x and grad_w in one launch)"}


class ConvDesc(ctypes.Structure):
    """Mirror of ``cimq_conv_desc``."""

    _fields_ = [
        ("batch", ctypes.c_int32), ("in_channels", ctypes.c_int32),
        ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32),
        ("out_channels", ctypes.c_int32), ("kernel_h", ctypes.c_int32), ("kernel_w", ctypes.c_int32),
        ("stride_h", ctypes.c_int32), ("stride_w", ctypes.c_int32),
        ("pad_h", ctypes.c_int32), ("pad_w", ctypes.c_int32),
        ("xbar", ctypes.c_int32),
        ("bits_w", ctypes.c_int32), ("bits_a", ctypes.c_int32),
        ("bs_w", ctypes.c_int32), ("bs_a", ctypes.c_int32),
        ("adc_bits", ctypes.c_float),
        ("input_kind", ctypes.c_int32),
        ("lsq_qp", ctypes.c_float),
        ("adc_variant", ctypes.c_int32),
        ("seed_lo", ctypes.c_uint32), ("seed_hi", ctypes.c_uint32),
        ("options", ctypes.c_int32),
    ]


class LsqDesc(ctypes.Structure):
    """Mirror of ``cimq_lsq_desc``."""

    _fields_ = [("qn_w", ctypes.c_float), ("qp_w", ctypes.c_float), ("gscale_a", ctypes.c_float),
                ("gscale_w", ctypes.c_float), ("nbits_alpha", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("wprep", ctypes.c_void_p)]


class QConvDesc(ctypes.Structure):
    """Mirror of ``cimq_qconv_desc``."""

    _fields_ = [
        ("batch", ctypes.c_int32), ("in_channels", ctypes.c_int32),
        ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32),
        ("out_channels", ctypes.c_int32), ("kernel_h", ctypes.c_int32), ("kernel_w", ctypes.c_int32),
        ("stride_h", ctypes.c_int32), ("stride_w", ctypes.c_int32),
        ("pad_h", ctypes.c_int32), ("pad_w", ctypes.c_int32),
        ("dilation_h", ctypes.c_int32), ("dilation_w", ctypes.c_int32), ("groups", ctypes.c_int32),
        ("code_min", ctypes.c_int32), ("code_max", ctypes.c_int32),
        ("has_bias", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class Pending(ctypes.Structure):
    """Mirror of ``cimq_pending`` (opaque; zero-initialised by ctypes)."""

    _fields_ = [("opaque", ctypes.c_uint64 * 2048)]


class Sizes(ctypes.Structure):
    """Mirror of ``cimq_sizes``."""

    _fields_ = [("ctx_bytes", ctypes.c_size_t), ("fwd_workspace_bytes", ctypes.c_size_t),
                ("bwd_workspace_bytes", ctypes.c_size_t), ("wprep_bytes", ctypes.c_size_t),
                ("module_ctx_bytes", ctypes.c_size_t)]


class PrepareItem(ctypes.Structure):
    """Mirror of ``cimq_prepare_item``."""

    _fields_ = [("desc", ctypes.POINTER(ConvDesc)), ("lsq", ctypes.POINTER(LsqDesc)),
                ("weight", ctypes.c_void_p), ("alpha_act", ctypes.c_void_p), ("alpha_weight", ctypes.c_void_p),
                ("alpha_cim", ctypes.c_void_p), ("binary_mask", ctypes.c_void_p), ("wprep", ctypes.c_void_p)]


_VP = ctypes.c_void_p
_lock = threading.Lock()
_lib = None


class CimqError(RuntimeError):
    pass


def _bind(lib):
    lib.cimq_abi_version.restype = ctypes.c_int
    lib.cimq_abi_version.argtypes = []
    lib.cimq_last_error.restype = ctypes.c_char_p
    lib.cimq_last_error.argtypes = []
    lib.cimq_query_sizes.restype = ctypes.c_int
    lib.cimq_query_sizes.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(Sizes)]
    lib.cimq_forward.restype = ctypes.c_int
    lib.cimq_forward.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 11
    lib.cimq_backward.restype = ctypes.c_int
    lib.cimq_backward.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 14
    lib.cimq_module_forward.restype = ctypes.c_int
    lib.cimq_module_forward.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 11
    lib.cimq_module_backward.restype = ctypes.c_int
    lib.cimq_module_backward.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 16
    lib.cimq_module_backward_tail.restype = ctypes.c_int
    lib.cimq_module_backward_tail.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 9
    lib.cimq_module_backward_params.restype = ctypes.c_int
    lib.cimq_module_backward_params.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 10
    lib.cimq_module_backward_chain.restype = ctypes.c_int
    lib.cimq_module_backward_chain.argtypes = ([ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 15 +
                                               [ctypes.POINTER(Pending), _VP])
    lib.cimq_pending_flush.restype = ctypes.c_int
    lib.cimq_pending_flush.argtypes = [ctypes.POINTER(Pending), _VP]
    lib.cimq_pending_jobs.restype = ctypes.c_int
    lib.cimq_pending_jobs.argtypes = [ctypes.POINTER(Pending)]
    lib.cimq_module_prepare.restype = ctypes.c_int
    lib.cimq_module_prepare.argtypes = [ctypes.c_int, ctypes.POINTER(PrepareItem), _VP]
    lib.cimq_module_shift_supported.restype = ctypes.c_int
    lib.cimq_module_shift_supported.argtypes = [ctypes.POINTER(ConvDesc)]
    lib.cimq_module_route.restype = ctypes.c_int
    lib.cimq_module_route.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(ctypes.c_int)]
    lib.cimq_module_shift_forward.restype = ctypes.c_int
    lib.cimq_module_shift_forward.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 12
    lib.cimq_module_shift_backward.restype = ctypes.c_int
    lib.cimq_module_shift_backward.argtypes = [ctypes.POINTER(ConvDesc), ctypes.POINTER(LsqDesc)] + [_VP] * 18
    lib.cimq_alpha_init.restype = ctypes.c_int
    lib.cimq_alpha_init.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 10
    lib.cimq_shift_forward.restype = ctypes.c_int
    lib.cimq_shift_forward.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 12
    lib.cimq_shift_backward.restype = ctypes.c_int
    lib.cimq_shift_backward.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 16
    lib.cimq_debug_partial_sums.restype = ctypes.c_int
    lib.cimq_debug_partial_sums.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 12
    lib.cimq_debug_state_codes.restype = ctypes.c_int
    lib.cimq_debug_state_codes.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 4
    lib.cimq_debug_recompute_codes.restype = ctypes.c_int
    lib.cimq_debug_recompute_codes.argtypes = [ctypes.POINTER(ConvDesc)] + [_VP] * 7
    _F, _LL, _I = ctypes.c_float, ctypes.c_longlong, ctypes.c_int
    lib.cimq_lsq_quantize_forward.restype = ctypes.c_int
    lib.cimq_lsq_quantize_forward.argtypes = [_VP, _LL, _VP, _F, _F, _I, _VP, _VP]
    lib.cimq_lsq_quantize_workspace_bytes.restype = ctypes.c_size_t
    lib.cimq_lsq_quantize_workspace_bytes.argtypes = [_LL]
    lib.cimq_lsq_quantize_backward.restype = ctypes.c_int
    lib.cimq_lsq_quantize_backward.argtypes = [_VP, _LL, _VP, _F, _F, _I, _VP, _VP, _VP, _VP, _VP]
    lib.cimq_qconv_sizes.restype = ctypes.c_int
    lib.cimq_qconv_sizes.argtypes = [ctypes.POINTER(QConvDesc), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_size_t)]
    lib.cimq_qconv_forward.restype = ctypes.c_int
    lib.cimq_qconv_forward.argtypes = [ctypes.POINTER(QConvDesc)] + [_VP] * 9
    lib.cimq_qconv_backward_scales.restype = ctypes.c_int
    lib.cimq_qconv_backward_scales.argtypes = [ctypes.POINTER(QConvDesc)] + [_VP] * 8
    lib.cimq_flat_sgd.restype = ctypes.c_int
    lib.cimq_flat_sgd.argtypes = [ctypes.c_longlong, _VP, _VP, _VP, _VP, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                  ctypes.c_int, _VP]
    lib.cimq_profile_start.restype = ctypes.c_int
    lib.cimq_profile_start.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.cimq_profile_read.restype = ctypes.c_int
    lib.cimq_profile_read.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_double)] * 4 + [ctypes.POINTER(ctypes.c_int)]
    lib.cimq_profile_stop.restype = ctypes.c_int
    lib.cimq_profile_stop.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    return lib


def load(path: str | None = None):
    """Load (once) and return the bound library; raises CimqError if unavailable."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise CimqError(f"libcimq.so not found at {p}; build it with "
                            f"`python -m cim_quantization_amd.build` (hipcc --offload-arch=gfx950)")
        lib = _bind(ctypes.CDLL(p))
        v = lib.cimq_abi_version()
        if v != ABI_VERSION:
            raise CimqError(f"libcimq ABI {v} != expected {ABI_VERSION}; rebuild")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().cimq_last_error().decode(errors="replace")
        raise CimqError(f"{what} failed (status {rc}): {msg}")


def make_desc(B, C, H, W, O, KH, KW, stride, padding, xbar, bits_w, bits_a, bs_w, bs_a, adc_bits,
              input_kind=CIMQ_INPUT_XQ, lsq_qp=0.0, adc_variant=CIMQ_ADC_LIBRARY, seed=0, options=0) -> ConvDesc:
    d = ConvDesc()
    d.batch, d.in_channels, d.in_h, d.in_w = int(B), int(C), int(H), int(W)
    d.out_channels, d.kernel_h, d.kernel_w = int(O), int(KH), int(KW)
    d.stride_h, d.stride_w = int(stride[0]), int(stride[1])
    d.pad_h, d.pad_w = int(padding[0]), int(padding[1])
    d.xbar = int(xbar)
    d.bits_w, d.bits_a, d.bs_w, d.bs_a = int(bits_w), int(bits_a), int(bs_w), int(bs_a)
    d.adc_bits = float(adc_bits)
    d.input_kind = int(input_kind)
    d.lsq_qp = float(lsq_qp)
    d.adc_variant = int(adc_variant)
    d.seed_lo, d.seed_hi = int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF
    d.options = int(options)
    return d


def make_lsq_desc(qn_w, qp_w, gscale_a, gscale_w, nbits_alpha, flags=0, wprep=None) -> LsqDesc:
    q = LsqDesc()
    q.qn_w, q.qp_w = float(qn_w), float(qp_w)
    q.gscale_a, q.gscale_w = float(gscale_a), float(gscale_w)
    q.nbits_alpha = int(nbits_alpha)
    q.flags = int(flags)
    q.wprep = wprep
    return q


def make_qconv_desc(B, C, H, W, O, KH, KW, stride, padding, dilation, groups, code_min, code_max,
                    has_bias) -> QConvDesc:
    d = QConvDesc()
    d.batch, d.in_channels, d.in_h, d.in_w = int(B), int(C), int(H), int(W)
    d.out_channels, d.kernel_h, d.kernel_w = int(O), int(KH), int(KW)
    d.stride_h, d.stride_w = int(stride[0]), int(stride[1])
    d.pad_h, d.pad_w = int(padding[0]), int(padding[1])
    d.dilation_h, d.dilation_w = int(dilation[0]), int(dilation[1])
    d.groups = int(groups)
    d.code_min, d.code_max = int(code_min), int(code_max)
    d.has_bias = 1 if has_bias else 0
    return d


def qconv_sizes(desc: QConvDesc):
    f, b = ctypes.c_size_t(), ctypes.c_size_t()
    check(load().cimq_qconv_sizes(ctypes.byref(desc), ctypes.byref(f), ctypes.byref(b)), "cimq_qconv_sizes")
    return f.value, b.value


def module_route(desc: ConvDesc):
    """(forward, grad_x, grad_w) CIMQ_ROUTE_* codes of the module entry points for ``desc``."""
    r = (ctypes.c_int * 3)()
    check(load().cimq_module_route(ctypes.byref(desc), r), "cimq_module_route")
    return tuple(r)


def query_sizes(desc: ConvDesc) -> Sizes:
    s = Sizes()
    check(load().cimq_query_sizes(ctypes.byref(desc), ctypes.byref(s)), "cimq_query_sizes")
    return s


class KernelTimer:
    """Sum of HIP-event-measured durations of every launch of one libcimq kernel."""

    def __init__(self, kernel: str, max_launches: int = 65536):
        self.kid = KERNEL_IDS[kernel]
        self.cap = max_launches
        self.total_ms = 0.0
        self.launches = 0
        self.algo_bytes = 0.0
        self.algo_flops = 0.0

    def __enter__(self):
        check(load().cimq_profile_start(self.kid, self.cap), "cimq_profile_start")
        return self

    def __exit__(self, *exc):
        ms, n = ctypes.c_double(), ctypes.c_int()
        b, f = ctypes.c_double(), ctypes.c_double()
        # per launch (cimq_profile_read, ABI 9): duration, algorithmic bytes, logical flops, MFMA ops
        cap = self.cap
        arr = [(ctypes.c_double * cap)() for _ in range(4)]
        got = ctypes.c_int()
        check(load().cimq_profile_read(cap, *arr, ctypes.byref(got)), "cimq_profile_read")
        k = min(cap, got.value)
        self.per_launch = [tuple(a[i] for a in arr) for i in range(k)]
        check(load().cimq_profile_stop(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b), ctypes.byref(f)),
              "cimq_profile_stop")
        self.total_ms, self.launches = ms.value, n.value
        self.algo_bytes, self.algo_flops = b.value, f.value
        return False

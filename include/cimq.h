/*
 * cimq.h -- C ABI of libcimq.so, the MI355X (gfx950) implementation of the CiM
 * partial-sum-quantised convolution of UtkarshSaxena1/CiM_Quantization.
 *
 * The reference path is pure PyTorch (models/_modules/lsq.py); its device work is
 * stock torch ops issued from Python.  libcimq replaces that device work with
 * hand-written CDNA4 HIP kernels.  The Python host layer (cim_quantization_amd)
 * binds these symbols with ctypes; any other FFI (cgo, JNI, N-API) can bind them the
 * same way.
 *
 * Conventions
 *  - Every pointer argument is DEVICE memory owned by the caller (e.g. a torch
 *    tensor's data_ptr()).  The library allocates nothing; scratch comes from the
 *    caller's ``ws`` of cimq_query_sizes()->*_workspace_bytes.
 *  - Scalars that live on the device in the reference (the LSQ step sizes sw/sa,
 *    alpha_cim, signed_act) are passed as device pointers: no host synchronisation.
 *  - All launches are stream-ordered on ``stream`` (a hipStream_t, passed as void*;
 *    NULL = the legacy default stream).  Functions are reentrant and keep no global
 *    mutable state apart from a thread-local error string.
 *  - Return value: 0 on success, otherwise a CIMQ_E* code; cimq_last_error() gives
 *    the message.  Nothing throws across the ABI.
 *
 * Tensor layouts (identical to the reference):
 *   x, grad_x      [B, C, H, W]              fp32, NCHW contiguous
 *   w_q, grad_w    [O, C, KH, KW]            fp32
 *   out, grad_out  [B, Ho*Wo, O]             fp32 (the Function's [B, P, O] output)
 *   alpha_q        [1, T, nbw, nba, 1, O]    fp32 (quantised alpha_cim), may be NULL
 *   binary_mask    [1, 1, nbw, nba, 1, 1]    int8 (wraps for 8-bit layers)
 *   signed_act     [1]                       fp32 buffer (0 or 1)
 */
#ifndef CIMQ_H
#define CIMQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CIMQ_ABI_VERSION 14

/* status codes */
#define CIMQ_OK 0
#define CIMQ_EINVAL 1      /* descriptor / argument rejected */
#define CIMQ_EUNSUPPORTED 2 /* valid for the reference but not implemented here */
#define CIMQ_EHIP 3        /* a HIP runtime call failed */

/* what ``x`` holds (cimq_conv_desc.input_kind) */
#define CIMQ_INPUT_XQ 0     /* x is x_q, the quantised activation handed to the Function (lsq.py:92) */
#define CIMQ_INPUT_RAW_LSQ 1 /* x is the raw activation; the LSQ act quantiser (lsq.py:547-549) is fused */

/* cimq_conv_desc.adc_variant: which ADC the partial sums go through.  Low byte = variant,
 * higher bits = CIMQ_ADC_F_* modifiers. */
#define CIMQ_ADC_LIBRARY 0     /* get_cim_output_signed's ADC (lsq.py:196-230), deterministic */
#define CIMQ_ADC_STOCHASTIC 1  /* the stochastic 1.5-bit ADC (lsq.py:205-221): 2 x 50 Bernoulli draws
                                  per partial sum from a Philox4x32-10 stream keyed by seed_lo/hi;
                                  the backward is the deterministic one (lsq.py:244-386) */
#define CIMQ_ADC_SHIFT_ROUND 2 /* scale + shift ADC clamp(round((u-beta)/alpha))*alpha + beta
                                  (test/test_backward_cimlayer_scale_shift.py:336-546, "ver2") */
#define CIMQ_ADC_SHIFT_SIGN 3  /* scale + shift sign ADC sign((u-beta)/alpha)*alpha + beta
                                  (test/test_backward_cimlayer_scale_shift.py:113-334, "adcless") */
#define CIMQ_ADC_F_PS_INT8 0x100     /* partial sums pass through an int8 buffer before the ADC
                                        (truncation + wrap, scale_shift.py:401) */
#define CIMQ_ADC_F_SHIFT_RANGE 0x200 /* ADC range Qp = 2^(b-1)-1, Qn = -2^(b-1) for every adc_bits
                                        but 1 (scale_shift.py:369-375) instead of the library's
                                        +-1 for 1.5 bits */

/* cimq_conv_desc.options */
#define CIMQ_OPT_RECOMPUTE 1 /* module entry points: where a recompute backward exists (CIMQ_ROUTE_R6: w3a3 16 -> 16,
                                3x3 stride 1, xbar 128, 32 wide) the forward writes no per-partial-sum state words
                                and the backward recomputes the partial sums -- a smaller ctx (module_ctx_bytes;
                                33.5 MB less per such layer at B = 256) for a slower backward on MI355X (DESIGN.md
                                section 10).  Ignored elsewhere.  Since ABI 14 */

/* cimq_lsq_desc.flags */
#define CIMQ_LSQ_ACCUMULATE_GRADS 1 /* cimq_module_backward adds the parameter gradients into
                                       grad_weight / grad_alpha_* (torch's AccumulateGrad,
                                       grad = grad + new) instead of overwriting them */
#define CIMQ_LSQ_SKIP_TAIL 2        /* cimq_module_backward stops after grad_x and the per-chunk
                                       grad_w / grad_alpha partials (left in ws); the caller runs
                                       cimq_module_backward_tail later, e.g. on a second stream
                                       (the parameter gradients are off the grad_x chain) */
#define CIMQ_LSQ_DEFER_GW 4         /* as SKIP_TAIL, and on layers whose grad_w is a kernel of its
                                       own (the v7 pair) that kernel is left out too: the caller
                                       runs cimq_module_backward_params (grad_w + the epilogue) on
                                       a second stream ordered after cimq_module_backward.  Since ABI 10 */

typedef struct cimq_conv_desc {
  int32_t batch, in_channels, in_h, in_w; /* B, C, H, W */
  int32_t out_channels, kernel_h, kernel_w; /* O, KH, KW (square kernels in the reference) */
  int32_t stride_h, stride_w, pad_h, pad_w;
  int32_t xbar;       /* crossbar rows per tile ("arr", lsq.py:166); multiple of 16 */
  int32_t bits_w, bits_a; /* nbits_w, nbits_a */
  int32_t bs_w, bs_a; /* weight / activation bit-slice widths */
  float adc_bits;     /* 0 (fp ADC), 1 (sign), 1.5 (ternary, alpha scaled), >1.5 (multi-level) */
  int32_t input_kind; /* CIMQ_INPUT_* */
  float lsq_qp;       /* CIMQ_INPUT_RAW_LSQ: act clamp max Qp_a = 2^bits_a - 1 (Qn_a = 0) */
  int32_t adc_variant; /* CIMQ_ADC_* | CIMQ_ADC_F_* (0: the library ADC) */
  uint32_t seed_lo, seed_hi; /* CIMQ_ADC_STOCHASTIC: Philox key of this call */
  int32_t options;    /* CIMQ_OPT_* bits (0: the defaults); was ``reserved`` before ABI 14 */
} cimq_conv_desc;

/* The LSQ quantisers of Conv2dLSQCiM.forward (lsq.py:544-571), for the module entry points. */
typedef struct cimq_lsq_desc {
  float qn_w, qp_w;         /* weight clamp range: -2^(bits_w-1), 2^(bits_w-1)-1 (lsq.py:553-555) */
  float gscale_a;           /* grad_scale factor of alpha_act: 1/sqrt(numel(x) * Qp_a) (lsq.py:547) */
  float gscale_w;           /* grad_scale factor of alpha_weight: 1/sqrt(numel(w) * Qp_w) (lsq.py:553) */
  int32_t nbits_alpha;      /* alpha_cim quantiser bits (lsq.py:566-571); ignored unless adc 1 / 1.5 */
  int32_t flags;            /* CIMQ_LSQ_* bits */
  const void* wprep;        /* NULL, or a buffer of cimq_sizes.wprep_bytes that cimq_module_prepare
                               filled for this descriptor pair and the current parameter values:
                               the module forward then runs only the activation quantiser, and it
                               and the backward read the weight-side state (w_q operands, alpha_q
                               thresholds, step sizes) from there instead of from ctx */
} cimq_lsq_desc;

typedef struct cimq_sizes {
  size_t ctx_bytes;           /* forward -> backward state, caller-owned device memory */
  size_t fwd_workspace_bytes; /* scratch for cimq_forward / cimq_alpha_init */
  size_t bwd_workspace_bytes; /* scratch for cimq_backward */
  size_t wprep_bytes;         /* weight-side state of the module entry points (cimq_module_prepare) */
  size_t module_ctx_bytes;    /* ctx of the module entry points (cimq_module_forward / _backward): smaller than
                                 ctx_bytes where their backward recomputes the partial sums instead of reading
                                 per-partial-sum state words (CIMQ_ROUTE_R6 under CIMQ_OPT_RECOMPUTE).  Since ABI 13 */
} cimq_sizes;

/* ABI version of the loaded library (compare with CIMQ_ABI_VERSION). */
int cimq_abi_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char* cimq_last_error(void);

/* Validate a descriptor and report the buffer sizes it needs.
 * Replaces the geometry bookkeeping of get_cim_output_signed.forward (lsq.py:115-170). */
int cimq_query_sizes(const cimq_conv_desc* d, cimq_sizes* out);

/* Forward of the CiM conv: act codes + bit slices, implicit-im2col int8 MFMA partial sums
 * per (tile, w-slice, a-slice), ADC requantisation and shift-and-add.
 * Replaces get_cim_output_signed.forward (lsq.py:92-237); with CIMQ_INPUT_RAW_LSQ it
 * also absorbs the activation quantiser of Conv2dLSQCiM.forward (lsq.py:547-549).
 * out = [B, P, O]; ctx receives what cimq_backward needs (the int8 ctx of lsq.py:99,160
 * and the parameters that stand in for the fp16 partial sums of lsq.py:192). */
int cimq_forward(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                 const float* sw, const float* alpha_q, const int8_t* binary_mask,
                 const float* signed_act, float* out, void* ctx, void* ws, void* stream);

/* Backward of the CiM conv.  Replaces get_cim_output_signed.backward (lsq.py:244-386):
 *   grad_x     [B,C,H,W]  d loss / d x_q (CIMQ_INPUT_XQ) or d loss / d x through the
 *                          fused LSQ quantiser (CIMQ_INPUT_RAW_LSQ)
 *   grad_w     [O,C,KH,KW] d loss / d w_q
 *   grad_alpha [1,T,nbw,nba,1,O] d loss / d alpha_q (adc 1 / 1.5 only, else may be NULL)
 *   grad_sa    [1]  CIMQ_INPUT_RAW_LSQ only: d loss / d sa from the LSQ graph (lsq.py:548-549)
 * ``x``, ``sa``, ``sw``, ``alpha_q``, ``binary_mask``, ``signed_act`` must be the same
 * buffers (same contents) that were given to cimq_forward with this ctx. */
int cimq_backward(const cimq_conv_desc* d, const float* grad_out, const float* x, const float* sa,
                  const float* sw, const float* alpha_q, const int8_t* binary_mask,
                  const float* signed_act, const void* ctx, float* grad_x, float* grad_w,
                  float* grad_alpha, float* grad_sa, void* ws, void* stream);

/* Forward of a whole Conv2dLSQCiM layer after its first-step initialisation (lsq.py:544-581):
 * the activation, weight and alpha_cim quantisers run inside the library on the raw
 * parameters, then the CiM conv; ``out`` is the module's NCHW output [B, O, Ho, Wo] (before
 * the optional bias).  Requires input_kind = CIMQ_INPUT_RAW_LSQ.  ``alpha_cim`` may be NULL
 * unless adc_bits is 1 or 1.5.  ``ctx`` must hold cimq_query_sizes()->module_ctx_bytes (ABI 13; ctx_bytes
 * is never smaller) and ``ws`` fwd_workspace_bytes. */
int cimq_module_forward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                        const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                        const int8_t* binary_mask, const float* signed_act, float* out, void* ctx, void* ws,
                        void* stream);

/* Backward of cimq_module_forward: from d loss / d out (NCHW) to the gradients of the raw
 * activation and of the four parameters (weight, alpha_act, alpha_weight, alpha_cim), through
 * the quantisers as torch's autograd differentiates them.  With CIMQ_LSQ_ACCUMULATE_GRADS in
 * q->flags the parameter gradients are added into the four grad buffers (grad_x is always
 * overwritten).  ctx must come from cimq_module_forward. */
int cimq_module_backward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out, const float* x,
                         const float* weight, const float* alpha_act, const float* alpha_weight,
                         const float* alpha_cim, const int8_t* binary_mask, const float* signed_act,
                         const void* ctx, float* grad_x, float* grad_weight, float* grad_alpha_act,
                         float* grad_alpha_weight, float* grad_alpha_cim, void* ws, void* stream);

/* The parameter-gradient epilogue of cimq_module_backward (slab reductions of grad_w and
 * grad_alpha, the weight / alpha_cim quantiser backward, the two step-size gradients) for a
 * backward run with CIMQ_LSQ_SKIP_TAIL: ``ctx`` and ``ws`` are that call's, unchanged, and the
 * stream must be ordered after it.  Replaces the torch autograd of lsq.py:547-571 into the
 * parameters.  q->flags as that call's (CIMQ_LSQ_ACCUMULATE_GRADS honoured). */
int cimq_module_backward_tail(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* weight,
                              const float* alpha_cim, const void* ctx, float* grad_weight, float* grad_alpha_act,
                              float* grad_alpha_weight, float* grad_alpha_cim, void* ws, void* stream);

/* The parameter-gradient half of a cimq_module_backward run with CIMQ_LSQ_DEFER_GW: the grad_w
 * kernel that call left out (if the layer has one of its own), then the epilogue of
 * cimq_module_backward_tail.  grad_out, ctx and ws are that call's, unchanged; the stream must be
 * ordered after it (grad_w reads only grad_out and the forward's state, so it overlaps the next
 * layer's grad_x when it runs on a second stream).  q->flags as that call's.  Since ABI 10. */
int cimq_module_backward_params(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                                const float* weight, const float* alpha_cim, const void* ctx, float* grad_weight,
                                float* grad_alpha_act, float* grad_alpha_weight, float* grad_alpha_cim, void* ws,
                                void* stream);

/* cimq_module_forward / cimq_module_backward for Conv2dLSQCiM(adc_shift=True): the per-tile scale +
 * shift ADC clamp(round((u - beta) / alpha_q), -1, 1) * alpha_q + beta of
 * test/test_backward_cimlayer_scale_shift.py:336-546 applied to the library's rescaled partial sum
 * u = fp16(ps) * sw * sa, with the three quantisers inside the library as for the library ADC.
 * Requires adc_variant = CIMQ_ADC_SHIFT_ROUND (no flags), adc_bits 1.5, input_kind =
 * CIMQ_INPUT_RAW_LSQ, nbw = nba = 2 or 3 and a layer the fast path takes (3x3, pad 1, stride 1 or 2,
 * power-of-two output width and channels); CIMQ_EUNSUPPORTED otherwise (the caller then quantises
 * in torch and calls cimq_shift_forward / cimq_shift_backward).  No prepared weight side
 * (q->wprep NULL), no CIMQ_LSQ_SKIP_TAIL.  beta_cim / grad_beta_cim: [1, T, nbw, nba, 1, O] like
 * alpha_cim; CIMQ_LSQ_ACCUMULATE_GRADS adds into grad_beta_cim as well.  Since ABI 8. */
int cimq_module_shift_supported(const cimq_conv_desc* d); /* 1 if the two calls below take d, else 0 */

/* Which kernels cimq_module_forward / cimq_module_backward run for d (the library ADC, the module entry
 * points): route[0] forward, route[1] grad_x, route[2] grad_w (+ grad_alpha_cim partials), each one of
 * the CIMQ_ROUTE_* codes below.  Pure host query, no device work.  Returns 0, or an error status for a
 * descriptor the module entry points refuse.  Since ABI 12. */
enum {
  CIMQ_ROUTE_GENERAL = 0,  /* the general kernels */
  CIMQ_ROUTE_V3 = 1,       /* forward: cim_fwd_v3_kernel */
  CIMQ_ROUTE_FWD5 = 2,     /* forward: cim_fwd5_kernel (slice-planar patch, round 5) */
  CIMQ_ROUTE_V7 = 3,       /* grad_x: cim_bwd_gx_v8_kernel / grad_w: cim_bwd_gw_v7_kernel */
  CIMQ_ROUTE_FUSED = 4,    /* grad_x and grad_w in cim_bwd_fused_kernel */
  CIMQ_ROUTE_C1 = 5,       /* the w8a8 first conv: cim_bwd_c1_kernel (both) */
  CIMQ_ROUTE_GX5 = 6,      /* grad_x: cim_bwd_gx5_kernel (per input pixel, round 5) */
  CIMQ_ROUTE_GW5 = 7,      /* grad_w: cim_bwd_gw5_kernel (A-ready patch, round 5) */
  CIMQ_ROUTE_DENSE = 8,    /* the dense 1x1 path */
  CIMQ_ROUTE_R6 = 9        /* grad_x and grad_w in cim_bwd_r6_kernel from RECOMPUTED partial sums (the forward
                              writes no state words; round 6, ABI 13; only under CIMQ_OPT_RECOMPUTE since ABI 14) */
};
int cimq_module_route(const cimq_conv_desc* d, int* route);
int cimq_module_shift_forward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                              const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                              const float* beta_cim, const int8_t* binary_mask, const float* signed_act, float* out,
                              void* ctx, void* ws, void* stream);
int cimq_module_shift_backward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                               const float* x, const float* weight, const float* alpha_act,
                               const float* alpha_weight, const float* alpha_cim, const float* beta_cim,
                               const int8_t* binary_mask, const float* signed_act, const void* ctx, float* grad_x,
                               float* grad_weight, float* grad_alpha_act, float* grad_alpha_weight,
                               float* grad_alpha_cim, float* grad_beta_cim, void* ws, void* stream);

/* One layer of cimq_module_prepare: its descriptors (as the forward will receive them; the
 * lsq descriptor's wprep and flags are ignored here) and raw parameters, and its output buffer
 * ``wprep`` (cimq_sizes.wprep_bytes, caller-owned device memory). */
typedef struct cimq_prepare_item {
  const cimq_conv_desc* desc;
  const cimq_lsq_desc* lsq;
  const float* weight;
  const float* alpha_act;
  const float* alpha_weight;
  const float* alpha_cim; /* NULL unless adc_bits is 1 or 1.5 */
  const int8_t* binary_mask;
  void* wprep;
} cimq_prepare_item;

/* The weight side of cimq_module_forward for n layers at once (lsq.py:552-571: w_q, alpha_q and
 * the step sizes, turned into the CiM kernels' operands and ADC / STE thresholds): one launch per
 * up to 7 layers instead of a few latency-bound workgroups inside every layer's prologue.  A
 * forward given q->wprep = items[i].wprep must see the same parameter values (e.g. prepare after
 * each optimizer step); the backward of that forward reads the buffer too, so it must not be
 * re-prepared in between. */
int cimq_module_prepare(int n, const cimq_prepare_item* items, void* stream);

/* Opaque, caller-owned host memory for cimq_module_backward_chain: zero-initialise it once.
 * 16 KB since ABI 11. */
typedef struct cimq_pending {
  uint64_t opaque[2048];
} cimq_pending;

/* cimq_module_backward for a chain of layers run back to back on ONE stream (a network's
 * backward pass): the parameter-gradient epilogue of each call (the grad_w / grad_alpha slab
 * sums, the LSQ and alpha_cim quantiser backwards) is not launched but left in ``pending``;
 * cimq_pending_flush launches every pending epilogue at once, packed: ceil(n/20) slab-sum (tail)
 * launches, the jobs sorted by slab count, then ceil(n/24) finish launches (since ABI 11; before,
 * each ran inside the next call's kernels).  A call also issues the pending ones first when 32 are
 * pending or when a pending one writes one of its gradient buffers.  The parameter gradients of a
 * call are therefore complete only after the flush (or a later call that issued them) has been
 * issued on the stream; every buffer the call used (ctx, ws, weight, alpha_cim, the four gradient
 * buffers) must stay valid and unreused until then -- in particular ``ws`` must not be handed to
 * another chained call before that.  Memory: each pending layer keeps its workspace alive, and a
 * workspace holds the layer's grad_w slabs (one per image on the fused / first-conv paths: about
 * 37.7 MB for a 64-channel ResNet-20 layer at B = 256), so the chain's peak is up to 32 workspaces;
 * flush more often (e.g. per segment of layers, as bench.Trainer does at world > 1) to bound it.
 * Same arguments as cimq_module_backward; CIMQ_LSQ_SKIP_TAIL and CIMQ_LSQ_DEFER_GW are refused. */
int cimq_module_backward_chain(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                               const float* x, const float* weight, const float* alpha_act,
                               const float* alpha_weight, const float* alpha_cim, const int8_t* binary_mask,
                               const float* signed_act, const void* ctx, float* grad_x, float* grad_weight,
                               float* grad_alpha_act, float* grad_alpha_weight, float* grad_alpha_cim, void* ws,
                               cimq_pending* pending, void* stream);
int cimq_pending_flush(cimq_pending* pending, void* stream);
/* The number of epilogues ``pending`` holds (not yet issued).  After a chained call it is 1 when
 * every earlier one has been issued: the caller may then release their buffers.  Since ABI 11. */
int cimq_pending_jobs(const cimq_pending* pending);

/* First-step alpha_cim initialisation (lsq.py:557-563 with get_analog_partial_sums_signed,
 * lsq.py:35-87): alpha_init[1,T,nbw,nba,1,O] = 2*mean_{b,p}|ps*sw*sa| / sqrt(Qp_adc), zeros
 * replaced by sw*sa.  Uses x, w_q, sa, sw like cimq_forward (ctx is scratch here). */
int cimq_alpha_init(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                    const float* sw, const int8_t* binary_mask, const float* signed_act,
                    float* alpha_init, void* ctx, void* ws, void* stream);

/* Forward of the scale + shift CiM conv (adc_variant CIMQ_ADC_SHIFT_ROUND / _SIGN): the
 * test Functions get_analog_partial_sums_autograd_ver2 / get_adcless_cim_output of
 * test/test_backward_cimlayer_scale_shift.py (:336-431 / :113-215) when x, w_q are the integer
 * x_int / w_int with sa = sw = 1, and this build's Conv2dLSQCiM(adc_shift=True) otherwise
 * (u = fp16(ps) * sw * sa as lsq.py:195 before the shifted ADC).  alpha and beta are
 * [1, T, nbw, nba, 1, O] fp32; the rest as cimq_forward. */
int cimq_shift_forward(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                       const float* sw, const float* alpha, const float* beta, const int8_t* binary_mask,
                       const float* signed_act, float* out, void* ctx, void* ws, void* stream);

/* Backward of cimq_shift_forward (scale_shift.py:437-546 / :240-334): grad_x, grad_w, and
 * grad_alpha / grad_beta [1, T, nbw, nba, 1, O]; grad_sa as cimq_backward (RAW_LSQ only). */
int cimq_shift_backward(const cimq_conv_desc* d, const float* grad_out, const float* x, const float* sa,
                        const float* sw, const float* alpha, const float* beta, const int8_t* binary_mask,
                        const float* signed_act, const void* ctx, float* grad_x, float* grad_w,
                        float* grad_alpha, float* grad_beta, float* grad_sa, void* ws, void* stream);

/* Diagnostic / parity hook: cimq_forward that also writes every integer partial sum
 * ps_out[B,T,nbw,nba,P,O] (int32; the reference keeps them as the fp16 ctx.ps_int of
 * lsq.py:169-192) and its ADC output adc_out (same shape, fp32, before the shift-and-add
 * mask: adc_out of lsq.py:197-230).  Used by the bit-exactness tests. */
int cimq_debug_partial_sums(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                            const float* sw, const float* alpha_q, const int8_t* binary_mask,
                            const float* signed_act, float* out, int32_t* ps_out, float* adc_out,
                            void* ctx, void* stream);

/* Parity hook for the production forward: decodes the per-partial-sum state words that the
 * fast forward (cim_fwd_v3_kernel on the v7 path) left in ``ctx`` -- the ADC code
 * (lsq.py:321-332: -1 / 0 / +1) and the STE pass bit (lsq.py:310-313) of every (tile, w-slice,
 * a-slice) partial sum -- into code_out / pass_out [B, T, nbw, nba, P, O] (int8 / uint8).
 * ``ctx`` must come from cimq_forward / cimq_module_forward with the same descriptor;
 * CIMQ_EUNSUPPORTED for layers whose forward writes no state words. */
int cimq_debug_state_codes(const cimq_conv_desc* d, const void* ctx, int8_t* code_out, uint8_t* pass_out,
                           void* stream);

/* Parity hook for the module layers whose backward recomputes the partial sums (CIMQ_ROUTE_R6, whose forward
 * leaves no state words): the ADC codes and STE pass bits as cimq_debug_state_codes gives them, produced by the
 * recomputing backward's own code path (cim_bwd_r6_kernel in its debug form) from x, signed_act and the ctx of
 * cimq_module_forward.  ``st_scratch`` is caller-owned device memory of T * B * Ho * Wo * O * 4 bytes.
 * CIMQ_EUNSUPPORTED for other layers.  Since ABI 13. */
int cimq_debug_recompute_codes(const cimq_conv_desc* d, const float* x, const float* signed_act, const void* ctx,
                               void* st_scratch, int8_t* code_out, uint8_t* pass_out, void* stream);

/* ---- plain LSQ modules (lsq.py:389-436 Conv2dLSQ, :591-617 LinearLSQ, :620-662 ActLSQ) ---- */

/* The LSQ quantiser out = round_pass(clamp(x / s, qn, qp)) [* s if scaled] over n fp32
 * elements (any float-aligned x, out: 16-byte aligned ones take vector loads), s = *s the grad-scaled step size (grad_scale(alpha, g),
 * lsq.py:407-412 / :608-611 / :653-656, evaluated by the caller).  Replaces those lines'
 * torch ops: ActLSQ's codes (scaled = 0), Conv2dLSQ's weight codes (0), LinearLSQ's w_q (1). */
int cimq_lsq_quantize_forward(const float* x, long long n, const float* s, float qn, float qp, int scaled,
                              float* out, void* stream);

/* Autograd of cimq_lsq_quantize_forward: grad_x (STE through round_pass, the clamp mask,
 * DivBackward wrt x) and grad_s[1] = d loss / d s (MulBackward's sum when scaled, then
 * DivBackward's -grad_t * ((x / s) / s)), reduced in a fixed order.  ``ws`` holds
 * cimq_lsq_quantize_workspace_bytes(n). */
size_t cimq_lsq_quantize_workspace_bytes(long long n);
int cimq_lsq_quantize_backward(const float* x, long long n, const float* s, float qn, float qp, int scaled,
                               const float* grad_out, float* grad_x, float* grad_s, void* ws, void* stream);

/* Conv2dLSQ's conv of integer codes (lsq.py:436): x_codes [B,C,H,W] and w_codes [O,C,KH,KW]
 * are fp32 tensors holding integers (ActLSQ / weight-quantiser codes) in [code_min, code_max]
 * (activations) and [-128, 127] (weights). */
typedef struct cimq_qconv_desc {
  int32_t batch, in_channels, in_h, in_w;
  int32_t out_channels, kernel_h, kernel_w;
  int32_t stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, groups; /* groups must be 1 */
  int32_t code_min, code_max; /* activation code range: within [-128, 127] or [0, 255] */
  int32_t has_bias;
  int32_t reserved;
} cimq_qconv_desc;

int cimq_qconv_sizes(const cimq_qconv_desc* d, size_t* fwd_workspace_bytes, size_t* bwd_workspace_bytes);

/* y0 = conv2d(x_codes, w_codes) (+ bias) on int8 MFMA (exact int32 sums, then fp32; the
 * reference's fp32 conv of the same integers is exact while |sum| < 2^24) and
 * y = (y0 * act_scale) * w_scale, both [B, O, Ho, Wo].  y0 is kept for the backward (the
 * tensor torch's MulBackward saves).  act_scale / w_scale: device pointers to one float. */
int cimq_qconv_forward(const cimq_qconv_desc* d, const float* x_codes, const float* w_codes, const float* act_scale,
                       const float* w_scale, const float* bias, float* y, float* y0, void* ws, void* stream);

/* Elementwise backward of y = (y0 * act_scale) * w_scale: grad_y0 = (grad_y * w_scale) * act_scale,
 * grad_scales[0] = sum grad_y * (y0 * act_scale) (d / d w_scale), grad_scales[1] =
 * sum (grad_y * w_scale) * y0 (d / d act_scale).  The conv's own input / weight gradients of
 * grad_y0 are plain fp32 convolutions (the caller's library conv). */
int cimq_qconv_backward_scales(const cimq_qconv_desc* d, const float* grad_y, const float* y0, const float* act_scale,
                               const float* w_scale, float* grad_y0, float* grad_scales, void* ws, void* stream);

/* Diagnostic kernel timer.  Until cimq_profile_stop(), every launch of kernel ``kernel_id``
 * (1 = partial-sum forward, 2 = grad_x, 3 = grad_w/grad_alpha, 4 = act-code prep, each over
 * all kernel variants; 5 / 6 / 7 = only the v7-path forward / grad_x / grad_w kernels; 8 = the
 * fused backward of the stride-1 w2a2 / w3a3 layers, role 2) is
 * bracketed by a hipEvent pair on its launch stream (at most ``max_launches``).  stop()
 * waits for the last event and returns the summed kernel time, the number of launches and
 * their summed algorithmic bytes / flops ("Roofline accounting"). */
int cimq_profile_start(int kernel_id, int max_launches);
int cimq_profile_stop(double* total_ms, int* launches, double* algo_bytes, double* algo_flops);
/* ABI 9: before cimq_profile_stop(), the first ``cap`` launches one by one -- HIP-event duration (ms),
 * the SURVEY 8(d) algorithmic bytes and logical flops, and the MFMA operations as issued (int8 bit-slice
 * products of the live slice pairs forward, three bf16 products per fp32-accurate backward MAC) -- and
 * in *launches the count recorded.  Lets a caller take max(t_HBM, t_MFMA) per launch. */
int cimq_profile_read(int cap, double* ms, double* algo_bytes, double* algo_flops, double* mfma_ops, int* launches);

/* One SGD step (momentum, per-element weight decay, no dampening / Nesterov: torch.optim.SGD's
 * update, examples/__init__.py:184-188) over n flat fp32 elements in one launch:
 *   d = grad + wd * param;  buf = first ? d : momentum * buf + d;  param -= lr * buf
 * (each operation rounded to fp32, no fused multiply-adds), then grad = 0 when zero_grad is set.
 * The bench's optimizer (dist.FlatSGD) on the flat parameter / gradient buffers.  Since ABI 11. */
int cimq_flat_sgd(long long n, float* param, float* grad, float* buf, const float* wd, float lr, float momentum,
                  int first, int zero_grad, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CIMQ_H */

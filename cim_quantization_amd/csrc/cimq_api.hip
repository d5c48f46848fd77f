// cimq_api.hip -- the extern "C" boundary of libcimq.so (declared in include/cimq.h).
// Host-side geometry validation, ctx / workspace carving and the kernel launch sequences
// that replace get_cim_output_signed.forward / backward (models/_modules/lsq.py:92-386).
#define CIMQ_TU_MAIN
#include "cimq_host.h"
#include "cimq_lsq.hip"

using namespace cimq;

namespace {

int prep_all(const Geo& g, const float* x, const float* w_q, const float* sa, const float* sw,
             const float* alpha_q, const int8_t* bmask, const float* signed_act, uint8_t* ctx,
             hipStream_t s, bool need_params, bool need_wgx, const float* beta = nullptr) {
  CtxLayout L = ctx_layout(g);
  const int blk = 256;
  {
    // one 4-element item per thread up to 8192 blocks (fewer, fatter blocks measured slower)
    int grid = cdiv(g.Nin, 4 * blk);
    if (grid > act_blocks()) grid = act_blocks();
    const int slot = prof_begin(KID_PREP_ACT, g, s);
    hipLaunchKernelGGL(prep_act_kernel, dim3(grid), dim3(blk), 0, s, g, x, sa, signed_act,
                       ctx + L.xcode, ctx + L.xhat);
    prof_end(slot, s);
    CIMQ_TRY(check_hip("prep_act"));
  }
  {
    int total = g.T * g.KS * g.NBLK * 64;
    hipLaunchKernelGGL(prep_wfrag_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, w_q, sw,
                       reinterpret_cast<v4i*>(wreg(g, ctx) + L.wfrag));
    CIMQ_TRY(check_hip("prep_wfrag"));
  }
  if (need_wgx) {
    const Plan7 p7 = v7_plan(g);
    // the general / v6 grad_x operands only where the v7 backward will not run
    if (!(p7.ok && (g.variant == VAR_LIBRARY || shift_stats_ok(g)))) {
      // the general grad_x operand where the v7 backward will not run
      int total = g.T * g.FBT * g.NKS * 64;
      hipLaunchKernelGGL(prep_wgx_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, w_q, sw,
                         reinterpret_cast<v4i*>(wreg(g, ctx) + L.wgx));
      CIMQ_TRY(check_hip("prep_wgx"));
    }
    if (p7.ok) {
      const int tc = g.T * p7.v.NCPBT * g.NKS * 64;
      hipLaunchKernelGGL(prep_wcy_kernel, dim3(cdiv(tc, blk)), dim3(blk), 0, s, g, w_q, sw, p7.v.NCPBT,
                         reinterpret_cast<v4i*>(wreg(g, ctx) + L.wcy));
      CIMQ_TRY(check_hip("prep_wcy"));
    }
    // cim_bwd_gx5_kernel's operand (x5_plan: the RAW_LSQ Function path runs that kernel too)
    CIMQ_TRY(launch_prep_wg5(g, w_q, sw, ctx, s));
  }
  Params pp = params_of(g, ctx);
  if (need_params) {
    if (hipMemsetAsync(pp.flags, 0, 16, s) != hipSuccess) return fail(CIMQ_EHIP, "memset flags");
    int total = g.T * g.nba * g.nbw * g.Opad + g.nbw * g.nba + (beta != nullptr ? g.Opad : 0);
    hipLaunchKernelGGL(prep_params_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, alpha_q, sw, sa,
                       bmask, pp, beta);
    CIMQ_TRY(check_hip("prep_params"));
  }
  return CIMQ_OK;
}

// layers whose backward is the separate v7 grad_x / grad_w pair: with CIMQ_LSQ_DEFER_GW the grad_w
// kernel leaves cimq_module_backward for cimq_module_backward_params (the fused / first-conv kernels
// and the general paths produce both in one pass)
static bool gw_deferrable(const Geo& g) {
  return g.variant == VAR_LIBRARY && v7_bwd(g) && !c1_plan(g).ok && !v9_plan(g).ok && !r6_bwd(g);
}

// parts: bit 0 grad_x (with everything a single-pass backward produces), bit 1 the deferred grad_w
// kernel of a gw_deferrable layer
int dispatch_bwd_any(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
                     const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused,
                     int parts = 3) {
  if (parts == 2 && !gw_deferrable(g)) return fail(CIMQ_EINVAL, "internal: grad_w alone on a single-pass backward");
  if (!v7_bwd(g)) {
    if (dense_plan(g)) {
      *lsq_fused = g.input_kind == CIMQ_INPUT_RAW_LSQ && dense_lsq_parts(g) > 0;
      return launch_dense_bwd(g, ctx, sw, gout, gx, ws, s, *lsq_fused ? x : nullptr, sa);
    }
    return launch_bwd_general(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
  }
  if (r6_bwd(g)) {  // the module path's w3a3 16-channel layers: recompute, no state words (cimq_r6.hip)
    if (!signed_act) return fail(CIMQ_EINVAL, "internal: the recompute backward needs signed_act");
    *lsq_fused = true;
    return launch_r6(g, r6_plan(g), ctx, sw, sa, signed_act, gout, x, gx, ws, s);
  }
  const PlanC1 pc = c1_plan(g);
  if (pc.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    *lsq_fused = lsq;
    return launch_c1(g, pc, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  }
  const Plan9 p9 = v9_plan(g);
  if (p9.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    *lsq_fused = lsq;
    return launch_fused(g, p9, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  }
  const Plan7 p7 = v7_plan(g);
  if (p7.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    *lsq_fused = lsq;
    if (g.NBP == 8) return launch_v7_n<8, 8>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
    if (g.nbw == 2) return launch_v7_n<2, 2>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
    return launch_v7_n<3, 3>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
  }
  if (dense_plan(g)) {
    *lsq_fused = g.input_kind == CIMQ_INPUT_RAW_LSQ && dense_lsq_parts(g) > 0;
    return launch_dense_bwd(g, ctx, sw, gout, gx, ws, s, *lsq_fused ? x : nullptr, sa);
  }
  return launch_bwd_general(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
}

int launch_reduce_galpha(const Geo& g, const uint8_t* ctx, uint8_t* ws, float cgrad, int init, const float* sw,
                         const float* sa, float* out, hipStream_t s) {
  WsLayout W = ws_layout(g);
  const long long nout = (long long)g.T * g.nbw * g.nba * g.Opad;
  hipLaunchKernelGGL(reduce_galpha_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, init ? W.nchunks : W.nchunks_bwd,
                     reinterpret_cast<const float*>(ws + W.ga_slab), params_of(g, const_cast<uint8_t*>(ctx)),
                     cgrad, init, sw, sa, (float)((double)g.B * g.P), (float)sqrt((double)g.qp), out);
  return check_hip("reduce_galpha");
}

// mask * cgrad * (slab sum over the backward's pixel chunks) -> [1, T, nbw, nba, 1, O]
int launch_reduce_slab(const Geo& g, const uint8_t* ctx, uint8_t* ws, size_t slab, float cgrad, const float* sw,
                       const float* sa, float* out, hipStream_t s) {
  WsLayout W = ws_layout(g);
  const long long nout = (long long)g.T * g.nbw * g.nba * g.Opad;
  hipLaunchKernelGGL(reduce_galpha_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, W.nchunks_bwd,
                     reinterpret_cast<const float*>(ws + slab), params_of(g, const_cast<uint8_t*>(ctx)), cgrad, 0,
                     sw, sa, 1.f, 1.f, out);
  return check_hip("reduce_slab");
}

// number of act-LSQ partials the backward leaves in ws (fused into the fused / v7 grad_x kernels,
// else one per lsq_act_bwd_kernel block)
int act_parts(const Geo& g) {
  if (v7_bwd(g)) {
    if (v9_plan(g).ok || c1_plan(g).ok || r6_bwd(g)) return g.B;
    const PlanX5 p5 = x5_plan(g);
    if (p5.ok) return p5.nblk;
    return g.B * v7_plan(g).v.nbands;
  }
  if (dense_plan(g) && g.input_kind == CIMQ_INPUT_RAW_LSQ && dense_lsq_parts(g) > 0) return dense_lsq_parts(g);
  int grid = cdiv(g.Nin, 256);
  return grid > kLsqParts ? kLsqParts : grid;
}

}  // namespace

extern "C" {

int cimq_abi_version(void) { return CIMQ_ABI_VERSION; }

const char* cimq_last_error(void) { return g_last_error.c_str(); }

int cimq_query_sizes(const cimq_conv_desc* d, cimq_sizes* out) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!out) return fail(CIMQ_EINVAL, "null output");
  out->ctx_bytes = ctx_layout(g).total;
  out->wprep_bytes = ctx_layout(g).wbytes;
  WsLayout W = ws_layout(g);
  out->fwd_workspace_bytes = W.total;
  out->bwd_workspace_bytes = W.total;
  Geo gm = g;
  gm.onchw = 1;  // the module entry points' layout: no state words where their backward recomputes
  out->module_ctx_bytes = ctx_layout(gm).total;
  return CIMQ_OK;
}

int cimq_forward(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                 const float* sw, const float* alpha_q, const int8_t* binary_mask,
                 const float* signed_act, float* out, void* ctx, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !out || !ctx)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && !alpha_q)
    return fail(CIMQ_EINVAL, "adc_bits 1 / 1.5 need alpha_q");
  if (g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN)
    return fail(CIMQ_EINVAL, "scale/shift ADC variants go through cimq_shift_forward");
  (void)ws;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, alpha_q, binary_mask, signed_act, c, s, true, true));
  return launch_fwd_any(g, c, sw, sa, out, nullptr, nullptr, s);
}

int cimq_shift_forward(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                       const float* sw, const float* alpha, const float* beta, const int8_t* binary_mask,
                       const float* signed_act, float* out, void* ctx, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (g.variant != VAR_SHIFT_ROUND && g.variant != VAR_SHIFT_SIGN)
    return fail(CIMQ_EINVAL, "cimq_shift_forward needs adc_variant CIMQ_ADC_SHIFT_ROUND or _SIGN");
  if (!x || !w_q || !sa || !sw || !alpha || !beta || !binary_mask || !signed_act || !out || !ctx)
    return fail(CIMQ_EINVAL, "null pointer argument");
  (void)ws;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, alpha, binary_mask, signed_act, c, s, true, true, beta));
  return launch_fwd_any(g, c, sw, sa, out, nullptr, nullptr, s);
}

int cimq_shift_backward(const cimq_conv_desc* d, const float* grad_out, const float* x, const float* sa,
                        const float* sw, const float* alpha, const float* beta, const int8_t* binary_mask,
                        const float* signed_act, const void* ctx, float* grad_x, float* grad_w,
                        float* grad_alpha, float* grad_beta, float* grad_sa, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  (void)alpha; (void)beta;
  if (g.variant != VAR_SHIFT_ROUND && g.variant != VAR_SHIFT_SIGN)
    return fail(CIMQ_EINVAL, "cimq_shift_backward needs adc_variant CIMQ_ADC_SHIFT_ROUND or _SIGN");
  if (!grad_out || !sa || !sw || !signed_act || !ctx || !grad_x || !grad_w || !grad_alpha || !grad_beta || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ && (!x || !grad_sa))
    return fail(CIMQ_EINVAL, "RAW_LSQ backward needs x and grad_sa");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  bool lsq_fused = false;
  if (v7_plan(g).ok && shift_stats_ok(g)) {
    // the shift ADC on the fast path (shift_fast): grad_x / grad_w from the state words as for the
    // library ADC (same STE mask), the step-size gradients from the statistics kernel
    if (!binary_mask) return fail(CIMQ_EINVAL, "null binary_mask");
    CIMQ_TRY(dispatch_bwd_any(g, c, sw, sa, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
    WsLayout W = ws_layout(g);
    const long long nout = (long long)g.T * g.FBT * 16 * g.Opad;
    hipLaunchKernelGGL(reduce_gw_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, W.nchunks_bwd,
                       reinterpret_cast<const float*>(w + W.gw_slab), sa, grad_w);
    CIMQ_TRY(check_hip("reduce_gw"));
    CIMQ_TRY(launch_shift_stats(g, c, sw, sa, grad_out, binary_mask, w, grad_alpha, grad_beta, s));
    if (g.input_kind == CIMQ_INPUT_RAW_LSQ) {
      if (!lsq_fused) return fail(CIMQ_EINVAL, "internal: unfused act-LSQ backward on the v7 path");
      hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, act_parts(g),
                         reinterpret_cast<float*>(w + W.lsq_part), grad_sa);
      CIMQ_TRY(check_hip("sum_partials"));
    }
    return CIMQ_OK;
  }
  CIMQ_TRY(launch_bwd_general(g, c, sw, sa, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
  WsLayout W = ws_layout(g);
  {
    const long long nout = (long long)g.T * g.FBT * 16 * g.Opad;
    hipLaunchKernelGGL(reduce_gw_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, W.nchunks_bwd,
                       reinterpret_cast<const float*>(w + W.gw_slab), sa, grad_w);
    CIMQ_TRY(check_hip("reduce_gw"));
  }
  // grad_alpha: sign variant sum sign * G / sqrt(numel * Qp) (scale_shift.py:283); round variant
  // without the factor (:491 commented out); grad_beta: sum over the clamped region / all of G
  const double numel = (double)g.B * g.T * g.nbw * g.nba * g.P * g.O;
  const float cgrad = g.variant == VAR_SHIFT_SIGN ? (float)(1.0 / sqrt(numel * (double)g.qp)) : 1.f;
  CIMQ_TRY(launch_reduce_slab(g, c, w, W.ga_slab, cgrad, sw, sa, grad_alpha, s));
  CIMQ_TRY(launch_reduce_slab(g, c, w, W.gb_slab, 1.f, sw, sa, grad_beta, s));
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ) {
    float* part = reinterpret_cast<float*>(w + W.lsq_part);
    int grid = cdiv(g.Nin, 256);
    if (grid > kLsqParts) grid = kLsqParts;
    hipLaunchKernelGGL(lsq_act_bwd_kernel, dim3(grid), dim3(256), 0, s, g.Nin, x, sa, g.lsq_qp, grad_x, part);
    CIMQ_TRY(check_hip("lsq_act_bwd"));
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, grid, part, grad_sa);
    CIMQ_TRY(check_hip("sum_partials"));
  }
  return CIMQ_OK;
}

int cimq_debug_partial_sums(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                            const float* sw, const float* alpha_q, const int8_t* binary_mask,
                            const float* signed_act, float* out, int32_t* ps_out, float* adc_out, void* ctx,
                            void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !out || !ps_out || !adc_out || !ctx)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && !alpha_q)
    return fail(CIMQ_EINVAL, "adc_bits 1 / 1.5 need alpha_q");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, alpha_q, binary_mask, signed_act, c, s, true, true));
  return launch_fwd_any(g, c, sw, sa, out, ps_out, adc_out, s);
}

int cimq_debug_state_codes(const cimq_conv_desc* d, const void* ctx, int8_t* code_out, uint8_t* pass_out,
                           void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!ctx || !code_out || !pass_out) return fail(CIMQ_EINVAL, "null pointer argument");
  if (!v7_plan(g).ok || c1_plan(g).ok)
    return fail(CIMQ_EUNSUPPORTED, "this layer's forward writes no v7 state words (the first conv's backward recomputes them)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  const long long n = (long long)g.T * g.M * g.O;
  hipLaunchKernelGGL(decode_state_kernel, dim3(std::min(cdiv(n, 256), 8192)), dim3(256), 0, s, g, g.NBP == 8 ? 1 : 0,
                     c + ctx_layout(g).st, code_out, pass_out);
  return check_hip("decode_state");
}

int cimq_debug_recompute_codes(const cimq_conv_desc* d, const float* x, const float* signed_act, const void* ctx,
                               void* st_scratch, int8_t* code_out, uint8_t* pass_out, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !signed_act || !ctx || !st_scratch || !code_out || !pass_out) return fail(CIMQ_EINVAL, "null pointer argument");
  g.onchw = 1;  // the module entry points' layer
  if (!r6_bwd(g)) return fail(CIMQ_EUNSUPPORTED, "this layer's module backward does not recompute the partial sums");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  const float* scal = reinterpret_cast<const float*>(wreg(g, c) + ctx_layout(g).lsq_scal);
  uint32_t* st = reinterpret_cast<uint32_t*>(st_scratch);
  CIMQ_TRY(launch_r6(g, r6_plan(g), c, scal + 1, scal, signed_act, nullptr, x, nullptr, nullptr, s, st));
  const long long n = (long long)g.T * g.M * g.O;
  hipLaunchKernelGGL(decode_state_kernel, dim3(std::min(cdiv(n, 256), 8192)), dim3(256), 0, s, g, 0,
                     reinterpret_cast<const uint8_t*>(st), code_out, pass_out);
  return check_hip("decode_state");
}

int cimq_backward(const cimq_conv_desc* d, const float* grad_out, const float* x, const float* sa,
                  const float* sw, const float* alpha_q, const int8_t* binary_mask,
                  const float* signed_act, const void* ctx, float* grad_x, float* grad_w,
                  float* grad_alpha, float* grad_sa, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  (void)alpha_q; (void)binary_mask;
  if (!grad_out || !sa || !sw || !signed_act || !ctx || !grad_x || !grad_w || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN)
    return fail(CIMQ_EINVAL, "scale/shift ADC variants go through cimq_shift_backward");
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ && (!x || !grad_sa))
    return fail(CIMQ_EINVAL, "RAW_LSQ backward needs x and grad_sa");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  bool lsq_fused = false;
  CIMQ_TRY(dispatch_bwd_any(g, c, sw, sa, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
  WsLayout W = ws_layout(g);
  {
    const long long nout = (long long)g.T * g.FBT * 16 * g.Opad;
    hipLaunchKernelGGL(reduce_gw_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, W.nchunks_bwd,
                       reinterpret_cast<const float*>(w + W.gw_slab), sa, grad_w);
    CIMQ_TRY(check_hip("reduce_gw"));
  }
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && grad_alpha) {
    const double numel = (double)g.B * g.T * g.nbw * g.nba * g.P * g.O;
    const float cgrad = (float)(1.0 / sqrt(numel * (double)g.qp));  // lsq.py:323,330
    CIMQ_TRY(launch_reduce_galpha(g, c, w, cgrad, 0, sw, sa, grad_alpha, s));
  }
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ) {
    float* part = reinterpret_cast<float*>(w + W.lsq_part);
    int nparts;
    if (lsq_fused) {
      nparts = act_parts(g);
    } else {
      int grid = cdiv(g.Nin, 256);
      if (grid > kLsqParts) grid = kLsqParts;
      hipLaunchKernelGGL(lsq_act_bwd_kernel, dim3(grid), dim3(256), 0, s, g.Nin, x, sa, g.lsq_qp, grad_x, part);
      CIMQ_TRY(check_hip("lsq_act_bwd"));
      nparts = grid;
    }
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, nparts, part, grad_sa);
    CIMQ_TRY(check_hip("sum_partials"));
  }
  return CIMQ_OK;
}

// the module backward's epilogue: grad_w + weight-LSQ backward, grad_alpha_cim, the step sizes;
// tail_blocks is the grid of its slab-sum launch
struct TailLaunch {
  int tail_blocks;
  Geo g;
  LsqArgs q;
  ModuleTail a;
};

static TailLaunch tail_job(const Geo& g, const LsqArgs& la, const cimq_lsq_desc* q, const uint8_t* c, uint8_t* w,
                      const float* weight, const float* alpha_cim, float* grad_weight, float* grad_alpha_act,
                      float* grad_alpha_weight, float* grad_alpha_cim, int gaq_ready = 0, bool packed = false) {
  const bool has_alpha = la.nbits_alpha > 0;
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  TailLaunch j;
  memset(&j, 0, sizeof(j));
  ModuleTail& a = j.a;
  a.gw_slab = reinterpret_cast<const float*>(w + W.gw_slab);
  a.ga_slab = reinterpret_cast<const float*>(w + W.ga_slab);
  a.scal = reinterpret_cast<const float*>(wreg(g, c) + L.lsq_scal);
  a.weight = weight;
  a.alpha_cim = alpha_cim;
  a.apart = reinterpret_cast<float*>(w + W.lsq_part);
  a.wpart = reinterpret_cast<float*>(w + W.wpart);
  a.gaq = reinterpret_cast<float*>(w + W.gaq);
  a.grad_weight = grad_weight;
  a.grad_alpha_act = grad_alpha_act;
  a.grad_alpha_w = grad_alpha_weight;
  a.grad_alpha_cim = grad_alpha_cim;
  a.ckj = params_of(g, const_cast<uint8_t*>(c)).ckj;
  a.cgrad = (float)(1.0 / sqrt((double)g.B * g.T * g.nbw * g.nba * g.P * g.O * (double)g.qp));  // lsq.py:323,330
  a.nchunks = W.nchunks_bwd;
  // few chunks and many outputs (the dense path's 8 chunks of a 1024 x 1024 layer): one output per
  // thread (16 k blocks of 64 outputs each took 67 us for 34 MB of slab)
  const long long nout_w = (long long)g.T * g.FBT * 16 * g.Opad;
  a.wide = (a.nchunks <= 16 && nout_w >= (1 << 18) && tune("WIDE_SLAB", 1)) ? 1 : 0;
  // otherwise, in a launch packed with the other layers' epilogues (cimq_pending_flush), float4
  // reads in 64-lane rows, 256 outputs per block (reduce_chunks4; 16-lane rows there: 85.7 -> 92.6
  // us); alone, one output per lane, 64 per block, so that a small layer still spreads over the chip
  // (a layer's tail 6.8 us against 9.1 with the float4 rows, cfg4)
  a.lpr = packed ? tune("TAIL_LPR_PACKED", 64) : tune("TAIL_LPR_SINGLE", 0);
  const int per_blk = a.wide ? 1024 : a.lpr == 0 ? 64 : 4 * a.lpr;
  a.nwb = cdiv(nout_w, per_blk);
  a.nga = has_alpha ? cdiv((long long)g.T * g.nbw * g.nba * g.Opad, per_blk) : 0;
  a.napart = act_parts(g);
  a.accum = (q->flags & CIMQ_LSQ_ACCUMULATE_GRADS) ? 1 : 0;
  a.gapart = (has_alpha && la.nalpha > kFinishInReg && tune("WIDE_TAIL", 1)) ? reinterpret_cast<float*>(w + W.gapart) : nullptr;
  a.gaq_ready = gaq_ready;
  j.g = g;
  j.q = la;
  j.tail_blocks = a.nwb + a.nga;
  return j;
}

static int launch_tail(const TailLaunch& j, hipStream_t s) {
  hipLaunchKernelGGL(module_bwd_tail_kernel, dim3(j.tail_blocks), dim3(1024), 0, s, j.g, j.q, j.a);
  return check_hip("module_bwd_tail");
}

static int launch_finish(const TailLaunch& j, hipStream_t s) {
  if (j.a.gapart)
    hipLaunchKernelGGL(module_bwd_finish_wide_kernel, dim3(cdiv(j.q.nalpha, 1024)), dim3(1024), 0, s, j.q, j.a);
  else
    hipLaunchKernelGGL(module_bwd_finish_kernel, dim3(1), dim3(1024), 0, s, j.q, j.a);
  return check_hip("module_bwd_finish");
}

static int module_tail(Geo g, const LsqArgs& la, const cimq_lsq_desc* q, const uint8_t* c, uint8_t* w,
                       const float* weight, const float* alpha_cim, float* grad_weight, float* grad_alpha_act,
                       float* grad_alpha_weight, float* grad_alpha_cim, hipStream_t s, int gaq_ready = 0) {
  const TailLaunch j = tail_job(g, la, q, c, w, weight, alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight,
                           grad_alpha_cim, gaq_ready);
  CIMQ_TRY(launch_tail(j, s));
  return launch_finish(j, s);
}

// cimq_pending (caller-owned host memory): the epilogues chained module backwards left behind,
// in call order, with each one's tail grid
constexpr int kPendingJobs = 32;
struct Pending {
  uint32_t magic;
  int n;
  int nblk[kPendingJobs];
  TailJob job[kPendingJobs];
};
static_assert(sizeof(Pending) <= sizeof(cimq_pending), "cimq_pending too small");
constexpr uint32_t kPendingMagic = 0x63696d70u;

static TailJob tail_job_of(const TailLaunch& c) {
  TailJob t;
  t.t = TailGeo{c.g.T, c.g.FBT, c.g.Opad, c.g.O, c.g.xbar, c.g.K, c.g.nbw, c.g.nba};
  t.q = c.q;
  t.a = c.a;
  return t;
}

// every pending tail (packs of kTailJobs per launch), then every finish: the launch boundary
// orders each finish after its tail's partials
static int pending_run(Pending* pd, hipStream_t s) {
  if (pd->magic != kPendingMagic) return CIMQ_OK;
  const int n = pd->n;
  pd->magic = 0;
  pd->n = 0;
  // the jobs with the longest blocks (most chunks per output) first, so that the grid does not
  // end on a round of them; the jobs are independent (pending_overlaps), their order is free
  int ord[kPendingJobs];
  for (int i = 0; i < n; ++i) ord[i] = i;
  if (tune("TAIL_SORT", 1))
    std::stable_sort(ord, ord + n, [&](int x, int y) { return pd->job[x].a.nchunks > pd->job[y].a.nchunks; });
  for (int i = 0; i < n;) {
    TailPack tp;
    tp.n = 0;
    int blk = 0;
    for (; i < n && tp.n < kTailJobs; ++i, ++tp.n) {
      tp.blk0[tp.n] = blk;
      tp.job[tp.n] = pd->job[ord[i]];
      blk += pd->nblk[ord[i]];
    }
    tp.blk0[tp.n] = blk;
    hipLaunchKernelGGL(module_tail_many_kernel, dim3(blk), dim3(1024), 0, s, tp);
    CIMQ_TRY(check_hip("module_tail_many"));
  }
  for (int i = 0; i < n;) {
    FinishPack fp;
    fp.n = 0;
    int blk = 0;
    for (; i < n && fp.n < kFinishJobs; ++i, ++fp.n) {
      const TailJob& t = pd->job[i];
      fp.blk0[fp.n] = blk;
      fp.job[fp.n].q = t.q;
      fp.job[fp.n].a = t.a;
      blk += t.a.gapart ? cdiv(t.q.nalpha, 1024) : 1;
    }
    fp.blk0[fp.n] = blk;
    hipLaunchKernelGGL(module_finish_many_kernel, dim3(blk), dim3(1024), 0, s, fp);
    CIMQ_TRY(check_hip("module_finish_many"));
  }
  return CIMQ_OK;
}

// a pending epilogue writing any gradient buffer this one writes (a layer run twice in one
// backward): the two must not share a launch
static bool pending_overlaps(const Pending* pd, const ModuleTail& a) {
  for (int i = 0; i < pd->n; ++i) {
    const ModuleTail& b = pd->job[i].a;
    if (b.grad_weight == a.grad_weight || b.grad_alpha_act == a.grad_alpha_act || b.grad_alpha_w == a.grad_alpha_w ||
        (a.grad_alpha_cim && b.grad_alpha_cim == a.grad_alpha_cim))
      return true;
  }
  return false;
}

static int lsq_args(const Geo& g, const cimq_lsq_desc* q, LsqArgs* a) {
  if (!q) return fail(CIMQ_EINVAL, "null LSQ descriptor");
  if (!(q->qn_w < q->qp_w) || !(q->gscale_a > 0.f) || !(q->gscale_w > 0.f))
    return fail(CIMQ_EINVAL, "bad LSQ descriptor");
  if (q->nbits_alpha < 0 || q->nbits_alpha > 16 || q->nbits_alpha == 1)
    return fail(CIMQ_EINVAL, "nbits_alpha must be 0 (no alpha_cim) or 2..16");
  a->qn_w = q->qn_w;
  a->qp_w = q->qp_w;
  a->gs_a = q->gscale_a;
  a->gs_w = q->gscale_w;
  a->nbits_alpha = q->nbits_alpha;
  a->nalpha = g.T * g.nbw * g.nba * g.O;
  if (q->flags & ~(CIMQ_LSQ_ACCUMULATE_GRADS | CIMQ_LSQ_SKIP_TAIL | CIMQ_LSQ_DEFER_GW))
    return fail(CIMQ_EINVAL, "unknown LSQ flags 0x%x", q->flags);
  return CIMQ_OK;
}

// the module prologue's arguments: activation side into ctx c, weight side into wreg(g, c)
static ModulePrep module_prep_args(const Geo& g, const float* x, const float* weight, const float* alpha_act,
                                   const float* alpha_weight, const float* alpha_cim, const int8_t* binary_mask,
                                   const float* signed_act, uint8_t* c, int* nwblk) {
  CtxLayout L = ctx_layout(g);
  uint8_t* wr = wreg(g, c);
  const Plan7 p7 = v7_plan(g);
  ModulePrep a;
  memset(&a, 0, sizeof(a));
  a.x = x;
  a.alpha_act = alpha_act;
  a.alpha_w = alpha_weight;
  a.weight = weight;
  a.alpha_cim = alpha_cim;
  a.signed_act = signed_act;
  a.bmask = binary_mask;
  a.xcf = c ? c + L.xcode : nullptr;
  a.xcb = c ? c + L.xhat : nullptr;
  a.wfrag = reinterpret_cast<v4i*>(wr + L.wfrag);
  a.wgx = reinterpret_cast<v4i*>(wr + L.wgx);
  a.wcy = reinterpret_cast<v4i*>(wr + L.wcy);
  a.pp = params_of(g, c);
  a.scal = reinterpret_cast<float*>(wr + L.lsq_scal);
  a.nact_blocks = (int)std::min<long long>(cdiv(g.Nin, 4 * 256), act_blocks());
  a.nwf = g.T * g.KS * g.NBLK * 64;
  a.nwg = p7.ok ? 0 : g.T * g.FBT * g.NKS * 64;       // general / dense grad_x operand
  a.ncpbt = p7.ok ? p7.v.NCPBT : 1;
  a.nwc = p7.ok ? g.T * p7.v.NCPBT * g.NKS * 64 : 0;  // v8 grad_x operand
  const Plan5 p5 = f5_plan(g);
  a.wf5 = reinterpret_cast<v4i*>(wr + L.wf5);
  a.f5 = f5w_of(p5.v);
  a.nw5 = (int)f5_frag_items(g, p5);  // cim_fwd5_kernel's weight operand
  a.wg5 = reinterpret_cast<v4i*>(wr + L.wg5);
  a.nwx5 = (int)(x5_frag_bytes(g) / 16);  // cim_bwd_gx5_kernel's weight operand
  a.wx6 = reinterpret_cast<v4i*>(wr + L.wx6);
  a.nwx6 = (int)(r6_frag_bytes(g) / 16);  // cim_bwd_r6_kernel's gx operand
  a.npp = g.T * g.nba * g.nbw * g.Opad + g.nbw * g.nba;
  *nwblk = std::max(1, std::min(cdiv(a.nwf + a.nwg + a.nwc + a.nw5 + a.nwx5 + a.nwx6 + a.npp, 256), 1024));
  return a;
}

// the checks every module entry point shares; applies q->wprep.  shift: the cimq_module_shift_*
// entry points (the shift ADC on the fast path, no prepared weight side)
static int module_geo(const cimq_conv_desc* d, const cimq_lsq_desc* q, Geo* g, LsqArgs* la, bool shift = false) {
  CIMQ_TRY(make_geo(d, g));
  if (g->input_kind != CIMQ_INPUT_RAW_LSQ) return fail(CIMQ_EINVAL, "module entry points take the raw activation");
  if (shift) {
    if (g->variant != VAR_SHIFT_ROUND || !v7_plan(*g).ok || !shift_stats_ok(*g))
      return fail(CIMQ_EUNSUPPORTED, "cimq_module_shift_*: the shift ADC on a fast-path layer only "
                                     "(adc_variant CIMQ_ADC_SHIFT_ROUND, adc 1.5, 2 or 3 equal slices, v7 shapes)");
    if (q && q->wprep) return fail(CIMQ_EINVAL, "cimq_module_shift_*: no prepared weight side");
  } else if (g->variant == VAR_SHIFT_ROUND || g->variant == VAR_SHIFT_SIGN) {
    return fail(CIMQ_EUNSUPPORTED, "the module entry points run the library / stochastic ADC only");
  }
  CIMQ_TRY(lsq_args(*g, q, la));
  g->wbase = reinterpret_cast<const unsigned char*>(q->wprep);
  return CIMQ_OK;
}

static int module_forward_impl(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                               const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                               const float* beta_cim, const int8_t* binary_mask, const float* signed_act, float* out,
                               void* ctx, void* ws, void* stream) {
  Geo g;
  LsqArgs la;
  CIMQ_TRY(module_geo(d, q, &g, &la, beta_cim != nullptr));
  if (!x || !weight || !alpha_act || !alpha_weight || !binary_mask || !signed_act || !out || !ctx || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || la.nbits_alpha == 0)) return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CtxLayout L = ctx_layout(g);
  float* scal = reinterpret_cast<float*>(wreg(g, c) + L.lsq_scal);
  {
    int nwblk;
    ModulePrep a = module_prep_args(g, x, weight, alpha_act, alpha_weight, has_alpha ? alpha_cim : nullptr,
                                    binary_mask, signed_act, c, &nwblk);
    if (beta_cim) {  // the shift ADC: beta into the thresholds, and the per-channel beta sums
      a.beta = beta_cim;
      a.npp += g.Opad;
      nwblk = std::max(1, std::min(cdiv(a.nwf + a.nwg + a.nwc + a.nw5 + a.nwx5 + a.nwx6 + a.npp, 256), 1024));
    }
    if (g.wbase) nwblk = 0;  // weight side prepared (cimq_module_prepare): the activation quantiser only
    if (fwd_actq_ok(g)) a.nact_blocks = 0;  // the forward's row staging quantises (stage_rows_q)
    if (a.nact_blocks + nwblk == 0) goto prepared;
    {
    const int slot = prof_begin(KID_PREP_ACT, g, s);
    ModulePrep aw = a;
    if (nwblk > 0 && has_alpha && la.nalpha > kFinishInReg && tune("WIDE_PREP", 1)) {  // wide alpha_cim: its max / min in 64 blocks first
      float* part = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) + ws_layout(g).lsq_part);
      hipLaunchKernelGGL(alpha_minmax_kernel, dim3(64), dim3(256), 0, s, alpha_cim, la.nalpha, part);
      aw.amm = part;
      aw.namm = 64;
    }
    hipLaunchKernelGGL(prep_module_kernel, dim3(a.nact_blocks + nwblk), dim3(256), 0, s, g, la, aw);
    prof_end(slot, s);
    CIMQ_TRY(check_hip("prep_module"));
    }
  }
prepared:
  const Plan3 p = v3_plan(g);
  if (p.ok) {
    g.onchw = 1;
    const ActQ aq{x, signed_act};
    return launch_fwd_any(g, c, scal + 1, scal, out, nullptr, nullptr, s, fwd_actq_ok(g) ? &aq : nullptr);
  }
  if (dense_plan(g)) return launch_fwd_any(g, c, scal + 1, scal, out, nullptr, nullptr, s);  // P = 1: NCHW is [B, P, O]
  // general kernels write [B, P, O]; the module returns NCHW
  WsLayout W = ws_layout(g);
  float* bpo = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) + W.bpo);
  CIMQ_TRY(launch_fwd_any(g, c, scal + 1, scal, bpo, nullptr, nullptr, s));
  hipLaunchKernelGGL(bpo_to_nchw_kernel, dim3(std::min(cdiv((long long)g.M * g.O, 256), 8192)), dim3(256), 0, s,
                     g, bpo, out);
  return check_hip("bpo_to_nchw");
}

int cimq_module_forward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                        const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                        const int8_t* binary_mask, const float* signed_act, float* out, void* ctx, void* ws,
                        void* stream) {
  return module_forward_impl(d, q, x, weight, alpha_act, alpha_weight, alpha_cim, nullptr, binary_mask, signed_act,
                             out, ctx, ws, stream);
}

int cimq_module_route(const cimq_conv_desc* d, int* route) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!route) return fail(CIMQ_EINVAL, "null route");
  if (g.input_kind != CIMQ_INPUT_RAW_LSQ) return fail(CIMQ_EINVAL, "module entry points take the raw activation");
  // the ctx / workspace layouts must not depend on state the entry points set only at launch (the
  // module path's NCHW flag): cimq_query_sizes, the prologue and the kernels compute them separately
  // (the module path's ctx may END earlier -- no state-word region where its backward recomputes them -- and
  // its backward's chunk / partial counts are that backward's; every offset and the workspace size agree)
  {
    Geo g1 = g;
    g1.onchw = 1;
    const CtxLayout a = ctx_layout(g), c = ctx_layout(g1);
    const WsLayout w0 = ws_layout(g), w1 = ws_layout(g1);
    if (c.total > a.total || a.wbytes != c.wbytes || a.st != c.st || a.wg5 != c.wg5 || a.wx6 != c.wx6 ||
        w0.total != w1.total || w0.gw_slab != w1.gw_slab || w0.ga_slab != w1.ga_slab || w0.lsq_part != w1.lsq_part ||
        (!r6_bwd(g1) && (w0.nchunks_bwd != w1.nchunks_bwd || act_parts(g) != act_parts(g1))))
      return fail(CIMQ_EINVAL, "internal: layouts depend on the output layout flag");
  }
  g.onchw = 1;  // the module path's layout (as module_forward_impl sets it)
  route[0] = route[1] = route[2] = CIMQ_ROUTE_GENERAL;
  // forward (module_forward_impl -> launch_fwd_any -> launch_fwd)
  if (v3_plan(g).ok) {
    route[0] = (fwd_actq_ok(g) && f5_plan(g).ok) ? CIMQ_ROUTE_FWD5 : CIMQ_ROUTE_V3;
  } else if (dense_plan(g)) {
    route[0] = CIMQ_ROUTE_DENSE;
  }
  // backward (dispatch_bwd_any)
  if (v7_bwd(g)) {
    if (r6_bwd(g)) {
      route[1] = route[2] = CIMQ_ROUTE_R6;
    } else if (c1_plan(g).ok) {
      route[1] = route[2] = CIMQ_ROUTE_C1;
    } else if (v9_plan(g).ok) {
      route[1] = route[2] = CIMQ_ROUTE_FUSED;
    } else if (v7_plan(g).ok) {
      route[1] = x5_plan(g).ok ? CIMQ_ROUTE_GX5 : CIMQ_ROUTE_V7;
      route[2] = g5_plan(g).ok ? CIMQ_ROUTE_GW5 : CIMQ_ROUTE_V7;
    }
  } else if (dense_plan(g)) {
    route[1] = route[2] = CIMQ_ROUTE_DENSE;
  }
  return CIMQ_OK;
}

int cimq_module_shift_supported(const cimq_conv_desc* d) {
  Geo g;
  if (make_geo(d, &g) != CIMQ_OK) return 0;
  return (g.input_kind == CIMQ_INPUT_RAW_LSQ && g.variant == VAR_SHIFT_ROUND && v7_plan(g).ok && shift_stats_ok(g))
             ? 1 : 0;
}

int cimq_module_shift_forward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                              const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                              const float* beta_cim, const int8_t* binary_mask, const float* signed_act, float* out,
                              void* ctx, void* ws, void* stream) {
  if (!beta_cim || !alpha_cim) return fail(CIMQ_EINVAL, "cimq_module_shift_forward needs alpha_cim and beta_cim");
  return module_forward_impl(d, q, x, weight, alpha_act, alpha_weight, alpha_cim, beta_cim, binary_mask, signed_act,
                             out, ctx, ws, stream);
}

static int module_backward_impl(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                                const float* x, const float* weight, const float* alpha_act,
                                const float* alpha_weight, const float* alpha_cim, const int8_t* binary_mask,
                                const float* signed_act, const void* ctx, float* grad_x, float* grad_weight,
                                float* grad_alpha_act, float* grad_alpha_weight, float* grad_alpha_cim, void* ws,
                                Pending* pend, void* stream) {
  Geo g;
  LsqArgs la;
  CIMQ_TRY(module_geo(d, q, &g, &la));
  (void)alpha_act; (void)alpha_weight; (void)binary_mask;
  if (!grad_out || !x || !weight || !signed_act || !ctx || !grad_x || !grad_weight || !grad_alpha_act ||
      !grad_alpha_weight || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || !grad_alpha_cim || la.nbits_alpha == 0))
    return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim and grad_alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const float* scal = reinterpret_cast<const float*>(wreg(g, c) + L.lsq_scal);
  const float* sa = scal;
  const float* sw = scal + 1;
  const Plan3 p = v3_plan(g);
  const float* gsrc = grad_out;
  if (p.ok) {
    g.onchw = 1;
  } else if (!dense_plan(g)) {  // (P = 1: NCHW grad_out is already [B, P, O])
    float* bpo = reinterpret_cast<float*>(w + W.bpo);
    hipLaunchKernelGGL(nchw_to_bpo_kernel, dim3(std::min(cdiv((long long)g.M * g.O, 256), 8192)), dim3(256), 0, s,
                       g, grad_out, bpo);
    CIMQ_TRY(check_hip("nchw_to_bpo"));
    gsrc = bpo;
  }
  bool lsq_fused = false;
  const bool defer = (q->flags & CIMQ_LSQ_DEFER_GW) && gw_deferrable(g);
  CIMQ_TRY(dispatch_bwd_any(g, c, sw, sa, signed_act, gsrc, x, grad_x, w, s, &lsq_fused, defer ? 1 : 3));
  // the act-LSQ partials: fused into the fast grad_x kernel, a separate pass otherwise
  float* part = reinterpret_cast<float*>(w + W.lsq_part);
  int nparts;
  if (lsq_fused) {
    nparts = act_parts(g);
  } else {
    int grid = cdiv(g.Nin, 256);
    if (grid > kLsqParts) grid = kLsqParts;
    hipLaunchKernelGGL(lsq_act_bwd_kernel, dim3(grid), dim3(256), 0, s, g.Nin, x, sa, g.lsq_qp, grad_x, part);
    CIMQ_TRY(check_hip("lsq_act_bwd"));
    nparts = grid;
  }
  if (nparts != act_parts(g)) return fail(CIMQ_EINVAL, "internal: act-LSQ partial count mismatch");
  if (pend) {
    // the epilogue joins the pending ones: cimq_pending_flush (or a full list, or a layer whose
    // gradient buffers a pending one writes) launches them all, packed.  Until then this layer's
    // ws (its grad_w slabs: B per-image slabs on the fused / first-conv paths, ~37.7 MB for a
    // 64-channel ResNet-20 layer at B = 256) stays in use: the chain's peak memory is up to
    // kPendingJobs workspaces (cimq.h states it; bench.Trainer flushes per segment at world > 1)
    const TailLaunch j = tail_job(g, la, q, c, w, weight, alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight,
                                  grad_alpha_cim, 0, true);
    if (pend->magic == kPendingMagic && (pend->n == kPendingJobs || pending_overlaps(pend, j.a)))
      CIMQ_TRY(pending_run(pend, s));
    if (pend->magic != kPendingMagic) pend->n = 0;
    pend->nblk[pend->n] = j.tail_blocks;
    pend->job[pend->n] = tail_job_of(j);
    ++pend->n;
    pend->magic = kPendingMagic;
    return CIMQ_OK;
  }
  // the caller runs cimq_module_backward_tail / _params
  if (q->flags & (CIMQ_LSQ_SKIP_TAIL | CIMQ_LSQ_DEFER_GW)) return CIMQ_OK;
  return module_tail(g, la, q, c, w, weight, alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight,
                     grad_alpha_cim, s);
}

int cimq_module_backward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out, const float* x,
                         const float* weight, const float* alpha_act, const float* alpha_weight,
                         const float* alpha_cim, const int8_t* binary_mask, const float* signed_act,
                         const void* ctx, float* grad_x, float* grad_weight, float* grad_alpha_act,
                         float* grad_alpha_weight, float* grad_alpha_cim, void* ws, void* stream) {
  return module_backward_impl(d, q, grad_out, x, weight, alpha_act, alpha_weight, alpha_cim, binary_mask, signed_act,
                              ctx, grad_x, grad_weight, grad_alpha_act, grad_alpha_weight, grad_alpha_cim, ws,
                              nullptr, stream);
}

int cimq_module_backward_chain(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                               const float* x, const float* weight, const float* alpha_act,
                               const float* alpha_weight, const float* alpha_cim, const int8_t* binary_mask,
                               const float* signed_act, const void* ctx, float* grad_x, float* grad_weight,
                               float* grad_alpha_act, float* grad_alpha_weight, float* grad_alpha_cim, void* ws,
                               cimq_pending* pending, void* stream) {
  if (!pending) return fail(CIMQ_EINVAL, "null cimq_pending");
  Pending* pd = reinterpret_cast<Pending*>(pending);
  if (pd->magic != 0 && pd->magic != kPendingMagic) return fail(CIMQ_EINVAL, "cimq_pending not initialised (zero it)");
  if (q && (q->flags & (CIMQ_LSQ_SKIP_TAIL | CIMQ_LSQ_DEFER_GW)))
    return fail(CIMQ_EINVAL, "CIMQ_LSQ_SKIP_TAIL / _DEFER_GW with the chained backward");
  return module_backward_impl(d, q, grad_out, x, weight, alpha_act, alpha_weight, alpha_cim, binary_mask, signed_act,
                              ctx, grad_x, grad_weight, grad_alpha_act, grad_alpha_weight, grad_alpha_cim, ws, pd,
                              stream);
}

int cimq_pending_jobs(const cimq_pending* pending) {
  const Pending* pd = reinterpret_cast<const Pending*>(pending);
  return (pd && pd->magic == kPendingMagic) ? pd->n : 0;
}

int cimq_pending_flush(cimq_pending* pending, void* stream) {
  if (!pending) return fail(CIMQ_EINVAL, "null cimq_pending");
  Pending* pd = reinterpret_cast<Pending*>(pending);
  if (pd->magic != 0 && pd->magic != kPendingMagic) return fail(CIMQ_EINVAL, "cimq_pending not initialised (zero it)");
  return pending_run(pd, reinterpret_cast<hipStream_t>(stream));
}

int cimq_module_backward_tail(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* weight,
                              const float* alpha_cim, const void* ctx, float* grad_weight, float* grad_alpha_act,
                              float* grad_alpha_weight, float* grad_alpha_cim, void* ws, void* stream) {
  Geo g;
  LsqArgs la;
  CIMQ_TRY(module_geo(d, q, &g, &la));
  if (!weight || !ctx || !grad_weight || !grad_alpha_act || !grad_alpha_weight || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || !grad_alpha_cim || la.nbits_alpha == 0))
    return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim and grad_alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  return module_tail(g, la, q, reinterpret_cast<const uint8_t*>(ctx), reinterpret_cast<uint8_t*>(ws), weight,
                     alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight, grad_alpha_cim,
                     reinterpret_cast<hipStream_t>(stream));
}

int cimq_module_backward_params(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                                const float* weight, const float* alpha_cim, const void* ctx, float* grad_weight,
                                float* grad_alpha_act, float* grad_alpha_weight, float* grad_alpha_cim, void* ws,
                                void* stream) {
  Geo g;
  LsqArgs la;
  CIMQ_TRY(module_geo(d, q, &g, &la));
  if (!(q->flags & CIMQ_LSQ_DEFER_GW)) return fail(CIMQ_EINVAL, "cimq_module_backward_params needs CIMQ_LSQ_DEFER_GW");
  if (!grad_out || !weight || !ctx || !grad_weight || !grad_alpha_act || !grad_alpha_weight || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || !grad_alpha_cim || la.nbits_alpha == 0))
    return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim and grad_alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  if (v3_plan(g).ok) g.onchw = 1;  // as module_backward_impl: the backward that ran was the module path's
  if (gw_deferrable(g)) {
    // the grad_w kernel cimq_module_backward left out (grad_out NCHW, as the v7 path reads it there)
    const float* scal = reinterpret_cast<const float*>(wreg(g, c) + ctx_layout(g).lsq_scal);
    bool lsq_fused = false;
    CIMQ_TRY(dispatch_bwd_any(g, c, scal + 1, scal, nullptr, grad_out, nullptr, nullptr, w, s, &lsq_fused, 2));
  }
  return module_tail(g, la, q, c, w, weight, alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight,
                     grad_alpha_cim, s);
}

int cimq_module_shift_backward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out,
                               const float* x, const float* weight, const float* alpha_act,
                               const float* alpha_weight, const float* alpha_cim, const float* beta_cim,
                               const int8_t* binary_mask, const float* signed_act, const void* ctx, float* grad_x,
                               float* grad_weight, float* grad_alpha_act, float* grad_alpha_weight,
                               float* grad_alpha_cim, float* grad_beta_cim, void* ws, void* stream) {
  Geo g;
  LsqArgs la;
  CIMQ_TRY(module_geo(d, q, &g, &la, true));
  (void)alpha_act; (void)alpha_weight; (void)beta_cim;
  if (!grad_out || !x || !weight || !alpha_cim || !binary_mask || !signed_act || !ctx || !grad_x || !grad_weight ||
      !grad_alpha_act || !grad_alpha_weight || !grad_alpha_cim || !grad_beta_cim || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (la.nbits_alpha == 0) return fail(CIMQ_EINVAL, "the shift ADC needs alpha_cim (nbits_alpha > 0)");
  if (q->flags & (CIMQ_LSQ_SKIP_TAIL | CIMQ_LSQ_DEFER_GW))
    return fail(CIMQ_EINVAL, "CIMQ_LSQ_SKIP_TAIL / _DEFER_GW with cimq_module_shift_backward");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const float* scal = reinterpret_cast<const float*>(wreg(g, c) + L.lsq_scal);
  g.onchw = 1;
  bool lsq_fused = false;
  CIMQ_TRY(dispatch_bwd_any(g, c, scal + 1, scal, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
  if (!lsq_fused)
    return fail(CIMQ_EINVAL, "internal: act-LSQ partials off the fused grad_x");
  // d loss / d alpha_q and grad_beta (scale_shift.py:488-501) from the statistics kernel, then the
  // module epilogue (grad_w + weight-LSQ backward, alpha_cim's quantiser, the step sizes) from there
  CIMQ_TRY(launch_shift_stats(g, c, scal + 1, scal, grad_out, binary_mask, w, reinterpret_cast<float*>(w + W.gaq),
                              grad_beta_cim, s, (q->flags & CIMQ_LSQ_ACCUMULATE_GRADS) ? 1 : 0));
  return module_tail(g, la, q, c, w, weight, alpha_cim, grad_weight, grad_alpha_act, grad_alpha_weight,
                     grad_alpha_cim, s, 1);
}

int cimq_module_prepare(int n, const cimq_prepare_item* items, void* stream) {
  if (n < 0 || (n > 0 && !items)) return fail(CIMQ_EINVAL, "bad prepare item list");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  PrepPack pk;
  memset(&pk, 0, sizeof(pk));
  int grid = 0;
  for (int i = 0; i < n; ++i) {
    const cimq_prepare_item& it = items[i];
    Geo g;
    LsqArgs la;
    if (!it.lsq) return fail(CIMQ_EINVAL, "item %d: null LSQ descriptor", i);
    cimq_lsq_desc q = *it.lsq;
    q.flags = 0;
    q.wprep = it.wprep;
    CIMQ_TRY(module_geo(it.desc, &q, &g, &la));
    if (!it.weight || !it.alpha_act || !it.alpha_weight || !it.binary_mask || !it.wprep)
      return fail(CIMQ_EINVAL, "item %d: null pointer argument", i);
    const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
    if (has_alpha && (!it.alpha_cim || la.nbits_alpha == 0))
      return fail(CIMQ_EINVAL, "item %d: adc 1 / 1.5 need alpha_cim", i);
    if (!has_alpha) la.nbits_alpha = 0;
    PrepJob& j = pk.job[pk.n];
    j.g = g;
    j.q = la;
    j.a = module_prep_args(g, nullptr, it.weight, it.alpha_act, it.alpha_weight, has_alpha ? it.alpha_cim : nullptr,
                           it.binary_mask, nullptr, nullptr, &j.nwblk);
    j.a.nact_blocks = 0;
    pk.blk0[pk.n] = grid;
    grid += j.nwblk;
    ++pk.n;
    if (pk.n == kPrepJobs || i == n - 1) {
      pk.blk0[pk.n] = grid;
      hipLaunchKernelGGL(prep_weights_many_kernel, dim3(grid), dim3(256), 0, s, pk);
      CIMQ_TRY(check_hip("prep_weights_many"));
      memset(&pk, 0, sizeof(pk));
      grid = 0;
    }
  }
  return CIMQ_OK;
}

int cimq_alpha_init(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                    const float* sw, const int8_t* binary_mask, const float* signed_act,
                    float* alpha_init, void* ctx, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !alpha_init || !ctx || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (!(g.mode == ADC_SIGN || g.mode == ADC_TERNARY))
    return fail(CIMQ_EINVAL, "alpha_cim exists only for adc_bits 1 / 1.5");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  // the init path slices activations unsigned (lsq.py:51); the fused-LSQ codes are never
  // negative there, so the signed and unsigned slicings coincide
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, nullptr, binary_mask, signed_act, c, s, false, false));
  {
    Params pp = params_of(g, c);
    if (hipMemsetAsync(pp.flags, 0, 16, s) != hipSuccess) return fail(CIMQ_EHIP, "memset flags");
  }
  CIMQ_TRY(launch_alpha_init_sums(g, c, sw, sa, signed_act, w, s));
  return launch_reduce_galpha(g, c, w, 0.f, 1, sw, sa, alpha_init, s);
}

// dist.FlatSGD's update: four elements per thread (the flat buffers are 256-B aligned torch
// allocations), the last n % 4 by thread 0 of block 0
__global__ __launch_bounds__(256) void flat_sgd_kernel(long long n, float* __restrict__ p, float* __restrict__ g,
                                                       float* __restrict__ buf, const float* __restrict__ wd, float lr,
                                                       float mom, int first, int zero_grad) {
  auto upd = [&](float pv, float gv, float bv, float w, float& po, float& bo) {
    const float d = gv + w * pv;
    bo = first ? d : mom * bv + d;
    po = pv - lr * bo;
  };
  const long long n4 = n >> 2;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += (long long)gridDim.x * blockDim.x) {
    const float4 pv = reinterpret_cast<const float4*>(p)[t], gv = reinterpret_cast<const float4*>(g)[t];
    const float4 wv = reinterpret_cast<const float4*>(wd)[t];
    const float4 bv = first ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4*>(buf)[t];
    float4 po, bo;
    upd(pv.x, gv.x, bv.x, wv.x, po.x, bo.x);
    upd(pv.y, gv.y, bv.y, wv.y, po.y, bo.y);
    upd(pv.z, gv.z, bv.z, wv.z, po.z, bo.z);
    upd(pv.w, gv.w, bv.w, wv.w, po.w, bo.w);
    reinterpret_cast<float4*>(p)[t] = po;
    reinterpret_cast<float4*>(buf)[t] = bo;
    if (zero_grad) reinterpret_cast<float4*>(g)[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (long long e = n4 << 2; e < n; ++e) {
      upd(p[e], g[e], first ? 0.f : buf[e], wd[e], p[e], buf[e]);
      if (zero_grad) g[e] = 0.f;
    }
}

int cimq_flat_sgd(long long n, float* param, float* grad, float* buf, const float* wd, float lr, float momentum,
                  int first, int zero_grad, void* stream) {
  if (n < 0) return fail(CIMQ_EINVAL, "negative element count");
  if (n == 0) return CIMQ_OK;
  if (!param || !grad || !buf || !wd) return fail(CIMQ_EINVAL, "null pointer argument");
  for (const void* q : {(const void*)param, (const void*)grad, (const void*)buf, (const void*)wd})
    if (reinterpret_cast<uintptr_t>(q) % 16 != 0) return fail(CIMQ_EINVAL, "cimq_flat_sgd: buffers must be 16-byte aligned");
  const long long n4 = n >> 2;
  const int grid = (int)std::max<long long>(1, std::min<long long>(cdiv(n4, 256), 2048));
  hipLaunchKernelGGL(flat_sgd_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), n, param, grad,
                     buf, wd, lr, momentum, first ? 1 : 0, zero_grad ? 1 : 0);
  return check_hip("flat_sgd");
}

int cimq_profile_start(int kernel_id, int max_launches) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.ev) return fail(CIMQ_EINVAL, "profiler already running");
  if (kernel_id < KID_FWD || kernel_id > KID_LAST || max_launches <= 0)
    return fail(CIMQ_EINVAL, "bad profiler arguments");
  p.ev = new hipEvent_t[2 * (size_t)max_launches];
  p.lb = new double[(size_t)max_launches];
  p.lf = new double[(size_t)max_launches];
  p.lm = new double[(size_t)max_launches];
  for (int i = 0; i < 2 * max_launches; ++i) {
    if (hipEventCreate(&p.ev[i]) != hipSuccess) {
      for (int k = 0; k < i; ++k) (void)hipEventDestroy(p.ev[k]);
      delete[] p.ev;
      delete[] p.lb;
      delete[] p.lf;
      delete[] p.lm;
      p.ev = nullptr;
      p.lb = p.lf = p.lm = nullptr;
      return fail(CIMQ_EHIP, "hipEventCreate");
    }
  }
  p.kid = kernel_id;
  p.cap = max_launches;
  p.n = 0;
  p.bytes = p.flops = 0;
  return CIMQ_OK;
}

int cimq_profile_read(int cap, double* ms, double* algo_bytes, double* algo_flops, double* mfma_ops, int* launches) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (!p.ev) return fail(CIMQ_EINVAL, "profiler not running");
  if (cap < 0 || (cap > 0 && (!ms || !algo_bytes || !algo_flops || !mfma_ops))) return fail(CIMQ_EINVAL, "bad buffers");
  const int n = std::min(cap, p.n);
  for (int i = 0; i < n; ++i) {
    float t = 0;
    if (hipEventSynchronize(p.ev[2 * i + 1]) != hipSuccess || hipEventElapsedTime(&t, p.ev[2 * i], p.ev[2 * i + 1]) != hipSuccess)
      return fail(CIMQ_EHIP, "hipEventElapsedTime");
    ms[i] = t;
    algo_bytes[i] = p.lb[i];
    algo_flops[i] = p.lf[i];
    mfma_ops[i] = p.lm[i];
  }
  if (launches) *launches = p.n;
  return CIMQ_OK;
}

int cimq_profile_stop(double* total_ms, int* launches, double* algo_bytes, double* algo_flops) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (!p.ev) return fail(CIMQ_EINVAL, "profiler not running");
  double tot = 0;
  int rc = CIMQ_OK;
  for (int i = 0; i < p.n; ++i) {
    float ms = 0;
    if (hipEventSynchronize(p.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, p.ev[2 * i], p.ev[2 * i + 1]) != hipSuccess) {
      rc = fail(CIMQ_EHIP, "hipEventElapsedTime");
      break;
    }
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = p.n;
  if (algo_bytes) *algo_bytes = p.bytes;
  if (algo_flops) *algo_flops = p.flops;
  for (int i = 0; i < 2 * p.cap; ++i) (void)hipEventDestroy(p.ev[i]);
  delete[] p.ev;
  delete[] p.lb;
  delete[] p.lf;
  delete[] p.lm;
  p.ev = nullptr;
  p.lb = p.lf = p.lm = nullptr;
  p.kid = KID_NONE;
  p.cap = p.n = 0;
  return rc;
}

}  // extern "C"

// cimq_part_bwd.hip -- backward launch sequences for layers outside the v7 plan (v5 / v6
// state-word kernels and the general recompute kernels, lsq.py:244-386) and the alpha_cim
// initialisation sums (lsq.py:35-87).  Own translation unit of libcimq.so.
#define CIMQ_TU_BWD
#include "cimq_host.h"

namespace cimq {

template <int NBP, int FBMAX, bool INIT>
int launch_gw(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
              const float* gout, uint8_t* ws, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const Plan3 p = v3_plan(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  dim3 grid(W.nchunks, g.T, (g.OB16 + 1) / 2);
  const int slot = INIT ? -1 : prof_begin(KID_BWD_GW, g, s);
  if (p.ok && !INIT) {
    auto kern = g.nbw <= 4 ? cim_bwd_gw_v5_kernel<NBP, FBMAX, 4> : cim_bwd_gw_v5_kernel<NBP, FBMAX, 8>;
    CIMQ_TRY(set_lds(kern, p.lds_gw));
    dim3 grid16(W.nchunks, g.T, g.OB16);
    hipLaunchKernelGGL(kern, grid16, dim3(256), p.lds_gw, s, g, p.v, ctx + L.st, ctx + L.xhat, pp, gout, W.rows,
                       reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
    prof_end(slot, s);
    return check_hip("cim_bwd_gw_v5");
  }
  if constexpr (INIT) {
    // alpha_cim init sums (the v3 kernel runs only in this mode)
    if (p.ok && p.lds_init <= kLdsMax - 512) {
      const size_t lds = p.lds_init;
      auto kern = g.KS == 1 ? cim_bwd_gw_v3_kernel<NBP, 1, FBMAX, true> : cim_bwd_gw_v3_kernel<NBP, 2, FBMAX, true>;
      CIMQ_TRY(set_lds(kern, lds));
      hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, p.v, ctx + L.xcode, ctx + L.xhat,
                         reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag), pp, sw, sa, gout, W.rows,
                         reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
      return check_hip("cim_bwd_gw_v3(init)");
    }
  }
  {
    const size_t lds = lds_gw(g);
    auto kern = cim_bwd_gw_kernel<NBP, FBMAX, INIT>;
    CIMQ_TRY(set_lds(kern, lds));
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, reinterpret_cast<const int8_t*>(ctx + L.xcode),
                       reinterpret_cast<const int8_t*>(ctx + L.xhat), reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag),
                       pp, sw, sa, signed_act, gout, W.rows, reinterpret_cast<float*>(ws + W.gw_slab),
                       reinterpret_cast<float*>(ws + W.ga_slab), reinterpret_cast<float*>(ws + W.gb_slab));
  }
  prof_end(slot, s);
  return check_hip("cim_bwd_gw");
}

// grad_x; returns through *lsq_fused whether the LSQ activation backward was applied
template <int NBP, int FBMAX>
int launch_gx(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
              const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const Plan3 p = v3_plan(g);
  const v4i* wf = reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag);
  const v4i* wg = reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wgx);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  *lsq_fused = false;
  if (p.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    float* part = reinterpret_cast<float*>(ws + W.lsq_part);
    dim3 grid(g.B * p.v.nbands);
    const bool two = p.v.NT <= 16;
    if (p.lds_gx6) {
      auto kern = two ? (lsq ? cim_bwd_gx_v6_kernel<NBP, 2, true> : cim_bwd_gx_v6_kernel<NBP, 2, false>)
                      : (lsq ? cim_bwd_gx_v6_kernel<NBP, 4, true> : cim_bwd_gx_v6_kernel<NBP, 4, false>);
      CIMQ_TRY(set_lds(kern, p.lds_gx6));
      const int slot = prof_begin(KID_BWD_GX, g, s);
      hipLaunchKernelGGL(kern, grid, dim3(512), p.lds_gx6, s, g, p.v, ctx + L.st,
                         reinterpret_cast<const uint4*>(wreg(g, ctx) + L.wtc), pp, sw, sa, gout, x, gx, part);
      prof_end(slot, s);
      *lsq_fused = lsq;
      return check_hip("cim_bwd_gx_v6");
    }
    auto kern = two ? (lsq ? cim_bwd_gx_v5_kernel<NBP, 2, true> : cim_bwd_gx_v5_kernel<NBP, 2, false>)
                    : (lsq ? cim_bwd_gx_v5_kernel<NBP, 4, true> : cim_bwd_gx_v5_kernel<NBP, 4, false>);
    CIMQ_TRY(set_lds(kern, p.lds_gx));
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL(kern, grid, dim3(512), p.lds_gx, s, g, p.v, ctx + L.st,
                       reinterpret_cast<const uint4*>(wreg(g, ctx) + L.wtc), pp, sw, sa, gout, x, gx, part);
    prof_end(slot, s);
    *lsq_fused = lsq;
    return check_hip("cim_bwd_gx_v5");
  }
  const int8_t* xc = reinterpret_cast<const int8_t*>(ctx + L.xcode);
  if (gx_lds_ok(g) && g.P >= 64) {  // one block per image: only when an image fills a 64-pixel tile
    const size_t lds = lds_tile(g) + sizeof(float) * g.C * g.HW;
    auto kern = cim_bwd_gx_kernel<NBP, FBMAX, true>;
    CIMQ_TRY(set_lds(kern, lds));
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL(kern, dim3(g.B), dim3(256), lds, s, g, xc, wf, wg, pp, sw, sa, gout, gx);
    prof_end(slot, s);
    return check_hip("cim_bwd_gx(lds)");
  }
  if (hipMemsetAsync(gx, 0, sizeof(float) * g.Nin, s) != hipSuccess) return fail(CIMQ_EHIP, "memset gx");
  const size_t lds = lds_tile(g);
  auto kern = cim_bwd_gx_kernel<NBP, FBMAX, false>;
  CIMQ_TRY(set_lds(kern, lds));
  const int slot = prof_begin(KID_BWD_GX, g, s);
  hipLaunchKernelGGL(kern, dim3(cdiv(g.M, 64), g.T), dim3(256), lds, s, g, xc, wf, wg, pp, sw, sa, gout, gx);
  prof_end(slot, s);
  CIMQ_TRY(check_hip("cim_bwd_gx(global)"));
  int grid = cdiv(g.Nin, 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(scale_kernel, dim3(grid), dim3(256), 0, s, gx, g.Nin, sw, g.nba);
  return check_hip("scale");
}

template <int NBP, int FBMAX>
int launch_bwd_all(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                   const float* signed_act, const float* gout, const float* x, float* gx, uint8_t* ws,
                   hipStream_t s, bool* lsq_fused) {
  CIMQ_TRY((launch_gx<NBP, FBMAX>(g, ctx, sw, sa, gout, x, gx, ws, s, lsq_fused)));
  CIMQ_TRY((launch_gw<NBP, FBMAX, false>(g, ctx, sw, sa, signed_act, gout, ws, s)));
  return CIMQ_OK;
}

template <int NBP>
int dispatch_bwd(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
                 const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused) {
  if (g.FBT <= 4) return launch_bwd_all<NBP, 4>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
  return launch_bwd_all<NBP, 8>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
}

template <int NBP>
int dispatch_init(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                  const float* signed_act, uint8_t* ws, hipStream_t s) {
  if (g.FBT <= 4) return launch_gw<NBP, 4, true>(g, ctx, sw, sa, signed_act, nullptr, ws, s);
  return launch_gw<NBP, 8, true>(g, ctx, sw, sa, signed_act, nullptr, ws, s);
}


int launch_bwd_general(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
                       const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused) {
  if (g.NBP == 4) return dispatch_bwd<4>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
  return dispatch_bwd<8>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
}

int launch_alpha_init_sums(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                           const float* signed_act, uint8_t* ws, hipStream_t s) {
  if (g.NBP == 4) return dispatch_init<4>(g, ctx, sw, sa, signed_act, ws, s);
  return dispatch_init<8>(g, ctx, sw, sa, signed_act, ws, s);
}

}  // namespace cimq

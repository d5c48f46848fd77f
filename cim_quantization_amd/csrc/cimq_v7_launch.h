// cimq_v7_launch.h -- launch sequence of the v7 backward (cim_bwd_gx_v8_kernel +
// cim_bwd_gw_v7_kernel, cimq_v7.hip) as a template over the slice-pair shape; each shape is
// instantiated in its own translation unit (cimq_part_v7_*.hip) so they compile in parallel.
// parts: bit 0 the grad_x kernel, bit 1 the grad_w kernel (CIMQ_LSQ_DEFER_GW launches them apart,
// grad_w on the caller's second stream).
#pragma once
#include "cimq_host.h"

namespace cimq {

template <int NBW, int NBA, int OBX>
int launch_v7_nb(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa,
                 const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq,
                 int parts) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  const uint32_t* st = reinterpret_cast<const uint32_t*>(ctx + L.st);
  const PlanX5 px5 = x5_plan(g);
  if ((parts & 3) == 3 && px5.ok && lsq && g.SH == 1 && tune("GXW5", 1)) {
    const PlanG5 pg5 = g5_plan(g);
    if (pg5.ok) return launch_gxw5(g, px5, pg5, ctx, sw, sa, gout, x, gx, ws, s);  // both kernels, one grid
  }
  if ((parts & 1) && px5.ok && lsq) {
    CIMQ_TRY(launch_gx5(g, px5, ctx, sw, sa, gout, x, gx, ws, s));
  } else if (parts & 1) {
    const int np = p.v.NPART;
#define CIMQ_GX8(L, S, N) cim_bwd_gx_v8_kernel<NBW, NBA, OBX, L, S, N>
#ifdef CIMQ_TUNING
#define CIMQ_GX8N(L, S) (np == 1 ? CIMQ_GX8(L, S, 1) : np == 2 ? CIMQ_GX8(L, S, 2) : CIMQ_GX8(L, S, 4))
#else  // v7_plan: NPART is 1 or 2 unless a tuning knob asks for 4
#define CIMQ_GX8N(L, S) (np == 1 ? CIMQ_GX8(L, S, 1) : CIMQ_GX8(L, S, 2))
#endif
    auto kern = g.SH == 1 ? (lsq ? CIMQ_GX8N(true, 1) : CIMQ_GX8N(false, 1)) : (lsq ? CIMQ_GX8N(true, 2) : CIMQ_GX8N(false, 2));
#undef CIMQ_GX8N
#undef CIMQ_GX8
    CIMQ_TRY(set_lds(kern, p.lds_gx));
    const int slot = prof_begin(KID_GX_V8, g, s);
    hipLaunchKernelGGL(kern, dim3(g.B * p.v.nbands), dim3(256 * np), p.lds_gx, s, g, p.v, st,
                       reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wcy), pp, sw, sa, gout, x, gx,
                       reinterpret_cast<float*>(ws + W.lsq_part));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("cim_bwd_gx_v8"));
  }
  if (parts & 2) {
    const PlanG5 p5 = g5_plan(g);
    if (p5.ok) return launch_gw5(g, p5, ctx, gout, ws, s);
    auto kern = g.SH == 1 ? cim_bwd_gw_v7_kernel<NBW, NBA, 1> : cim_bwd_gw_v7_kernel<NBW, NBA, 2>;
    CIMQ_TRY(set_lds(kern, p.lds_gw));
    const int slot = prof_begin(KID_GW_V7, g, s);
    hipLaunchKernelGGL(kern, dim3(p.v.nchunks, p.pairs), dim3(256), p.lds_gw, s, g, p.v, st, ctx + L.xhat, pp,
                       gout, reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("cim_bwd_gw_v7"));
  }
  return CIMQ_OK;
}

template <int NBW, int NBA>
int launch_v7_n(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa,
                const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq,
                int parts) {
  if constexpr (NBW * NBA > 10) {
    return launch_v7_nb<NBW, NBA, 1>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);  // v7_plan: OB16 == 1
  } else {
    if (g.OB16 == 1) return launch_v7_nb<NBW, NBA, 1>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
    if (g.OB16 == 2) return launch_v7_nb<NBW, NBA, 2>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
    return launch_v7_nb<NBW, NBA, 4>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq, parts);
  }
}


}  // namespace cimq

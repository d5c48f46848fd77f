// cimq_part_bwd.hip -- backward launch sequences for layers outside the v7 and dense plans (the
// general recompute kernels, lsq.py:244-386: every ADC variant, any conv geometry; deterministic,
// no atomics) and the alpha_cim initialisation sums (lsq.py:35-87).  Own translation unit of
// libcimq.so.
#define CIMQ_TU_BWD
#include "cimq_host.h"

namespace cimq {

// grad_w + grad_alpha (beta) slabs, or the alpha_cim init sums (INIT), on the general kernel
template <int NBP, int FBMAX, bool INIT>
int launch_gw(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
              const float* gout, uint8_t* ws, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  dim3 grid(W.nchunks, g.T, g.OB16);  // one 16-channel output block per workgroup
  const int slot = INIT ? -1 : prof_begin(KID_BWD_GW, g, s);
  const size_t lds = lds_gw(g);
  auto kern = cim_bwd_gw_kernel<NBP, FBMAX, INIT>;
  CIMQ_TRY(set_lds(kern, lds));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, reinterpret_cast<const int8_t*>(ctx + L.xcode),
                     reinterpret_cast<const int8_t*>(ctx + L.xhat), reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag),
                     pp, sw, sa, signed_act, gout, W.rows, reinterpret_cast<float*>(ws + W.gw_slab),
                     reinterpret_cast<float*>(ws + W.ga_slab), reinterpret_cast<float*>(ws + W.gb_slab));
  prof_end(slot, s);
  return check_hip("cim_bwd_gw");
}

// grad_x: the unfolded product per (64-pixel tile, crossbar tile), then the fixed-order fold
// (the act-LSQ backward runs after it, lsq_act_bwd_kernel)
template <int NBP, int FBMAX>
int launch_gx(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* gout, float* gx,
              uint8_t* ws, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const v4i* wf = reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag);
  const v4i* wg = reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wgx);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  float* gxu = reinterpret_cast<float*>(ws + W.gxu);
  const int8_t* xc = reinterpret_cast<const int8_t*>(ctx + L.xcode);
  const size_t lds = lds_tile(g);
  auto kern = cim_bwd_gx_kernel<NBP, FBMAX>;
  CIMQ_TRY(set_lds(kern, lds));
  const int slot = prof_begin(KID_BWD_GX, g, s);
  hipLaunchKernelGGL(kern, dim3(cdiv(g.M, 64), g.T), dim3(256), lds, s, g, xc, wf, wg, pp, sw, sa, gout, gxu);
  CIMQ_TRY(check_hip("cim_bwd_gx"));
  hipLaunchKernelGGL(fold_gx_kernel, dim3(std::min(cdiv(g.Nin, 256), 8192)), dim3(256), 0, s, g, gxu, sw, gx);
  prof_end(slot, s);
  return check_hip("fold_gx");
}

template <int NBP, int FBMAX>
int launch_bwd_all(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                   const float* signed_act, const float* gout, const float* x, float* gx, uint8_t* ws,
                   hipStream_t s, bool* lsq_fused) {
  (void)x;
  *lsq_fused = false;
  CIMQ_TRY((launch_gx<NBP, FBMAX>(g, ctx, sw, sa, gout, gx, ws, s)));
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

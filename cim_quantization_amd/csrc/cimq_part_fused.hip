// cimq_part_fused.hip -- launch of the one-kernel backwards: cimq_fused.hip for the stride-1 3x3 w2a2 /
// w3a3 layers v9_plan accepts, cimq_c1.hip for the w8a8 first conv (c1_plan); one workgroup per image,
// grad_x + grad_w + grad_alpha partials.
// Own translation unit of libcimq.so.
#include "cimq_host.h"

namespace cimq {

template <int NB, int OBX>
static int launch_fused_nb(const Geo& g, const Plan9& p, const uint8_t* ctx, const float* sw, const float* sa,
                           const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  auto kern = lsq ? cim_bwd_fused_kernel<NB, OBX, true> : cim_bwd_fused_kernel<NB, OBX, false>;
  CIMQ_TRY(set_lds(kern, p.v.lds));
  const int slot = prof_begin(KID_FUSED, g, s);
  hipLaunchKernelGGL(kern, dim3(g.B), dim3(512), p.v.lds, s, g, p.v,
                     reinterpret_cast<const uint32_t*>(ctx + L.st), reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wcy),
                     pp, sw, sa, gout, reinterpret_cast<const uint32_t*>(ctx + L.xhat), x, gx,
                     reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab),
                     reinterpret_cast<float*>(ws + W.lsq_part));
  prof_end(slot, s);
  return check_hip("cim_bwd_fused");
}

template <int NB>
static int launch_fused_n(const Geo& g, const Plan9& p, const uint8_t* ctx, const float* sw, const float* sa,
                          const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  if (g.OB16 == 1) return launch_fused_nb<NB, 1>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  if (g.OB16 == 2) return launch_fused_nb<NB, 2>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  return launch_fused_nb<NB, 4>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
}

int launch_fused(const Geo& g, const Plan9& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
                 const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  if (g.nbw == 2) return launch_fused_n<2>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  return launch_fused_n<3>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
}

int launch_c1(const Geo& g, const PlanC1& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
              const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  auto kern = lsq ? cim_bwd_c1_kernel<true> : cim_bwd_c1_kernel<false>;
  CIMQ_TRY(set_lds(kern, p.v.lds));
  const int slot = prof_begin(KID_FUSED, g, s);
  hipLaunchKernelGGL(kern, dim3(g.B), dim3(512), p.v.lds, s, g, p.v, ctx + L.xcode, ctx + L.xhat,
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag), reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wcy),
                     pp, sw, sa, gout, x, gx, reinterpret_cast<float*>(ws + W.gw_slab),
                     reinterpret_cast<float*>(ws + W.ga_slab), reinterpret_cast<float*>(ws + W.lsq_part));
  prof_end(slot, s);
  return check_hip("cim_bwd_c1");
}

}  // namespace cimq

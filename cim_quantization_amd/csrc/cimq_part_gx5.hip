// cimq_part_gx5.hip -- launch of the per-input-pixel grad_x kernel of the 16 -> 16-channel 32-wide w3a3
// layers (cimq_gx5.hip, lsq.py:336-386 + lsq.py:549).  Own translation unit of libcimq.so.
#define CIMQ_TU_GX5
#include "cimq_host.h"

namespace cimq {

int launch_gx5(const Geo& g, const PlanX5& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
               const float* x, float* gx, uint8_t* ws, hipStream_t s) {
  if (!p.ok) return fail(CIMQ_EINVAL, "internal: cim_bwd_gx5 off its plan");
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  auto kern = p.v.CBN == 2 ? cim_bwd_gx5_kernel<2> : cim_bwd_gx5_kernel<1>;
  CIMQ_TRY(set_lds(kern, p.lds));
  const int slot = prof_begin(KID_GX_V8, g, s);
  hipLaunchKernelGGL(kern, dim3(p.nblk), dim3(512), p.lds, s, g, p.v, reinterpret_cast<const uint32_t*>(ctx + L.st),
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wg5), params_of(g, const_cast<uint8_t*>(ctx)), sw,
                     sa, gout, x, gx, reinterpret_cast<float*>(ws + W.lsq_part));
  prof_end(slot, s);
  return check_hip("cim_bwd_gx5");
}

int launch_prep_wg5(const Geo& g, const float* w_q, const float* sw, uint8_t* ctx, hipStream_t s) {
  const int total = (int)(x5_frag_bytes(g) / 16);
  if (total == 0) return CIMQ_OK;
  CtxLayout L = ctx_layout(g);
  hipLaunchKernelGGL(prep_wg5_kernel, dim3(cdiv(total, 256)), dim3(256), 0, s, g, w_q, sw, total,
                     reinterpret_cast<v4i*>(wreg(g, ctx) + L.wg5));
  return check_hip("prep_wg5");
}

}  // namespace cimq

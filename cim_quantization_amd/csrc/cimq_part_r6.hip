// cimq_part_r6.hip -- launch of the recompute backward of the w3a3 16 -> 16 stride-1 module layers (cimq_r6.hip,
// lsq.py:244-386 + lsq.py:549).  Own translation unit of libcimq.so.
#define CIMQ_TU_R6
#include "cimq_host.h"

namespace cimq {

int launch_r6(const Geo& g, const PlanR6& p, const uint8_t* ctx, const float* sw, const float* sa, const float* sgn,
              const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, uint32_t* st_dbg) {
  if (!p.ok || !g.onchw || !sgn || !x) return fail(CIMQ_EINVAL, "internal: cim_bwd_r6 off its plan");
  if (!st_dbg && (!gout || !gx || !ws)) return fail(CIMQ_EINVAL, "internal: cim_bwd_r6 without its buffers");
  CtxLayout L = ctx_layout(g);
  const uint8_t* wr = wreg(g, ctx);
  auto kern = st_dbg ? cim_bwd_r6_kernel<true> : cim_bwd_r6_kernel<false>;
  CIMQ_TRY(set_lds(kern, p.lds));
  const WsLayout W = ws_layout(g);
  if (!st_dbg && W.nchunks_bwd != g.B) return fail(CIMQ_EINVAL, "internal: cim_bwd_r6 slab count mismatch");
  const int slot = st_dbg ? -1 : prof_begin(KID_FUSED, g, s);
  // one workgroup per image (the B chunks of the slabs, the B act-LSQ partials)
  hipLaunchKernelGGL(kern, dim3(g.B), dim3(512), p.lds, s, g, p.v, reinterpret_cast<const v4i*>(wr + L.wf5),
                     reinterpret_cast<const v4i*>(wr + L.wx6), params_of(g, const_cast<uint8_t*>(ctx)), sw, sa, sgn, x,
                     gout, gx, ws ? reinterpret_cast<float*>(ws + W.gw_slab) : nullptr,
                     ws ? reinterpret_cast<float*>(ws + W.ga_slab) : nullptr,
                     ws ? reinterpret_cast<float*>(ws + W.lsq_part) : nullptr, st_dbg);
  prof_end(slot, s);
  return check_hip("cim_bwd_r6");
}

}  // namespace cimq

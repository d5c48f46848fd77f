// cimq_part_gw5.hip -- launch of the grad_w / grad_alpha kernel of the w3a3 stride-1 16 / 32-channel layers
// (cimq_gw5.hip, lsq.py:321-356).  Own translation unit of libcimq.so.
#define CIMQ_TU_GW5
#include "cimq_host.h"

namespace cimq {

int launch_gw5(const Geo& g, const PlanG5& p, const uint8_t* ctx, const float* gout, uint8_t* ws, hipStream_t s) {
  if (!p.ok) return fail(CIMQ_EINVAL, "internal: cim_bwd_gw5 off its plan");
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  if (W.nchunks_bwd != p.v.nchunks) return fail(CIMQ_EINVAL, "internal: cim_bwd_gw5 slab count mismatch");
  G5 v = p.v;
  v.codes = ctx_codes(g) ? 1 : 0;  // the forward wrote code bytes (cim_fwd5_kernel on the module path)
  // the row-block split compiled in: 16 input channels (every block in input-channel block 0) and 32 (blocks 0 / 1)
  const int sp = !tune("GW5_SP8", 1) ? 0 : g.C == 16 ? 8 : (g.C == 32 && tune("GW5_SP78", 1)) ? 78 : 0;
#define CIMQ_GW5_K(SS_, C_) (sp == 8 ? cim_bwd_gw5_kernel<SS_, C_, 8> : sp == 78 ? cim_bwd_gw5_kernel<SS_, C_, 78> \
                                                                       : cim_bwd_gw5_kernel<SS_, C_, 0>)
  auto kern = g.SH == 2 ? (v.codes ? CIMQ_GW5_K(2, true) : CIMQ_GW5_K(2, false))
                        : (v.codes ? CIMQ_GW5_K(1, true) : CIMQ_GW5_K(1, false));
#undef CIMQ_GW5_K
  CIMQ_TRY(set_lds(kern, p.lds));
  const int slot = prof_begin(KID_GW_V7, g, s);
  hipLaunchKernelGGL(kern, dim3(p.v.nchunks, p.pairs), dim3(512), p.lds, s, g, v,
                     reinterpret_cast<const uint32_t*>(ctx + L.st), reinterpret_cast<const uint32_t*>(ctx + L.xhat),
                     params_of(g, const_cast<uint8_t*>(ctx)), gout, reinterpret_cast<const uint32_t*>(ctx + L.alut),
                     reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
  prof_end(slot, s);
  return check_hip("cim_bwd_gw5");
}

}  // namespace cimq

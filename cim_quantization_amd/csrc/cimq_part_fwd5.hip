// cimq_part_fwd5.hip -- launch of the w3a3 module forward on the slice-planar patch (cimq_fwd5.hip,
// lsq.py:141-233 with the activation quantiser of lsq.py:544-549).  Own translation unit of libcimq.so.
#define CIMQ_TU_FWD5
#include "cimq_host.h"

namespace cimq {

int launch_fwd5(const Geo& g, const Plan5& p, uint8_t* ctx, const float* sw, const float* sa, float* out,
                hipStream_t s, const ActQ* aq) {
  if (!p.ok || !aq || !g.onchw) return fail(CIMQ_EINVAL, "internal: cim_fwd5 off its plan");
  CtxLayout L = ctx_layout(g);
  // the state words and ctx only where the backward reads them (not where cim_bwd_r6_kernel recomputes)
  const bool wst = !r6_bwd(g);
  auto kern = p.nob == 2 ? (wst ? cim_fwd5_kernel<2, true> : cim_fwd5_kernel<2, false>)
                         : (wst ? cim_fwd5_kernel<1, true> : cim_fwd5_kernel<1, false>);
  CIMQ_TRY(set_lds(kern, p.lds));
  // 4 waves per SIMD: two 512-thread blocks per CU (one output block each) or one 1024-thread block (two),
  // a grid-stride walk over the 128-pixel m-tiles; the output-block groups in y
  const int ny = g.OB16 / p.nob;
  const int per_ob = std::max(1, tune("FWD5_GRID", p.nob == 2 ? 256 : 512) / ny);
  dim3 grid(std::min(p.v.nmt, per_ob), ny);
  const int slot = prof_begin(KID_FWD_V7, g, s);
  F5 v = p.v;
  v.codes = ctx_codes(g) ? 1 : 0;  // one code byte per ctx element (grad_w is cim_bwd_gw5_kernel)
  hipLaunchKernelGGL(kern, grid, dim3(512 * p.nob), p.lds, s, g, v, reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wf5),
                     params_of(g, ctx), sw, sa, aq->x, aq->signed_act, out,
                     reinterpret_cast<uint32_t*>(ctx + L.st), reinterpret_cast<uint32_t*>(ctx + L.xhat),
                     reinterpret_cast<uint32_t*>(ctx + L.alut));
  prof_end(slot, s);
  return check_hip("cim_fwd5");
}

}  // namespace cimq

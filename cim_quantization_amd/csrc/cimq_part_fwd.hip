// cimq_part_fwd.hip -- forward launch sequences (lsq.py:166-233): the v3 fast-path kernel and
// the general kernel (also the partial-sum debug hook).  Own translation unit of libcimq.so.
#include "cimq_host.h"

namespace cimq {

template <int NBP, int KS>
int launch_fwd_v3(const Geo& g, const Plan3& p, uint8_t* ctx, const float* sw, const float* sa, float* out,
                  hipStream_t s, const ActQ* aq) {
  CtxLayout L = ctx_layout(g);
  // compact state words when the v7 backward will read them
  const bool cst = v7_plan(g).ok;
  // OBM: 16-channel output blocks per block (register arrays sized for exactly that)
  const int obm = std::min(p.v.obm, g.OB16 <= 2 ? g.OB16 : 4);
  // CST: compact state words with nbw = nba = CST fixed at compile time (v7_plan's slice pairs)
  void (*kern)(Geo, V3, const uint8_t*, const v4i*, Params, const float*, const float*, float*, uint8_t*,
               const float*, const float*, uint8_t*);
  if (!cst) {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 0, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 0, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 0, 4>;
  } else if constexpr (NBP == 8) {
    // v7_plan: w8a8 with one 16-channel block; the first conv's backward (c1_plan) recomputes the state
    kern = c1_plan(g).ok ? cim_fwd_v3_kernel<8, KS, 9, 1> : cim_fwd_v3_kernel<8, KS, 8, 1>;
  } else if (g.nbw == 2) {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 2, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 2, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 2, 4>;
  } else {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 3, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 3, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 3, 4>;
  }
  // the fused activation quantiser's word table (after the kernel's other LDS)
  const size_t lds = p.lds_fwd + (aq ? (size_t)kActLutMax * 2 * 4 : 0);
  CIMQ_TRY(set_lds(kern, lds));
  // grid: about three resident 256-thread blocks per CU (measured: 768 blocks for w3a3, 1024
  // for the 236-VGPR w8a8 instance)
  dim3 grid(std::min(p.v.nmt, tune("FWD_GRID", NBP == 8 ? 1024 : 768)), cdiv(g.OB16, obm));
  const int slot = prof_begin(cst ? KID_FWD_V7 : KID_FWD, g, s);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, p.v, ctx + L.xcode,
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag), params_of(g, ctx), sw, sa, out, ctx + L.st,
                     aq ? aq->x : nullptr, aq ? aq->signed_act : nullptr, aq ? ctx + L.xhat : nullptr);
  prof_end(slot, s);
  return check_hip("cim_fwd_v3");
}

template <int NBP, bool DBG>
int launch_fwd(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, int* ps_dbg,
               float* adc_dbg, hipStream_t s, const ActQ* aq) {
  CtxLayout L = ctx_layout(g);
  const Plan3 p = v3_plan(g);
  if (p.ok && !DBG) {
    if (aq) {
      const Plan5 p5 = f5_plan(g);
      if (p5.ok) return launch_fwd5(g, p5, ctx, sw, sa, out, s, aq);
    }
    if (g.KS == 1) return launch_fwd_v3<NBP, 1>(g, p, ctx, sw, sa, out, s, aq);
    return launch_fwd_v3<NBP, 2>(g, p, ctx, sw, sa, out, s, aq);
  }
  if (p.ok) {
    // the debug forward is the general kernel; the fast one still fills the state words the
    // fast backward reads (same out values)
    if (g.KS == 1) CIMQ_TRY((launch_fwd_v3<NBP, 1>(g, p, ctx, sw, sa, out, s, nullptr)));
    else CIMQ_TRY((launch_fwd_v3<NBP, 2>(g, p, ctx, sw, sa, out, s, nullptr)));
  }
  dim3 grid(cdiv(g.M, 64), cdiv(g.OB16, 4));
  const size_t lds = lds_tile(g);
  auto kern = cim_fwd_kernel<NBP, DBG>;
  CIMQ_TRY(set_lds(kern, lds));
  const int slot = DBG ? -1 : prof_begin(KID_FWD, g, s);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, reinterpret_cast<const int8_t*>(ctx + L.xcode),
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag), params_of(g, ctx), sw, sa, out, ps_dbg,
                     adc_dbg);
  prof_end(slot, s);
  return check_hip("cim_fwd");
}


int launch_fwd_any(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, int* ps_dbg,
                   float* adc_dbg, hipStream_t s, const ActQ* aq) {
  if (aq && (!fwd_actq_ok(g) || ps_dbg)) return fail(CIMQ_EINVAL, "internal: fused activation quantiser off its plan");
  if (dense_plan(g)) {
    // the dense GEMM path (its state words feed the dense backward); the debug hook then reruns
    // the general kernel for the partial sums (same out values)
    CIMQ_TRY(launch_dense_fwd(g, ctx, sw, sa, out, s));
    if (!ps_dbg) return CIMQ_OK;
  }
  if (ps_dbg) {
    if (g.NBP == 4) return launch_fwd<4, true>(g, ctx, sw, sa, out, ps_dbg, adc_dbg, s, nullptr);
    return launch_fwd<8, true>(g, ctx, sw, sa, out, ps_dbg, adc_dbg, s, nullptr);
  }
  if (g.NBP == 4) return launch_fwd<4, false>(g, ctx, sw, sa, out, nullptr, nullptr, s, aq);
  return launch_fwd<8, false>(g, ctx, sw, sa, out, nullptr, nullptr, s, nullptr);
}

}  // namespace cimq

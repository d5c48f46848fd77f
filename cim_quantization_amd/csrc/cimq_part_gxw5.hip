// cimq_part_gxw5.hip -- grad_x and grad_w of a w3a3 16 / 32-channel stride-1 module layer in ONE launch: the
// workgroups of cim_bwd_gx5_kernel first, then those of cim_bwd_gw5_kernel, each running its own body
// (cimq_gx5.hip, cimq_gw5.hip; lsq.py:321-386 + lsq.py:549).  The two kernels read the same state words and
// grad_out and are independent; as one grid, grad_w's workgroups start on the CUs grad_x's last workgroups
// leave idle, and the launch gap between them goes.  Own translation unit of libcimq.so.
#define CIMQ_TU_GXW5
#include "cimq_host.h"

namespace cimq {

template <int CBN, bool CODES, int SP>
__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
void cim_bwd_gxw5_kernel(Geo g, X5 vx, G5 vw, const uint32_t* __restrict__ st, const v4i* __restrict__ wg5, Params pp,
                         const float* __restrict__ sw_p, const float* __restrict__ sa_p, const float* __restrict__ gout,
                         const float* __restrict__ x, float* __restrict__ gx, float* __restrict__ gsa_part,
                         const uint32_t* __restrict__ xcb, const uint32_t* __restrict__ cal, float* __restrict__ gw_slab,
                         float* __restrict__ ga_slab, int ngx) {
  const int b = (int)blockIdx.x;
  if (b < ngx) {
    gx5_body<CBN>(b, ngx, g, vx, st, wg5, pp, sw_p, sa_p, gout, x, gx, gsa_part);
  } else {
    const int t = b - ngx, by = t / vw.nchunks;
    gw5_body<1, CODES, SP>(t - by * vw.nchunks, by, g, vw, st, xcb, pp, gout, cal, gw_slab, ga_slab);
  }
}

int launch_gxw5(const Geo& g, const PlanX5& px, const PlanG5& pw, const uint8_t* ctx, const float* sw, const float* sa,
                const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s) {
  if (!px.ok || !pw.ok || g.SH != 1 || !(g.C == 16 || g.C == 32)) return fail(CIMQ_EINVAL, "internal: cim_bwd_gxw5 off its plans");
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  if (W.nchunks_bwd != pw.v.nchunks) return fail(CIMQ_EINVAL, "internal: cim_bwd_gxw5 slab count mismatch");
  G5 vw = pw.v;
  vw.codes = ctx_codes(g) ? 1 : 0;  // the forward wrote code bytes (cim_fwd5_kernel on the module path)
  // x5_plan: C = 16 -> one 16-channel input block (gw5's row-block split at 8), C = 32 -> two (splits 8 and 7)
  auto kern = px.v.CBN == 1 ? (vw.codes ? cim_bwd_gxw5_kernel<1, true, 8> : cim_bwd_gxw5_kernel<1, false, 8>)
                            : (vw.codes ? cim_bwd_gxw5_kernel<2, true, 78> : cim_bwd_gxw5_kernel<2, false, 78>);
  const size_t lds = std::max(px.lds, pw.lds);
  CIMQ_TRY(set_lds(kern, lds));
  const int ngw = pw.v.nchunks * pw.pairs;
  // timed as the fused family (grad_x + grad_w of the layer in one launch: its algorithmic bytes are read gy
  // and x once, write gx; its MFMA work both contractions), not as grad_x alone
  const int slot = prof_begin(KID_FUSED, g, s);
  hipLaunchKernelGGL(kern, dim3(px.nblk + ngw), dim3(512), lds, s, g, px.v, vw, reinterpret_cast<const uint32_t*>(ctx + L.st),
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wg5), params_of(g, const_cast<uint8_t*>(ctx)), sw, sa,
                     gout, x, gx, reinterpret_cast<float*>(ws + W.lsq_part), reinterpret_cast<const uint32_t*>(ctx + L.xhat),
                     reinterpret_cast<const uint32_t*>(ctx + L.alut), reinterpret_cast<float*>(ws + W.gw_slab),
                     reinterpret_cast<float*>(ws + W.ga_slab), px.nblk);
  prof_end(slot, s);
  return check_hip("cim_bwd_gxw5");
}

}  // namespace cimq

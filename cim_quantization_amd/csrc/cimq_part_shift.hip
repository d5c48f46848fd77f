// cimq_part_shift.hip -- grad_alpha / grad_beta of the scale + shift ADC (Conv2dLSQCiM(adc_shift=True),
// test/test_backward_cimlayer_scale_shift.py:437-501 applied to the library's rescaled partial sum) on
// the fast path.  Own translation unit of libcimq.so.
//
// The forward (cim_fwd_v3_kernel, shift_fast layers) leaves the STE pass bit and the ADC code of every
// partial sum in the v7 state words, and grad_x / grad_w need nothing else (the STE mask is the
// library's).  The step-size gradients need the partial sum itself:
//   grad_alpha[i,k,j,o] = mask_kj * sum_{b,p} q * g,   q = rint(v) - v where the ADC input v =
//                         (u - beta) / alpha is inside the clamp range, else the clamped code (:488-495)
//   grad_beta[i,k,j,o]  = mask_kj * sum_{b,p} [v clamped] * g                                  (:496-501)
// with u = fp16(ps) * sw * sa.  shift_stats_kernel recomputes each partial sum on the int8 MFMA from
// the forward's slice words and weight fragments (no fp16 ps buffer) and takes q from a table of the
// partial sum's possible values per (tile, pair, channel) -- built by shift_qtab_kernel with the
// reference's fp32 op chain (u_var, one IEEE division), so q matches the reference's term for term at
// an LDS lookup per partial sum.  Sums are per-lane registers, a fixed shuffle / LDS tree per block and
// a fixed-order sum over the pixel chunks (shift_combine_kernel): bit-identical run to run, no atomics.
#include "cimq_host.h"

namespace cimq {

// q of one partial sum: the ADC input v = (u - beta) / alpha in the reference's fp32 op chain (u_var,
// one IEEE division, scale_shift.py:469), the code clamp(rint(v), -1, 1), and q = rint(v) - v inside the
// STE range, the clamped code outside (:484-495).  |q| == 1 exactly iff v is clamped (inside, |q| <= 1/2).
__device__ inline float shift_q(int p, float sw, float sa, float al, float be, float thr_hi, float thr_lo) {
  const float v = (((ps_half(p) * sw) * sa) - be) / al;
  const float code = clamp_nan(rintf(v), -1.f, 1.f);
  const bool clamped = (v >= thr_hi) || (v <= thr_lo);
  return clamped ? code : code - v;
}
__device__ __noinline__ float shift_q_ool(int p, float sw, float sa, float al, float be, float thr_hi, float thr_lo) {
  return shift_q(p, sw, sa, al, be, thr_hi, thr_lo);
}

// q tables: for every (tile i, o-block ob, slice pair kj, channel col) and partial sum ps in [-R, R],
// q(ps) -- [T][OB16][NKJ][16][2R + 1] floats; the statistics kernel looks them up instead of dividing
__global__ void shift_qtab_kernel(Geo g, Params pp, const float* __restrict__ sw_p, const float* __restrict__ sa_p,
                                  int R, float* __restrict__ qtab) {
  const int NE = 2 * R + 1, nkj = g.nbw * g.nba;
  const long long total = (long long)g.T * g.OB16 * nkj * 16 * NE;
  const float sw = *sw_p, sa = *sa_p;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(t % NE);
    long long r = t / NE;
    const int col = (int)(r % 16); r /= 16;
    const int kj = (int)(r % nkj); r /= nkj;
    const int ob = (int)(r % g.OB16), i = (int)(r / g.OB16);
    const int k = kj / g.nba, j = kj - k * g.nba, o = ob * 16 + col;
    const int pi = pidx(g, i, j, k, o);
    qtab[t] = shift_q(e - R, sw, sa, pp.alpha[pi], pp.beta[pi], g.thr_hi, g.thr_lo);
  }
}

// block = 256 threads (4 waves of 16 output pixels) over the 64-pixel m-tiles mt = blockIdx.x + k*nsc,
// for one crossbar tile i and one 16-channel block ob (blockIdx.y = i * OB16 + ob).  LUT: the block's q
// table ([NKJ][16][2R + 1]) in LDS; a partial sum outside [-R, R] (slice artifacts) evaluates q directly.
template <int KS, int NS, bool LUT>
__global__ __launch_bounds__(256) void shift_stats_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                          const v4i* __restrict__ wfrag, Params pp,
                                                          const float* __restrict__ sw_p,
                                                          const float* __restrict__ sa_p,
                                                          const float* __restrict__ gout,
                                                          const float* __restrict__ qtab, int R,
                                                          float* __restrict__ slab, int nsc) {
  constexpr int NKJ = NS * NS;
  constexpr int NBP = 4;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int i = blockIdx.y / g.OB16, ob = blockIdx.y - i * g.OB16;
  // input channels of tile i: the patch holds only those
  const int c_lo = (i * g.xbar) / g.KHW, c_hi = (min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
  const int ncx = c_hi - c_lo + 1;
  const int NE = 2 * R + 1;
  uint8_t* cur = smem;
  float* tab = reinterpret_cast<float*>(cur); cur += LUT ? al16((size_t)NKJ * 16 * NE * 4) : 0;
  uint8_t* patch = cur; cur += al16((size_t)ncx * v.RH * v.WP * NBP);
  int* ptab = reinterpret_cast<int*>(cur); cur += (size_t)KS * 64 * 4;
  float* red = reinterpret_cast<float*>(cur);  // [4 waves][2 * NKJ][16 channels]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int o = ob * 16 + r16;  // this lane's channel (MFMA column)
  const bool ov = o < g.O;
  build_ptab(g, i, KS, v.RH, v.WP, ptab, c_lo);
  zero_lds(reinterpret_cast<uint32_t*>(patch), ncx * v.RH * v.WP * NBP / 4);
  if (LUT) {
    const float4* src = reinterpret_cast<const float4*>(qtab + (size_t)blockIdx.y * NKJ * 16 * NE);
    const int n4 = NKJ * 16 * NE / 4;  // a multiple of 16 floats per block: 16-byte rows
    batched_copy<4>(n4, reinterpret_cast<float4*>(tab), [&](int idx) -> float4 { return src[idx]; });
  }
  const float sw = *sw_p, sa = *sa_p;
  float al[NKJ], be[NKJ];
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) {
    const int k = kj / NS, j = kj - k * NS;
    al[kj] = pp.alpha[pidx(g, i, j, k, o)];
    be[kj] = pp.beta[pidx(g, i, j, k, o)];
  }
  v4i wk[NS][KS];  // tile i's weight fragments of this o-block, every slice k (fixed for the block)
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wk[k][ks] = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + ob) * WAVE + lane];
  float qs[NKJ], cs[NKJ];
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) qs[kj] = cs[kj] = 0.f;
  const int Wo = 1 << v.lw;
  const int pl = wave * 16 + r16;  // this lane's gather pixel (A row) within the m-tile
  const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & (Wo - 1)) * g.SW;
  const int tpi = g.P >> 6;
  for (int mt = blockIdx.x; mt < v.nmt; mt += nsc) {
    const int b = mt / tpi, p0 = (mt - b * tpi) * 64;
    __syncthreads();
    stage_rows<NBP>(g, v.WP, v.RH, xcf, b, (p0 >> v.lw) * g.SH - g.PH, patch, c_lo, ncx);
    __syncthreads();
    v4i xs[NBP][KS];
    gather_xs<NBP, KS>(patch, rb, ptab, g4, xs);
    // grad_out of pixels mt*64 + 16*wave + 4*g4 + r (MFMA output rows), channel o
    float gv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 64 + wave * 16 + 4 * g4 + r;
      const int pm = p0 + wave * 16 + 4 * g4 + r;
      gv[r] = ov ? (g.onchw ? gout[((size_t)b * g.O + o) * g.P + pm] : gout[(size_t)m * g.O + o]) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        v4i ps = {0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[k][ks], ps, 0, 0, 0);
        const int kj = k * NS + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float q;
          const int e = ps[r] + R;
          if (LUT && (unsigned)e < (unsigned)NE) q = tab[(kj * 16 + r16) * NE + e];
          else q = shift_q_ool(ps[r], sw, sa, al[kj], be[kj], g.thr_hi, g.thr_lo);
          qs[kj] += q * gv[r];
          cs[kj] += (fabsf(q) == 1.f) ? gv[r] : 0.f;  // clamped: grad_beta's region
        }
      }
    }
  }
  // the four pixel groups of a channel (lanes r16 + 16 g4), then the four waves in a fixed order
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) {
    float a = qs[kj], c = cs[kj];
    a = rows4_sum(a);
    c = rows4_sum(c);
    if (g4 == 0) {
      red[(wave * 2 * NKJ + kj) * 16 + r16] = a;
      red[(wave * 2 * NKJ + NKJ + kj) * 16 + r16] = c;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * NKJ * 16; t += blockDim.x) {
    const int w2 = 2 * NKJ * 16;
    const float sum = (red[t] + red[w2 + t]) + (red[2 * w2 + t] + red[3 * w2 + t]);
    const int which = t / (NKJ * 16), rem = t - which * NKJ * 16, kj = rem >> 4, col = rem & 15;
    slab[(((size_t)blockIdx.x * g.T + i) * 2 + which) * NKJ * g.Opad + (size_t)kj * g.Opad + ob * 16 + col] = sum;
  }
}

// The w8a8 first conv under the shift ADC (K <= 32: one K-step, 64 slice pairs, 36 live under the
// int8-wrapped mask): the same sums with slice k a rolled loop (eight live accumulator pairs at a time;
// a full unroll of the 64 pairs would hold 128 of them), q evaluated directly (its table, 64 pairs x
// 16 channels x 55 partial sums, exceeds LDS), and each slice's sums folded over the four pixel rows of
// a lane by half-wave swaps into the wave's LDS region -- still a fixed order, no atomics.
__global__ __launch_bounds__(256) void shift_stats8_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                           const v4i* __restrict__ wfrag, Params pp,
                                                           const float* __restrict__ sw_p,
                                                           const float* __restrict__ sa_p,
                                                           const float* __restrict__ gout, float* __restrict__ slab,
                                                           int nsc) {
  constexpr int NS = 8, NKJ = 64, NBP = 8;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int i = blockIdx.y / g.OB16, ob = blockIdx.y - i * g.OB16;
  const int c_lo = (i * g.xbar) / g.KHW, c_hi = (min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
  const int ncx = c_hi - c_lo + 1;
  uint8_t* cur = smem;
  float* red = reinterpret_cast<float*>(cur); cur += (size_t)4 * 2 * NKJ * 16 * 4;   // [wave][q | c][kj][16]
  float2* abl = reinterpret_cast<float2*>(cur); cur += (size_t)NKJ * 16 * 8;          // alpha, beta [kj][16]
  v4i* wkl = reinterpret_cast<v4i*>(cur); cur += (size_t)NS * 64 * 16;                // weight slices [k][lane]
  int* ptab = reinterpret_cast<int*>(cur); cur += 64 * 4;
  uint8_t* patch = cur;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int o = ob * 16 + r16;
  const bool ov = o < g.O;
  build_ptab(g, i, 1, v.RH, v.WP, ptab, c_lo);
  zero_lds(reinterpret_cast<uint32_t*>(patch), ncx * v.RH * v.WP * NBP / 4);
  for (int t = threadIdx.x; t < 4 * 2 * NKJ * 16; t += blockDim.x) red[t] = 0.f;
  for (int t = threadIdx.x; t < NKJ * 16; t += blockDim.x) {
    const int kj = t >> 4, col = t & 15, k = kj / NS, j = kj - k * NS;
    const int oc = min(ob * 16 + col, g.O - 1);
    abl[t] = make_float2(pp.alpha[pidx(g, i, j, k, oc)], pp.beta[pidx(g, i, j, k, oc)]);
  }
  for (int t = threadIdx.x; t < NS * 64; t += blockDim.x)
    wkl[t] = wfrag[((size_t)i * g.NBLK + (t >> 6) * g.OB16 + ob) * WAVE + (t & 63)];
  __syncthreads();
  // pairs with a nonzero mask (the others add mask * sum = 0 in shift_combine_kernel)
  const uint64_t live = __builtin_amdgcn_ballot_w64(pp.ckj[lane] != 0.f);
  const float sw = *sw_p, sa = *sa_p;
  const int Wo = 1 << v.lw;
  const int pl = wave * 16 + r16;
  const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & (Wo - 1)) * g.SW;
  const int tpi = g.P >> 6;
  float* rq = red + (size_t)wave * 2 * NKJ * 16;
  for (int mt = blockIdx.x; mt < v.nmt; mt += nsc) {
    const int b = mt / tpi, p0 = (mt - b * tpi) * 64;
    __syncthreads();
    stage_rows<NBP>(g, v.WP, v.RH, xcf, b, (p0 >> v.lw) * g.SH - g.PH, patch, c_lo, ncx);
    __syncthreads();
    v4i xs[NBP][1];
    gather_xs<NBP, 1>(patch, rb, ptab, g4, xs);
    float gv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 64 + wave * 16 + 4 * g4 + r;
      const int pm = p0 + wave * 16 + 4 * g4 + r;
      gv[r] = ov ? (g.onchw ? gout[((size_t)b * g.O + o) * g.P + pm] : gout[(size_t)m * g.O + o]) : 0.f;
    }
#pragma unroll 1
    for (int k = 0; k < NS; ++k) {
      const v4i wkk = wkl[k * 64 + lane];
      const unsigned lk = (unsigned)(live >> (8 * k)) & 0xFFu;
      float qs[NS], cs[NS];
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        qs[j] = cs[j] = 0.f;
        if (!((lk >> j) & 1u)) continue;  // uniform
        const v4i ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][0], wkk, v4i{0, 0, 0, 0}, 0, 0, 0);
        const float2 ab = abl[(k * NS + j) * 16 + r16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float q = shift_q(ps[r], sw, sa, ab.x, ab.y, g.thr_hi, g.thr_lo);
          qs[j] += q * gv[r];
          cs[j] += (fabsf(q) == 1.f) ? gv[r] : 0.f;  // clamped: grad_beta's region
        }
      }
      // the lane's four pixel rows -> every lane of the channel (two half-wave swaps), then lane row
      // g4 adds pairs j = g4 and g4 + 4 of this slice to the wave's region
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        auto fold = [](float x) {
          const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
          const float h = __uint_as_float(a[0]) + __uint_as_float(a[1]);
          const auto c = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
          return __uint_as_float(c[0]) + __uint_as_float(c[1]);
        };
        qs[j] = fold(qs[j]);
        cs[j] = fold(cs[j]);
      }
      const float q0 = g4 == 0 ? qs[0] : g4 == 1 ? qs[1] : g4 == 2 ? qs[2] : qs[3];
      const float q1 = g4 == 0 ? qs[4] : g4 == 1 ? qs[5] : g4 == 2 ? qs[6] : qs[7];
      const float c0 = g4 == 0 ? cs[0] : g4 == 1 ? cs[1] : g4 == 2 ? cs[2] : cs[3];
      const float c1 = g4 == 0 ? cs[4] : g4 == 1 ? cs[5] : g4 == 2 ? cs[6] : cs[7];
      float* d = rq + (k * NS + g4) * 16 + r16;
      d[0] += q0;
      d[4 * 16] += q1;
      d[NKJ * 16] += c0;
      d[NKJ * 16 + 4 * 16] += c1;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * NKJ * 16; t += blockDim.x) {
    const int w2 = 2 * NKJ * 16;
    const float sum = (red[t] + red[w2 + t]) + (red[2 * w2 + t] + red[3 * w2 + t]);
    const int which = t / (NKJ * 16), rem = t - which * NKJ * 16, kj = rem >> 4, col = rem & 15;
    slab[(((size_t)blockIdx.x * g.T + i) * 2 + which) * NKJ * g.Opad + (size_t)kj * g.Opad + ob * 16 + col] = sum;
  }
}

// fixed-order sum over the pixel chunks, times the binary mask: [1, T, nbw, nba, 1, O] each.  One wave
// per output: lane l sums chunks l, l + 64, ..., then a fixed butterfly (deterministic)
__global__ __launch_bounds__(256) void shift_combine_kernel(Geo g, const float* __restrict__ slab, int nsc,
                                                            const int8_t* __restrict__ bmask,
                                                            float* __restrict__ grad_alpha,
                                                            float* __restrict__ grad_beta, int accum_beta) {
  const int nkj = g.nbw * g.nba;
  const int total = g.T * nkj * g.O;
  const int lane = threadIdx.x & 63;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < total; t += gridDim.x * 4) {
    const int o = t % g.O, r = t / g.O;
    const int j = r % g.nba, r2 = r / g.nba;
    const int k = r2 % g.nbw, i = r2 / g.nbw;
    const int kj = k * g.nba + j;
    float a = 0.f, c = 0.f;
    for (int ch = lane; ch < nsc; ch += 64) {
      const size_t base = (((size_t)ch * g.T + i) * 2) * nkj * g.Opad + (size_t)kj * g.Opad + o;
      a += slab[base];
      c += slab[base + (size_t)nkj * g.Opad];
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      a += __shfl_xor(a, d);
      c += __shfl_xor(c, d);
    }
    if (lane == 0) {
      const float mk = (float)bmask[kj];  // binary_mask[0, 0, k, j, 0, 0]
      grad_alpha[t] = a * mk;
      grad_beta[t] = accum_beta ? grad_beta[t] + c * mk : c * mk;  // torch's AccumulateGrad when asked
    }
  }
}

typedef void (*StatsKernel)(Geo, V3, const uint8_t*, const v4i*, Params, const float*, const float*, const float*,
                            const float*, int, float*, int);
template <int KS, int NS, bool LUT>
StatsKernel stats_ptr() {
  return shift_stats_kernel<KS, NS, LUT>;
}

int launch_shift_stats(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
                       const int8_t* bmask, uint8_t* ws, float* grad_alpha, float* grad_beta, hipStream_t s,
                       int accum_beta) {
  const Plan3 p = v3_plan(g);
  if (!p.ok || !shift_stats_ok(g)) return fail(CIMQ_EUNSUPPORTED, "internal: shift statistics off the fast path");
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const int nsc = shift_chunks(g);
  const int nkj = g.nbw * g.nba;
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  float* slab = reinterpret_cast<float*>(ws + W.ss_slab);
  if (g.NBP == 8) {  // the w8a8 first conv (shift_stats_ok: one K-step)
    const int ncx = (std::min(g.K, g.xbar) - 1) / g.KHW + 1;
    const size_t lds = (size_t)4 * 2 * 64 * 16 * 4 + (size_t)64 * 16 * 8 + (size_t)8 * 64 * 16 + 64 * 4 +
                       a16((size_t)ncx * p.v.RH * p.v.WP * 8);
    CIMQ_TRY(set_lds(shift_stats8_kernel, lds));
    hipLaunchKernelGGL(shift_stats8_kernel, dim3(nsc, g.T * g.OB16), dim3(256), lds, s, g, p.v, ctx + L.xcode,
                       reinterpret_cast<const v4i*>(wreg(g, const_cast<uint8_t*>(ctx)) + L.wfrag), pp, sw, sa, gout,
                       slab, nsc);
    CIMQ_TRY(check_hip("shift_stats8"));
    const int total = g.T * nkj * g.O;
    hipLaunchKernelGGL(shift_combine_kernel, dim3(std::min(cdiv(total, 4), 2048)), dim3(256), 0, s, g, slab, nsc,
                       bmask, grad_alpha, grad_beta, accum_beta);
    return check_hip("shift_combine");
  }
  const bool lut = shift_table_fits(g);
  const int R = shift_table_range(g);
  float* qtab = reinterpret_cast<float*>(ws + W.qtab);
  if (lut) {
    const long long nt = (long long)g.T * g.OB16 * nkj * 16 * (2 * R + 1);
    hipLaunchKernelGGL(shift_qtab_kernel, dim3((unsigned)std::min<long long>(cdiv(nt, 256), 2048)), dim3(256), 0, s, g,
                       pp, sw, sa, R, qtab);
    CIMQ_TRY(check_hip("shift_qtab"));
  }
  int ncmax = 1;
  for (int i = 0; i < g.T; ++i) {
    const int c_lo = (i * g.xbar) / g.KHW, c_hi = (std::min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
    ncmax = std::max(ncmax, c_hi - c_lo + 1);
  }
  const size_t lds = (lut ? a16((size_t)nkj * 16 * (2 * R + 1) * 4) : 0) + a16((size_t)ncmax * p.v.RH * p.v.WP * 4) +
                     (size_t)g.KS * 64 * 4 + (size_t)4 * 2 * nkj * 16 * 4;
  StatsKernel kern;
  if (g.KS == 1 && g.nbw == 2) kern = lut ? stats_ptr<1, 2, true>() : stats_ptr<1, 2, false>();
  else if (g.KS == 1) kern = lut ? stats_ptr<1, 3, true>() : stats_ptr<1, 3, false>();
  else if (g.nbw == 2) kern = lut ? stats_ptr<2, 2, true>() : stats_ptr<2, 2, false>();
  else kern = lut ? stats_ptr<2, 3, true>() : stats_ptr<2, 3, false>();
  CIMQ_TRY(set_lds(kern, lds));
  hipLaunchKernelGGL(kern, dim3(nsc, g.T * g.OB16), dim3(256), lds, s, g, p.v, ctx + L.xcode,
                     reinterpret_cast<const v4i*>(wreg(g, const_cast<uint8_t*>(ctx)) + L.wfrag), pp, sw, sa, gout,
                     qtab, R, slab, nsc);
  CIMQ_TRY(check_hip("shift_stats"));
  const int total = g.T * nkj * g.O;
  hipLaunchKernelGGL(shift_combine_kernel, dim3(std::min(cdiv(total, 4), 2048)), dim3(256), 0, s, g, slab, nsc,
                     bmask, grad_alpha, grad_beta, accum_beta);
  return check_hip("shift_combine");
}

}  // namespace cimq

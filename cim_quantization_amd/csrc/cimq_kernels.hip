// cimq_kernels.hip -- CDNA4 (gfx950) kernels for the CiM partial-sum-quantised conv.
//
// Data flow (one layer):
//   prep_act      x (fp32) -> packed per-element act bit-slice codes + int8 ctx code
//   prep_weight   w_q      -> int8 MFMA fragments of the weight slices (forward / ps
//                             recompute), bf16 fragments of the truncated slices (grad_x)
//   prep_params   alpha_q, sw, sa -> integer ADC thresholds + STE intervals per
//                             (tile, a-slice, w-slice, out-channel)
//   cim_fwd       implicit im2col -> v_mfma_i32_16x16x64_i8 partial sums -> ADC -> shift-add
//   cim_bwd_gx    transposed ps recompute -> STE weights E -> bf16x3 MFMA -> col2im in LDS
//   cim_bwd_gw    ps recompute -> STE weights D, ADC codes -> bf16x3 MFMA over pixels -> slabs
//   reduce_*      deterministic slab sums (grad_w, grad_alpha, alpha init), LSQ backward
//
// Every integer step (codes, slices, partial sums, ADC codes, STE masks) is bit-exact with
// the reference's fp32 op sequence; the float reductions are fp32 (bf16x3 on MFMA).
#include "cimq_device.h"

namespace cimq {

#define WAVE 64

// =========================================================================================
// prep_act: per input element, the forward bit-slice integers and the backward ctx slices
// =========================================================================================
// x_int = x_q / sa (lsq.py:97); with RAW_LSQ, x_q = round_pass(clamp(x/sa,0,Qp))*sa first
// (lsq.py:549).  Forward slices follow slicing_act / slicing_act_signed on x_int
// (lsq.py:146-149) and are stored as rint() int8s (|residue| << 0.5, so the int8 MAC gives
// round(ps_ref)).  Backward slices are those of the int8 ctx code int8(x_int) (lsq.py:99,
// truncation + wrap) as re-sliced by the backward (lsq.py:290-295).  Both are written as
// NBP-byte words per element (byte j = slice j), once, so no kernel re-slices per gather.
__device__ inline void pack_word(int8_t (&v)[8], int nbp, uint8_t* dst, long long idx) {
  uint32_t lo = (uint8_t)v[0] | ((uint32_t)(uint8_t)v[1] << 8) | ((uint32_t)(uint8_t)v[2] << 16) |
                ((uint32_t)(uint8_t)v[3] << 24);
  if (nbp == 4) {
    reinterpret_cast<uint32_t*>(dst)[idx] = lo;
  } else {
    uint2 w;
    w.x = lo;
    w.y = (uint8_t)v[4] | ((uint32_t)(uint8_t)v[5] << 8) | ((uint32_t)(uint8_t)v[6] << 16) |
          ((uint32_t)(uint8_t)v[7] << 24);
    reinterpret_cast<uint2*>(dst)[idx] = w;
  }
}

__device__ inline void act_item(const Geo& g, const float* __restrict__ x, float sa, bool sgn,
                                uint8_t* __restrict__ xcf, uint8_t* __restrict__ xcb, long long idx) {
  float v = x[idx];
  float xq;
  if (g.input_kind == 1) {
    float t = v / sa;
    float c = clamp_nan(t, 0.f, g.lsq_qp);
    float r = rintf(c);
    float rp = (r - c) + c;  // round_pass value
    xq = rp * sa;
  } else {
    xq = v;
  }
  const float xi = xq / sa;
  const float xh = (float)to_i8_wrap(xi);
  int8_t fw[8], bw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f, sb = 0.f;
    if (j < g.nba) {
      s = sgn ? slice_signed(xi, j, g.bsa) : slice_unsigned(xi, j, g.bsa);
      sb = sgn ? slice_signed(xh, j, g.bsa) : slice_unsigned(xh, j, g.bsa);
    }
    fw[j] = (j < g.nba) ? (int8_t)clamp_i8(s) : (int8_t)0;
    bw[j] = (j < g.nba) ? (int8_t)clamp_i8(sb) : (int8_t)0;
  }
  pack_word(fw, g.NBP, xcf, idx);
  pack_word(bw, g.NBP, xcb, idx);
}

// Slice words of one element, NBP-specialised.  When x_int is an exact integer (the common
// case: fl(fl(r*sa)/sa) == r) the floor / remainder chain of slicing_act(_signed) reduces to
// shifts and masks of that integer, bit for bit (floor-mod by 2^b of an integer is its low b
// bits in two's complement); other values (the 6 - eps slice artifacts) take the float path.
// NBA_C > 0: nba = NBA_C and bsa = 1 at compile time (the unrolled digit loop has no runtime
// bounds); 0: read from g
template <int NBP, int NBA_C = 0>
__device__ inline void act_words_xq(const Geo& g, float xq, float sa, bool sgn, uint32_t (&fwd)[NBP / 4],
                                    uint32_t (&bwd)[NBP / 4]) {
  const int nba = NBA_C > 0 ? NBA_C : g.nba;
  const int bsa = NBA_C > 0 ? 1 : g.bsa;
  const float xi = xq / sa;
  const int xhi = to_i8_wrap(xi);
  const int mask = (1 << bsa) - 1;
  // forward digits without branches for |xi| < 2^23: with F = floor(m) and fr = m - F (both
  // exact), m = xi (unsigned) or |xi| (signed, digits negated for xi < 0), the reference's
  // chain gives digit 0 = rint((F mod 2^b) + fr) -- 2^b for the 6 - eps artifacts -- and digit
  // j = (F >> b*j) mod 2^b (floor(floor(m) / 2^s) = floor(m / 2^s)); larger |xi| or NaN take
  // the float chain below
  const bool fast = fabsf(xi) < 8388608.f;
  const float m = sgn ? fabsf(xi) : xi;
  const float F = floorf(m);
  const int Fi = fast ? (int)F : 0;
  const float fr = m - F;
  const bool negd = sgn && xi < 0.f;
#pragma unroll
  for (int w = 0; w < NBP / 4; ++w) { fwd[w] = 0u; bwd[w] = 0u; }
#pragma unroll
  for (int j = 0; j < NBP; ++j) {
    if (j < nba) {
      const int sh = bsa * j;
      const int sb = sgn ? (xhi >= 0 ? ((xhi >> sh) & mask) : -(((-xhi) >> sh) & mask)) : ((xhi >> sh) & mask);
      int d = (j == 0) ? min((int)rintf((float)(Fi & mask) + fr), 127) : ((Fi >> sh) & mask);
      const int sf = negd ? -d : d;
      fwd[j >> 2] |= (uint32_t)(uint8_t)(int8_t)sf << (8 * (j & 3));
      bwd[j >> 2] |= (uint32_t)(uint8_t)(int8_t)sb << (8 * (j & 3));
    }
  }
  if (!fast) {
#pragma unroll
    for (int w = 0; w < NBP / 4; ++w) fwd[w] = 0u;
#pragma unroll
    for (int j = 0; j < NBP; ++j) {
      if (j < nba) {
        const int sf = clamp_i8(sgn ? slice_signed(xi, j, bsa) : slice_unsigned(xi, j, bsa));
        fwd[j >> 2] |= (uint32_t)(uint8_t)(int8_t)sf << (8 * (j & 3));
      }
    }
  }
}

// x_q of one element: with RAW_LSQ the activation quantiser round_pass(clamp(x/sa,0,Qp))*sa
// (lsq.py:549), else the input itself
__device__ inline float act_xq(const Geo& g, float v, float sa) {
  if (g.input_kind != 1) return v;
  const float t = v / sa;
  const float c = clamp_nan(t, 0.f, g.lsq_qp);
  const float r = rintf(c);
  const float rp = (r - c) + c;  // round_pass value
  return rp * sa;
}

template <int NBP, int NBA_C = 0>
__device__ inline void act_words(const Geo& g, float v, float sa, bool sgn, uint32_t (&fwd)[NBP / 4],
                                 uint32_t (&bwd)[NBP / 4]) {
  act_words_xq<NBP, NBA_C>(g, act_xq(g, v, sa), sa, sgn, fwd, bwd);
}

// RAW_LSQ: the words depend on the element only through the integer code r = rint(clamp(x/sa,
// 0, Qp)) -- round_pass gives rp = (r - c) + c = r exactly for c in [0, Qp], so x_q = r * sa --
// so a block tabulates the Qp + 1 words once (with the same act_words_xq) and each element
// takes the quantiser's division, clamp and rint, then a table lookup; a NaN code (NaN input)
// takes the element-wise chain.  lut: [Qp + 1][fwd words, bwd words] in LDS.
constexpr int kActLutMax = 256;
template <int NBP, int NBA_C>
__device__ inline void act_lut_build(const Geo& g, float sa, bool sgn, uint32_t* lut) {
  const int nl = (int)g.lsq_qp + 1;
  for (int r = threadIdx.x; r < nl; r += blockDim.x) {
    uint32_t f[NBP / 4], b[NBP / 4];
    act_words_xq<NBP, NBA_C>(g, (float)r * sa, sa, sgn, f, b);
#pragma unroll
    for (int w = 0; w < NBP / 4; ++w) {
      lut[r * (NBP / 2) + w] = f[w];
      lut[r * (NBP / 2) + NBP / 4 + w] = b[w];
    }
  }
  __syncthreads();
}
template <int NBP, int NBA_C>
__device__ inline void act_words_lut(const Geo& g, float v, float sa, bool sgn, const uint32_t* lut,
                                     uint32_t (&fwd)[NBP / 4], uint32_t (&bwd)[NBP / 4]) {
  const float c = clamp_nan(v / sa, 0.f, g.lsq_qp);
  const float r = rintf(c);
  if (r == r) {
    const int e = (int)r * (NBP / 2);
    if (NBP == 4) {
      const uint2 t = *reinterpret_cast<const uint2*>(lut + e);
      fwd[0] = t.x;
      bwd[0] = t.y;
    } else {
      const uint4 t = *reinterpret_cast<const uint4*>(lut + e);
      fwd[0] = t.x;
      fwd[NBP / 4 - 1] = t.y;
      bwd[0] = t.z;
      bwd[NBP / 4 - 1] = t.w;
    }
  } else {
    act_words<NBP, NBA_C>(g, v, sa, sgn, fwd, bwd);
  }
}

// four consecutive elements (idx4 = 4 * t): one 16-B load, 16-B (NBP 4) or 2 x 16-B stores
template <int NBP, int NBA_C = 0>
__device__ inline void act_item4(const Geo& g, const float* __restrict__ x, float sa, bool sgn,
                                 uint8_t* __restrict__ xcf, uint8_t* __restrict__ xcb, long long t,
                                 const uint32_t* lut = nullptr) {
  const float4 v4 = reinterpret_cast<const float4*>(x)[t];
  const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
  uint32_t f[4][NBP / 4], b[4][NBP / 4];
  if (lut) {
#pragma unroll
    for (int e = 0; e < 4; ++e) act_words_lut<NBP, NBA_C>(g, vv[e], sa, sgn, lut, f[e], b[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) act_words<NBP, NBA_C>(g, vv[e], sa, sgn, f[e], b[e]);
  }
  if (NBP == 4) {
    reinterpret_cast<uint4*>(xcf)[t] = make_uint4(f[0][0], f[1][0], f[2][0], f[3][0]);
    reinterpret_cast<uint4*>(xcb)[t] = make_uint4(b[0][0], b[1][0], b[2][0], b[3][0]);
  } else {
    reinterpret_cast<uint4*>(xcf)[2 * t] = make_uint4(f[0][0], f[0][NBP / 4 - 1], f[1][0], f[1][NBP / 4 - 1]);
    reinterpret_cast<uint4*>(xcf)[2 * t + 1] = make_uint4(f[2][0], f[2][NBP / 4 - 1], f[3][0], f[3][NBP / 4 - 1]);
    reinterpret_cast<uint4*>(xcb)[2 * t] = make_uint4(b[0][0], b[0][NBP / 4 - 1], b[1][0], b[1][NBP / 4 - 1]);
    reinterpret_cast<uint4*>(xcb)[2 * t + 1] = make_uint4(b[2][0], b[2][NBP / 4 - 1], b[3][0], b[3][NBP / 4 - 1]);
  }
}

// all elements of x: vectorised when Nin % 4 == 0 (W % 4 == 0), element-wise otherwise
template <int NBP, int NBA_C>
__device__ inline void act_range_sel(const Geo& g, const float* __restrict__ x, float sa, bool sgn,
                                     uint8_t* __restrict__ xcf, uint8_t* __restrict__ xcb, long long first,
                                     long long step, uint32_t* lut) {
  const long long n4 = g.Nin / 4;
  const bool tab = lut && g.input_kind == 1 && g.lsq_qp >= 0.f && g.lsq_qp < (float)kActLutMax;
  if (tab) act_lut_build<NBP, NBA_C>(g, sa, sgn, lut);  // block-uniform condition: every thread syncs
  for (long long t = first; t < n4; t += step) act_item4<NBP, NBA_C>(g, x, sa, sgn, xcf, xcb, t, tab ? lut : nullptr);
}

// lut: LDS for the RAW_LSQ word table (kActLutMax * NBP / 2 words), or null; called by every
// thread of the block
__device__ inline void act_range(const Geo& g, const float* __restrict__ x, float sa, bool sgn,
                                 uint8_t* __restrict__ xcf, uint8_t* __restrict__ xcb, long long first,
                                 long long step, uint32_t* lut = nullptr) {
  if (g.Nin % 4 == 0) {
    const long long n4 = g.Nin / 4;
    // the 1-bit-slice cases of the CIFAR / QuantLinear configs with compile-time digit loops
    const int sel = g.bsa != 1 ? 0 : g.nba;
    if (sel == 3)
      act_range_sel<4, 3>(g, x, sa, sgn, xcf, xcb, first, step, lut);
    else if (sel == 2)
      act_range_sel<4, 2>(g, x, sa, sgn, xcf, xcb, first, step, lut);
    else if (sel == 4)
      act_range_sel<4, 4>(g, x, sa, sgn, xcf, xcb, first, step, lut);
    else if (sel == 8)
      act_range_sel<8, 8>(g, x, sa, sgn, xcf, xcb, first, step, lut);
    else if (g.NBP == 4)
      for (long long t = first; t < n4; t += step) act_item4<4>(g, x, sa, sgn, xcf, xcb, t);
    else
      for (long long t = first; t < n4; t += step) act_item4<8>(g, x, sa, sgn, xcf, xcb, t);
  } else {
    for (long long idx = first; idx < g.Nin; idx += step) act_item(g, x, sa, sgn, xcf, xcb, idx);
  }
}

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void prep_act_kernel(Geo g, const float* __restrict__ x, const float* __restrict__ sa_p,
                                const float* __restrict__ signed_p, uint8_t* __restrict__ xcf,
                                uint8_t* __restrict__ xcb) {
  const float sa = *sa_p;
  const bool sgn = (*signed_p) != 0.f;
  act_range(g, x, sa, sgn, xcf, xcb, (long long)blockIdx.x * blockDim.x + threadIdx.x,
            (long long)gridDim.x * blockDim.x);
}
#endif

// =========================================================================================
// prep_weight: MFMA fragments of the weight bit slices
// =========================================================================================
// w_int = w_q / sw (lsq.py:98), w_unf = w_int.view(O,-1).t() (lsq.py:153), signed slices
// (lsq.py:155).  Forward / ps-recompute operand: rint(slice) as int8, stored in the exact
// per-lane order of v_mfma_i32_16x16x64_i8: wfrag[i][ks][nb][lane][16 bytes], lane l holding
// rows n = nb*16 + (l&15) (n = k*Opad + o) and contraction f = i*xbar + ks*64 + 16*(l>>4) + e.
// grad_x operand: int8(slice) (lsq.py:160 truncation) as bf16, wgx[i][fb][s][lane][8]:
// lane l holds f = i*xbar + fb*16 + (l&15), kappa = (2s + (e>>2))*16 + 4*(l>>4) + (e&3).
// Source of the integer weights w_int = w_q / sw: either a materialised w_q (Function entry
// points) or the raw weight run through the LSQ quantiser in place (module entry points:
// w_q = round_pass(clamp(w / sw, Qn, Qp)) * sw, lsq.py:555, the same fp32 op sequence).
struct WSrc {
  const float* w;
  float sw;
  int raw;
  float qn, qp;
  __device__ float wint(const Geo& g, int o, int f) const {
    const float v = w[(size_t)o * g.K + f];
    if (!raw) return v / sw;
    const float c = clamp_nan(v / sw, qn, qp);
    const float wq = round_pass_value(c) * sw;
    return wq / sw;
  }
};

__device__ inline float wslice(const Geo& g, const WSrc& ws, int f, int n) {
  const int k = n / g.Opad, o = n - k * g.Opad;
  if (f >= g.K || o >= g.O || k >= g.nbw) return 0.f;
  return slice_signed(ws.wint(g, o, f), k, g.bsw);
}

__device__ inline void wfrag_item(const Geo& g, const WSrc& ws, v4i* __restrict__ wfrag, int t) {
  const int lane = t % WAVE;
  int r = t / WAVE;
  const int nb = r % g.NBLK;
  r /= g.NBLK;
  const int ks = r % g.KS;
  const int i = r / g.KS;
  const int flo = i * g.xbar, fhi = min(flo + g.xbar, g.K);
  const int n = nb * 16 + (lane & 15);
  uint32_t wd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int f = flo + ks * 64 + 16 * (lane >> 4) + e;
    int v = 0;
    if (f < fhi) v = clamp_i8(wslice(g, ws, f, n));
    wd[e >> 2] |= ((uint32_t)(uint8_t)(int8_t)v) << (8 * (e & 3));
  }
  v4i o;
  o.x = (int)wd[0]; o.y = (int)wd[1]; o.z = (int)wd[2]; o.w = (int)wd[3];
  wfrag[t] = o;
}

__device__ inline void wgx_item(const Geo& g, const WSrc& ws, v4i* __restrict__ wgx, int t) {
  const int lane = t % WAVE;
  int r = t / WAVE;
  const int s = r % g.NKS;
  r /= g.NKS;
  const int fb = r % g.FBT;
  const int i = r / g.FBT;
  const int flo = i * g.xbar, fhi = min(flo + g.xbar, g.K);
  const int f = flo + fb * 16 + (lane & 15);
  uint32_t wd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kb = 2 * s + (e >> 2);
    const int kap = kb * 16 + 4 * (lane >> 4) + (e & 3);
    float v = 0.f;
    if (f < fhi && kb < g.NBLK) v = (float)to_i8_wrap(wslice(g, ws, f, kap));
    const uint32_t h = bf16_bits(v);
    wd[e >> 1] |= h << (16 * (e & 1));
  }
  v4i o;
  o.x = (int)wd[0]; o.y = (int)wd[1]; o.z = (int)wd[2]; o.w = (int)wd[3];
  wgx[t] = o;
}

// v8 grad_x operand (cimq_v7.hip): the same int8(slice) values as wgx with the MFMA rows
// re-ordered so that row rho = 4*q + kw of cp-block cpb is weight row f = cp*KW + kw,
// cp = cpb*4 + q = c*KH + kh (rho & 3 == 3 and rows outside tile i are zero): one lane of the
// product then holds all KW taps of one (c, kh) for its pixel.  wcy[i][cb][s][lane][8 bf16],
// cpb = cpb_lo(i) + cb, cpb_lo(i) = ((i*xbar) / KW) / 4, cb < ncpbt.
__device__ inline void wcy_item(const Geo& g, const WSrc& ws, int ncpbt, v4i* __restrict__ wcy, int t) {
  const int lane = t % WAVE;
  int r = t / WAVE;
  const int s = r % g.NKS;
  r /= g.NKS;
  const int cb = r % ncpbt;
  const int i = r / ncpbt;
  const int flo = i * g.xbar, fhi = min(flo + g.xbar, g.K);
  const int rho = lane & 15;
  const int cp = ((flo / g.KW) / 4 + cb) * 4 + (rho >> 2), kw = rho & 3;
  const int c = cp / g.KH, kh = cp - c * g.KH;
  const int f = c * g.KHW + kh * g.KW + kw;
  const bool ok = kw < g.KW && c < g.C && f >= flo && f < fhi;
  uint32_t wd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kb = 2 * s + (e >> 2);
    const int kap = kb * 16 + 4 * (lane >> 4) + (e & 3);
    float v = 0.f;
    if (ok && kb < g.NBLK) v = (float)to_i8_wrap(wslice(g, ws, f, kap));
    wd[e >> 1] |= (uint32_t)bf16_bits(v) << (16 * (e & 1));
  }
  v4i o;
  o.x = (int)wd[0]; o.y = (int)wd[1]; o.z = (int)wd[2]; o.w = (int)wd[3];
  wcy[t] = o;
}


#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void prep_wfrag_kernel(Geo g, const float* __restrict__ w_q, const float* __restrict__ sw_p,
                                  v4i* __restrict__ wfrag) {
  const WSrc ws{w_q, *sw_p, 0, 0.f, 0.f};
  const int total = g.T * g.KS * g.NBLK * WAVE;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x)
    wfrag_item(g, ws, wfrag, t);
}
#endif

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void prep_wgx_kernel(Geo g, const float* __restrict__ w_q, const float* __restrict__ sw_p,
                                v4i* __restrict__ wgx) {
  const WSrc ws{w_q, *sw_p, 0, 0.f, 0.f};
  const int total = g.T * g.FBT * g.NKS * WAVE;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x)
    wgx_item(g, ws, wgx, t);
}
#endif

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void prep_wcy_kernel(Geo g, const float* __restrict__ w_q, const float* __restrict__ sw_p, int ncpbt,
                                v4i* __restrict__ wcy) {
  const WSrc ws{w_q, *sw_p, 0, 0.f, 0.f};
  const int total = g.T * ncpbt * g.NKS * WAVE;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x)
    wcy_item(g, ws, ncpbt, wcy, t);
}
#endif

// =========================================================================================
// prep_params: ADC thresholds and STE intervals by exact binary search over integer ps
// =========================================================================================
// The ADC code and the STE mask are monotone step functions of the integer partial sum
// (each op in u = fp16(ps)*sw*sa, u/alpha, rint, clamp is monotone for sw*sa > 0 and
// alpha > 0), so they are captured exactly by integer thresholds found with the very
// same fp32 ops.  Anything else (alpha_q <= 0 / NaN -- e.g. all-equal alpha_cim gives
// NaN, lsq.py:570-571 -- or non-positive scales) sets flags[0]: kernels then evaluate
// the ADC literally per partial sum.
__device__ inline int first_true_ternary_hi(int lo, int hi, float sw, float sa, float a) {
  // smallest p in [lo, hi] with rint(u/a) >= 1 ; hi+1 if none
  int L = lo, R = hi + 1;
  while (L < R) {
    int mid = L + ((R - L) >> 1);
    float q = rintf(u_of(mid, sw, sa) / a);
    if (q >= 1.f) R = mid; else L = mid + 1;
  }
  return L;
}
__device__ inline int last_true_ternary_lo(int lo, int hi, float sw, float sa, float a) {
  // largest p in [lo, hi] with rint(u/a) <= -1 ; lo-1 if none
  int L = lo - 1, R = hi;
  while (L < R) {
    int mid = L + ((R - L + 1) >> 1);
    float q = rintf(u_of(mid, sw, sa) / a);
    if (q <= -1.f) L = mid; else R = mid - 1;
  }
  return L;
}

// Source of alpha_q: a materialised alpha_q, or alpha_cim through its quantiser in place
// (alpha_q = clamp(round_pass(a / scale), 1, 2^b - 1) * scale, lsq.py:566-571).
struct ASrc {
  const float* a;
  int raw;
  float scale, qp_al;
  __device__ float get(int e) const {
    if (!raw) return a[e];
    const float t = a[e] / scale;
    return clamp_nan(round_pass_value(t), 1.f, qp_al) * scale;
  }
};

__device__ inline bool scales_ok(float sw, float sa) {
  return (sw * sa > 0.f) && isfinite(sw * sa) && isfinite(sw) && isfinite(sa);
}

// one (i, j, k, o) entry (t < npar) or one (k, j) coefficient triple (t >= npar); returns
// whether the entry needs the literal ADC
__device__ inline bool params_item(const Geo& g, const ASrc& as, float sw, float sa,
                                   const int8_t* __restrict__ bmask, const Params& pp, int t,
                                   const float* __restrict__ beta = nullptr) {
  const int npar = g.T * g.nba * g.nbw * g.Opad;
  const int nkj = g.nbw * g.nba;
  if (t >= npar + nkj) {  // shift ADC: sum_{i,k,j} beta * mask of channel o, added to every output
    const int o = t - npar - nkj;
    float b = 0.f;
    if (beta != nullptr && o < g.O)
      for (int i = 0; i < g.T; ++i)
        for (int k = 0; k < g.nbw; ++k)
          for (int j = 0; j < g.nba; ++j)
            b += beta[((i * g.nbw + k) * g.nba + j) * g.O + o] * (float)bmask[k * g.nba + j];
    pp.bsum[o] = b;
    return false;
  }
  if (t >= npar) {  // per-(k,j) float coefficients
    const int kj = t - npar, k = kj / g.nba, j = kj - k * g.nba;
    const float mk = (float)bmask[k * g.nba + j];  // binary_mask[0,0,k,j,0,0]
    pp.ckj[kj] = mk;
    pp.ckj[nkj + kj] = mk * pow2f(-g.bsa * j);      // E weight: 2^-(bsa*j) * mask
    pp.ckj[2 * nkj + kj] = mk * pow2f(-g.bsw * k);  // D weight: 2^-(bsw*k) * mask
    return false;
  }
  int r = t;
  const int o = r % g.Opad; r /= g.Opad;
  const int k = r % g.nbw; r /= g.nbw;
  const int j = r % g.nba;
  const int i = r / g.nba;
  const float mk = (float)bmask[k * g.nba + j];
  float a = 1.f;
  if (has_alpha(g) && as.a != nullptr && o < g.O)
    a = as.get(((i * g.nbw + k) * g.nba + j) * g.O + o);  // alpha[0,i,k,j,0,o]
  pp.alpha[t] = a;
  pp.beta[t] = (beta != nullptr && o < g.O) ? beta[((i * g.nbw + k) * g.nba + j) * g.O + o] : 0.f;
  pp.coef[t] = a * mk;
  const int lo = -g.psmax - 1, hi = g.psmax + 1;
  bool literal = false;
  int thi = hi + 1, tlo = lo - 1, mlo = hi + 1, mhi = lo - 1;
  if (g.mode == ADC_SIGN || g.mode == ADC_TERNARY) {
    if (!(scales_ok(sw, sa) && a > 0.f && isfinite(a))) literal = true;
  }
  // the variants are evaluated per partial sum, except the shift ADC of the fast path
  const bool sf = shift_fast(g);
  const float be = pp.beta[t];
  if (g.variant != VAR_LIBRARY && !sf) literal = true;
  if (sf && !isfinite(be)) literal = true;
  if (!literal) {
    if (sf) {
      // v = (u - beta) / alpha (scale_shift.py:421): code +1 <=> rint(v) >= 1, -1 <=> rint(v) <= -1
      int L = lo, R = hi + 1;
      while (L < R) {
        const int mid = L + ((R - L) >> 1);
        if (rintf(psb_value(g, mid, sw, sa, a, be)) >= 1.f) R = mid; else L = mid + 1;
      }
      thi = L;
      L = lo - 1; R = hi;
      while (L < R) {
        const int mid = L + ((R - L + 1) >> 1);
        if (rintf(psb_value(g, mid, sw, sa, a, be)) <= -1.f) L = mid; else R = mid - 1;
      }
      tlo = L;
    } else if (g.mode == ADC_TERNARY) {
      thi = first_true_ternary_hi(lo, hi, sw, sa, a);
      tlo = last_true_ternary_lo(lo, hi, sw, sa, a);
    }
    // STE interval: psb(p) monotone non-decreasing in p
    {
      int L = lo, R = hi + 1;  // first p with psb > thr_lo  (i.e. not "<= thr_lo")
      while (L < R) {
        int mid = L + ((R - L) >> 1);
        float b = sf ? psb_value(g, mid, sw, sa, a, be) : psb_literal(mid, g.mode, sw, sa, a);
        if (b > g.thr_lo) R = mid; else L = mid + 1;
      }
      mlo = L;
      L = lo - 1; R = hi;  // last p with psb < thr_hi
      while (L < R) {
        int mid = L + ((R - L + 1) >> 1);
        float b = sf ? psb_value(g, mid, sw, sa, a, be) : psb_literal(mid, g.mode, sw, sa, a);
        if (b < g.thr_hi) L = mid; else R = mid - 1;
      }
      mhi = L;
    }
  }
  pp.thi[t] = thi;
  pp.tlo[t] = tlo;
  // STE interval as (lo, span): pass <=> (unsigned)(ps - lo) <= (unsigned)span
  if (mhi >= mlo) { pp.mlo[t] = mlo; pp.mhi[t] = mhi - mlo; }
  else { pp.mlo[t] = -(1 << 30); pp.mhi[t] = 0; }
  return literal;
}

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void prep_params_kernel(Geo g, const float* __restrict__ alpha_q, const float* __restrict__ sw_p,
                                   const float* __restrict__ sa_p, const int8_t* __restrict__ bmask,
                                   Params pp, const float* __restrict__ beta) {
  const float sw = *sw_p, sa = *sa_p;
  const ASrc as{alpha_q, 0, 0.f, 0.f};
  const int total = g.T * g.nba * g.nbw * g.Opad + g.nbw * g.nba + (beta != nullptr ? g.Opad : 0);
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x)
    if (params_item(g, as, sw, sa, bmask, pp, t, beta)) pp.flags[0] = 1;  // every writer stores 1
}
#endif

// =========================================================================================
// shared tile machinery: implicit im2col of the packed act codes into LDS
// =========================================================================================
// LDS image of one crossbar tile for 64 output pixels: As[j][row][KTP] int8 (row = pixel,
// contiguous f), built from the packed per-element codes; out-of-image taps are 0 (the
// zero padding of nn.Unfold).  Tables: foff[f] = c*H*W + kh*W + kw, fkk[f] = kh<<16|kw
// (-1 = beyond the tile), rowinfo[r] = {img base + ih0*W + iw0, ih0, iw0, valid}.
struct TileSmem {
  int8_t* As;     // [nba][64][KTP]
  int* foff;      // [KS*64]
  int* fkk;       // [KS*64]
  int4* rowinfo;  // [64]
};

__device__ inline void build_rowinfo(const Geo& g, int m0, int4* rowinfo) {
  const int t = threadIdx.x;
  if (t < 64) {
    const int m = m0 + t;
    int4 ri = make_int4(0, 0, 0, 0);
    if (m < g.M) {
      const int b = m / g.P, p = m - b * g.P;
      const int oh = p / g.Wo, ow = p - oh * g.Wo;
      const int ih0 = oh * g.SH - g.PH, iw0 = ow * g.SW - g.PW;
      ri = make_int4(b * g.C * g.HW + ih0 * g.W + iw0, ih0, iw0, 1);
    }
    rowinfo[t] = ri;
  }
}

__device__ inline void build_ftable(const Geo& g, int i, int* foff, int* fkk) {
  const int flo = i * g.xbar, flen = min(g.xbar, g.K - flo);
  for (int t = threadIdx.x; t < g.KS * 64; t += blockDim.x) {
    if (t < flen) {
      const int f = flo + t;
      const int c = f / g.KHW, rem = f - c * g.KHW;
      const int kh = rem / g.KW, kw = rem - kh * g.KW;
      foff[t] = c * g.HW + kh * g.W + kw;
      fkk[t] = (kh << 16) | kw;
    } else {
      foff[t] = 0;
      fkk[t] = -1;
    }
  }
}

// Gather one element's packed code (all slices) for pixel row r and tile column t.
template <int NBP>
__device__ inline uint2 gather_code(const Geo& g, const int8_t* __restrict__ xcode, const int4 ri,
                                    int fo, int fk) {
  uint2 c = make_uint2(0, 0);
  if (fk >= 0 && ri.w) {
    const int kh = fk >> 16, kw = fk & 0xFFFF;
    const int ih = ri.y + kh, iw = ri.z + kw;
    if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) {
      const long long idx = (long long)ri.x + fo;
      if (NBP == 4) c.x = reinterpret_cast<const uint32_t*>(xcode)[idx];
      else c = reinterpret_cast<const uint2*>(xcode)[idx];
    }
  }
  return c;
}

// Build As for the 64 pixels of rowinfo and tile (foff/fkk): each work item is 4
// consecutive tile columns of one pixel; the per-slice bytes are transposed into one
// dword per slice plane.
template <int NBP>
__device__ inline void build_As(const Geo& g, const int8_t* __restrict__ xcode, const TileSmem& sm) {
  const int quads = g.KS * 16;
  const int items = 64 * quads;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int r = it / quads, q = it - r * quads;
    const int4 ri = sm.rowinfo[r];
    uint32_t pl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = 4 * q + e;
      const uint2 c = gather_code<NBP>(g, xcode, ri, sm.foff[t], sm.fkk[t]);
#pragma unroll
      for (int j = 0; j < 4; ++j) pl[j] |= ((c.x >> (8 * j)) & 0xFFu) << (8 * e);
      if (NBP == 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) pl[4 + j] |= ((c.y >> (8 * j)) & 0xFFu) << (8 * e);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < g.nba) *reinterpret_cast<uint32_t*>(sm.As + ((size_t)j * 64 + r) * g.KTP + 4 * q) = pl[j];
  }
}

// Load the 16-byte MFMA operand of slice plane j for row (base16 + (lane&15)).
__device__ inline v4i load_xfrag(const Geo& g, const int8_t* As, int j, int row, int ks, int lane) {
  const int8_t* p = As + ((size_t)j * 64 + row) * g.KTP + ks * 64 + 16 * (lane >> 4);
  return *reinterpret_cast<const v4i*>(p);
}

// =========================================================================================
// cim_fwd: partial sums + ADC + shift-and-add   (lsq.py:166-233)
// =========================================================================================
// Block = 64 output pixels x one 64-column output-channel group; wave w owns pixels
// [16w, 16w+16).  For every tile i, a-slice j, w-slice k:  ps = X_j(16 x tile) . W_k(tile x 16)
// on v_mfma_i32_16x16x64_i8 (exact integers), then the ADC code and out += code*alpha*mask.
// DBG: additionally write every integer partial sum and its ADC output (before the
// shift-and-add mask) in the reference's [B, T, nbw, nba, P, O] order (the ctx.ps_int of
// lsq.py:192 and adc_out of lsq.py:197-230) -- the parity hook of cimq_debug_partial_sums.
template <int NBP, bool DBG>
__global__ __launch_bounds__(256) void cim_fwd_kernel(Geo g, const int8_t* __restrict__ xcode,
                                                      const v4i* __restrict__ wfrag, Params pp,
                                                      const float* __restrict__ sw_p,
                                                      const float* __restrict__ sa_p,
                                                      float* __restrict__ out, int* __restrict__ ps_dbg,
                                                      float* __restrict__ adc_dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  TileSmem sm;
  sm.As = reinterpret_cast<int8_t*>(smem);
  size_t off = (size_t)g.nba * 64 * g.KTP;
  sm.foff = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.fkk = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.rowinfo = reinterpret_cast<int4*>(smem + off);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * 64;
  const int og = blockIdx.y;
  const int nob = min(4, g.OB16 - og * 4);
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0) || g.mode != ADC_TERNARY || g.variant != VAR_LIBRARY;
  const int nkj = g.nbw * g.nba;

  build_rowinfo(g, m0, sm.rowinfo);
  float acc_out[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc_out[a][b] = 0.f;

  for (int i = 0; i < g.T; ++i) {
    __syncthreads();
    build_ftable(g, i, sm.foff, sm.fkk);
    __syncthreads();
    build_As<NBP>(g, xcode, sm);
    __syncthreads();
    for (int j = 0; j < g.nba; ++j) {
      v4i a[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        if (ks < g.KS) a[ks] = load_xfrag(g, sm.As, j, wave * 16 + r16, ks, lane);
      for (int k = 0; k < g.nbw; ++k) {
        const float mk = pp.ckj[k * g.nba + j];
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) {
          if (ob < nob) {
            const int nb = k * g.OB16 + og * 4 + ob;
            v4i acc = {0, 0, 0, 0};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
              if (ks < g.KS)
                acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                    a[ks], wfrag[((size_t)(i * g.KS + ks) * g.NBLK + nb) * WAVE + lane], acc, 0, 0, 0);
            const int o = (og * 4 + ob) * 16 + r16;
            const int pi = pidx(g, i, j, k, o);
            if (DBG) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int m = m0 + wave * 16 + 4 * g4 + r;
                if (m < g.M && o < g.O) {
                  const int b = m / g.P, p = m - b * g.P;
                  const size_t di = ((((size_t)b * g.T + i) * g.nbw + k) * g.nba + j) * g.P * g.O +
                                    (size_t)p * g.O + o;
                  ps_dbg[di] = acc[r];
                  float adc;
                  if (!literal) {
                    const float q = (acc[r] >= pp.thi[pi]) ? 1.f : ((acc[r] <= pp.tlo[pi]) ? -1.f : 0.f);
                    adc = q * pp.alpha[pi];
                  } else {
                    adc = adc_value(g, acc[r], sw, sa, pp.alpha[pi], pp.beta[pi], (uint64_t)di);
                  }
                  adc_dbg[di] = adc;
                }
              }
            }
            if (!literal) {
              const int thi = pp.thi[pi], tlo = pp.tlo[pi];
              const float cf = pp.coef[pi];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int ps = acc[r];
                float v = (ps >= thi) ? cf : 0.f;
                v -= (ps <= tlo) ? cf : 0.f;
                acc_out[ob][r] += v;
              }
            } else {
              const float al = pp.alpha[pi], be = pp.beta[pi];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                uint64_t eid = 0;  // element id of the stochastic ADC's draws: [B, T, nbw, nba, P, O] order
                if (g.variant == VAR_STOCHASTIC) {
                  const int m = m0 + wave * 16 + 4 * g4 + r;
                  const int b = m / g.P, p = m - b * g.P;
                  eid = ((((uint64_t)b * g.T + i) * g.nbw + k) * g.nba + j) * (uint64_t)g.P * g.O + (uint64_t)p * g.O + o;
                }
                const float adc = adc_value(g, acc[r], sw, sa, al, be, eid);
                acc_out[ob][r] += adc * mk;
              }
            }
          }
        }
      }
    }
  }
  (void)nkj;
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    if (ob < nob) {
      const int o = (og * 4 + ob) * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wave * 16 + 4 * g4 + r;
        if (m < g.M && o < g.O) out[(size_t)m * g.O + o] = acc_out[ob][r];
      }
    }
  }
}

// =========================================================================================
// cim_bwd_gx: grad wrt the activation   (lsq.py:338-382, closed form)
// =========================================================================================
//   gx_unf[m,f] = sum_{k,o} g[m,o] * E_k[m,i(f),o] * w^_k[f,o]
//   E_k = sum_j 2^-(bsa*j) * mask[k,j] * STE[m,i,k,j,o]
// ps is recomputed TRANSPOSED (rows kappa=(k,o), columns = pixels) so each accumulator is
// directly the B operand of the next bf16 MFMA (contraction over kappa, no LDS transpose);
// g*E is split into three bf16 terms.  Block = (64 pixels, crossbar tile blockIdx.y): the
// tiles' f ranges are disjoint, so every unfolded value gxu[m][f] is written by exactly one
// lane; fold_gx_kernel then applies the nn.Fold adjoint (lsq.py:382) in a fixed order -- no
// atomics anywhere, bit-identical run to run.
template <int NBP, int FBMAX>
__global__ __launch_bounds__(256) void cim_bwd_gx_kernel(Geo g, const int8_t* __restrict__ xcode,
                                                         const v4i* __restrict__ wfrag,
                                                         const v4i* __restrict__ wgx, Params pp,
                                                         const float* __restrict__ sw_p,
                                                         const float* __restrict__ sa_p,
                                                         const float* __restrict__ gout,
                                                         float* __restrict__ gxu) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  TileSmem sm;
  sm.As = reinterpret_cast<int8_t*>(smem);
  size_t off = (size_t)g.nba * 64 * g.KTP;
  sm.foff = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.fkk = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.rowinfo = reinterpret_cast<int4*>(smem + off);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0) || g.variant != VAR_LIBRARY;
  const int nkj = g.nbw * g.nba;
  const int m0 = blockIdx.x * 64;
  const int i = blockIdx.y;
  const int flo = i * g.xbar, flen = min(g.xbar, g.K - flo);

  build_rowinfo(g, m0, sm.rowinfo);
  build_ftable(g, i, sm.foff, sm.fkk);
  __syncthreads();
  build_As<NBP>(g, xcode, sm);
  __syncthreads();

  const int mcol = m0 + wave * 16 + r16;  // this lane's pixel (accumulator column)
  const bool mvalid = sm.rowinfo[wave * 16 + r16].w != 0;
  v4f gxa[FBMAX];
#pragma unroll
  for (int fb = 0; fb < FBMAX; ++fb) gxa[fb] = v4f{0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < g.NBLK; kc += 8) {  // chunk of 8 kappa-blocks (4 MFMA K-steps)
    float E[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) E[a][b] = 0.f;
    for (int j = 0; j < g.nba; ++j) {
      v4i xb[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        if (ks < g.KS) xb[ks] = load_xfrag(g, sm.As, j, wave * 16 + r16, ks, lane);
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int kb = kc + kk;
        if (kb < g.NBLK) {
          v4i acc = {0, 0, 0, 0};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            if (ks < g.KS)
              acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                  wfrag[((size_t)(i * g.KS + ks) * g.NBLK + kb) * WAVE + lane], xb[ks], acc, 0, 0, 0);
          const int k = kb / g.OB16;
          const int obase = (kb - k * g.OB16) * 16 + 4 * g4;
          const float ce = pp.ckj[nkj + k * g.nba + j];
          const int pi = pidx(g, i, j, k, obase);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            bool pass;
            if (!literal) {
              pass = (unsigned)(acc[r] - pp.mlo[pi + r]) <= (unsigned)pp.mhi[pi + r];
            } else {
              const float b = psb_value(g, acc[r], sw, sa, pp.alpha[pi + r], pp.beta[pi + r]);
              pass = ste_pass(b, g.thr_hi, g.thr_lo);
            }
            E[kk][r] += pass ? ce : 0.f;
          }
        }
      }
    }
    // B operands: (g * E)[kappa, pixel], kappa-step s covers kappa-blocks kc+2s, kc+2s+1
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kb0 = kc + 2 * s;
      if (kb0 < g.NBLK) {
        uint32_t hi[4] = {0, 0, 0, 0}, mi[4] = {0, 0, 0, 0}, lo[4] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int kb = kb0 + (e >> 2);
          const int r = e & 3;
          float av = 0.f;
          if (kb < g.NBLK && mvalid) {
            const int k = kb / g.OB16;
            const int o = (kb - k * g.OB16) * 16 + 4 * g4 + r;
            if (o < g.O) av = gout[(size_t)mcol * g.O + o] * E[2 * s + (e >> 2)][r];
          }
          uint16_t h, md, l;
          split3(av, h, md, l);
          hi[e >> 1] |= (uint32_t)h << (16 * (e & 1));
          mi[e >> 1] |= (uint32_t)md << (16 * (e & 1));
          lo[e >> 1] |= (uint32_t)l << (16 * (e & 1));
        }
        const v8bf bh = as_v8bf(v4i{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]});
        const v8bf bm = as_v8bf(v4i{(int)mi[0], (int)mi[1], (int)mi[2], (int)mi[3]});
        const v8bf bl = as_v8bf(v4i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]});
        const int sg = kc / 2 + s;
#pragma unroll
        for (int fb = 0; fb < FBMAX; ++fb) {
          if (fb < g.FBT) {
            const v8bf wa = as_v8bf(wgx[((size_t)(i * g.FBT + fb) * g.NKS + sg) * WAVE + lane]);
            gxa[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bh, gxa[fb], 0, 0, 0);
            gxa[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bm, gxa[fb], 0, 0, 0);
            gxa[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bl, gxa[fb], 0, 0, 0);
          }
        }
      }
    }
  }
  // gx_unf[pixel, f] of this tile's rows (accumulator row fb*16 + 4*g4 + r, column = pixel)
  if (mvalid) {
    float* dst = gxu + (size_t)mcol * g.K + flo;
#pragma unroll
    for (int fb = 0; fb < FBMAX; ++fb) {
      if (fb < g.FBT) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = fb * 16 + 4 * g4 + r;
          if (t < flen) dst[t] = gxa[fb][r];
        }
      }
    }
  }
}

// nn.Fold adjoint of the unfold (lsq.py:382): every input element sums its (kh, kw) window
// taps of gx_unf in a fixed order, times sw / nba (lsq.py:362-376's slice recombination).
// Dilation is ignored, as by the reference's Unfold of the forward (lsq.py:141).
#ifdef CIMQ_TU_BWD  // non-template kernel: defined in one translation unit only
__global__ void fold_gx_kernel(Geo g, const float* __restrict__ gxu, const float* __restrict__ sw_p,
                               float* __restrict__ gx) {
  const float scale = (*sw_p) / (float)g.nba;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < g.Nin;
       idx += (long long)gridDim.x * blockDim.x) {
    const int iw = (int)(idx % g.W);
    long long r = idx / g.W;
    const int ih = (int)(r % g.H);
    r /= g.H;
    const int c = (int)(r % g.C);
    const int b = (int)(r / g.C);
    float a = 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int th = ih + g.PH - kh;
      if (th < 0 || th % g.SH != 0) continue;
      const int oh = th / g.SH;
      if (oh >= g.Ho) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int tw = iw + g.PW - kw;
        if (tw < 0 || tw % g.SW != 0) continue;
        const int ow = tw / g.SW;
        if (ow >= g.Wo) continue;
        const size_t m = (size_t)b * g.P + (size_t)oh * g.Wo + ow;
        a += gxu[m * g.K + (size_t)c * g.KHW + kh * g.KW + kw];
      }
    }
    gx[idx] = a * scale;
  }
}
#endif

// =========================================================================================
// cim_bwd_gw: grad wrt the weights and alpha_cim; alpha_cim init   (lsq.py:321-369, 35-87)
// =========================================================================================
//   gw[f,o] = (sa/nbw) * sum_j sum_m xhat_j[m,f] * g[m,o] * D_j[m,i(f),o]
//   D_j = sum_k 2^-(bsw*k) * mask[k,j] * STE[m,i,k,j,o]
//   galpha[i,k,j,o] = c * mask[k,j] * sum_m code[m,i,k,j,o] * g[m,o]
// Block = (tile i, 32-channel group, pixel chunk).  ps is recomputed in the natural
// orientation (rows = pixels), so g*D is directly the B operand of a bf16 MFMA that
// contracts over (pixel, a-slice) against the int8 ctx slices xhat_j (lsq.py:290-295).
// INIT mode accumulates sum_m |ps*sw*sa| instead (fp32 partial sums of lsq.py:64).
template <int NBP, int FBMAX, bool INIT>
__global__ __launch_bounds__(256) void cim_bwd_gw_kernel(Geo g, const int8_t* __restrict__ xcode,
                                                         const int8_t* __restrict__ xhat,
                                                         const v4i* __restrict__ wfrag, Params pp,
                                                         const float* __restrict__ sw_p,
                                                         const float* __restrict__ sa_p,
                                                         const float* __restrict__ signed_p,
                                                         const float* __restrict__ gout, int rows_per_chunk,
                                                         float* __restrict__ gw_slab,
                                                         float* __restrict__ ga_slab,
                                                         float* __restrict__ gb_slab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  TileSmem sm;
  sm.As = reinterpret_cast<int8_t*>(smem);
  size_t off = (size_t)g.nba * 64 * g.KTP;
  sm.foff = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.fkk = reinterpret_cast<int*>(smem + off); off += sizeof(int) * g.KS * 64;
  sm.rowinfo = reinterpret_cast<int4*>(smem + off); off += sizeof(int4) * 64;
  const int tlen = g.KS * 64;
  const int nkj = g.nbw * g.nba;
  constexpr int NOBG = 1;  // 16-channel output blocks per workgroup (LDS: the per-wave sums below)
  const int ncol = 16 * NOBG;
  // [4 waves][nkj][ncol]: sums of code*g (INIT: of |u|), one writer lane per slot and wave, the
  // waves added in a fixed order at the end -- no atomics, bit-identical run to run
  float* qacc = reinterpret_cast<float*>(smem + off);
  off += sizeof(float) * 4 * nkj * ncol;
  // [FBT*16][ncol] block sum of grad_w: built after the pixel loop, in the act-tile region (free by then)
  float* gwacc = reinterpret_cast<float*>(smem);
  float* qbacc = reinterpret_cast<float*>(smem + off);  // [4 waves][nkj][ncol]: sum beta_term*g (shift variants only)
  off += is_shift(g) ? sizeof(float) * 4 * nkj * ncol : 0;
  int8_t* Xb = reinterpret_cast<int8_t*>(smem + off);   // [nba][tlen][64] bwd slices, f-major

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int i = blockIdx.y;
  const int og = blockIdx.z;  // channel group: o-blocks NOBG*og ..
  const int nob = min(NOBG, g.OB16 - og * NOBG);
  const int mc = blockIdx.x;
  const int mbeg = mc * rows_per_chunk, mend = min(mbeg + rows_per_chunk, g.M);
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0) || g.variant != VAR_LIBRARY;
  const bool ternary_fast = (!literal) && g.mode == ADC_TERNARY;
  const bool has_code = has_alpha(g);
  const bool shift = is_shift(g);

  for (int t = threadIdx.x; t < 4 * nkj * ncol; t += blockDim.x) qacc[t] = 0.f;
  if (!INIT && shift)
    for (int t = threadIdx.x; t < 4 * nkj * ncol; t += blockDim.x) qbacc[t] = 0.f;
  v4f gwa[FBMAX][2];
#pragma unroll
  for (int a = 0; a < FBMAX; ++a) { gwa[a][0] = v4f{0, 0, 0, 0}; gwa[a][1] = v4f{0, 0, 0, 0}; }

  build_ftable(g, i, sm.foff, sm.fkk);
  for (int m0 = mbeg; m0 < mend; m0 += 64) {
    __syncthreads();
    build_rowinfo(g, m0, sm.rowinfo);
    if (threadIdx.x < 64 && m0 + (int)threadIdx.x >= mend) sm.rowinfo[threadIdx.x].w = 0;
    __syncthreads();
    build_As<NBP>(g, xcode, sm);
    if (!INIT) {
      // backward act slices of the int8 ctx code (lsq.py:290-295), f-major: Xb[j][t][row]
      for (int it = threadIdx.x; it < tlen * 16; it += blockDim.x) {
        const int t = it >> 4, rq = (it & 15) * 4;
        const int fk = sm.fkk[t];
        uint32_t pl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int4 ri = sm.rowinfo[rq + e];
          const uint2 c = gather_code<NBP>(g, xhat, ri, sm.foff[t], fk);
#pragma unroll
          for (int j = 0; j < 4; ++j) pl[j] |= ((c.x >> (8 * j)) & 0xFFu) << (8 * e);
          if (NBP == 8) {
#pragma unroll
            for (int j = 0; j < 4; ++j) pl[4 + j] |= ((c.y >> (8 * j)) & 0xFFu) << (8 * e);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < g.nba) *reinterpret_cast<uint32_t*>(Xb + ((size_t)j * tlen + t) * 64 + rq) = pl[j];
      }
    }
    __syncthreads();

    const int rowbase = wave * 16 + 4 * g4;  // this lane's 4 accumulator rows (pixels)
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
      if (ob < nob) {
        const int ocol = ob * 16 + r16;
        const int o = og * ncol + ocol;
        float gval[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + rowbase + r;
          gval[r] = (!INIT && o < g.O && sm.rowinfo[rowbase + r].w) ? gout[(size_t)m * g.O + o] : 0.f;
        }
        float D[8][4];
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) D[a][b] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j < g.nba) {
            v4i xa[4];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
              if (ks < g.KS) xa[ks] = load_xfrag(g, sm.As, j, wave * 16 + r16, ks, lane);
            for (int k = 0; k < g.nbw; ++k) {
              const int nb = k * g.OB16 + og * NOBG + ob;
              v4i acc = {0, 0, 0, 0};
#pragma unroll
              for (int ks = 0; ks < 4; ++ks)
                if (ks < g.KS)
                  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                      xa[ks], wfrag[((size_t)(i * g.KS + ks) * g.NBLK + nb) * WAVE + lane], acc, 0, 0, 0);
              const int pi = pidx(g, i, j, k, o);
              const int kj = k * g.nba + j;
              float qs = 0.f, qb = 0.f;
              if (INIT) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float u = ((float)acc[r] * sw) * sa;  // fp32 ps (no fp16 store), lsq.py:64,84
                  qs += fabsf(u);
                }
              } else {
                const float cd = pp.ckj[2 * nkj + kj];
                if (ternary_fast) {
                  const int mlo = pp.mlo[pi], mhi = pp.mhi[pi], thi = pp.thi[pi], tlo = pp.tlo[pi];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const int p = acc[r];
                    D[j][r] += ((unsigned)(p - mlo) <= (unsigned)mhi) ? cd : 0.f;
                    const float q = (p >= thi) ? 1.f : ((p <= tlo) ? -1.f : 0.f);
                    qs += q * gval[r];
                  }
                } else {
                  const float al = pp.alpha[pi], be = pp.beta[pi];
                  const int mlo = pp.mlo[pi], mhi = pp.mhi[pi];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const int p = acc[r];
                    const float b = psb_value(g, p, sw, sa, al, be);
                    const bool pass = literal ? ste_pass(b, g.thr_hi, g.thr_lo) : ((unsigned)(p - mlo) <= (unsigned)mhi);
                    D[j][r] += pass ? cd : 0.f;
                    if (has_code) qs += alpha_term(g, b) * gval[r];
                    if (shift) qb += beta_term(g, b) * gval[r];
                  }
                }
              }
              // lanes l, l^16, l^32, l^48 share the column: fold the 16 pixel rows, then LDS
              qs = rows4_sum(qs);
              if (shift) {
                qb = rows4_sum(qb);
              }
              if (g4 == 0 && (INIT || has_code)) {
                qacc[(wave * nkj + kj) * ncol + ocol] += qs;
                if (!INIT && shift) qbacc[(wave * nkj + kj) * ncol + ocol] += qb;
              }
            }
          }
        }
        if (!INIT) {
          // gw MFMA: contraction over kappa = (pixel row r of this lane's 4, a-slice j)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if (2 * s < g.nba) {
              uint32_t hi[4] = {0, 0, 0, 0}, mi[4] = {0, 0, 0, 0}, lo[4] = {0, 0, 0, 0};
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const int j = 2 * s + (e >> 2), r = e & 3;
                const float bv = (j < g.nba) ? gval[r] * D[j][r] : 0.f;
                uint16_t h, md, l;
                split3(bv, h, md, l);
                hi[e >> 1] |= (uint32_t)h << (16 * (e & 1));
                mi[e >> 1] |= (uint32_t)md << (16 * (e & 1));
                lo[e >> 1] |= (uint32_t)l << (16 * (e & 1));
              }
              const v8bf bh = as_v8bf(v4i{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]});
              const v8bf bm = as_v8bf(v4i{(int)mi[0], (int)mi[1], (int)mi[2], (int)mi[3]});
              const v8bf bl = as_v8bf(v4i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]});
#pragma unroll
              for (int fb = 0; fb < FBMAX; ++fb) {
                if (fb < g.FBT) {
                  const int t = fb * 16 + r16;
                  uint32_t ad[4] = {0, 0, 0, 0};
#pragma unroll
                  for (int h2 = 0; h2 < 2; ++h2) {
                    const int j = 2 * s + h2;
                    uint32_t bytes = 0;
                    if (j < g.nba)
                      bytes = *reinterpret_cast<const uint32_t*>(Xb + ((size_t)j * tlen + t) * 64 + rowbase);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                      const float xv = (float)(int8_t)((bytes >> (8 * r)) & 0xFF);
                      const int e = h2 * 4 + r;
                      ad[e >> 1] |= (uint32_t)bf16_bits(xv) << (16 * (e & 1));
                    }
                  }
                  const v8bf xa8 = as_v8bf(v4i{(int)ad[0], (int)ad[1], (int)ad[2], (int)ad[3]});
                  v4f accw = gwa[fb][ob];
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa8, bh, accw, 0, 0, 0);
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa8, bm, accw, 0, 0, 0);
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa8, bl, accw, 0, 0, 0);
                  gwa[fb][ob] = accw;
                }
              }
            }
          }
        }
      }
    }
  }

  // ---- block reductions -> slabs (deterministic: the waves in a fixed order, no atomics) ----
  if (!INIT) {
    __syncthreads();
    for (int t = threadIdx.x; t < g.FBT * 16 * ncol; t += blockDim.x) gwacc[t] = 0.f;
    for (int w = 0; w < 4; ++w) {
      __syncthreads();
      if (wave == w) {
#pragma unroll
        for (int fb = 0; fb < FBMAX; ++fb)
          if (fb < g.FBT)
#pragma unroll
            for (int ob = 0; ob < 2; ++ob)
              if (ob < nob)
#pragma unroll
                for (int r = 0; r < 4; ++r) gwacc[(fb * 16 + 4 * g4 + r) * ncol + ob * 16 + r16] += gwa[fb][ob][r];
      }
    }
  }
  __syncthreads();
  const int wq = nkj * ncol;
  for (int t = threadIdx.x; t < nkj * ncol; t += blockDim.x) {
    const int q = t / ncol, col = t - q * ncol;
    const int o = og * ncol + col;
    if (o < g.Opad) {
      const int k = q / g.nba, j = q - k * g.nba;
      const float qv = ((qacc[t] + qacc[wq + t]) + qacc[2 * wq + t]) + qacc[3 * wq + t];
      ga_slab[(((size_t)mc * g.T + i) * nkj + (size_t)k * g.nba + j) * g.Opad + o] = qv;
      if (!INIT && shift)
        gb_slab[(((size_t)mc * g.T + i) * nkj + (size_t)k * g.nba + j) * g.Opad + o] =
            ((qbacc[t] + qbacc[wq + t]) + qbacc[2 * wq + t]) + qbacc[3 * wq + t];
    }
  }
  if (INIT) return;
  for (int t = threadIdx.x; t < g.FBT * 16 * ncol; t += blockDim.x) {
    const int fl = t / ncol, col = t - fl * ncol;
    const int o = og * ncol + col;
    if (o < g.Opad) gw_slab[(((size_t)mc * g.T + i) * (g.FBT * 16) + fl) * g.Opad + o] = gwacc[t];
  }
}

// =========================================================================================
// LSQ activation quantiser backward (autograd of lsq.py:547-549, fused-module path)
// =========================================================================================
//   y1 = x/sa ; c = clamp(y1,0,Qp) ; x_q = round_pass(c)*sa
//   g_y1 = (0<=y1<=Qp) ? g*sa : 0 ;  g_x = g_y1/sa
//   g_sa = sum(g*round(c)) + sum(-g_y1*((x/sa)/sa))
#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void lsq_act_bwd_kernel(long long n, const float* __restrict__ x, const float* __restrict__ sa_p,
                                   float qp, float* __restrict__ gx_inout, float* __restrict__ partial) {
  __shared__ float sred[256];
  const float sa = *sa_p;
  float acc = 0.f;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (long long)gridDim.x * blockDim.x) {
    const float xv = x[idx];
    const float gq = gx_inout[idx];
    const float y1 = xv / sa;
    const float c = clamp_nan(y1, 0.f, qp);
    const float r = rintf(c);
    const float rp = (r - c) + c;
    const bool pass = (y1 >= 0.f) && (y1 <= qp);
    const float gy = pass ? gq * sa : 0.f;
    gx_inout[idx] = gy / sa;
    acc += gq * rp;
    acc += -(gy * (y1 / sa));
  }
  sred[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sred[threadIdx.x] += sred[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sred[0];
}
#endif

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ void sum_partials_kernel(int n, const float* __restrict__ partial, float* __restrict__ out) {
  __shared__ float sred[256];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partial[i];
  sred[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sred[threadIdx.x] += sred[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = sred[0];
}
#endif

}  // namespace cimq

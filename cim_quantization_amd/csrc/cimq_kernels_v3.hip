// cimq_kernels_v3.hip -- fast path for layers whose output image splits into whole-row
// 64-pixel tiles (P % 64 == 0 and Wo | 64: every conv of the CIFAR ResNets).  Same
// arithmetic as the general kernels in cimq_kernels.hip (bit-exact integer partial sums, ADC
// codes and STE masks; fp32-accurate bf16x3 backward GEMMs); the data movement is built for
// CDNA4:
//   * the packed activation slice words of a pixel strip (or, for grad_x, of a band of input
//     rows) are staged into LDS once with batched 16-byte loads, zero-padded like nn.Unfold;
//   * each wave gathers the int8 MFMA operand of ITS 16 pixels straight from that patch
//     (16 LDS words per 64-deep K-step, v_perm byte transposes give every bit slice at once),
//     so there is no im2col buffer, no LDS round trip and no barrier between the waves;
//   * per-tile weight fragments, ADC thresholds and STE intervals live in LDS; every index
//     into them is a table lookup or a shift (no integer division in the inner loops);
//   * grad_x blocks own a band of input rows and fold (nn.Fold adjoint) into an LDS
//     accumulator with the same geometry as the patch -- the fold address of (pixel, f) is
//     the gather address -- then apply the fused LSQ activation backward and store once;
//   * grad_w keeps its accumulators in registers across the block's pixel chunk and folds the
//     four waves together in LDS once, at the end.
#pragma once
#include "cimq_kernels.hip"

namespace cimq {

// host-computed plan of the fast path (cimq_api.hip: v3_plan)
struct V3 {
  int lw;          // log2(Wo)
  int RH;          // strip patch rows: (64/Wo - 1)*SH + KH
  int obm;         // forward: 16-channel output blocks per block (1, 2 or 4)
  int WP;          // patch row length: W + 2*PW
  int RI, nbands;  // grad_x: owned input rows per block, bands per image
  int RHB;         // grad_x: max band patch rows
  int NPB;         // grad_x: max output pixels per band, rounded up to 16
  int fwd_res;     // forward: every tile's weights / thresholds resident in LDS
  int nmt;         // M / 64
  int NCG;         // grad_w: max input channels one tile touches
  int NCBT;        // grad_x: max 16-channel blocks one tile touches
  int CB;          // grad_x: 16-channel blocks of the output tile grid (ceil(C/16))
  int NT;          // grad_x: max output tiles (16 positions x 16 channels) per band
  int pf;          // forward, non-resident tiles: the next tile's weight side prefetched in registers
};

// floor(n / d) for 0 <= n < 2^22 (inv = 1.f / d): float estimate + one correction step
__device__ inline int fdiv(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  if (r < 0) q -= 1;
  else if (r >= d) q += 1;
  return q;
}

__device__ inline size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }

// Batched global -> LDS copy: every thread issues U independent loads before its first LDS
// store, so a block waits about one memory latency per U*blockDim elements instead of one
// per element.  src(idx) returns element idx; it lands in dst[idx].
template <int U, typename T, typename Src>
__device__ inline void batched_copy(int n, T* dst, Src src) {
  const int nt = blockDim.x;
  for (int base = threadIdx.x; base < n; base += U * nt) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * nt < n) v[u] = src(base + u * nt);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * nt < n) dst[base + u * nt] = v[u];
  }
}

// ---------------------------------------------------------------------------------------
// patch staging: rows [ih_first, ih_first + RHx) of image b -> LDS [C][RHx][WP] words of
// NBP bytes; data columns only (the 2*PW padding columns are zeroed once per block).  Rows
// outside the image are written as zeros.
// ---------------------------------------------------------------------------------------
__device__ inline void zero_lds(uint32_t* p, int nwords) {
  for (int t = threadIdx.x; t < nwords; t += blockDim.x) p[t] = 0u;
}

template <int NBP>
__device__ inline void stage_rows(const Geo& g, int WP, int RHx, const uint8_t* __restrict__ xc, int b,
                                  int ih_first, uint8_t* patch, int c0 = 0, int ncx = -1) {
  const int QW = g.W * NBP / 16;  // 16-byte vectors per row
  const int nrow = (ncx < 0 ? g.C : ncx) * RHx;
  const int n = nrow * QW;
  const uint4* src = reinterpret_cast<const uint4*>(xc) + ((size_t)b * g.C + c0) * g.H * QW;
  const int nt = blockDim.x;
  // item -> (row, q) by a shift when QW is a power of two, row -> (c, rr) by a 24-bit
  // multiply-shift (exact for row * RHx < 2^20); 32-bit offsets from the image's base: no
  // quarter-rate 32/64-bit multiplies per item
  const bool pq = (QW & (QW - 1)) == 0;
  const int lq = 31 - __builtin_clz(QW);
  const bool mag_ok = nrow * RHx < (1 << 20);
  const unsigned mag = ((1u << 20) + RHx - 1) / RHx;
  const float invQ = 1.f / (float)QW, invR = 1.f / (float)RHx;
  const int HQ = g.H * QW, rowb = WP * NBP, colb = g.PW * NBP;
  for (int base = threadIdx.x; base < n; base += 8 * nt) {
    uint4 v[8];
    int d[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * nt;
      d[u] = -1;
      if (idx < n) {
        const int row = pq ? (idx >> lq) : fdiv(idx, QW, invQ), q = pq ? (idx & (QW - 1)) : idx - row * QW;
        const int c = mag_ok ? (int)(__umul24((unsigned)row, mag) >> 20) : fdiv(row, RHx, invR);
        const int rr = row - c * RHx;
        const int ih = ih_first + rr;
        d[u] = row * rowb + colb + q * 16;
        v[u] = make_uint4(0, 0, 0, 0);
        if ((unsigned)ih < (unsigned)g.H) v[u] = src[c * HQ + ih * QW + q];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (d[u] >= 0) {
        uint32_t* p = reinterpret_cast<uint32_t*>(patch + d[u]);
        p[0] = v[u].x; p[1] = v[u].y; p[2] = v[u].z; p[3] = v[u].w;
      }
    }
  }
}

// stage_rows for the module forward with the LSQ activation quantiser fused (NBP 4): the rows are read
// as fp32 x and turned into slice words on the way into LDS -- act_words_lut, the same table and the
// same element chain as the prologue's act_range, so the words are bit-identical -- and the block
// that owns input rows [own_lo, own_hi) also writes their backward (ctx) words to xcb.  The forward
// slice words are never stored.
// lut: [Qp + 1][fwd, bwd] from act_lut_build plus, at entry Qp + 1, the words of a NaN element
// (act_words of any NaN: every step of its chain is independent of the NaN's sign and payload)
__device__ inline uint2 act_words_tab(float v, float sa, float qp, int nan_e, const uint32_t* lut) {
  const float c = clamp_nan(v / sa, 0.f, qp);
  const float r = rintf(c);
  const int e = (r == r) ? (int)r : nan_e;
  return *reinterpret_cast<const uint2*>(lut + 2 * e);
}
template <int NBA_C>
__device__ inline void act_lut_build_q(const Geo& g, float sa, bool sgn, uint32_t* lut) {
  if (threadIdx.x == 0) {
    uint32_t f[1], b[1];
    act_words<4, NBA_C>(g, __int_as_float(0x7fc00000), sa, sgn, f, b);
    const int e = (int)g.lsq_qp + 1;
    lut[2 * e] = f[0];
    lut[2 * e + 1] = b[0];
  }
  act_lut_build<4, NBA_C>(g, sa, sgn, lut);  // entries 0 .. Qp, then the block barrier
}
__device__ inline void stage_rows_q(const Geo& g, int WP, int RHx, const float* __restrict__ x, float sa,
                                    const uint32_t* lut, int b, int ih_first, uint8_t* patch,
                                    uint8_t* __restrict__ xcb, int own_lo, int own_hi) {
  const int nan_e = (int)g.lsq_qp + 1;
  const int QW = g.W >> 2;  // 4-element items per row (W % 4 == 0)
  const int nrow = g.C * RHx;
  const int n = nrow * QW;
  const bool pq = (QW & (QW - 1)) == 0;
  const int lq = 31 - __builtin_clz(QW);
  const float invQ = 1.f / (float)QW, invR = 1.f / (float)RHx;
  const size_t img = (size_t)b * g.C * g.H;
  for (int base = threadIdx.x; base < n; base += 4 * (int)blockDim.x) {
    float4 v[4];
    int d[4], ihs[4], cs[4], qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = base + u * (int)blockDim.x;
      d[u] = -1;
      if (idx < n) {
        const int row = pq ? (idx >> lq) : fdiv(idx, QW, invQ), q = pq ? (idx & (QW - 1)) : idx - row * QW;
        const int c = fdiv(row, RHx, invR);
        const int ih = ih_first + (row - c * RHx);
        d[u] = row * WP * 4 + g.PW * 4 + q * 16;
        ihs[u] = ih;
        cs[u] = c;
        qs[u] = q;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)ih < (unsigned)g.H)
          v[u] = reinterpret_cast<const float4*>(x)[((img + (size_t)c * g.H + ih) * g.W >> 2) + q];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (d[u] < 0) continue;
      uint32_t* p = reinterpret_cast<uint32_t*>(patch + d[u]);
      if ((unsigned)ihs[u] >= (unsigned)g.H) {
        p[0] = p[1] = p[2] = p[3] = 0u;
        continue;
      }
      const uint2 w0 = act_words_tab(v[u].x, sa, g.lsq_qp, nan_e, lut);
      const uint2 w1 = act_words_tab(v[u].y, sa, g.lsq_qp, nan_e, lut);
      const uint2 w2 = act_words_tab(v[u].z, sa, g.lsq_qp, nan_e, lut);
      const uint2 w3 = act_words_tab(v[u].w, sa, g.lsq_qp, nan_e, lut);
      p[0] = w0.x; p[1] = w1.x; p[2] = w2.x; p[3] = w3.x;
      if (ihs[u] >= own_lo && ihs[u] < own_hi)
        reinterpret_cast<uint4*>(xcb)[((img + (size_t)cs[u] * g.H + ihs[u]) * g.W >> 2) + qs[u]] =
            make_uint4(w0.y, w1.y, w2.y, w3.y);
    }
  }
}

// ptab[t] (t < KS*64) for tile i: patch word offset of contraction row f = i*xbar + t relative
// to a pixel's window origin; 0 for t outside the tile (the weight operand is zero there).
__device__ inline void build_ptab(const Geo& g, int i, int KSx, int RHx, int WP, int* ptab, int c0 = 0) {
  for (int t = threadIdx.x; t < KSx * 64; t += blockDim.x) {
    const int f = i * g.xbar + t;
    int off = 0;
    if (t < g.xbar && f < g.K) {
      const int c = fdiv(f, g.KHW, 1.f / (float)g.KHW), rem = f - c * g.KHW;
      const int kh = fdiv(rem, g.KW, 1.f / (float)g.KW), kw = rem - kh * g.KW;
      off = ((c - c0) * RHx + kh) * WP + kw;
    }
    ptab[t] = off;
  }
}

// 4x4 byte transpose: P_j byte e = w_e byte j
__device__ inline void tr4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t (&P)[4]) {
  const uint32_t t01l = __builtin_amdgcn_perm(w1, w0, 0x05010400u);
  const uint32_t t01h = __builtin_amdgcn_perm(w1, w0, 0x07030602u);
  const uint32_t t23l = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
  const uint32_t t23h = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
  P[0] = __builtin_amdgcn_perm(t23l, t01l, 0x05040100u);
  P[1] = __builtin_amdgcn_perm(t23l, t01l, 0x07060302u);
  P[2] = __builtin_amdgcn_perm(t23h, t01h, 0x05040100u);
  P[3] = __builtin_amdgcn_perm(t23h, t01h, 0x07060302u);
}

// The int8 MFMA operand of one pixel (this lane's column / row l&15) for tile i:
// xs[j][ks] byte e = slice j of the element at contraction index t = ks*64 + 16*(l>>4) + e.
template <int NBP, int KS>
__device__ inline void gather_xs(const uint8_t* patch, int rb, const int* ptab, int g4, v4i (&xs)[NBP][KS],
                                 int ksn = KS) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks >= ksn) break;
    const int4* pt = reinterpret_cast<const int4*>(ptab + ks * 64 + 16 * g4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 o4 = pt[q];
      const int oo[4] = {o4.x, o4.y, o4.z, o4.w};
      uint32_t w[4], wh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (NBP == 4) {
          w[e] = reinterpret_cast<const uint32_t*>(patch)[rb + oo[e]];
        } else {
          const uint2 t = reinterpret_cast<const uint2*>(patch)[rb + oo[e]];
          w[e] = t.x;
          wh[e] = t.y;
        }
      }
      uint32_t P[4];
      tr4(w[0], w[1], w[2], w[3], P);
#pragma unroll
      for (int j = 0; j < 4; ++j) xs[j][ks][q] = (int)P[j];
      if (NBP == 8) {
        tr4(wh[0], wh[1], wh[2], wh[3], P);
#pragma unroll
        for (int j = 0; j < 4; ++j) xs[4 + j][ks][q] = (int)P[j];
      }
    }
  }
}

// fp32 -> three bf16 parts (hi + mid + lo), 8 values -> 3 MFMA operands
// (a, b) -> bf16 hi / mid / lo pairs, low half a: round-to-nearest-even conversions and exact fp32
// remainders (hi + mid + lo reproduces a to fp32 accuracy), one v_cvt_pk_bf16_f32 per level for both values
__device__ inline uint32_t pk_bf16(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ inline void split3_pk(float a, float b, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = pk_bf16(a, b);
  float ra = a - __uint_as_float(hi << 16), rb = b - __uint_as_float(hi & 0xffff0000u);
  mid = pk_bf16(ra, rb);
  ra = ra - __uint_as_float(mid << 16);
  rb = rb - __uint_as_float(mid & 0xffff0000u);
  lo = pk_bf16(ra, rb);
}
__device__ inline void split3x8(const float (&v)[8], v8bf& bh, v8bf& bm, v8bf& bl) {
  v4i h, m, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    uint32_t a, b, c;
    split3_pk(v[2 * e], v[2 * e + 1], a, b, c);
    h[e] = (int)a;
    m[e] = (int)b;
    l[e] = (int)c;
  }
  bh = __builtin_bit_cast(v8bf, h);
  bm = __builtin_bit_cast(v8bf, m);
  bl = __builtin_bit_cast(v8bf, l);
}

// literal (threshold-free) per-partial-sum paths, kept out of line: degenerate alpha / scales
__device__ __noinline__ float adc_literal_sum(v4i ps, int mode, float sw, float sa, float al, float qn, float qp,
                                             float mk, int r) {
  return adc_literal(ps[r], mode, sw, sa, al, qn, qp) * mk;
}
__device__ __noinline__ float ste_literal(int p, int mode, float sw, float sa, float al, float thr_hi, float thr_lo) {
  const float bb = psb_literal(p, mode, sw, sa, al);
  return ste_pass(bb, thr_hi, thr_lo) ? 1.f : 0.f;
}
__device__ __noinline__ float code_literal(int p, int mode, float sw, float sa, float al, float qn, float qp,
                                           float thr_hi, float thr_lo) {
  const float bb = psb_literal(p, mode, sw, sa, al);
  return alpha_code_literal(bb, mode, qn, qp, thr_hi, thr_lo);
}
// the shift ADC's literal path (shift_fast layers with a degenerate alpha / beta / scale): adc * mask
// (scale_shift.py:421-429) and the state bits of the partial sum (v = (u - beta) / alpha: STE pass
// unless v >= Qp + 1e-5 or v <= Qn - 1e-5, :469-484; code clamp(rint(v), -1, 1))
// (scalar arguments only, as the helpers above: a Geo by reference would put it on the stack and
// cost the whole kernel registers; shift_fast fixes ps_int8 = 0 and the range -1 .. 1)
__device__ __noinline__ float shift_adc_literal(int p, float sw, float sa, float al, float be, float mk) {
  const float u = (ps_half(p) * sw) * sa;  // u_var without the int8 buffer
  const float v = (u - be) / al;
  const float t = clamp_nan(rintf(v), -1.f, 1.f) * al;
  return (t + be) * mk;
}
__device__ __noinline__ uint32_t shift_state_literal(int p, float sw, float sa, float al, float be, float thr_hi,
                                                     float thr_lo) {
  const float v = (((ps_half(p) * sw) * sa) - be) / al;
  const bool pass = !(v >= thr_hi || v <= thr_lo);
  const float code = clamp_nan(rintf(v), -1.f, 1.f);
  return (pass ? 1u : 0u) | ((code != 0.f) ? 2u : 0u) | ((code < 0.f) ? 4u : 0u);
}

// ---------------------------------------------------------------------------------------
// forward: out[m, o] = sum_{i,j,k} ADC(ps_ijk[m, o]) * mask   (lsq.py:166-233)
// block = 64-pixel m-tiles (grid-stride) x one 64-wide o-group; wave w = pixels 16w..16w+15.
// ---------------------------------------------------------------------------------------
// state bits of one partial sum: bit 0 STE pass (lsq.py:310-313), bit 1 ADC code != 0, bit 2
// ADC code < 0 (lsq.py:321-332)
__device__ inline uint32_t st_bits(bool pass, float code) {
  return (pass ? 1u : 0u) | ((code != 0.f) ? 2u : 0u) | ((code < 0.f) ? 4u : 0u);
}

// shift a bit in: x * 2 + c in one v_addc_co_u32 whose carry-in is the compare's lane mask
// (the compiler spends a cndmask + shift/or on the plain expression)
// The ctx's code -> word table region (CtxLayout::alut, 1,280 bytes) also carries a format word at entry
// kCalFlag: cim_fwd5_kernel writes kCodesMagic there when it stores one activation code byte per ctx element
// (ctx_codes), and cim_bwd_gw5_kernel's code-byte instance checks it -- a ctx written in the other format
// (a forward / backward planned differently, e.g. a tuning knob changed in between) yields NaN grad_w and
// grad_alpha partials instead of silently reading words as codes.
constexpr int kCalFlag = 300;
constexpr uint32_t kCodesMagic = 0xC0DE5EEDu;

__device__ inline uint32_t shin(uint32_t x, uint64_t m) {
  uint32_t r;
  uint64_t co;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(x), "s"(m));
  return r;
}
// ternary ADC term: hi ? cf : (lo ? -cf : 0) from the two compare masks (two cndmasks; the
// plain expression makes the compiler rematerialise the masks as 0/1 vectors)
__device__ inline float adc3(float cf, uint64_t mhi, uint64_t mlo) {
  float a, r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(a) : "v"(cf), "s"(mhi));
  asm("v_cndmask_b32_e64 %0, %1, -%2, %3" : "=v"(r) : "v"(a), "v"(cf), "s"(mlo));
  return r;
}

// CST: compact state words (cimq_v7.hip) -- one uint32 per (tile i, pixel m, channel o) at
// st32[(i*M + m)*O + o], bits 3*(k*nba + j) + {0: STE pass, 1: code != 0, 2: code < 0}.
// CST > 0 also fixes nbw = nba = CST at compile time: the ternary-threshold path then runs
// (CSTA = 9: CST 8 without writing the state words -- the first conv's backward recomputes them)
// fully unrolled (every slice pair's MFMAs issued before its ADC work, state bits shifted in).
template <int NBP, int KS, int CSTA, int OBM>
__global__ __launch_bounds__(256) void cim_fwd_v3_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                         const v4i* __restrict__ wfrag, Params pp,
                                                         const float* __restrict__ sw_p,
                                                         const float* __restrict__ sa_p, float* __restrict__ out,
                                                         uint8_t* __restrict__ st, const float* __restrict__ xin,
                                                         const float* __restrict__ sgn_p, uint8_t* __restrict__ xcb) {
  // CSTA 9: the w8a8 fast path of CST 8 without the state words (cimq_c1.hip recomputes them)
  // xin (module path, NBP 4): the activation quantiser fused into the row staging (stage_rows_q)
  constexpr int CST = CSTA == 9 ? 8 : CSTA;
  constexpr bool WST = CSTA != 9;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int og = blockIdx.y;
  const int NOB = min(OBM, g.OB16);
  const int nob = min(OBM, g.OB16 - og * OBM);
  const int TT = v.fwd_res ? g.T : 1;
  const int nkj = g.nbw * g.nba;
  uint8_t* cur = smem;
  uint8_t* patch = cur; cur += al16((size_t)g.C * v.RH * v.WP * NBP);
  int* ptab = reinterpret_cast<int*>(cur); cur += (size_t)g.T * KS * 64 * 4;
  v4i* wfl = reinterpret_cast<v4i*>(cur); cur += (size_t)TT * g.nbw * NOB * KS * 1024;   // [tt][k][ob][ks][64]
  int4* prm = reinterpret_cast<int4*>(cur); cur += (size_t)TT * nkj * NOB * 16 * 16;    // [tt][j][k][NOB*16]
  float* cfl = reinterpret_cast<float*>(cur); cur += (size_t)TT * nkj * NOB * 16 * 4;   // coef, same order
  float* ckl = reinterpret_cast<float*>(cur);
  // the quantiser's word table [Qp + 1][fwd, bwd] after ckl (launch_fwd_v3 sizes it in)
  uint32_t* alut = reinterpret_cast<uint32_t*>(cur + al16((size_t)3 * g.nbw * g.nba * 4));

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const bool flag_lit = (pp.flags[0] != 0);
  const bool literal = flag_lit || g.mode != ADC_TERNARY;
  const bool has_code = (g.mode == ADC_SIGN || g.mode == ADC_TERNARY);
  const int Wo = 1 << v.lw;

  // index math by shifts (NOB in {1, 2, 4}, KS in {1, 2}) and a float-reciprocal division
  // by nbw: integer division is ~30 VALU each, and this prologue runs once per block
  const int lnob = NOB == 4 ? 2 : NOB - 1;
  const float inv_nbw = 1.f / (float)g.nbw;
  // the ADC thresholds and coefficients of tile i (the weight side's small part)
  auto stage_prm = [&](int i, int tt) {
    if (!flag_lit) {
      batched_copy<2>(nkj * NOB * 16, prm + (size_t)tt * nkj * NOB * 16, [&](int idx) -> int4 {
        const int col = idx & ((16 << lnob) - 1), jk = idx >> (4 + lnob);
        const int j = fdiv(jk, g.nbw, inv_nbw), k = jk - j * g.nbw;
        const int o = og * OBM * 16 + col;
        int4 p = make_int4(0, 0, 0, 0);
        if (o < g.Opad) {
          const int pi = pidx(g, i, j, k, o);
          p = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
        }
        return p;
      });
      batched_copy<4>(nkj * NOB * 16, cfl + (size_t)tt * nkj * NOB * 16, [&](int idx) -> float {
        const int col = idx & ((16 << lnob) - 1), jk = idx >> (4 + lnob);
        const int j = fdiv(jk, g.nbw, inv_nbw), k = jk - j * g.nbw;
        const int o = og * OBM * 16 + col;
        return (o < g.Opad) ? pp.coef[pidx(g, i, j, k, o)] : 0.f;
      });
    }
  };
  auto stage_tile = [&](int i, int tt) {
    batched_copy<4>(g.nbw * NOB * KS * 64, wfl + (size_t)tt * g.nbw * NOB * KS * 64, [&](int idx) -> v4i {
      const int l = idx & 63, fr = idx >> 6;
      const int ks = KS == 1 ? 0 : (fr & 1), kob = KS == 1 ? fr : (fr >> 1);
      const int k = kob >> lnob, ob = kob - (k << lnob);
      v4i w = {0, 0, 0, 0};
      if (ob < nob) w = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * OBM + ob) * WAVE + l];
      return w;
    });
    stage_prm(i, tt);
  };

  // every tile's weight side at once (fwd_res): one batched pass per array over all tiles, so its
  // loads are in flight together (tile by tile it took T x 3 dependent round trips: 8-9 us of a
  // 40-45 us launch on the 16x16 / 8x8 layers)
  auto stage_all = [&]() {
    const int nw = g.nbw * NOB * KS * 64, np = nkj * NOB * 16;
    const float inv_nw = 1.f / (float)nw, inv_np = 1.f / (float)np;
    batched_copy<8>(g.T * nw, wfl, [&](int t) -> v4i {
      const int i = fdiv(t, nw, inv_nw), idx = t - i * nw;
      const int l = idx & 63, fr = idx >> 6;
      const int ks = KS == 1 ? 0 : (fr & 1), kob = KS == 1 ? fr : (fr >> 1);
      const int k = kob >> lnob, ob = kob - (k << lnob);
      v4i w = {0, 0, 0, 0};
      if (ob < nob) w = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * OBM + ob) * WAVE + l];
      return w;
    });
    if (!flag_lit) {
      batched_copy<8>(g.T * np, prm, [&](int t) -> int4 {
        const int i = fdiv(t, np, inv_np), idx = t - i * np;
        const int col = idx & ((16 << lnob) - 1), jk = idx >> (4 + lnob);
        const int j = fdiv(jk, g.nbw, inv_nbw), k = jk - j * g.nbw;
        const int o = og * OBM * 16 + col;
        int4 p = make_int4(0, 0, 0, 0);
        if (o < g.Opad) {
          const int pi = pidx(g, i, j, k, o);
          p = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
        }
        return p;
      });
      batched_copy<8>(g.T * np, cfl, [&](int t) -> float {
        const int i = fdiv(t, np, inv_np), idx = t - i * np;
        const int col = idx & ((16 << lnob) - 1), jk = idx >> (4 + lnob);
        const int j = fdiv(jk, g.nbw, inv_nbw), k = jk - j * g.nbw;
        const int o = og * OBM * 16 + col;
        return (o < g.Opad) ? pp.coef[pidx(g, i, j, k, o)] : 0.f;
      });
    }
  };

  // non-resident tiles with a compile-time slice count (CST > 0): the next tile's weight fragments
  // are loaded into registers while the current tile computes and stored after the tile barrier
  // (the 16x16 / 8x8 layers, whose tiles do not all fit in LDS, spent 8-9 us per launch staging
  // them tile by tile); the thresholds are still staged at the barrier (in registers too they cost
  // the 32-channel layers a wave per SIMD)
  constexpr int PFW = CST > 0 ? (CST * OBM * KS * 64 + 255) / 256 : 1;
  const bool pfx = CST > 0 && !v.fwd_res && v.pf && blockDim.x == 256;  // uniform
  v4i pw[PFW];
  auto load_tile = [&](int i) {
    const int nw = g.nbw * NOB * KS * 64;
#pragma unroll
    for (int u = 0; u < PFW; ++u) {
      const int idx = threadIdx.x + u * 256;
      pw[u] = v4i{0, 0, 0, 0};
      if (idx < nw) {
        const int l = idx & 63, fr = idx >> 6;
        const int ks = KS == 1 ? 0 : (fr & 1), kob = KS == 1 ? fr : (fr >> 1);
        const int k = kob >> lnob, ob = kob - (k << lnob);
        if (ob < nob) pw[u] = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * OBM + ob) * WAVE + l];
      }
    }
  };
  auto store_tile = [&]() {
    const int nw = g.nbw * NOB * KS * 64;
#pragma unroll
    for (int u = 0; u < PFW; ++u)
      if ((int)threadIdx.x + u * 256 < nw) wfl[threadIdx.x + u * 256] = pw[u];
  };

  for (int i = 0; i < g.T; ++i) build_ptab(g, i, KS, v.RH, v.WP, ptab + i * KS * 64);
  for (int t = threadIdx.x; t < 3 * nkj; t += blockDim.x) ckl[t] = pp.ckj[t];
  if (pfx) load_tile(0);  // in flight through the prologue and the first row staging
  if (v.fwd_res)
#ifndef CIMQ_EXP_FWD_NOSTAGEW  // attribution builds only (tools/kernel_experiment.py)
    stage_all();
#endif
  zero_lds(reinterpret_cast<uint32_t*>(patch), g.C * v.RH * v.WP * NBP / 4);
  const bool actq = NBP == 4 && xin != nullptr;  // uniform
  const float sa_q = actq ? *sa_p : 0.f;
  const bool sgn_q = actq && *sgn_p != 0.f;
  if (actq) act_lut_build_q<(CST == 2 || CST == 3) ? CST : 0>(g, sa_q, sgn_q, alut);  // syncs the block

  __syncthreads();
  // w8a8: is binary_mask the standard int8-wrapped one (zero exactly where j + k >= 8)?
  const bool std8 = CST != 8 ||
                    __builtin_amdgcn_ballot_w64(lane < nkj && ((ckl[lane < nkj ? lane : 0] != 0.f) != ((lane >> 3) + (lane & 7) < 8))) == 0ull;
  const int pl = wave * 16 + r16;  // this lane's gather pixel within the m-tile
  const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & (Wo - 1)) * g.SW;
  const int tiles_per_img = g.P >> 6;

  const float inv_tpi = 1.f / (float)tiles_per_img, inv_p = 1.f / (float)g.P;
  for (int mt = blockIdx.x; mt < v.nmt; mt += gridDim.x) {
    const int b = fdiv(mt, tiles_per_img, inv_tpi), p0 = (mt - b * tiles_per_img) * 64;
    const int oh0 = p0 >> v.lw;
    __syncthreads();
#ifndef CIMQ_EXP_FWD_NOSTAGEX
    if (actq) {
      // input rows this m-tile owns (written once to xcb): its output rows' stride-spans, to the
      // image's end for its last m-tile; one o-group's blocks write them
      const int own_lo = blockIdx.y == 0 ? oh0 * g.SH : 0;
      const int own_hi = blockIdx.y == 0 ? (p0 + 64 == g.P ? g.H : (oh0 + (64 >> v.lw)) * g.SH) : 0;
      if constexpr (NBP == 4)
        stage_rows_q(g, v.WP, v.RH, xin, sa_q, alut, b, oh0 * g.SH - g.PH, patch, xcb, own_lo, own_hi);
    } else {
      stage_rows<NBP>(g, v.WP, v.RH, xcf, b, oh0 * g.SH - g.PH, patch);
    }
#endif
    __syncthreads();
    float acc[OBM][4];
#pragma unroll
    for (int a = 0; a < OBM; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][c] = 0.f;
    for (int i = 0; i < g.T; ++i) {
      if (!v.fwd_res) {
        __syncthreads();
#ifndef CIMQ_EXP_FWD_NOSTAGEW
        if (pfx) {
          // the weight fragments from the registers loaded a tile ago; the ADC thresholds as before
          store_tile();
          stage_prm(i, 0);
          load_tile(i + 1 < g.T ? i + 1 : 0);  // the next tile (tile 0 again for the next m-tile)
        } else {
          stage_tile(i, 0);
        }
#endif
        __syncthreads();
      }
      const int tt = v.fwd_res ? i : 0;
      const int ksn = (min(g.xbar, g.K - i * g.xbar) + 63) >> 6;  // K-steps holding data in tile i
      v4i xs[NBP][KS];
      // (the fast path runs every K-step: ptab and the weight operand are zero past the tile)
#ifdef CIMQ_EXP_FWD_NOGATHER  // attribution builds only: operands without the LDS gather
#pragma unroll
      for (int j = 0; j < NBP; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xs[j][ks] = v4i{lane + mt, j + i, ks, rb};
#else
      gather_xs<NBP, KS>(patch, rb, ptab + i * KS * 64, g4, xs, (CST > 0 && !literal && std8) ? KS : ksn);
#endif
      const v4i* wt = wfl + (size_t)tt * g.nbw * NOB * KS * 64;
      const int4* pt = prm + (size_t)tt * nkj * NOB * 16;
      const float* ct = cfl + (size_t)tt * nkj * NOB * 16;
      uint32_t stc[OBM][4];
#pragma unroll
      for (int a = 0; a < OBM; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) stc[a][c] = 0u;
      // plane state words (more than 10 slice pairs, NBP 8): per (i, m, o) three 64-bit planes
      // -- STE pass, code != 0, code < 0 -- bit k*nba + j each (cimq_v7.hip)
      constexpr bool PLF = (NBP == 8) && CST;
      uint64_t pl[OBM][4][3];
#pragma unroll
      for (int a = 0; a < OBM; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) pl[a][c][0] = pl[a][c][1] = pl[a][c][2] = 0ull;
      if (CST > 0 && !literal && std8) {
        // fast path: slice pairs kj = k*CST + j in descending order, so that shifting each
        // state bit in from the bottom leaves bit 3*kj + {0,1,2} (interleaved words) or bit
        // kj of each 64-bit plane (PLF) where cimq_v7.hip reads it.  w8a8 (CST 8) runs it only
        // with the standard int8-wrapped binary_mask (_quan_base.py:207-214), whose pairs with
        // j + k >= 8 are 0: they add adc * 0 = 0 to the output and G * 0 = 0 to every gradient,
        // so neither their MFMAs nor their ADC run and their state bits stay 0 (exact: this path
        // has finite ADC outputs).  Any other mask takes the per-pair loop below.
        constexpr int NS = CST > 0 ? CST : 1;

        uint32_t sw3[OBM][4][PLF ? 6 : 1];
#pragma unroll
        for (int a = 0; a < OBM; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int q = 0; q < (PLF ? 6 : 1); ++q) sw3[a][c][q] = 0u;
#pragma unroll
        for (int k = NS - 1; k >= 0; --k) {
#pragma unroll
          for (int ob = 0; ob < OBM; ++ob) {
            if (ob < nob) {
              v4i wk[KS];
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) wk[ks] = wt[((k * NOB + ob) * KS + ks) * 64 + lane];
              v4i ps[NS];
#pragma unroll
              for (int j = 0; j < NS; ++j) {
                if (CST != 8 || j + k < 8) {  // compile time once unrolled (w8a8: standard mask only)
                  // (the first K-step from the inline zero accumulator: no register clearing)
                  ps[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][0], wk[0], v4i{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                  for (int ks = 1; ks < KS; ++ks) ps[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[ks], ps[j], 0, 0, 0);
                } else {
                  ps[j] = v4i{0, 0, 0, 0};  // (a mask-0 pair: never read)
                }
              }
#pragma unroll
              for (int j = NS - 1; j >= 0; --j) {
                const int kj = k * NS + j;
                if (CST == 8 && j + k >= 8) {  // mask-0 pair of the wrapped 8-bit mask: zero state bits
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    if constexpr (!WST) continue;
                    if constexpr (PLF) {
                      const int wd = kj >= 32 ? 1 : 0;
                      sw3[ob][r][wd] <<= 1;
                      sw3[ob][r][2 + wd] <<= 1;
                      sw3[ob][r][4 + wd] <<= 1;
                    } else {
                      sw3[ob][r][0] <<= 3;
                    }
                  }
                  continue;
                }
                const int pcol = (j * NS + k) * NOB * 16 + ob * 16 + r16;
                const int4 pv = pt[pcol];
                const float cf = ct[pcol];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
#ifdef CIMQ_EXP_FWD_NOADC  // attribution builds only: no ADC, no state bits
                  acc[ob][r] += (float)(ps[j][r] + pv.x) * cf;
                  continue;
#endif
#ifdef CIMQ_EXP_FWD_NOSTATE  // attribution builds only: the ADC without the state bits
                  {
                    const uint64_t mhi = __builtin_amdgcn_ballot_w64(ps[j][r] >= pv.x);
                    const uint64_t mlo = __builtin_amdgcn_ballot_w64(ps[j][r] <= pv.y);
                    acc[ob][r] += adc3(cf, mhi, mlo);
                    continue;
                  }
#endif
                  const uint64_t mhi = __builtin_amdgcn_ballot_w64(ps[j][r] >= pv.x);
                  const uint64_t mlo = __builtin_amdgcn_ballot_w64(ps[j][r] <= pv.y);
                  acc[ob][r] += adc3(cf, mhi, mlo);
                  if constexpr (!WST) continue;  // (CSTA 9: no state words -- and none of their bits)
                  const uint64_t mps = __builtin_amdgcn_ballot_w64((unsigned)(ps[j][r] - pv.z) <= (unsigned)pv.w);
                  const uint64_t mnz = mhi | mlo;
                  if constexpr (PLF) {
                    const int wd = kj >= 32 ? 1 : 0;
                    sw3[ob][r][wd] = shin(sw3[ob][r][wd], mps);
                    sw3[ob][r][2 + wd] = shin(sw3[ob][r][2 + wd], mnz);
                    sw3[ob][r][4 + wd] = shin(sw3[ob][r][4 + wd], mlo);
                  } else {
                    sw3[ob][r][0] = shin(shin(shin(sw3[ob][r][0], mlo), mnz), mps);
                  }
                }
              }
            }
          }
        }
#pragma unroll
        for (int a = 0; a < OBM; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if constexpr (PLF) {
#pragma unroll
              for (int q = 0; q < 3; ++q)
                pl[a][c][q] = (uint64_t)sw3[a][c][2 * q] | ((uint64_t)sw3[a][c][2 * q + 1] << 32);
            } else {
              stc[a][c] = sw3[a][c][0];
            }
          }
      }
      for (int k = 0; k < ((CST > 0 && !literal && std8) ? 0 : g.nbw); ++k) {
#pragma unroll
        for (int ob = 0; ob < OBM; ++ob) {
          if (ob < nob) {
            const int o = (og * OBM + ob) * 16 + r16;
            v4i wk[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) wk[ks] = wt[((k * NOB + ob) * KS + ks) * 64 + lane];
            uint32_t stw[4] = {0u, 0u, 0u, 0u};
            uint32_t tq[4][3] = {{0u, 0u, 0u}, {0u, 0u, 0u}, {0u, 0u, 0u}, {0u, 0u, 0u}};
#pragma unroll
            for (int j = 0; j < NBP; ++j) {
              if (j < g.nba) {
                v4i ps = {0, 0, 0, 0};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) if (ks < ksn) ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[ks], ps, 0, 0, 0);
                const int pcol = (j * g.nbw + k) * NOB * 16 + ob * 16 + r16;
                if (!literal) {
                  const int4 pv = pt[pcol];
                  const float cf = ct[pcol];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const bool hi = ps[r] >= pv.x, lo = ps[r] <= pv.y;
                    float a = hi ? cf : 0.f;
                    a = lo ? -cf : a;
                    acc[ob][r] += a;
                    const bool pass = (unsigned)(ps[r] - pv.z) <= (unsigned)pv.w;
                    if (PLF) {
                      tq[r][0] |= (pass ? 1u : 0u) << j;
                      tq[r][1] |= ((hi || lo) ? 1u : 0u) << j;
                      tq[r][2] |= (lo ? 1u : 0u) << j;
                    } else {
                      stw[r] |= ((pass ? 1u : 0u) | ((hi || lo) ? 2u : 0u) | (lo ? 4u : 0u)) << (3 * j);
                    }
                  }
                } else if (is_shift(g)) {
                  const float al = pp.alpha[pidx(g, i, j, k, o)], be = pp.beta[pidx(g, i, j, k, o)];
                  const float mk = ckl[k * g.nba + j];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    acc[ob][r] += shift_adc_literal(ps[r], sw, sa, al, be, mk);
                    const uint32_t sb = shift_state_literal(ps[r], sw, sa, al, be, g.thr_hi, g.thr_lo);
                    if (PLF) {
                      tq[r][0] |= (sb & 1u) << j;
                      tq[r][1] |= ((sb >> 1) & 1u) << j;
                      tq[r][2] |= ((sb >> 2) & 1u) << j;
                    } else {
                      stw[r] |= sb << (3 * j);
                    }
                  }
                } else {
                  const float al = pp.alpha[pidx(g, i, j, k, o)];
                  const float mk = ckl[k * g.nba + j];
                  const int4 pv = pt[pcol];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    acc[ob][r] += adc_literal_sum(ps, g.mode, sw, sa, al, g.qn, g.qp, mk, r);
                    const bool pass = flag_lit ? (ste_literal(ps[r], g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f)
                                               : ((unsigned)(ps[r] - pv.z) <= (unsigned)pv.w);
                    const float code =
                        has_code ? code_literal(ps[r], g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo) : 0.f;
                    const uint32_t sb = st_bits(pass, code);
                    if (PLF) {
                      tq[r][0] |= (sb & 1u) << j;
                      tq[r][1] |= ((sb >> 1) & 1u) << j;
                      tq[r][2] |= ((sb >> 2) & 1u) << j;
                    } else {
                      stw[r] |= sb << (3 * j);
                    }
                  }
                }
              }
            }
            if (PLF) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 3; ++q) pl[ob][r][q] |= (uint64_t)tq[r][q] << (g.nba * k);
            } else if (CST) {
#pragma unroll
              for (int r = 0; r < 4; ++r) stc[ob][r] |= stw[r] << (3 * g.nba * k);
            }
          }
        }
      }
#if defined(CIMQ_EXP_FWD_NOSTATE) || defined(CIMQ_EXP_FWD_NOADC)
      if (false) {
#else
      if (CST && WST) {
#endif
#pragma unroll
        for (int ob = 0; ob < OBM; ++ob) {
          const int o = (og * OBM + ob) * 16 + r16;
          if (ob < nob && o < g.O) {
            const size_t e0 = ((size_t)i * g.M + (size_t)mt * 64 + wave * 16 + 4 * g4) * g.O + o;
            if (PLF) {
              uint2* s64 = reinterpret_cast<uint2*>(st);
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                  s64[(e0 + (size_t)r * g.O) * 3 + q] = make_uint2((uint32_t)pl[ob][r][q], (uint32_t)(pl[ob][r][q] >> 32));
            } else {
              uint32_t* s32 = reinterpret_cast<uint32_t*>(st) + e0;
#pragma unroll
              for (int r = 0; r < 4; ++r) s32[(size_t)r * g.O] = stc[ob][r];
            }
          }
        }
      }
    }
    // acc[ob][r]: pixel wave*16 + 4*g4 + r, channel (og*4 + ob)*16 + r16
#pragma unroll
    for (int ob = 0; ob < OBM; ++ob) {
      const int o = (og * OBM + ob) * 16 + r16;
      if (ob < nob && o < g.O) {
        if (is_shift(g) && !literal) {
          // the threshold path sums code * alpha * mask; the shift ADC adds beta * mask per pair
          const float bs = pp.bsum[o];
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[ob][r] += bs;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!g.onchw) out[((size_t)mt * 64 + wave * 16 + 4 * g4 + r) * g.O + o] = acc[ob][r];
        if (g.onchw) {
          const int m4 = mt * 64 + wave * 16 + 4 * g4;  // M < 2^24 (v3_plan)
          const int bb = fdiv(m4, g.P, inv_p), pq = m4 - bb * g.P;
          *reinterpret_cast<float4*>(out + ((size_t)bb * g.O + o) * g.P + pq) =
              make_float4(acc[ob][0], acc[ob][1], acc[ob][2], acc[ob][3]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// coalesced, thread-parallel slab reductions: 64 consecutive outputs x 4 chunk lanes / block
// ---------------------------------------------------------------------------------------
// 64 consecutive outputs per block, blockDim/64 chunk lanes per output; every lane keeps four
// independent loads in flight.  Returns the sum in the threads of the first wave.
__device__ inline float reduce_chunks(const float* __restrict__ slab, size_t chunk_stride, int nchunks,
                                      size_t idx, float* red) {
  // 8 independent loads in flight per lane: the few reducer blocks are latency-bound
  const int sub = threadIdx.x >> 6, nsub = blockDim.x >> 6;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int c = sub;
  for (; c + 7 * nsub < nchunks; c += 8 * nsub) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += slab[(size_t)(c + u * nsub) * chunk_stride + idx];
  }
  for (; c < nchunks; c += nsub) a[0] += slab[(size_t)c * chunk_stride + idx];
  red[threadIdx.x] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  float v = 0.f;
  if (sub == 0)
    for (int t = 0; t < nsub; ++t) v += red[threadIdx.x + 64 * t];
  return v;
}

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ __launch_bounds__(1024) void reduce_gw_v3_kernel(Geo g, int nchunks, const float* __restrict__ gw_slab,
                                                            const float* __restrict__ sa_p,
                                                            float* __restrict__ grad_w) {
  __shared__ float red[1024];
  const size_t rows = (size_t)g.T * g.FBT * 16;  // (tile, f-in-tile)
  const size_t nout = rows * g.Opad;
  const size_t idx = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const float v = reduce_chunks(gw_slab, nout, nchunks, idx < nout ? idx : 0, red);
  if ((threadIdx.x >> 6) == 0 && idx < nout) {
    const int o = (int)(idx % g.Opad);
    const size_t row = idx / g.Opad;
    const int i = (int)(row / (g.FBT * 16)), fl = (int)(row - (size_t)i * g.FBT * 16);
    const int f = i * g.xbar + fl;
    if (o < g.O && fl < g.xbar && f < g.K) grad_w[(size_t)o * g.K + f] = v * ((*sa_p) / (float)g.nbw);
  }
}
#endif

#ifdef CIMQ_TU_MAIN  // non-template kernel: defined in one translation unit only
__global__ __launch_bounds__(1024) void reduce_galpha_v3_kernel(Geo g, int nchunks, const float* __restrict__ ga_slab,
                                                                Params pp, float cgrad, int init,
                                                                const float* __restrict__ sw_p,
                                                                const float* __restrict__ sa_p, float count,
                                                                float sqrt_qp, float* __restrict__ out) {
  __shared__ float red[1024];
  const int nkj = g.nbw * g.nba;
  const size_t nout = (size_t)g.T * nkj * g.Opad;
  const size_t idx = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const float s = reduce_chunks(ga_slab, nout, nchunks, idx < nout ? idx : 0, red);
  if ((threadIdx.x >> 6) == 0 && idx < nout) {
    const int o = (int)(idx % g.Opad);
    const size_t q = idx / g.Opad;  // (i, k, j)
    if (o < g.O) {
      const int kj = (int)(q % nkj);
      const int i = (int)(q / nkj);
      const int k = kj / g.nba, j = kj - k * g.nba;
      const size_t dst = (((size_t)i * g.nbw + k) * g.nba + j) * g.O + o;  // [1,T,nbw,nba,1,O]
      if (init) {
        const float mean = s / count;
        const float v = (2.0f * mean) / sqrt_qp;
        out[dst] = (v == 0.f) ? (1.0f * (*sw_p)) * (*sa_p) : v;  // lsq.py:560-561
      } else {
        out[dst] = (cgrad * pp.ckj[kj]) * s;
      }
    }
  }
}
#endif

}  // namespace cimq

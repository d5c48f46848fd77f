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
  int WP;          // patch row length: W + 2*PW
  int RI, nbands;  // grad_x: owned input rows per block, bands per image
  int RHB;         // grad_x: max band patch rows
  int NPB;         // grad_x: max output pixels per band, rounded up to 16
  int fwd_res;     // forward: every tile's weights / thresholds resident in LDS
  int nmt;         // M / 64
  int NCG;         // grad_w: max input channels one tile touches
  int CB;          // grad_x: 16-channel blocks of the output tile grid (ceil(C/16))
  int NT;          // grad_x: max output tiles (16 positions x 16 channels) per band
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
  const int n = (ncx < 0 ? g.C : ncx) * RHx * QW;
  const float invQ = 1.f / (float)QW, invR = 1.f / (float)RHx;
  const uint4* src = reinterpret_cast<const uint4*>(xc) + ((size_t)b * g.C + c0) * g.H * QW;
  const int nt = blockDim.x;
  for (int base = threadIdx.x; base < n; base += 8 * nt) {
    uint4 v[8];
    int d[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * nt;
      d[u] = -1;
      if (idx < n) {
        const int row = fdiv(idx, QW, invQ), q = idx - row * QW;
        const int c = fdiv(row, RHx, invR), rr = row - c * RHx;
        const int ih = ih_first + rr;
        d[u] = ((c * RHx + rr) * WP + g.PW) * NBP + q * 16;
        v[u] = make_uint4(0, 0, 0, 0);
        if (ih >= 0 && ih < g.H) v[u] = src[((size_t)c * g.H + ih) * QW + q];
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

// the same rows of the backward ctx slices, widened to bf16 (exact small integers):
// element word = NBP bf16 = NBP/2 dwords, dword s = {bf16(slice 2s), bf16(slice 2s+1)}
__device__ inline uint32_t bf16x2_of_bytes(uint32_t w, int sh) {
  const float lo = (float)(int8_t)((w >> sh) & 0xFF);
  const float hi = (float)(int8_t)((w >> (sh + 8)) & 0xFF);
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}

template <int NBP>
__device__ inline void stage_rows_bf16(const Geo& g, int WP, int RHx, const uint8_t* __restrict__ xc, int b,
                                       int ih_first, uint8_t* patch) {
  const int QW = g.W * NBP / 16;
  const int n = g.C * RHx * QW;
  const float invQ = 1.f / (float)QW, invR = 1.f / (float)RHx;
  const uint4* src = reinterpret_cast<const uint4*>(xc) + (size_t)b * g.C * g.H * QW;
  const int nt = blockDim.x;
  for (int base = threadIdx.x; base < n; base += 4 * nt) {
    uint4 v[4];
    int d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = base + u * nt;
      d[u] = -1;
      if (idx < n) {
        const int row = fdiv(idx, QW, invQ), q = idx - row * QW;
        const int c = fdiv(row, RHx, invR), rr = row - c * RHx;
        const int ih = ih_first + rr;
        d[u] = ((c * RHx + rr) * WP + g.PW) * (2 * NBP) + q * 32;
        v[u] = make_uint4(0, 0, 0, 0);
        if (ih >= 0 && ih < g.H) v[u] = src[((size_t)c * g.H + ih) * QW + q];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (d[u] >= 0) {
        uint32_t* p = reinterpret_cast<uint32_t*>(patch + d[u]);
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          p[2 * e] = bf16x2_of_bytes(w[e], 0);
          p[2 * e + 1] = bf16x2_of_bytes(w[e], 16);
        }
      }
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
      const int c = f / g.KHW, rem = f - c * g.KHW;
      const int kh = rem / g.KW, kw = rem - kh * g.KW;
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
__device__ inline void gather_xs(const uint8_t* patch, int rb, const int* ptab, int g4, v4i (&xs)[NBP][KS]) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
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
__device__ inline void split3x8(const float (&v)[8], v8bf& bh, v8bf& bm, v8bf& bl) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    const float r1 = v[e] - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    bh[e] = h;
    bm[e] = m;
    bl[e] = (__bf16)r2;
  }
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

// ---------------------------------------------------------------------------------------
// forward: out[m, o] = sum_{i,j,k} ADC(ps_ijk[m, o]) * mask   (lsq.py:166-233)
// block = 64-pixel m-tiles (grid-stride) x one 64-wide o-group; wave w = pixels 16w..16w+15.
// ---------------------------------------------------------------------------------------
template <int NBP, int KS>
__global__ __launch_bounds__(256) void cim_fwd_v3_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                         const v4i* __restrict__ wfrag, Params pp,
                                                         const float* __restrict__ sw_p,
                                                         const float* __restrict__ sa_p, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int og = blockIdx.y;
  const int NOB = min(4, g.OB16);
  const int nob = min(4, g.OB16 - og * 4);
  const int TT = v.fwd_res ? g.T : 1;
  const int nkj = g.nbw * g.nba;
  uint8_t* cur = smem;
  uint8_t* patch = cur; cur += al16((size_t)g.C * v.RH * v.WP * NBP);
  int* ptab = reinterpret_cast<int*>(cur); cur += (size_t)g.T * KS * 64 * 4;
  v4i* wfl = reinterpret_cast<v4i*>(cur); cur += (size_t)TT * g.nbw * NOB * KS * 1024;   // [tt][k][ob][ks][64]
  int4* prm = reinterpret_cast<int4*>(cur); cur += (size_t)TT * nkj * NOB * 16 * 16;    // [tt][j][k][NOB*16]
  float* ckl = reinterpret_cast<float*>(cur);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0) || g.mode != ADC_TERNARY;
  const int Wo = 1 << v.lw;

  auto stage_tile = [&](int i, int tt) {
    batched_copy<4>(g.nbw * NOB * KS * 64, wfl + (size_t)tt * g.nbw * NOB * KS * 64, [&](int idx) -> v4i {
      const int l = idx & 63, fr = idx >> 6;
      const int ks = fr % KS, kob = fr / KS, k = kob / NOB, ob = kob - k * NOB;
      v4i w = {0, 0, 0, 0};
      if (ob < nob) w = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * 4 + ob) * WAVE + l];
      return w;
    });
    if (!literal) {
      batched_copy<2>(nkj * NOB * 16, prm + (size_t)tt * nkj * NOB * 16, [&](int idx) -> int4 {
        const int col = idx % (NOB * 16), jk = idx / (NOB * 16), k = jk % g.nbw, j = jk / g.nbw;
        const int o = og * 64 + col;
        int4 p = make_int4(0, 0, 0, 0);
        if (o < g.Opad) {
          const int pi = pidx(g, i, j, k, o);
          p = make_int4(pp.thi[pi], pp.tlo[pi], __float_as_int(pp.coef[pi]), 0);
        }
        return p;
      });
    }
  };

  for (int i = 0; i < g.T; ++i) build_ptab(g, i, KS, v.RH, v.WP, ptab + i * KS * 64);
  for (int t = threadIdx.x; t < 3 * nkj; t += blockDim.x) ckl[t] = pp.ckj[t];
  if (v.fwd_res)
    for (int i = 0; i < g.T; ++i) stage_tile(i, i);
  zero_lds(reinterpret_cast<uint32_t*>(patch), g.C * v.RH * v.WP * NBP / 4);

  const int pl = wave * 16 + r16;  // this lane's gather pixel within the m-tile
  const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & (Wo - 1)) * g.SW;
  const int tiles_per_img = g.P >> 6;

  for (int mt = blockIdx.x; mt < v.nmt; mt += gridDim.x) {
    const int b = mt / tiles_per_img, p0 = (mt - b * tiles_per_img) * 64;
    const int oh0 = p0 >> v.lw;
    __syncthreads();
    stage_rows<NBP>(g, v.WP, v.RH, xcf, b, oh0 * g.SH - g.PH, patch);
    __syncthreads();
    float acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][c] = 0.f;
    for (int i = 0; i < g.T; ++i) {
      if (!v.fwd_res) {
        __syncthreads();
        stage_tile(i, 0);
        __syncthreads();
      }
      const int tt = v.fwd_res ? i : 0;
      v4i xs[NBP][KS];
      gather_xs<NBP, KS>(patch, rb, ptab + i * KS * 64, g4, xs);
      const v4i* wt = wfl + (size_t)tt * g.nbw * NOB * KS * 64;
      const int4* pt = prm + (size_t)tt * nkj * NOB * 16;
      for (int k = 0; k < g.nbw; ++k) {
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) {
          if (ob < nob) {
            v4i wk[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) wk[ks] = wt[((k * NOB + ob) * KS + ks) * 64 + lane];
#pragma unroll
            for (int j = 0; j < NBP; ++j) {
              if (j < g.nba) {
                v4i ps = {0, 0, 0, 0};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[ks], ps, 0, 0, 0);
                if (!literal) {
                  const int4 pv = pt[(j * g.nbw + k) * NOB * 16 + ob * 16 + r16];
                  const float cf = __int_as_float(pv.z);
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    float a = (ps[r] >= pv.x) ? cf : 0.f;
                    a = (ps[r] <= pv.y) ? -cf : a;
                    acc[ob][r] += a;
                  }
                } else {
                  const int o = (og * 4 + ob) * 16 + r16;
                  const float al = pp.alpha[pidx(g, i, j, k, o)];
                  const float mk = ckl[k * g.nba + j];
#pragma unroll
                  for (int r = 0; r < 4; ++r) acc[ob][r] += adc_literal_sum(ps, g.mode, sw, sa, al, g.qn, g.qp, mk, r);
                }
              }
            }
          }
        }
      }
    }
    // acc[ob][r]: pixel wave*16 + 4*g4 + r, channel (og*4 + ob)*16 + r16
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      const int o = (og * 4 + ob) * 16 + r16;
      if (ob < nob && o < g.O) {
#pragma unroll
        for (int r = 0; r < 4; ++r) out[((size_t)mt * 64 + wave * 16 + 4 * g4 + r) * g.O + o] = acc[ob][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// grad_x (+ fused LSQ activation backward) as a transposed implicit GEMM: block = one band of
// RI input rows of one image.  Per tile i and 32-wide kappa chunk:
//   phase A  G_i[m, kappa] = g[m, o] * E_i[m, kappa],  E_i = sum_j cE_kj * STE_ijk[m, o]
//            (ps recomputed on the int8 MFMA for every output pixel m touching the band),
//            split into bf16 hi/mid/lo rows in LDS;
//   phase B  gx[q, c] += sum_{kh,kw} sum_kappa G_i[m(q,kh,kw), kappa] * int8(w_k[(c,kh,kw), o])
//            on bf16 MFMA, q = input position of the band, c = channel (lsq.py:257-317).
// The nn.Fold adjoint is folded into the MFMA K dimension (kh, kw, kappa): every wave owns
// its output tiles in registers for the whole kernel, so there are no atomics; the LSQ
// activation backward is applied in registers and gx stored once.
// ---------------------------------------------------------------------------------------
template <int NBP, int KS, int TPW, bool LSQ>
__global__ __launch_bounds__(512) void cim_bwd_gx_v4_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                            const v4i* __restrict__ wfrag,
                                                            const uint4* __restrict__ wtc, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p,
                                                            const float* __restrict__ gout,
                                                            const float* __restrict__ x, float* __restrict__ gx,
                                                            float* __restrict__ gsa_part) {
  // TPW: output tiles per wave (host guarantees NT <= 8 * TPW)
  constexpr int GPB = 40;   // G / W row pitch in bf16: 32 kappa + 8 pad (bank spread, 16-B rows)
  constexpr int KX = 3;     // max kernel height / width (host guarantees KH, KW <= 3)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int nkj = g.nbw * g.nba;
  const int b = blockIdx.x / v.nbands, band = blockIdx.x - b * v.nbands;
  const int r0 = band * v.RI, r1 = min(g.H, r0 + v.RI);
  const int nrow = r1 - r0;
  int oh_lo = r0 + g.PH - (g.KH - 1);
  oh_lo = oh_lo <= 0 ? 0 : (oh_lo + g.SH - 1) / g.SH;
  const int oh_hi = min(g.Ho - 1, (r1 - 1 + g.PH) / g.SH);
  const int nro = oh_hi - oh_lo + 1;
  const int npb = nro << v.lw;
  const int RHb = (nro - 1) * g.SH + g.KH;
  const int ih_first = oh_lo * g.SH - g.PH;
  const int Cp = v.CB * 16;
  const int ZROW = v.NPB;  // all-zero G row

  uint8_t* cur = smem;
  uint8_t* patch = cur; cur += al16((size_t)g.C * v.RHB * v.WP * NBP);
  __bf16* Gs = reinterpret_cast<__bf16*>(cur); cur += al16((size_t)3 * (v.NPB + 1) * GPB * 2);  // [part][row][GPB]
  __bf16* Wb = reinterpret_cast<__bf16*>(cur); cur += al16((size_t)g.KHW * Cp * GPB * 2);       // [khw][c][GPB]
  v4i* wfl = reinterpret_cast<v4i*>(cur); cur += (size_t)g.NBLK * KS * 1024;                    // [kb][ks][64]
  int2* msl = reinterpret_cast<int2*>(cur); cur += al16((size_t)nkj * g.Opad * 8);              // [j][k][Opad]
  int* ptab = reinterpret_cast<int*>(cur); cur += KS * 64 * 4;
  float* ckl = reinterpret_cast<float*>(cur); cur += al16(3 * nkj * 4);
  int* kbt = reinterpret_cast<int*>(cur); cur += al16((size_t)g.NBLK * 4);  // kb -> (k << 16) | o-block
  float* red = reinterpret_cast<float*>(cur);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0);
  const bool gvec = (g.O & 3) == 0;
  const int PART = (v.NPB + 1) * GPB;  // bf16 elements per split part

  zero_lds(reinterpret_cast<uint32_t*>(patch), g.C * RHb * v.WP * NBP / 4);
  for (int t = threadIdx.x; t < 3 * GPB / 2; t += blockDim.x) {
    const int part = t / (GPB / 2), w = t - part * (GPB / 2);
    reinterpret_cast<uint32_t*>(Gs + part * PART + ZROW * GPB)[w] = 0u;
  }
  for (int t = threadIdx.x; t < 3 * nkj; t += blockDim.x) ckl[t] = pp.ckj[t];
  for (int t = threadIdx.x; t < g.NBLK; t += blockDim.x) kbt[t] = ((t / g.OB16) << 16) | (t % g.OB16);
  __syncthreads();
  stage_rows<NBP>(g, v.WP, RHb, xcf, b, ih_first, patch);

  // this wave's output tiles: t = wave + NW*u -> (q-block, c-block); per tile the G row of
  // every tap for this lane's A-operand position q = qb*16 + r16, and x at the lane's four
  // accumulator positions q = qb*16 + 4*g4 + r (channel cb*16 + r16)
  const int nq = nrow * g.W;
  const int QBb = (nq + 15) >> 4;
  const int NTb = QBb * v.CB;
  // per tile: this lane's A-operand position relative to the band's first output row
  // (ihp = ih + PH - oh_lo*SH, iwp = iw + PW; -1 when the position is padding)
  int ihp[TPW], iwp[TPW];
  float xpre[TPW][4];
  v4f acc[TPW];
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    acc[u] = v4f{0.f, 0.f, 0.f, 0.f};
    const int t = wave + NW * u;
    const int qb = t / v.CB, cb = t - qb * v.CB;
    const int q = qb * 16 + r16;
    const int ih = r0 + q / g.W, iw = q - (q / g.W) * g.W;
    ihp[u] = (t < NTb && q < nq) ? ih + g.PH - oh_lo * g.SH : -(1 << 20);
    iwp[u] = iw + g.PW;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qa = qb * 16 + 4 * g4 + r, c = cb * 16 + r16;
      xpre[u][r] = 0.f;
      if (LSQ && t < NTb && qa < nq && c < g.C) xpre[u][r] = x[(((size_t)b * g.C + c) * g.H + r0) * g.W + qa];
    }
  }

  const int ngrp = (npb + 15) >> 4;
  const float* gimg = gout + ((size_t)b * g.P + ((size_t)oh_lo << v.lw)) * g.O;

  for (int i = 0; i < g.T; ++i) {
    const int ci0 = (i * g.xbar) / g.KHW, ci1 = (min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
    __syncthreads();
    batched_copy<2>(g.NBLK * KS * 64, wfl, [&](int idx) -> v4i {
      return wfrag[(size_t)i * KS * g.NBLK * 64 + ((idx >> 6) % KS) * g.NBLK * 64 + ((idx >> 6) / KS) * 64 + (idx & 63)];
    });
    if (!literal) {
      const int npi = nkj * g.Opad;
      batched_copy<2>(npi, msl, [&](int idx) -> int2 { return make_int2(pp.mlo[i * npi + idx], pp.mhi[i * npi + idx]); });
    }
    build_ptab(g, i, KS, RHb, v.WP, ptab);

    for (int kc = 0; kc < g.NKS; ++kc) {
      __syncthreads();
      // W rows of this tile and kappa chunk: Wb[khw][c][kappa] (zero for (c, khw) outside tile i)
      {
        const int nvec = g.KHW * Cp * 4;  // 16-B pieces: 4 data pieces per (khw, c) row
        for (int base = threadIdx.x; base < nvec; base += 4 * blockDim.x) {
          uint4 val[4];
          int dst[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int idx = base + u * blockDim.x;
            dst[u] = -1;
            if (idx < nvec) {
              const int row = idx >> 2, q8 = idx & 3;  // row = khw * Cp + c
              const int khw = row / Cp, c = row - khw * Cp;
              const int f = c * g.KHW + khw;
              val[u] = make_uint4(0, 0, 0, 0);
              if (c < g.C && f >= i * g.xbar && f < min(g.K, (i + 1) * g.xbar))
                val[u] = wtc[((size_t)row * g.NKS + kc) * 4 + q8];
              dst[u] = row * (GPB / 8) + q8;
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (dst[u] >= 0) reinterpret_cast<uint4*>(Wb)[dst[u]] = val[u];
        }
      }
      // phase A: G rows of kappa blocks 2kc, 2kc+1 for every band output pixel
      for (int u = wave; u < ngrp * 2; u += NW) {
        const int grp = u >> 1, h2 = u & 1;
        const int kb = 2 * kc + h2;
        const int plr = grp * 16 + r16;
        const bool pvalid = plr < npb;
        const int pl = min(plr, npb - 1);
        float G[4] = {0.f, 0.f, 0.f, 0.f};
        if (kb < g.NBLK) {
          const int kt = kbt[kb];
          const int k = kt >> 16, ob0 = (kt & 0xFFFF) * 16 + 4 * g4;
          float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (pvalid) {
            const float* grow = gimg + (size_t)pl * g.O;
            if (gvec && ob0 + 4 <= g.O) {
              gv = *reinterpret_cast<const float4*>(grow + ob0);
            } else {
              if (ob0 + 0 < g.O) gv.x = grow[ob0 + 0];
              if (ob0 + 1 < g.O) gv.y = grow[ob0 + 1];
              if (ob0 + 2 < g.O) gv.z = grow[ob0 + 2];
              if (ob0 + 3 < g.O) gv.w = grow[ob0 + 3];
            }
          }
          const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & ((1 << v.lw) - 1)) * g.SW;
          v4i xs[NBP][KS];
          gather_xs<NBP, KS>(patch, rb, ptab, g4, xs);
          v4i wk[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) wk[ks] = wfl[(kb * KS + ks) * 64 + lane];
          float E[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < NBP; ++j) {
            if (j < g.nba) {
              v4i ps = {0, 0, 0, 0};
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(wk[ks], xs[j][ks], ps, 0, 0, 0);
              const float ce = ckl[nkj + k * g.nba + j];
              if (!literal) {
                const int4* ms = reinterpret_cast<const int4*>(msl + (j * g.nbw + k) * g.Opad + ob0);
                const int4 m01 = ms[0], m23 = ms[1];
                E[0] += ((unsigned)(ps[0] - m01.x) <= (unsigned)m01.y) ? ce : 0.f;
                E[1] += ((unsigned)(ps[1] - m01.z) <= (unsigned)m01.w) ? ce : 0.f;
                E[2] += ((unsigned)(ps[2] - m23.x) <= (unsigned)m23.y) ? ce : 0.f;
                E[3] += ((unsigned)(ps[3] - m23.z) <= (unsigned)m23.w) ? ce : 0.f;
              } else {
                const int pi = pidx(g, i, j, k, ob0);
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  E[r] += ste_literal(ps[r], g.mode, sw, sa, pp.alpha[pi + r], g.thr_hi, g.thr_lo) * ce;
              }
            }
          }
          G[0] = gv.x * E[0];
          G[1] = gv.y * E[1];
          G[2] = gv.z * E[2];
          G[3] = gv.w * E[3];
        }
        if (pvalid) {
          // lane holds kappa (chunk-local) h2*16 + 4*g4 + r of pixel pl: 4 consecutive bf16 per part
          uint32_t ph[2], pm[2], pl2[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            float a0 = G[2 * e], a1 = G[2 * e + 1];
            const __bf16 h0 = (__bf16)a0, h1 = (__bf16)a1;
            const float s0 = a0 - (float)h0, s1 = a1 - (float)h1;
            const __bf16 m0 = (__bf16)s0, m1 = (__bf16)s1;
            const __bf16 l0 = (__bf16)(s0 - (float)m0), l1 = (__bf16)(s1 - (float)m1);
            ph[e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
            pm[e] = (uint32_t)__builtin_bit_cast(uint16_t, m0) | ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
            pl2[e] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
          }
          const int off = plr * GPB + h2 * 16 + 4 * g4;
          *reinterpret_cast<uint2*>(Gs + off) = make_uint2(ph[0], ph[1]);
          *reinterpret_cast<uint2*>(Gs + PART + off) = make_uint2(pm[0], pm[1]);
          *reinterpret_cast<uint2*>(Gs + 2 * PART + off) = make_uint2(pl2[0], pl2[1]);
        }
      }
      __syncthreads();
      // phase B: every owned output tile, every tap
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int t = wave + NW * u;
        const int qb = t / v.CB, cb = t - qb * v.CB;
        if (t < NTb && cb * 16 <= ci1 && cb * 16 + 15 >= ci0) {
          v4f a = acc[u];
#pragma unroll
          for (int kh = 0; kh < KX; ++kh) {
#pragma unroll
            for (int kw = 0; kw < KX; ++kw) {
              if (kh < g.KH && kw < g.KW) {
                // G row of output pixel m(q, kh, kw): the all-zero row when it does not exist
                const int ohs = ihp[u] - kh, ows = iwp[u] - kw;
                int row = ZROW;
                if (ohs >= 0 && ows >= 0 && (ohs % g.SH) == 0 && (ows % g.SW) == 0) {
                  const int oh = ohs / g.SH, ow = ows / g.SW;
                  if (oh < nro && ow < g.Wo) row = (oh << v.lw) + ow;
                }
                const int khw = kh * g.KW + kw;
                const v8bf gh = *reinterpret_cast<const v8bf*>(Gs + row * GPB + 8 * g4);
                const v8bf gm = *reinterpret_cast<const v8bf*>(Gs + PART + row * GPB + 8 * g4);
                const v8bf gl = *reinterpret_cast<const v8bf*>(Gs + 2 * PART + row * GPB + 8 * g4);
                const v8bf wv = *reinterpret_cast<const v8bf*>(Wb + (khw * Cp + cb * 16 + r16) * GPB + 8 * g4);
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh, wv, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm, wv, a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gl, wv, a, 0, 0, 0);
              }
            }
          }
          acc[u] = a;
        }
      }
    }
  }
  // epilogue from registers: acc[u][r] = gx_raw[q = qb*16 + 4*g4 + r, c = cb*16 + r16]
  const float scale = sw / (float)g.nba;
  float part = 0.f;
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    const int t = wave + NW * u;
    const int qb = t / v.CB, cb = t - qb * v.CB;
    const int c = cb * 16 + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qa = qb * 16 + 4 * g4 + r;
      if (t < NTb && qa < nq && c < g.C) {
        const size_t gi = (((size_t)b * g.C + c) * g.H + r0) * g.W + qa;
        const float gqv = acc[u][r] * scale;
        if (LSQ) {
          // autograd of round_pass(clamp(x/sa, 0, Qp)) * sa (lsq.py:549)
          const float xv = xpre[u][r];
          const float y1 = xv / sa;
          const float cl = clamp_nan(y1, 0.f, g.lsq_qp);
          const float rr2 = rintf(cl);
          const float rp = (rr2 - cl) + cl;
          const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
          const float gy = pass ? gqv * sa : 0.f;
          gx[gi] = gy / sa;
          part += gqv * rp;
          part += -(gy * (y1 / sa));
        } else {
          gx[gi] = gqv;
        }
      }
    }
  }
  if (LSQ) {
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if (lane == 0) red[wave] = part;
    __syncthreads();
    if (threadIdx.x == 0) {
      float sacc = 0.f;
      for (int w = 0; w < NW; ++w) sacc += red[w];
      gsa_part[blockIdx.x] = sacc;
    }
  }
}

// One grad_w pixel tile in one round of loads: forward slice rows (-> patch) and backward
// slice rows (-> patchB, widened to bf16) of channels [c0, c0 + ncx) -- the channels tile i
// touches.  Every thread issues up to 4 + 4 16-byte loads before its first LDS store.
template <int NBP>
__device__ inline void stage_gw_mtile(const Geo& g, int WP, int RHx, const uint8_t* __restrict__ xcf,
                                      const uint8_t* __restrict__ xcb, int b, int ih_first, int c0, int ncx,
                                      uint8_t* patch, uint8_t* patchB) {
  const int QW = g.W * NBP / 16;
  const int n = ncx * RHx * QW;
  const float invQ = 1.f / (float)QW, invR = 1.f / (float)RHx;
  const size_t img = ((size_t)b * g.C + c0) * g.H * QW;
  const uint4* sf = reinterpret_cast<const uint4*>(xcf) + img;
  const uint4* sb = reinterpret_cast<const uint4*>(xcb) + img;
  const int nt = blockDim.x;
  for (int base = threadIdx.x; base < n; base += 4 * nt) {
    uint4 vf[4], vb[4];
    int d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = base + u * nt;
      d[u] = -1;
      if (idx < n) {
        const int row = fdiv(idx, QW, invQ), q = idx - row * QW;
        const int c = fdiv(row, RHx, invR), rr = row - c * RHx;
        const int ih = ih_first + rr;
        d[u] = ((c * RHx + rr) * WP + g.PW) * NBP + q * 16;
        vf[u] = make_uint4(0, 0, 0, 0);
        vb[u] = make_uint4(0, 0, 0, 0);
        if (ih >= 0 && ih < g.H) {
          const size_t si = ((size_t)c * g.H + ih) * QW + q;
          vf[u] = sf[si];
          vb[u] = sb[si];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (d[u] >= 0) {
        uint32_t* pf = reinterpret_cast<uint32_t*>(patch + d[u]);
        pf[0] = vf[u].x; pf[1] = vf[u].y; pf[2] = vf[u].z; pf[3] = vf[u].w;
        uint32_t* pb = reinterpret_cast<uint32_t*>(patchB + 2 * d[u]);
        const uint32_t w[4] = {vb[u].x, vb[u].y, vb[u].z, vb[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pb[2 * e] = bf16x2_of_bytes(w[e], 0);
          pb[2 * e + 1] = bf16x2_of_bytes(w[e], 16);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// grad_w + grad_alpha (and the alpha_cim init sums): block = (pixel chunk, tile i, 32 cols)
//   D_j[m, o] = sum_k cD_kj * STE_ijk[m, o]
//   gw_i[f, o] += sum_{j, m} xhat_j[m, f] * (g[m, o] * D_j[m, o])     (bf16x3 MFMA)
//   ga[i, k, j, o] += sum_m code_ijk[m, o] * g[m, o]                   (lsq.py:257-333)
// Only the input channels of tile i are staged; grad_out is read straight from memory, one
// pixel tile ahead.
// ---------------------------------------------------------------------------------------
template <int NBP, int KS, int FBX, bool INIT>
__global__ __launch_bounds__(256) void cim_bwd_gw_v3_kernel(Geo g, V3 v, const uint8_t* __restrict__ xcf,
                                                            const uint8_t* __restrict__ xcb,
                                                            const v4i* __restrict__ wfrag, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p,
                                                            const float* __restrict__ gout, int rows_per_chunk,
                                                            float* __restrict__ gw_slab,
                                                            float* __restrict__ ga_slab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int nkj = g.nbw * g.nba;
  const int i = blockIdx.y, og = blockIdx.z;
  const int NOB = min(2, g.OB16);
  const int nob = min(2, g.OB16 - og * 2);
  const int c0 = (i * g.xbar) / g.KHW;
  const int ncx = (min(g.K, (i + 1) * g.xbar) - 1) / g.KHW - c0 + 1;
  const size_t pf = al16((size_t)v.NCG * v.RH * v.WP * NBP);
  const size_t pbsz = INIT ? 0 : al16((size_t)v.NCG * v.RH * v.WP * NBP * 2);
  const size_t gwsz = INIT ? 0 : (size_t)g.FBT * 16 * 32 * 4;

  uint8_t* cur = smem;
  uint8_t* patch = cur;
  uint8_t* patchB = cur + pf;
  float* gwacc = reinterpret_cast<float*>(cur);  // aliases the patches after the pixel loop
  cur += max(pf + pbsz, gwsz);
  int* ptab = reinterpret_cast<int*>(cur); cur += KS * 64 * 4;
  v4i* wfl = reinterpret_cast<v4i*>(cur); cur += (size_t)g.nbw * NOB * KS * 1024;     // [k][ob][ks][64]
  int4* prm = reinterpret_cast<int4*>(cur); cur += (size_t)nkj * NOB * 16 * 16;       // [j][k][NOB*16]
  float* qacc = reinterpret_cast<float*>(cur); cur += al16((size_t)nkj * 32 * 4);
  float* ckl = reinterpret_cast<float*>(cur);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int mbeg = blockIdx.x * rows_per_chunk, mend = min(mbeg + rows_per_chunk, g.M);
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = (pp.flags[0] != 0);
  const bool ternary_fast = (!literal) && g.mode == ADC_TERNARY;
  const bool has_code = (g.mode == ADC_SIGN || g.mode == ADC_TERNARY);
  const int Wo = 1 << v.lw;

  for (int t = threadIdx.x; t < nkj * 32; t += blockDim.x) qacc[t] = 0.f;
  for (int t = threadIdx.x; t < 3 * nkj; t += blockDim.x) ckl[t] = pp.ckj[t];
  build_ptab(g, i, KS, v.RH, v.WP, ptab, c0);
  batched_copy<4>(g.nbw * NOB * KS * 64, wfl, [&](int idx) -> v4i {
    const int l = idx & 63, fr = idx >> 6;
    const int ks = fr % KS, kob = fr / KS, k = kob / NOB, ob = kob - k * NOB;
    v4i w = {0, 0, 0, 0};
    if (ob < nob) w = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * 2 + ob) * WAVE + l];
    return w;
  });
  batched_copy<2>(nkj * NOB * 16, prm, [&](int idx) -> int4 {
    const int col = idx % (NOB * 16), jk = idx / (NOB * 16), k = jk % g.nbw, j = jk / g.nbw;
    const int o = og * 32 + col;
    int4 p = make_int4(0, 0, 0, 0);
    if (o < g.Opad) {
      const int pi = pidx(g, i, j, k, o);
      p = make_int4(pp.mlo[pi], pp.mhi[pi], pp.thi[pi], pp.tlo[pi]);
    }
    return p;
  });
  zero_lds(reinterpret_cast<uint32_t*>(patch), (int)((pf + pbsz) / 4));
  __syncthreads();

  // gather column pixel (i8 operand) and this lane's 4 accumulator-row pixels
  const int pl = wave * 16 + r16;
  const int rb = ((pl >> v.lw) * g.SH) * v.WP + (pl & (Wo - 1)) * g.SW;
  int rb4[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = wave * 16 + 4 * g4 + r;
    rb4[r] = ((q >> v.lw) * g.SH) * v.WP + (q & (Wo - 1)) * g.SW;
  }
  int ptf[FBX];
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) ptf[fb] = (fb < g.FBT) ? ptab[fb * 16 + r16] : 0;

  // grad_out of this lane's accumulator rows (4 pixels) for its column in each o-block
  auto load_gv = [&](int m0, float (&dst)[2][4]) {
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
      const int o = og * 32 + ob * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dst[ob][r] = 0.f;
        if (!INIT && m0 < mend && ob < nob && o < g.O)
          dst[ob][r] = gout[(size_t)(m0 + wave * 16 + 4 * g4 + r) * g.O + o];
      }
    }
  };
  float gnext[2][4];
  load_gv(mbeg, gnext);

  v4f gwa[FBX][2];
#pragma unroll
  for (int a = 0; a < FBX; ++a) {
    gwa[a][0] = v4f{0.f, 0.f, 0.f, 0.f};
    gwa[a][1] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  const int tiles_per_img = g.P >> 6;

  for (int m0 = mbeg; m0 < mend; m0 += 64) {
    const int mt = m0 >> 6;
    const int b = mt / tiles_per_img, p0 = (mt - b * tiles_per_img) * 64;
    const int ih_first = (p0 >> v.lw) * g.SH - g.PH;
    __syncthreads();
    if (INIT) stage_rows<NBP>(g, v.WP, v.RH, xcf, b, ih_first, patch, c0, ncx);
    else stage_gw_mtile<NBP>(g, v.WP, v.RH, xcf, xcb, b, ih_first, c0, ncx, patch, patchB);
    float gcur[2][4];
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) gcur[ob][r] = gnext[ob][r];
    __syncthreads();
    load_gv(m0 + 64, gnext);

    v4i xs[NBP][KS];
    gather_xs<NBP, KS>(patch, rb, ptab, g4, xs);
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
      if (ob < nob) {
        const int ocol = ob * 16 + r16;
        const float* gval = gcur[ob];
        float D[NBP][4];
#pragma unroll
        for (int j = 0; j < NBP; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) D[j][r] = 0.f;
        for (int k = 0; k < g.nbw; ++k) {
          v4i wk[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) wk[ks] = wfl[((k * NOB + ob) * KS + ks) * 64 + lane];
#pragma unroll
          for (int j = 0; j < NBP; ++j) {
            if (j < g.nba) {
              v4i ps = {0, 0, 0, 0};
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[ks], ps, 0, 0, 0);
              const int kj = k * g.nba + j;
              float qs = 0.f;
              if (INIT) {
#pragma unroll
                for (int r = 0; r < 4; ++r) qs += fabsf(((float)ps[r] * sw) * sa);  // lsq.py:64,84
              } else {
                const float cd = ckl[2 * nkj + kj];
                const int4 pv = prm[(j * g.nbw + k) * NOB * 16 + ocol];
                if (ternary_fast) {
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const int p = ps[r];
                    D[j][r] += ((unsigned)(p - pv.x) <= (unsigned)pv.y) ? cd : 0.f;
                    float q = (p >= pv.z) ? gval[r] : 0.f;
                    q = (p <= pv.w) ? -gval[r] : q;
                    qs += q;
                  }
                } else {
                  const int o = og * 32 + ocol;
                  const float al = pp.alpha[pidx(g, i, j, k, o)];
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const int p = ps[r];
                    const bool pass = literal ? (ste_literal(p, g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f)
                                              : ((unsigned)(p - pv.x) <= (unsigned)pv.y);
                    D[j][r] += pass ? cd : 0.f;
                    if (has_code) qs += code_literal(p, g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo) * gval[r];
                  }
                }
              }
              if (INIT || has_code) {
                qs += __shfl_xor(qs, 16);
                qs += __shfl_xor(qs, 32);
                if (g4 == 0) atomicAdd(&qacc[kj * 32 + ocol], qs);
              }
            }
          }
        }
        if (!INIT) {
          // B operands (k = (j-pair half h2, pixel r)) for every j-pair, then the f-blocks
          constexpr int NS = NBP / 2;
          v8bf bh[NS], bm[NS], bl[NS];
#pragma unroll
          for (int s2 = 0; s2 < NS; ++s2) {
            float ev[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int j = 2 * s2 + (e >> 2), r = e & 3;
              ev[e] = (j < g.nba) ? gval[r] * D[j][r] : 0.f;
            }
            split3x8(ev, bh[s2], bm[s2], bl[s2]);
          }
          const uint32_t* pB = reinterpret_cast<const uint32_t*>(patchB);
#pragma unroll
          for (int fb = 0; fb < FBX; ++fb) {
            if (fb < g.FBT) {
              v4f accw = gwa[fb][ob];
#pragma unroll
              for (int s2 = 0; s2 < NS; ++s2) {
                if (2 * s2 < g.nba) {
                  uint32_t d[4];
#pragma unroll
                  for (int r = 0; r < 4; ++r) d[r] = pB[(rb4[r] + ptf[fb]) * NS + s2];
                  v4i a;
                  a[0] = (int)__builtin_amdgcn_perm(d[1], d[0], 0x05040100u);
                  a[1] = (int)__builtin_amdgcn_perm(d[3], d[2], 0x05040100u);
                  a[2] = (int)__builtin_amdgcn_perm(d[1], d[0], 0x07060302u);
                  a[3] = (int)__builtin_amdgcn_perm(d[3], d[2], 0x07060302u);
                  const v8bf xa = as_v8bf(a);
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, bh[s2], accw, 0, 0, 0);
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, bm[s2], accw, 0, 0, 0);
                  accw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, bl[s2], accw, 0, 0, 0);
                }
              }
              gwa[fb][ob] = accw;
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (!INIT) {
    for (int t = threadIdx.x; t < g.FBT * 16 * 32; t += blockDim.x) gwacc[t] = 0.f;
    __syncthreads();
#pragma unroll
    for (int fb = 0; fb < FBX; ++fb)
      if (fb < g.FBT)
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
          if (ob < nob)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              atomicAdd(&gwacc[(fb * 16 + 4 * g4 + r) * 32 + ob * 16 + r16], gwa[fb][ob][r]);
    __syncthreads();
  }
  const int mc = blockIdx.x;
  for (int t = threadIdx.x; t < nkj * 32; t += blockDim.x) {
    const int q = t >> 5, col = t & 31;
    const int o = og * 32 + col;
    if (o < g.Opad) ga_slab[(((size_t)mc * g.T + i) * nkj + q) * g.Opad + o] = qacc[t];
  }
  if (INIT) return;
  for (int t = threadIdx.x; t < g.FBT * 16 * 32; t += blockDim.x) {
    const int fl = t >> 5, col = t & 31;
    const int o = og * 32 + col;
    if (o < g.Opad) gw_slab[(((size_t)mc * g.T + i) * (g.FBT * 16) + fl) * g.Opad + o] = gwacc[t];
  }
}

// ---------------------------------------------------------------------------------------
// coalesced, thread-parallel slab reductions: 64 consecutive outputs x 4 chunk lanes / block
// ---------------------------------------------------------------------------------------
__device__ inline float reduce_chunks(const float* __restrict__ slab, size_t chunk_stride, int nchunks,
                                      size_t idx, float* red) {
  const int sub = threadIdx.x >> 6;  // 0..3
  float s = 0.f;
  for (int c = sub; c < nchunks; c += 4) s += slab[(size_t)c * chunk_stride + idx];
  red[threadIdx.x] = s;
  __syncthreads();
  float v = 0.f;
  if (sub == 0) v = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192];
  return v;
}

__global__ __launch_bounds__(256) void reduce_gw_v3_kernel(Geo g, int nchunks, const float* __restrict__ gw_slab,
                                                           const float* __restrict__ sa_p,
                                                           float* __restrict__ grad_w) {
  __shared__ float red[256];
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

__global__ __launch_bounds__(256) void reduce_galpha_v3_kernel(Geo g, int nchunks, const float* __restrict__ ga_slab,
                                                               Params pp, float cgrad, int init,
                                                               const float* __restrict__ sw_p,
                                                               const float* __restrict__ sa_p, float count,
                                                               float sqrt_qp, float* __restrict__ out) {
  __shared__ float red[256];
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

}  // namespace cimq

// cimq_part_dense.hip -- the CiM conv as a dense GEMM: 1x1 kernels on 1x1 images (BASELINE
// cfg5, "QuantLinear 1024->1024 w4a4, 128-row tiles, batch 4096": Conv2dLSQCiM(k=1) on [B, C, 1, 1],
// SURVEY section 0).  With P = 1 the activations are a [B][C] matrix and the CiM tile of lsq.py:166-185
// is a contiguous run of xbar channels, so every step is a plain tiled GEMM:
//
//   forward  ps[m, i, k, j, o] = sum_{c in tile i} x_j[m, c] * w_k[o, c]      (v_mfma_i32_16x16x64_i8)
//            out[m, o] = sum_{i,k,j} ADC(ps) * mask                           (lsq.py:195-233)
//   grad_x   gx[m, c]  = sw/nba * sum_{k,o} What_k[c, o] * g[m, o] * E_ik[m, o]   (c in tile i)
//   grad_w   gw[c, o]  = sa/nbw * sum_j sum_m xhat_j[m, c] * g[m, o] * D_ij[m, o]
//            (both v_mfma_f32_16x16x32_bf16, the fp32 operand split hi/mid/lo: lsq.py:336-386)
//
// The forward leaves per (tile i, row m, channel o) a uint2 of three 16-bit planes -- STE pass,
// ADC code != 0, code < 0, bit k*nba + j -- instead of the fp16 partial sums (lsq.py:169-192);
// the backward kernels decode E / D / the ADC code from them.  grad_w and grad_alpha leave
// per-chunk slabs in the layout the module epilogue reduces (module_bwd_tail_kernel).
// Own translation unit of libcimq.so.
#define CIMQ_TU_DENSE
#include "cimq_host.h"

namespace cimq {

// pass-bit masks of a 16-bit plane: all j of weight slice k / all k of activation slice j
__device__ inline uint32_t dmask_k(int k, int nba) { return ((1u << nba) - 1u) << (k * nba); }
__device__ inline uint32_t dmask_j(int j, int nbw, int nba) {
  uint32_t m = 0;
  for (int k = 0; k < nbw; ++k) m |= 1u << (k * nba + j);
  return m;
}

// ---------------------------------------------------------------------------------------------
// forward: block = 64 rows x 64 channels, wave w = rows 16w..16w+15 x four 16-channel blocks
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA, int KS>
__global__ __launch_bounds__(256) void dense_fwd_kernel(Geo g, const uint8_t* __restrict__ xcf,
                                                        const v4i* __restrict__ wfrag, Params pp,
                                                        const float* __restrict__ sw_p, const float* __restrict__ sa_p,
                                                        float* __restrict__ out, uint2* __restrict__ st) {
  constexpr int NKJ = NBW * NBA;
  __shared__ int4 prm[NKJ * 64];  // this tile's ADC / STE thresholds, [j][k][64 channels]
  __shared__ float cfl[NKJ * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * 64, og = blockIdx.y;
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = pp.flags[0] != 0;
  const int mrow = m0 + wave * 16 + r16;  // this lane's A row
  float acc[4][4];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[ob][r] = 0.f;
  for (int i = 0; i < g.T; ++i) {
    __syncthreads();
    for (int t = threadIdx.x; t < NKJ * 64; t += 256) {
      const int col = t & 63, jk = t >> 6, j = jk / NBW, k = jk - j * NBW;
      const int pi = pidx(g, i, j, k, og * 64 + col);
      prm[t] = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
      cfl[t] = pp.coef[pi];
    }
    __syncthreads();
    // A operands: slice j of the 16 channels c0 .. c0+15 of row mrow, c0 = i*xbar + 64ks + 16 g4
    // (4-byte slice words, byte j = slice j: a 4x4 byte transpose per 4 channels)
    v4i xs[NBA][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = i * g.xbar + ks * 64 + 16 * g4;
      uint32_t w[16];
      if (c0 < g.C) {
        const uint4* src = reinterpret_cast<const uint4*>(xcf + ((size_t)mrow * g.C + c0) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 t4 = src[q];
          w[4 * q] = t4.x; w[4 * q + 1] = t4.y; w[4 * q + 2] = t4.z; w[4 * q + 3] = t4.w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) w[e] = 0u;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t P[4];
        tr4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], P);
#pragma unroll
        for (int j = 0; j < NBA; ++j) xs[j][ks][q] = (int)P[j];
      }
    }
    uint32_t sp[4][4], sz[4][4], sn[4][4];  // the three 16-bit state planes of (channel block, row)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[ob][r] = sz[ob][r] = sn[ob][r] = 0u;
    // slice pairs in descending kj = k*nba + j order: shifting each bit in from the bottom leaves it at bit kj
#pragma unroll
    for (int k = NBW - 1; k >= 0; --k) {
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) {
        v4i wk[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wk[ks] = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * 4 + ob) * 64 + lane];
        v4i ps[NBA];
#pragma unroll
        for (int j = 0; j < NBA; ++j) {
          ps[j] = v4i{0, 0, 0, 0};
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) ps[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][ks], wk[ks], ps[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = NBA - 1; j >= 0; --j) {
          const int pcol = (j * NBW + k) * 64 + ob * 16 + r16;
          const int4 pv = prm[pcol];
          const float cf = cfl[pcol];
          if (!literal) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint64_t mhi = __builtin_amdgcn_ballot_w64(ps[j][r] >= pv.x);
              const uint64_t mlo = __builtin_amdgcn_ballot_w64(ps[j][r] <= pv.y);
              const uint64_t mps = __builtin_amdgcn_ballot_w64((unsigned)(ps[j][r] - pv.z) <= (unsigned)pv.w);
              acc[ob][r] += adc3(cf, mhi, mlo);
              sp[ob][r] = shin(sp[ob][r], mps);
              sz[ob][r] = shin(sz[ob][r], mhi | mlo);
              sn[ob][r] = shin(sn[ob][r], mlo);
            }
          } else {
            // degenerate alpha / scales: the literal ADC per partial sum (as cim_fwd_v3_kernel)
            const int o = og * 64 + ob * 16 + r16;
            const float al = pp.alpha[pidx(g, i, j, k, o)];
            const float mk = pp.ckj[k * NBA + j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              acc[ob][r] += adc_literal_sum(ps[j], g.mode, sw, sa, al, g.qn, g.qp, mk, r);
              const bool pass = ste_literal(ps[j][r], g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f;
              const float code = code_literal(ps[j][r], g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo);
              sp[ob][r] = (sp[ob][r] << 1) | (pass ? 1u : 0u);
              sz[ob][r] = (sz[ob][r] << 1) | (code != 0.f ? 1u : 0u);
              sn[ob][r] = (sn[ob][r] << 1) | (code < 0.f ? 1u : 0u);
            }
          }
        }
      }
    }
    // state of rows m0 + 16w + 4g4 + r (MFMA output rows), channel og*64 + 16ob + r16
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      const int o = og * 64 + ob * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t m = (size_t)m0 + wave * 16 + 4 * g4 + r;
        st[((size_t)i * g.M + m) * g.O + o] = make_uint2((sp[ob][r] & 0xFFFFu) | (sz[ob][r] << 16), sn[ob][r] & 0xFFFFu);
      }
    }
  }
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o = og * 64 + ob * 16 + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r) out[((size_t)m0 + wave * 16 + 4 * g4 + r) * g.O + o] = acc[ob][r];
  }
}

// ---------------------------------------------------------------------------------------------
// grad_x: block = 128 rows x one crossbar tile's channels (FBT blocks of 16); wave w = rows
// 32w..32w+31 (two MFMA row blocks).  A = G_i (rows m, built from the state planes and g in
// registers), B = the int8 ctx weight slices as bf16 (wgx_item: columns c, kappa = (k, o) order).
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
__global__ __launch_bounds__(256) void dense_gx_kernel(Geo g, const uint2* __restrict__ st, const v4i* __restrict__ wgx,
                                                       Params pp, const float* __restrict__ sw_p,
                                                       const float* __restrict__ gout, float* __restrict__ gx) {
  constexpr int NKJ = NBW * NBA;
  constexpr int FBX = 8;  // dense plan: xbar <= 128
  __shared__ float cel[NKJ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * 128 + wave * 32, i = blockIdx.y;
  for (int t = threadIdx.x; t < NKJ; t += 256) cel[t] = pp.ckj[NKJ + t];
  __syncthreads();
  bool std_mask;  // cE_kj = 2^(bsw*k) for every j: E_k = 2^(bsw*k) * popcount(pass bits of slice k)
  {
    const int kl = lane < NKJ ? lane / NBA : 0;
    std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cel[lane < NKJ ? lane : 0] != ldexpf(1.f, g.bsw * kl)) == 0ull;
  }
  v4f acc[2][FBX];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int fb = 0; fb < FBX; ++fb) acc[h][fb] = v4f{0.f, 0.f, 0.f, 0.f};
  const v4i* wt = wgx + (size_t)i * g.FBT * g.NKS * 64 + lane;
  for (int s = 0; s < g.NKS; ++s) {
    v8bf Gh[2], Gm[2], Gl[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // row block h: rows m0 + 16h + r16
      const size_t m = (size_t)m0 + 16 * h + r16;
      float Gv[8];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {  // kappa block kb = 2s + hh: (k, o-block), 4 channels o0 .. o0+3
        const int kb = 2 * s + hh;
        if (kb < g.NBLK) {
          const int k = kb / g.OB16, o0 = (kb - k * g.OB16) * 16 + 4 * g4;
          const uint4* sp4 = reinterpret_cast<const uint4*>(st + ((size_t)i * g.M + m) * g.O + o0);
          const uint4 a = sp4[0], b = sp4[1];
          const float4 gg = *reinterpret_cast<const float4*>(gout + m * g.O + o0);
          const uint32_t pw[4] = {a.x, a.z, b.x, b.z};  // pass planes (low 16 bits)
          const float gv[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float E;
            if (std_mask) {
              E = ldexpf((float)__popc(pw[e] & dmask_k(k, NBA)), g.bsw * k);
            } else {
              E = 0.f;
#pragma unroll
              for (int j = 0; j < NBA; ++j) E += ((pw[e] >> (k * NBA + j)) & 1u) ? cel[k * NBA + j] : 0.f;
            }
            Gv[4 * hh + e] = gv[e] * E;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) Gv[4 * hh + e] = 0.f;
        }
      }
      split3x8(Gv, Gh[h], Gm[h], Gl[h]);
    }
#pragma unroll
    for (int fb = 0; fb < FBX; ++fb) {
      if (fb >= g.FBT) break;
      const v8bf bw = as_v8bf(wt[((size_t)fb * g.NKS + s) * 64]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[h][fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Gh[h], bw, acc[h][fb], 0, 0, 0);
        acc[h][fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Gm[h], bw, acc[h][fb], 0, 0, 0);
        acc[h][fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Gl[h], bw, acc[h][fb], 0, 0, 0);
      }
    }
  }
  const float scale = *sw_p / (float)NBA;
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) {
    if (fb >= g.FBT) break;
    const int c = i * g.xbar + fb * 16 + r16;
    if (c < g.C && fb * 16 < g.xbar) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) gx[((size_t)m0 + 16 * h + 4 * g4 + r) * g.C + c] = acc[h][fb][r] * scale;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// grad_w + grad_alpha partials: block = (row chunk, tile i, 64 channels o); wave w = channel block
// 4 blockIdx.z + w.  K-step = 32 rows: A = xhat_j[m, c] of the tile's channels (built once per
// step by the whole block into LDS), B = g * D_j (registers).  grad_alpha: sum of code * g.
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
__global__ __launch_bounds__(256) void dense_gw_kernel(Geo g, int rows_per_chunk, const uint2* __restrict__ st,
                                                       const uint8_t* __restrict__ xcb, Params pp,
                                                       const float* __restrict__ gout, float* __restrict__ gw_slab,
                                                       float* __restrict__ ga_slab) {
  constexpr int NKJ = NBW * NBA;
  constexpr int FBX = 8;
  __shared__ v4i As[FBX * NBA * 64];  // [fb][j][64 lanes]: 8 bf16 of rows c, contraction 8 rows m
  __shared__ float cdl[NKJ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int chunk = blockIdx.x, i = blockIdx.y;
  const int o = (blockIdx.z * 4 + wave) * 16 + r16;  // this lane's B column
  for (int t = threadIdx.x; t < NKJ; t += 256) cdl[t] = pp.ckj[2 * NKJ + t];
  __syncthreads();
  bool std_mask;  // cD_kj = 2^(bsa*j) for every k: D_j = 2^(bsa*j) * popcount(pass bits of slice j)
  {
    const int kl = lane < NKJ ? lane / NBA : 0, jl = lane < NKJ ? lane - kl * NBA : 0;
    std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cdl[lane < NKJ ? lane : 0] != ldexpf(1.f, g.bsa * jl)) == 0ull;
  }
  v4f acc[FBX];
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) acc[fb] = v4f{0.f, 0.f, 0.f, 0.f};
  float qa[NKJ];
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) qa[kj] = 0.f;
  const int mlo = chunk * rows_per_chunk, mhi = min(g.M, mlo + rows_per_chunk);
  for (int ms = mlo; ms < mhi; ms += 32) {
    __syncthreads();
    // A fragments of the step: item (fb, l) = rows c = i*xbar + 16fb + (l&15), rows m = ms + 8(l>>4) + e
    for (int it = threadIdx.x; it < g.FBT * 64; it += 256) {
      const int fb = it >> 6, l = it & 63;
      const int c = i * g.xbar + fb * 16 + (l & 15);
      uint32_t w[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int m = ms + 8 * (l >> 4) + e;
        w[e] = (c < g.C && fb * 16 < g.xbar && m < mhi) ? reinterpret_cast<const uint32_t*>(xcb)[(size_t)m * g.C + c] : 0u;
      }
#pragma unroll
      for (int j = 0; j < NBA; ++j) {
        uint32_t pk[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const float f0 = (float)(int8_t)((w[2 * e2] >> (8 * j)) & 0xFFu);
          const float f1 = (float)(int8_t)((w[2 * e2 + 1] >> (8 * j)) & 0xFFu);
          pk[e2] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);  // exact bf16
        }
        As[(fb * NBA + j) * 64 + l] = v4i{(int)pk[0], (int)pk[1], (int)pk[2], (int)pk[3]};
      }
    }
    __syncthreads();
    // B: rows m = ms + 8 g4 + e of channel o
    float gv[8];
    uint2 sv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = ms + 8 * g4 + e;
      const bool ok = m < mhi;
      gv[e] = ok ? gout[(size_t)m * g.O + o] : 0.f;
      sv[e] = ok ? st[((size_t)i * g.M + m) * g.O + o] : make_uint2(0u, 0u);
    }
    // grad_alpha partials (lsq.py:321-333): code * g, code from the nz / neg planes
#pragma unroll
    for (int kj = 0; kj < NKJ; ++kj) {
      float q = qa[kj];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t nz = (sv[e].x >> (16 + kj)) & 1u, ng = (sv[e].y >> kj) & 1u;
        const float code = nz ? (ng ? -1.f : 1.f) : 0.f;
        q = __builtin_fmaf(code, gv[e], q);
      }
      qa[kj] = q;
    }
#pragma unroll
    for (int j = 0; j < NBA; ++j) {
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float D;
        if (std_mask) {
          D = ldexpf((float)__popc(sv[e].x & dmask_j(j, NBW, NBA)), g.bsa * j);
        } else {
          D = 0.f;
#pragma unroll
          for (int k = 0; k < NBW; ++k) D += ((sv[e].x >> (k * NBA + j)) & 1u) ? cdl[k * NBA + j] : 0.f;
        }
        d[e] = gv[e] * D;
      }
      v8bf bh, bm, bl;
      split3x8(d, bh, bm, bl);
#pragma unroll
      for (int fb = 0; fb < FBX; ++fb) {
        if (fb >= g.FBT) break;
        const v8bf a = as_v8bf(As[(fb * NBA + j) * 64 + lane]);
        acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh, acc[fb], 0, 0, 0);
        acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm, acc[fb], 0, 0, 0);
        acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl, acc[fb], 0, 0, 0);
      }
    }
  }
  // acc[fb][r]: row c = 16fb + 4g4 + r of the tile, column o
  const int FR = g.FBT * 16;
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) {
    if (fb >= g.FBT) break;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      gw_slab[(((size_t)chunk * g.T + i) * FR + fb * 16 + 4 * g4 + r) * g.Opad + o] = acc[fb][r];
  }
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) {
    float q = qa[kj];
    q += __shfl_xor(q, 16);
    q += __shfl_xor(q, 32);
    if (g4 == 0) ga_slab[(((size_t)chunk * g.T + i) * NKJ + kj) * g.Opad + o] = q;
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
int launch_dense_fwd_n(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  auto kern = g.KS == 1 ? dense_fwd_kernel<NBW, NBA, 1> : dense_fwd_kernel<NBW, NBA, 2>;
  const int slot = prof_begin(KID_FWD, g, s);
  hipLaunchKernelGGL(kern, dim3(g.M / 64, g.O / 64), dim3(256), 0, s, g, ctx + L.xcode,
                     reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wfrag), params_of(g, ctx), sw, sa, out,
                     reinterpret_cast<uint2*>(ctx + L.st));
  prof_end(slot, s);
  return check_hip("dense_fwd");
}

template <int NBW, int NBA>
int launch_dense_bwd_n(const Geo& g, const uint8_t* ctx, const float* sw, const float* gout, float* gx, uint8_t* ws,
                       hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  const uint2* st = reinterpret_cast<const uint2*>(ctx + L.st);
  {
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL((dense_gx_kernel<NBW, NBA>), dim3(g.M / 128, g.T), dim3(256), 0, s, g, st,
                       reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wgx), pp, sw, gout, gx);
    prof_end(slot, s);
    CIMQ_TRY(check_hip("dense_gx"));
  }
  {
    const int slot = prof_begin(KID_BWD_GW, g, s);
    hipLaunchKernelGGL((dense_gw_kernel<NBW, NBA>), dim3(W.nchunks_bwd, g.T, g.O / 64), dim3(256), 0, s, g,
                       dense_rows_per_chunk(g), st, ctx + L.xhat, pp, gout, reinterpret_cast<float*>(ws + W.gw_slab),
                       reinterpret_cast<float*>(ws + W.ga_slab));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("dense_gw"));
  }
  return CIMQ_OK;
}

#define CIMQ_DENSE_SEL(F, ...)                                                     \
  switch (g.nbw * 8 + g.nba) {                                                     \
    case 1 * 8 + 1: return F<1, 1>(__VA_ARGS__);                                   \
    case 2 * 8 + 2: return F<2, 2>(__VA_ARGS__);                                   \
    case 3 * 8 + 3: return F<3, 3>(__VA_ARGS__);                                   \
    case 4 * 8 + 4: return F<4, 4>(__VA_ARGS__);                                   \
    default: return fail(CIMQ_EUNSUPPORTED, "dense path: no instance for nbw=%d nba=%d", g.nbw, g.nba); \
  }

int launch_dense_fwd(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, hipStream_t s) {
  CIMQ_DENSE_SEL(launch_dense_fwd_n, g, ctx, sw, sa, out, s)
}

int launch_dense_bwd(const Geo& g, const uint8_t* ctx, const float* sw, const float* gout, float* gx, uint8_t* ws,
                     hipStream_t s) {
  CIMQ_DENSE_SEL(launch_dense_bwd_n, g, ctx, sw, gout, gx, ws, s)
}

}  // namespace cimq

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
// The forward leaves per (tile i, row m, channel o) a uint2 instead of the fp16 partial sums
// (lsq.py:169-192): .x the ADC codes as 2-bit two's-complement fields (bits 2kj, 2kj+1 of slice
// pair kj = k*nba + j: 00 = 0, 01 = +1, 11 = -1), .y the STE pass bits (bit kj); the backward
// kernels decode E / D from the pass bits and grad_alpha's code * g from the fields.  grad_w and grad_alpha leave
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

// One partial sum's ternary ADC and state bits in one block of instructions: the three compare
// masks live in SGPRs only between their compare and their use (left to the compiler, the
// compares of all 16 partial sums of a slice-pair group are hoisted and their masks spill).
//   acc += hi ? cf : (lo ? -cf : 0);  pass / hi / lo shifted in at bit 0 of sp / shi / slo
// The subtraction stays compiler code: it is the first read of the MFMA result, so the hazard
// recognizer pads it (it does not look into inline asm); the asm reads ps only after it.
__device__ inline void adc_ps(int ps, int4 pv, float cf, float& acc, uint32_t& sp, uint32_t& shi, uint32_t& slo) {
  const int t = (int)((unsigned)ps - (unsigned)pv.z);
  uint64_t mh, ml, mp, co;
  float a;
  asm("v_cmp_ge_i32_e64 %[mh], %[ps], %[thi]\n\t"
      "v_cmp_le_i32_e64 %[ml], %[ps], %[tlo]\n\t"
      "v_cmp_le_u32_e64 %[mp], %[t], %[span]\n\t"
      "v_cndmask_b32_e64 %[a], 0, %[cf], %[mh]\n\t"
      "v_cndmask_b32_e64 %[a], %[a], -%[cf], %[ml]\n\t"
      "v_add_f32_e32 %[acc], %[acc], %[a]\n\t"
      "v_addc_co_u32_e64 %[sp], %[co], %[sp], %[sp], %[mp]\n\t"
      "v_addc_co_u32_e64 %[shi], %[co], %[shi], %[shi], %[mh]\n\t"
      "v_addc_co_u32_e64 %[slo], %[co], %[slo], %[slo], %[ml]"
      : [mh] "=&s"(mh), [ml] "=&s"(ml), [mp] "=&s"(mp), [co] "=&s"(co), [a] "=&v"(a),
        [acc] "+v"(acc), [sp] "+v"(sp), [shi] "+v"(shi), [slo] "+v"(slo)
      : [ps] "v"(ps), [t] "v"(t), [thi] "v"(pv.x), [tlo] "v"(pv.y), [span] "v"(pv.w), [cf] "v"(cf));
}

// bit b of a 16-bit plane -> bit 2b
__device__ inline uint32_t spread16(uint32_t x) {
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  return (x | (x << 1)) & 0x55555555u;
}

// ---------------------------------------------------------------------------------------------
// forward: block = 64 rows x 64 channels, wave w = rows 16w..16w+15 x four 16-channel blocks (in turn)
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA, int KS, bool LIT>
__device__ inline void dense_fwd_body(const Geo& g, const uint8_t* __restrict__ xcf, const v4i* __restrict__ wfrag,
                                      const Params& pp, float sw, float sa, float* __restrict__ out,
                                      uint2* __restrict__ st, int4* prm, float* cfl, float4* accs, int m0,
                                      int og) {
  constexpr int NKJ = NBW * NBA;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int mrow = m0 + wave * 16 + r16;  // this lane's A row
  // out accumulators of the four channel blocks in LDS ([wave][ob][lane]); one block's in registers
  float4* acc_l = accs + wave * 4 * 64 + lane;
  for (int i = 0; i < g.T; ++i) {
#ifdef CIMQ_EXP_DENSE_NOPRM
    if (!LIT && i == 0) {
#else
    if (!LIT) {
#endif
      __syncthreads();
      for (int t = threadIdx.x; t < NKJ * 64; t += 256) {
        const int col = t & 63, jk = t >> 6, j = jk / NBW, k = jk - j * NBW;
        const int pi = pidx(g, i, j, k, og * 64 + col);
        prm[t] = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
        cfl[t] = pp.coef[pi];
      }
      __syncthreads();
    }
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
    // one 16-channel block at a time: its three 16-bit state planes live only across the slice pairs
#pragma unroll 1
    for (int ob = 0; ob < 4; ++ob) {
      float acc[4];
      if (i == 0) {
        acc[0] = acc[1] = acc[2] = acc[3] = 0.f;
      } else {
        const float4 a4 = acc_l[ob * 64];
        acc[0] = a4.x; acc[1] = a4.y; acc[2] = a4.z; acc[3] = a4.w;
      }
      uint32_t sp[4], sz[4], sn[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[r] = sz[r] = sn[r] = 0u;
      // slice pairs in descending kj = k*nba + j order: shifting each bit in from the bottom leaves it at bit kj
#pragma unroll
      for (int k = NBW - 1; k >= 0; --k) {
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
          if (!LIT) {
            const int pcol = (j * NBW + k) * 64 + ob * 16 + r16;
            const int4 pv = prm[pcol];
            const float cf = cfl[pcol];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#ifdef CIMQ_EXP_DENSE_NOADC  // attribution builds only (tools/kernel_experiment.py): wrong results
              acc[r] += (float)ps[j][r] * cf + (float)pv.x;
#else
              adc_ps(ps[j][r], pv, cf, acc[r], sp[r], sz[r], sn[r]);
#endif
          } else {
            // degenerate alpha / scales: the literal ADC per partial sum (as cim_fwd_v3_kernel)
            const int o = og * 64 + ob * 16 + r16;
            const float al = pp.alpha[pidx(g, i, j, k, o)];
            const float mk = pp.ckj[k * NBA + j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              acc[r] += adc_literal_sum(ps[j], g.mode, sw, sa, al, g.qn, g.qp, mk, r);
              const bool pass = ste_literal(ps[j][r], g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f;
              const float code = code_literal(ps[j][r], g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo);
              sp[r] = (sp[r] << 1) | (pass ? 1u : 0u);
              sz[r] = (sz[r] << 1) | (code > 0.f ? 1u : 0u);
              sn[r] = (sn[r] << 1) | (code < 0.f ? 1u : 0u);
            }
          }
        }
      }
      // state of rows m0 + 16w + 4g4 + r (MFMA output rows), channel og*64 + 16ob + r16
      const int o = og * 64 + ob * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t m = (size_t)m0 + wave * 16 + 4 * g4 + r;
        // code fields: lo -> 11, hi -> 01 (lo wins, as the ADC's second select)
        const uint32_t code = spread16(sz[r] | sn[r]) | (spread16(sn[r]) << 1);
#ifndef CIMQ_EXP_DENSE_NOSTORE
        st[((size_t)i * g.M + m) * g.O + o] = make_uint2(code, sp[r] & 0xFFFFu);
#else
        if (code == 0x12345u) st[m] = make_uint2(code, sp[r]);
#endif
      }
      if (i + 1 < g.T) {
        acc_l[ob * 64] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) out[((size_t)m0 + wave * 16 + 4 * g4 + r) * g.O + o] = acc[r];
      }
    }
  }
}

// The threshold path: one 64 x 64 tile per block.  Exits at once when the prologue set the
// literal-ADC flag (dense_fwd_lit_kernel then does the work).
template <int NBW, int NBA, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void dense_fwd_kernel(
    Geo g, const uint8_t* __restrict__ xcf, const v4i* __restrict__ wfrag, Params pp, const float* __restrict__ sw_p,
    const float* __restrict__ sa_p, float* __restrict__ out, uint2* __restrict__ st) {
  __shared__ int4 prm[NBW * NBA * 64];  // this tile's ADC / STE thresholds, [j][k][64 channels]
  __shared__ float cfl[NBW * NBA * 64];
  __shared__ float4 accs[4 * 4 * 64];
  if (__builtin_amdgcn_readfirstlane(pp.flags[0]) != 0) return;
  dense_fwd_body<NBW, NBA, KS, false>(g, xcf, wfrag, pp, 0.f, 0.f, out, st, prm, cfl, accs, blockIdx.x * 64,
                                      blockIdx.y);
}

// The threshold path on 128 x 64 tiles (512 threads, wave w = rows 16w..16w+15): the weight fragments
// and the ADC / STE thresholds of a crossbar tile are staged ONCE per block into LDS and read by its eight
// waves (the 64-row form above re-read the tile's weight fragments from L2 in every wave: 1 GB per cfg5
// forward).  The weight fragments go in two halves (output blocks 0-1, then 2-3) so a block stays under
// 80 KB of LDS: two blocks per CU.  Per partial sum the ADC / state bits are adc_ps, in the same order:
// out and the state words are bit-identical to dense_fwd_kernel's.
template <int NBW, int NBA, int KS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void dense_fwd8_kernel(
    Geo g, const uint8_t* __restrict__ xcf, const v4i* __restrict__ wfrag, Params pp, float* __restrict__ out,
    uint2* __restrict__ st) {
  constexpr int NKJ = NBW * NBA;
  constexpr int NWH = KS * NBW * 2 * 64;  // v4i of one half's weight fragments
  __shared__ int4 prm[NKJ * 64];          // [j][k][64 channels]: thi, tlo, mlo, span
  __shared__ float cfl[NKJ * 64];
  __shared__ v4i wkl[NWH];                // [ks][k][2 output blocks][64 lanes]
  __shared__ float4 accs[8 * 4 * 64];     // [wave][output block][lane]: out across the tiles
  if (__builtin_amdgcn_readfirstlane(pp.flags[0]) != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * 128, og = blockIdx.y;
  const int mrow = m0 + wave * 16 + r16;  // this lane's A row
  float4* acc_l = accs + wave * 4 * 64 + lane;
  auto stage_w = [&](int i, int half) {
    for (int t = threadIdx.x; t < NWH; t += 512) {
      const int l = t & 63, obh = (t >> 6) & 1, kk = t >> 7, k = kk % NBW, ks = kk / NBW;
      wkl[t] = wfrag[((size_t)(i * KS + ks) * g.NBLK + k * g.OB16 + og * 4 + half * 2 + obh) * 64 + l];
    }
  };
  for (int i = 0; i < g.T; ++i) {
    // A operands of this wave's rows (issued first: they do not depend on the barrier)
    uint32_t w[KS][16];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = i * g.xbar + ks * 64 + 16 * g4;
#ifdef CIMQ_EXP_DENSE_NOX
      if (true) {
#pragma unroll
        for (int e = 0; e < 16; ++e) w[ks][e] = (uint32_t)(mrow * 131 + c0 * 7 + e) & 0x01010101u;
      } else if (c0 < g.C) {
#else
      if (c0 < g.C) {
#endif
        const uint4* src = reinterpret_cast<const uint4*>(xcf + ((size_t)mrow * g.C + c0) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 t4 = src[q];
          w[ks][4 * q] = t4.x; w[ks][4 * q + 1] = t4.y; w[ks][4 * q + 2] = t4.z; w[ks][4 * q + 3] = t4.w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) w[ks][e] = 0u;
      }
    }
    __syncthreads();  // the previous tile's readers of prm / wkl are done
#ifdef CIMQ_EXP_DENSE_NOSTAGE
    if (i == 0)
#endif
    for (int t = threadIdx.x; t < NKJ * 64; t += 512) {
      const int col = t & 63, jk = t >> 6, j = jk / NBW, k = jk - j * NBW;
      const int pi = pidx(g, i, j, k, og * 64 + col);
      prm[t] = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
      cfl[t] = pp.coef[pi];
    }
#ifdef CIMQ_EXP_DENSE_NOSTAGE
    if (i == 0)
#endif
    stage_w(i, 0);
    v4i xs[NBA][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t P[4];
        tr4(w[ks][4 * q], w[ks][4 * q + 1], w[ks][4 * q + 2], w[ks][4 * q + 3], P);
#pragma unroll
        for (int j = 0; j < NBA; ++j) xs[j][ks][q] = (int)P[j];
      }
    __syncthreads();
#pragma unroll 1
    for (int ob = 0; ob < 4; ++ob) {
      if (ob == 2) {
        __syncthreads();  // half 0 read by every wave
#ifndef CIMQ_EXP_DENSE_NOSTAGE
        stage_w(i, 1);
#endif
        __syncthreads();
      }
      float acc[4];
      if (i == 0) {
        acc[0] = acc[1] = acc[2] = acc[3] = 0.f;
      } else {
        const float4 a4 = acc_l[ob * 64];
        acc[0] = a4.x; acc[1] = a4.y; acc[2] = a4.z; acc[3] = a4.w;
      }
      uint32_t sp[4], sz[4], sn[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[r] = sz[r] = sn[r] = 0u;
#pragma unroll
      for (int k = NBW - 1; k >= 0; --k) {
        v4i wk[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wk[ks] = wkl[((ks * NBW + k) * 2 + (ob & 1)) * 64 + lane];
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
#pragma unroll
          for (int r = 0; r < 4; ++r)
#ifdef CIMQ_EXP_DENSE_NOADC
            acc[r] += (float)ps[j][r] * cf + (float)pv.x;
#else
            adc_ps(ps[j][r], pv, cf, acc[r], sp[r], sz[r], sn[r]);
#endif
        }
      }
      const int o = og * 64 + ob * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t m = (size_t)m0 + wave * 16 + 4 * g4 + r;
        const uint32_t code = spread16(sz[r] | sn[r]) | (spread16(sn[r]) << 1);
#ifndef CIMQ_EXP_DENSE_NOSTORE
        st[((size_t)i * g.M + m) * g.O + o] = make_uint2(code, sp[r] & 0xFFFFu);
#else
        if (code == 0x12345u) st[m] = make_uint2(code, sp[r]);
#endif
      }
      if (i + 1 < g.T) {
        acc_l[ob * 64] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) out[((size_t)m0 + wave * 16 + 4 * g4 + r) * g.O + o] = acc[r];
      }
    }
  }
}

// Degenerate alpha_q / scales (flag set): the literal ADC per partial sum, a few blocks looping
// over the tiles (its out-of-line calls kept out of the threshold kernel's register budget).
template <int NBW, int NBA, int KS>
__global__ __launch_bounds__(256) void dense_fwd_lit_kernel(Geo g, const uint8_t* __restrict__ xcf,
                                                            const v4i* __restrict__ wfrag, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p, float* __restrict__ out,
                                                            uint2* __restrict__ st) {
  __shared__ float4 accs[4 * 4 * 64];
  if (__builtin_amdgcn_readfirstlane(pp.flags[0]) == 0) return;
  const float sw = *sw_p, sa = *sa_p;
  const int nm = g.M / 64, ntile = nm * (g.O / 64);
  for (int t = blockIdx.x; t < ntile; t += gridDim.x)
    dense_fwd_body<NBW, NBA, KS, true>(g, xcf, wfrag, pp, sw, sa, out, st, nullptr, nullptr, accs, (t % nm) * 64, t / nm);
}

// ---------------------------------------------------------------------------------------------
// grad_x: block = 128 rows x one crossbar tile (<= 8 blocks of 16 channels), 16 waves in two roles.
// Per K-step of 32 kappa = (k, o): the 8 builder waves (8..15) write the A operand
// G_i[m, kappa] = g[m, o] * E_ik[m, o] of the NEXT step (hi / mid / lo bf16) into LDS -- builder b
// the rows 16b..16b+15, each lane one MFMA fragment -- while the 8 MFMA waves (0..7) multiply this
// step's G, rows 32(w&3)..+31, by the channel blocks 4(w>>2)..+3 (B: the int8 ctx weight slices as
// bf16, wgx_item layout, read from global one step ahead).  One barrier per step; the two roles
// share each SIMD (4 waves), so the split products and the MFMAs overlap.  K-steps run o-pair
// major, slice k minor: a builder lane loads each of its state words and g values once, one o-pair
// ahead.
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
__global__ __launch_bounds__(1024) void dense_gx_kernel(Geo g, const uint2* __restrict__ st, const v4i* __restrict__ wgx,
                                                        Params pp, const float* __restrict__ sw_p,
                                                        const float* __restrict__ gout, float* __restrict__ gx,
                                                        const float* __restrict__ x, const float* __restrict__ sa_p,
                                                        float* __restrict__ gsa_part) {
  constexpr int NKJ = NBW * NBA;
  __shared__ v4i Gs[2 * 3 * 8 * 64];  // [buffer][hi/mid/lo][16-row block][lane]
  __shared__ float cel[NKJ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.x * 128, i = blockIdx.y;
  const bool builder = wave >= 8;
  for (int t = threadIdx.x; t < NKJ; t += 1024) cel[t] = pp.ckj[NKJ + t];
  __syncthreads();
  const int hp = g.OB16 / 2;  // o-pairs (O % 64 == 0)
  const int nsteps = NBW * hp;
  if (builder) {
    bool std_mask;  // cE_kj = 2^(bsw*k) for every j: E_k = 2^(bsw*k) * popcount(pass bits of slice k)
    {
      const int kl = lane < NKJ ? lane / NBA : 0;
      std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cel[lane < NKJ ? lane : 0] != ldexpf(1.f, g.bsw * kl)) == 0ull;
    }
    const int bw = wave - 8;
    // row m0 + 16 bw + r16, kappa channels 32p + 4g4 + e (e < 4) and 32p + 16 + 4g4 + e
    const size_t mb = (size_t)m0 + 16 * bw + r16;
    const uint2* strow = st + ((size_t)i * g.M + mb) * g.O + 4 * g4;
    const float* grow = gout + mb * g.O + 4 * g4;
    uint4 sa0, sa1, sb0, sb1, na0, na1, nb0, nb1;
    float4 ga, gb, nga, ngb;
    auto load_p = [&](int p, uint4& a0, uint4& a1, uint4& b0, uint4& b1, float4& fa, float4& fb) {
      const uint4* s4 = reinterpret_cast<const uint4*>(strow + 32 * p);
      a0 = s4[0]; a1 = s4[1]; b0 = s4[8]; b1 = s4[9];
      fa = *reinterpret_cast<const float4*>(grow + 32 * p);
      fb = *reinterpret_cast<const float4*>(grow + 32 * p + 16);
    };
    auto build = [&](int k, int buf) {
      const uint32_t pw[8] = {sa0.y, sa0.w, sa1.y, sa1.w, sb0.y, sb0.w, sb1.y, sb1.w};  // pass bits
      const float gv[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
      float Gv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float E;
        if (std_mask) {
          E = ldexpf((float)__popc(pw[e] & dmask_k(k, NBA)), g.bsw * k);
        } else {
          E = 0.f;
#pragma unroll
          for (int j = 0; j < NBA; ++j) E += ((pw[e] >> (k * NBA + j)) & 1u) ? cel[k * NBA + j] : 0.f;
        }
        Gv[e] = gv[e] * E;
      }
      v8bf h, md, lo;
      split3x8(Gv, h, md, lo);
      v4i* dst = Gs + (buf * 3 * 8 + bw) * 64 + lane;
      dst[0] = as_v4i(h);
      dst[8 * 64] = as_v4i(md);
      dst[16 * 64] = as_v4i(lo);
    };
    load_p(0, sa0, sa1, sb0, sb1, ga, gb);
    if (hp > 1) load_p(1, na0, na1, nb0, nb1, nga, ngb);
    build(0, 0);
    __syncthreads();
    for (int t = 0; t < nsteps; ++t) {
      const int tn = t + 1;
      if (tn < nsteps) {
        const int k = tn % NBW;
        if (k == 0) {  // next o-pair: its words arrived during the last NBW steps; fetch the one after
          sa0 = na0; sa1 = na1; sb0 = nb0; sb1 = nb1; ga = nga; gb = ngb;
          const int pn = tn / NBW + 1;
          if (pn < hp) load_p(pn, na0, na1, nb0, nb1, nga, ngb);
        }
        build(k, tn & 1);
      }
      __syncthreads();
    }
    return;
  }
  const int rg = wave & 3, chh = wave >> 2;
  auto step_s = [&](int t) { return (t % NBW) * hp + t / NBW; };
  const int nf = min(4, g.FBT - 4 * chh);  // this wave's channel blocks (0 when the tile has 4)
  const v4i* wt = wgx + ((size_t)i * g.FBT + 4 * chh) * g.NKS * 64 + lane;
  v4i bc[4], bn[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) bc[f] = f < nf ? wt[((size_t)f * g.NKS + step_s(0)) * 64] : v4i{0, 0, 0, 0};
  __syncthreads();
  v4f acc[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[h][f] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < nsteps; ++t) {
    const int tn = t + 1;
    if (tn < nsteps) {
      const int sn = step_s(tn);
#pragma unroll
      for (int f = 0; f < 4; ++f) bn[f] = f < nf ? wt[((size_t)f * g.NKS + sn) * 64] : v4i{0, 0, 0, 0};
    }
    if (nf > 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const v4i* src = Gs + ((t & 1) * 3 * 8 + 2 * rg + h) * 64 + lane;
        const v8bf ah = as_v8bf(src[0]), am = as_v8bf(src[8 * 64]), al = as_v8bf(src[16 * 64]);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const v8bf bwv = as_v8bf(bc[f]);
          acc[h][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bwv, acc[h][f], 0, 0, 0);
          acc[h][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bwv, acc[h][f], 0, 0, 0);
          acc[h][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bwv, acc[h][f], 0, 0, 0);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < 4; ++f) bc[f] = bn[f];
  }
  const float scale = *sw_p / (float)NBA;
  // with x: the LSQ activation quantiser's backward fused into the store (as lsq_act_bwd_kernel,
  // the same operations: autograd of round_pass(clamp(x / sa, 0, Qp)) * sa, lsq.py:549) and this
  // block's partial of d loss / d sa
  const float sa = x ? *sa_p : 1.f;
  float gsum = 0.f;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    if (f >= nf) break;
    const int c = i * g.xbar + (4 * chh + f) * 16 + r16;
    if (c < g.C) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const size_t e = ((size_t)m0 + 32 * rg + 16 * h + 4 * g4 + r) * g.C + c;
          const float gq = acc[h][f][r] * scale;
          if (x) {
            const float y1 = x[e] / sa;
            const float cl = clamp_nan(y1, 0.f, g.lsq_qp);
            const float rr = rintf(cl);
            const float rp = (rr - cl) + cl;
            const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
            const float gy = pass ? gq * sa : 0.f;
            gx[e] = gy / sa;
            gsum += gq * rp;
            gsum += -(gy * (y1 / sa));
          } else {
            gx[e] = gq;
          }
        }
    }
  }
  if (x) {  // one partial per MFMA wave (the builder waves have returned: no block barrier here)
    for (int o = 32; o > 0; o >>= 1) gsum += __shfl_xor(gsum, o);
    if (lane == 0) gsa_part[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + wave] = gsum;
  }
}

// ---------------------------------------------------------------------------------------------
// grad_w + grad_alpha partials: block = (row chunk, tile i, 128 channels o), 8 waves; wave w =
// channel block 8 blockIdx.z + w.  K-step = 32 rows: A = xhat_j[m, c] of the tile's channels,
// built by the whole block into LDS one step ahead (double buffer, its words loaded two steps
// ahead), B = g * D_j (registers).  grad_alpha: sum over the rows of code * g per slice pair.
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
__global__ __launch_bounds__(512) void dense_gw_kernel(Geo g, int rows_per_chunk, const uint2* __restrict__ st,
                                                       const uint8_t* __restrict__ xcb, Params pp,
                                                       const float* __restrict__ gout, float* __restrict__ gw_slab,
                                                       float* __restrict__ ga_slab) {
  constexpr int NKJ = NBW * NBA;
  constexpr int FBX = 8;
  __shared__ v4i As[2 * FBX * NBA * 64];  // [buffer][fb][j][64 lanes]: 8 bf16 of rows c, contraction 8 rows m
  __shared__ float cdl[NKJ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int chunk = blockIdx.x, i = blockIdx.y;
  const int ob = blockIdx.z * 8 + wave;
  const bool oact = ob * 16 < g.O;     // waves past the last channel block only build A
  const int o = min(ob * 16 + r16, g.O - 1);  // this lane's B column
  for (int t = threadIdx.x; t < NKJ; t += 512) cdl[t] = pp.ckj[2 * NKJ + t];
  __syncthreads();
  bool std_mask;  // cD_kj = 2^(bsa*j) for every k: D_j = 2^(bsa*j) * popcount(pass bits of slice j)
  {
    const int kl = lane < NKJ ? lane / NBA : 0, jl = lane < NKJ ? lane - kl * NBA : 0;
    std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cdl[lane < NKJ ? lane : 0] != ldexpf(1.f, g.bsa * jl)) == 0ull;
  }
  // A builder: item (fb, l) = thread, rows c = i*xbar + 16fb + (l&15), rows m = ms + 8(l>>4) + e
  const int ifb = threadIdx.x >> 6;
  const bool ibld = ifb < g.FBT;
  const int ic = i * g.xbar + ifb * 16 + r16;
  const bool icok = ibld && ic < g.C && ifb * 16 < g.xbar;
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(xcb) + (icok ? ic : 0);
  const int mlo = chunk * rows_per_chunk, mhi = min(g.M, mlo + rows_per_chunk);
  uint32_t aw[8];
  auto load_a = [&](int ms) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int m = ms + 8 * g4 + e;
      aw[e] = (icok && m < mhi) ? xw[(size_t)m * g.C] : 0u;
    }
  };
  auto build_a = [&](int buf) {
    if (!ibld) return;
#pragma unroll
    for (int j = 0; j < NBA; ++j) {
      uint32_t pk[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        const float f0 = (float)(int8_t)((aw[2 * e2] >> (8 * j)) & 0xFFu);
        const float f1 = (float)(int8_t)((aw[2 * e2 + 1] >> (8 * j)) & 0xFFu);
        pk[e2] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);  // exact bf16
      }
      As[((buf * FBX + ifb) * NBA + j) * 64 + lane] = v4i{(int)pk[0], (int)pk[1], (int)pk[2], (int)pk[3]};
    }
  };
  v4f acc[FBX];
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) acc[fb] = v4f{0.f, 0.f, 0.f, 0.f};
  float qa[NKJ];
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) qa[kj] = 0.f;
  load_a(mlo);
  build_a(0);
  if (mlo + 32 < mhi) load_a(mlo + 32);
  __syncthreads();
  int cur = 0;
  for (int ms = mlo; ms < mhi; ms += 32) {
    if (oact) {
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
      // grad_alpha partials (lsq.py:321-333): code * g, code the 2-bit field of slice pair kj
#pragma unroll
      for (int kj = 0; kj < NKJ; ++kj) {
        float q = qa[kj];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // the field sign-extended by shifts (the sbfe builtin's result is converted as unsigned)
          const int code = (int)(sv[e].x << (30 - 2 * kj)) >> 30;
          q = __builtin_fmaf((float)code, gv[e], q);
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
            D = ldexpf((float)__popc(sv[e].y & dmask_j(j, NBW, NBA)), g.bsa * j);
          } else {
            D = 0.f;
#pragma unroll
            for (int k = 0; k < NBW; ++k) D += ((sv[e].y >> (k * NBA + j)) & 1u) ? cdl[k * NBA + j] : 0.f;
          }
          d[e] = gv[e] * D;
        }
        v8bf bh, bm, bl;
        split3x8(d, bh, bm, bl);
#pragma unroll
        for (int fb = 0; fb < FBX; ++fb) {
          if (fb >= g.FBT) break;
          const v8bf a = as_v8bf(As[((cur * FBX + fb) * NBA + j) * 64 + lane]);
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh, acc[fb], 0, 0, 0);
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm, acc[fb], 0, 0, 0);
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl, acc[fb], 0, 0, 0);
        }
      }
    }
    if (ms + 32 < mhi) {
      build_a(cur ^ 1);
      if (ms + 64 < mhi) load_a(ms + 64);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (!oact) return;
  // acc[fb][r]: row c = 16fb + 4g4 + r of the tile, column o
  const int FR = g.FBT * 16;
  const int oo = ob * 16 + r16;
#pragma unroll
  for (int fb = 0; fb < FBX; ++fb) {
    if (fb >= g.FBT) break;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      gw_slab[(((size_t)chunk * g.T + i) * FR + fb * 16 + 4 * g4 + r) * g.Opad + oo] = acc[fb][r];
  }
#pragma unroll
  for (int kj = 0; kj < NKJ; ++kj) {
    float q = qa[kj];
    q = rows4_sum(q);
    if (g4 == 0) ga_slab[(((size_t)chunk * g.T + i) * NKJ + kj) * g.Opad + oo] = q;
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
template <int NBW, int NBA>
int launch_dense_fwd_n(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  auto klit = g.KS == 1 ? dense_fwd_lit_kernel<NBW, NBA, 1> : dense_fwd_lit_kernel<NBW, NBA, 2>;
  const uint8_t* wr = wreg(g, ctx);
  uint2* st = reinterpret_cast<uint2*>(ctx + L.st);
  const int slot = prof_begin(KID_FWD, g, s);
  if (tune("DENSE_FWD8", 1)) {  // 128-row blocks, weight side staged once per block (dense_plan: M % 128 == 0)
    auto kern = g.KS == 1 ? dense_fwd8_kernel<NBW, NBA, 1> : dense_fwd8_kernel<NBW, NBA, 2>;
    hipLaunchKernelGGL(kern, dim3(g.M / 128, g.O / 64), dim3(512), 0, s, g, ctx + L.xcode,
                       reinterpret_cast<const v4i*>(wr + L.wfrag), params_of(g, ctx), out, st);
  } else {
    auto kern = g.KS == 1 ? dense_fwd_kernel<NBW, NBA, 1> : dense_fwd_kernel<NBW, NBA, 2>;
    hipLaunchKernelGGL(kern, dim3(g.M / 64, g.O / 64), dim3(256), 0, s, g, ctx + L.xcode,
                       reinterpret_cast<const v4i*>(wr + L.wfrag), params_of(g, ctx), sw, sa, out, st);
  }
  prof_end(slot, s);
  hipLaunchKernelGGL(klit, dim3(32), dim3(256), 0, s, g, ctx + L.xcode, reinterpret_cast<const v4i*>(wr + L.wfrag),
                     params_of(g, ctx), sw, sa, out, st);
  return check_hip("dense_fwd");
}

template <int NBW, int NBA>
int launch_dense_bwd_n(const Geo& g, const uint8_t* ctx, const float* sw, const float* gout, float* gx, uint8_t* ws,
                       hipStream_t s, const float* x, const float* sa) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  const uint2* st = reinterpret_cast<const uint2*>(ctx + L.st);
  {
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL((dense_gx_kernel<NBW, NBA>), dim3(g.M / 128, g.T), dim3(1024), 0, s, g, st,
                       reinterpret_cast<const v4i*>(wreg(g, ctx) + L.wgx), pp, sw, gout, gx, x, sa,
                       reinterpret_cast<float*>(ws + W.lsq_part));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("dense_gx"));
  }
  {
    const int slot = prof_begin(KID_BWD_GW, g, s);
    hipLaunchKernelGGL((dense_gw_kernel<NBW, NBA>), dim3(W.nchunks_bwd, g.T, cdiv(g.O, 128)), dim3(512), 0, s, g,
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
                     hipStream_t s, const float* x, const float* sa) {
  CIMQ_DENSE_SEL(launch_dense_bwd_n, g, ctx, sw, gout, gx, ws, s, x, sa)
}

}  // namespace cimq

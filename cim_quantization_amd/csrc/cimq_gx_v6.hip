// cimq_gx_v6.hip -- grad_x of the CiM conv (lsq.py:257-317 with the nn.Fold adjoint,
// lsq.py:336-386) as a pipelined transposed implicit GEMM.
//
// Same decomposition as cim_bwd_gx_v5_kernel (block = band of RI input rows of one image,
// every wave owns its output tiles in registers, no atomics, LSQ act backward in the
// epilogue), with the two latencies that dominated v5 taken off the critical path:
//   * grad_out is the same for every (tile i, kappa chunk): the band's [O][npb] (NCHW) or
//     [npb][O] slab is brought into LDS once, by LDS-DMA, instead of per chunk from global;
//   * the forward's state words of chunk n+1 are LDS-DMA'd into the other half of a double
//     buffer while phase A / phase B of chunk n run, so phase A reads only LDS.
// The DMA is issued from inline asm (global_load_lds_dwordx4), so the compiler neither
// waits for it at LDS reads nor at the mid-chunk barrier; it is retired explicitly with
// s_waitcnt vmcnt(0) before the end-of-chunk barrier.
#pragma once
#include "cimq_kernels_v3.hip"

namespace cimq {

__device__ inline uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// 16 bytes from each lane's gsrc to lds_wave_base + 16 * lane (wave-uniform base)
__device__ inline void glds16(const void* gsrc, uint32_t lds_wave_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_wave_base)
               : "memory");
}

__device__ inline void wait_vmem_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// workgroup barrier that retires LDS traffic only (an LDS-DMA may stay in flight across it)
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA copy of n16 16-byte pieces: piece t from src(t) to lds + 16 t (lane-linear per wave)
template <typename Src>
__device__ inline void glds_copy(int n16, uint8_t* lds, Src src) {
  const int lane = threadIdx.x & 63;
  for (int t = threadIdx.x; t - lane < n16; t += blockDim.x) {
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(lds) + (uint32_t)(t - lane) * 16u);
    if (t < n16) glds16(src(t), base);
  }
}

template <int NBP, int TPW, bool LSQ>
__global__ __launch_bounds__(512, 2) void cim_bwd_gx_v6_kernel(Geo g, V3 v, const uint8_t* __restrict__ st,
                                                            const uint4* __restrict__ wtc, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p,
                                                            const float* __restrict__ gout,
                                                            const float* __restrict__ x, float* __restrict__ gx,
                                                            float* __restrict__ gsa_part) {
  typedef typename StWord<NBP>::T SW;
  constexpr int GP = 40;   // G row pitch in bf16: 32 kappa + 8 pad (phase-A stores 2-way at most)
  constexpr int KX = 3;
  constexpr int PQ = 64 * (int)sizeof(SW);  // bytes of one (quad, 16-channel block) state piece
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
  const int nquad = npb >> 2;
  const int Cp = v.CB * 16;
  const int ZROW = v.NPB;
  const int PART = (v.NPB + 1) * GP;
  const int NQ = v.NPB >> 2;
  const size_t STB = al16((size_t)2 * NQ * PQ);  // one state buffer: [kbl][quad][PQ]
  const int NCR = v.NCBT * 16;                     // W rows per tap in one W buffer
  const size_t WBB = al16((size_t)g.KHW * NCR * 64);  // one W buffer: [khw][NCR][32 kappa] bf16

  uint8_t* cur = smem;
  __bf16* Gs = reinterpret_cast<__bf16*>(cur); cur += al16((size_t)3 * PART * 2);
  uint8_t* wbuf = cur; cur += 2 * WBB;
  float* gS = reinterpret_cast<float*>(cur); cur += al16((size_t)g.O * v.NPB * 4);
  uint8_t* stb = cur; cur += 2 * STB;
  float* ckl = reinterpret_cast<float*>(cur); cur += al16(3 * nkj * 4);
  float* red = reinterpret_cast<float*>(cur);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const size_t MQ = (size_t)g.M >> 2;
  const size_t m_band = (size_t)b * g.P + ((size_t)oh_lo << v.lw);
  const int nchunk = g.T * g.NKS;

  // state words of chunk n = (i, kc) -> state buffer n & 1
  auto issue_states = [&](int n) {
    const int i = n / g.NKS, kc = n - i * g.NKS;
    const int nkbl = min(2, g.NBLK - 2 * kc);
    constexpr int PP = PQ / 16;
    const int per = nquad * PP;
    glds_copy(nkbl * per, stb + (size_t)(n & 1) * STB, [&](int t) -> const void* {
      const int kbl = t / per, rem = t - kbl * per;
      const int qd = rem / PP, part = rem - qd * PP;
      const int kb = 2 * kc + kbl;
      const int k = kb / g.OB16, ob = kb - k * g.OB16;
      const size_t w = ((((size_t)(i * g.nbw + k) * MQ + (m_band >> 2) + qd) * g.O + ob * 16) * 4);
      return st + w * sizeof(SW) + part * 16;
    });
  };

  // W rows of chunk n = (i, kc), the channel blocks tile i touches -> W buffer n & 1.  The
  // 16-B kappa pieces of a row are XOR-swizzled by ((row >> 2) & 3) so the phase-B B-operand
  // reads (16 rows x one piece per lane group) hit 16 distinct bank groups.
  auto issue_w = [&](int n) {
    const int i = n / g.NKS, kc = n - i * g.NKS;
    const int cb0 = ((i * g.xbar) / g.KHW) >> 4;
    const int cb1 = ((min(g.K, (i + 1) * g.xbar) - 1) / g.KHW) >> 4;
    const int nr = (cb1 - cb0 + 1) * 16;
    glds_copy(g.KHW * nr * 4, wbuf + (size_t)(n & 1) * WBB, [&](int t) -> const void* {
      const int row = t >> 2, pz = t & 3;  // row = khw * nr + local channel
      const int khw = row / nr, cl = row - khw * nr;
      const int q = pz ^ ((cl >> 2) & 3);
      return wtc + (((size_t)(i * g.KHW + khw) * Cp + cb0 * 16 + cl) * g.NKS + kc) * 4 + q;
    });
  };

  // prologue: grad_out slab and chunk 0's state words by DMA; small tables by plain loads
  {
    const int n4 = g.O * npb / 4;
    if (g.onchw) {
      const int q4 = npb >> 2;
      glds_copy(n4, reinterpret_cast<uint8_t*>(gS), [&](int t) -> const void* {
        const int o = t / q4, p4 = t - o * q4;
        return gout + ((size_t)b * g.O + o) * g.P + ((size_t)oh_lo << v.lw) + 4 * p4;
      });
    } else {
      glds_copy(n4, reinterpret_cast<uint8_t*>(gS),
                [&](int t) -> const void* { return gout + m_band * g.O + 4 * (size_t)t; });
    }
  }
  issue_states(0);
  issue_w(0);
  for (int t = threadIdx.x; t < 3 * GP / 2; t += blockDim.x) {
    const int part = t / (GP / 2), w = t - part * (GP / 2);
    reinterpret_cast<uint32_t*>(Gs + part * PART + ZROW * GP)[w] = 0u;
  }
  for (int t = threadIdx.x; t < 3 * nkj; t += blockDim.x) ckl[t] = pp.ckj[t];

  const int nq = nrow * g.W;
  const int QBb = (nq + 15) >> 4;
  const int NTb = QBb * v.CB;
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
  constexpr int RIX = (TPW <= 2) ? TPW * KX * KX : 1;
  int rowidx[RIX];
  auto grow_of = [&](int u, int kh, int kw) -> int {
    const int ohs = ihp[u] - kh, ows = iwp[u] - kw;
    int row = ZROW;
    if (ohs >= 0 && ows >= 0 && (ohs % g.SH) == 0 && (ows % g.SW) == 0) {
      const int oh = ohs / g.SH, ow = ows / g.SW;
      if (oh < nro && ow < g.Wo) row = (oh << v.lw) + ow;
    }
    return row;
  };
  if constexpr (TPW <= 2) {
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
      for (int kh = 0; kh < KX; ++kh)
#pragma unroll
        for (int kw = 0; kw < KX; ++kw) rowidx[(u * KX + kh) * KX + kw] = grow_of(u, kh, kw);
  }
  wait_vmem_all();
  __syncthreads();

  for (int n = 0; n < nchunk; ++n) {
    const int i = n / g.NKS, kc = n - i * g.NKS;
    const int ci0 = (i * g.xbar) / g.KHW, ci1 = (min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
    const int cb0 = ci0 >> 4;
    const int nr = ((ci1 >> 4) - cb0 + 1) * 16;
    const __bf16* Wb = reinterpret_cast<const __bf16*>(wbuf + (size_t)(n & 1) * WBB);
    if (n + 1 < nchunk) {
      issue_states(n + 1);
      issue_w(n + 1);
    }
    // phase A: one item = 4 pixels x 4 consecutive kappa (same k, 4 channels), from LDS
    const uint8_t* sb = stb + (size_t)(n & 1) * STB;
    for (int it = threadIdx.x; it < nquad * 8; it += blockDim.x) {
      const int qd = it >> 3, kq = it & 7;
      const int kbl = kq >> 2, kb = 2 * kc + kbl;
      float G[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) G[r][e] = 0.f;
      if (kb < g.NBLK) {
        const int k = kb / g.OB16;
        const int o0 = (kb - k * g.OB16) * 16 + (kq & 3) * 4;
        SW sv[4][4];  // [channel e][pixel r]
        const uint8_t* sp = sb + ((size_t)kbl * nquad + qd) * PQ + (kq & 3) * 4 * 4 * sizeof(SW);
        if (sizeof(SW) == 2) {
          const uint4 a0 = reinterpret_cast<const uint4*>(sp)[0];
          const uint4 a1 = reinterpret_cast<const uint4*>(sp)[1];
          const uint32_t w8[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int r = 0; r < 4; ++r) sv[e][r] = (SW)(w8[2 * e + (r >> 1)] >> (16 * (r & 1)));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint4 a = reinterpret_cast<const uint4*>(sp)[e];
            sv[e][0] = a.x; sv[e][1] = a.y; sv[e][2] = a.z; sv[e][3] = a.w;
          }
        }
        float gv[4][4];  // [pixel r][channel e]
        if (g.onchw) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float4 t4 = *reinterpret_cast<const float4*>(gS + (size_t)(o0 + e) * npb + 4 * qd);
            gv[0][e] = t4.x; gv[1][e] = t4.y; gv[2][e] = t4.z; gv[3][e] = t4.w;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float4 t4 = *reinterpret_cast<const float4*>(gS + (size_t)(4 * qd + r) * g.O + o0);
            gv[r][0] = t4.x; gv[r][1] = t4.y; gv[r][2] = t4.z; gv[r][3] = t4.w;
          }
        }
#pragma unroll
        for (int j = 0; j < NBP; ++j) {
          if (j < g.nba) {
            const float ce = ckl[nkj + k * g.nba + j];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int e = 0; e < 4; ++e) G[r][e] += ((sv[e][r] >> (3 * j)) & 1u) ? ce : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) G[r][e] *= gv[r][e];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        uint32_t ph[2], pm[2], pl2[2];
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          const float a0 = G[r][2 * e2], a1 = G[r][2 * e2 + 1];
          const __bf16 h0 = (__bf16)a0, h1 = (__bf16)a1;
          const float s0 = a0 - (float)h0, s1 = a1 - (float)h1;
          const __bf16 m0b = (__bf16)s0, m1b = (__bf16)s1;
          const __bf16 l0 = (__bf16)(s0 - (float)m0b), l1 = (__bf16)(s1 - (float)m1b);
          ph[e2] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
          pm[e2] = (uint32_t)__builtin_bit_cast(uint16_t, m0b) | ((uint32_t)__builtin_bit_cast(uint16_t, m1b) << 16);
          pl2[e2] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
        }
        const int off = (4 * qd + r) * GP + kq * 4;
        *reinterpret_cast<uint2*>(Gs + off) = make_uint2(ph[0], ph[1]);
        *reinterpret_cast<uint2*>(Gs + PART + off) = make_uint2(pm[0], pm[1]);
        *reinterpret_cast<uint2*>(Gs + 2 * PART + off) = make_uint2(pl2[0], pl2[1]);
      }
    }
    lds_barrier();
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
              int row;
              if constexpr (TPW <= 2) row = rowidx[(u * KX + kh) * KX + kw];
              else row = grow_of(u, kh, kw);
              const int khw = kh * g.KW + kw;
              const v8bf gh = *reinterpret_cast<const v8bf*>(Gs + row * GP + 8 * g4);
              const v8bf gm = *reinterpret_cast<const v8bf*>(Gs + PART + row * GP + 8 * g4);
              const v8bf gl = *reinterpret_cast<const v8bf*>(Gs + 2 * PART + row * GP + 8 * g4);
              const v8bf wv = *reinterpret_cast<const v8bf*>(
                  Wb + (khw * nr + (cb - cb0) * 16 + r16) * 32 + 8 * (g4 ^ ((r16 >> 2) & 3)));
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh, wv, a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gm, wv, a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gl, wv, a, 0, 0, 0);
            }
          }
        }
        acc[u] = a;
      }
    }
    wait_vmem_all();  // chunk n+1's state words have landed (this wave's share)
    __syncthreads();
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

}  // namespace cimq

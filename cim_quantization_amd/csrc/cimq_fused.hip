// cimq_fused.hip -- the whole backward of a stride-1 3x3 CiM conv layer in ONE kernel
// (lsq.py:244-386): grad_x with the nn.Fold adjoint and the fused act-LSQ backward, grad_w
// and the grad_alpha_cim partials, from the forward's compact state words (cimq_v7.hip).
//
// The two v7 kernels read the same state words and grad_out, decode the same STE masks and
// each keeps its chip busy for only a few waves per SIMD.  Here one workgroup owns one image and
// walks it top to bottom in steps of 64 output pixels (64 / W rows), one crossbar tile at a time
// (a "unit" = step x tile).  Its eight waves split by role:
//
//  * waves 0-3 (grad_x, as cim_bwd_gx_v8_kernel): wave = one 16-pixel MFMA column group; builds
//    G_i[(k, o), m] = g[m, o] * E_k from the state words in registers (bf16 hi / mid / lo),
//    contracts it against the int8 weight slices on v_mfma_f32_16x16x32_bf16, folds kw by DPP
//    lane shifts and kh over an LDS ring of output rows;
//  * waves 4-7 (grad_w, as cim_bwd_gw_v7_kernel): wave = (16-channel output block, a share of the
//    tile's 16-row groups); builds B = g * D_j for the step's 64 pixels (two 32-deep K-steps) and
//    contracts it against the activation slices, which all eight waves stage per unit into bf16
//    planes [j][kw][c][row][col] (kw pre-shifted: every A fragment is one aligned 16-B read);
//    grad_alpha_cim partials sum code * g over the same pixels.
//
// Every unit's global loads (its state words, the step's grad_out, the activation words) are issued
// one unit ahead into registers (a few 16-B pieces per thread, coalesced) and staged into LDS at the
// unit's start, so their latency hides behind the previous unit's MFMA / VALU work.
// grad_w accumulates in LDS across the image's steps (or goes straight to the slab when the image
// is one step); the slabs [image][tile][row][o] are summed in a fixed order by the module tail /
// reduce kernels: bit-identical run to run, no atomics.
#pragma once
#include <type_traits>

#include "cimq_v7.hip"

namespace cimq {

struct V9 {
  int lw;        // log2(W)
  int R;         // output rows per step (64 / W)
  int nsteps;    // H / R
  int SWD, NSEG; // ring segments (as V7): min(16, W) columns, W / SWD per row
  int RSLOT;     // ring rows
  int NCPBT;     // (c, kh)-row blocks of 4 per tile (the v8 grad_x operand wcy)
  int lcin;      // log2(C), or -1
  int NCG;       // most input channels one tile touches (staged plane channels)
  int CPITCH;    // plane channel pitch (bf16): PROWS * W + 8 (the 8-element zero pad)
  int KWP;       // (j, kw) plane pitch (bf16)
  int PROWS;     // staged input rows per step: R + 2
  int NGRP;      // 16-row groups of K
  int gwl;       // 1: grad_w accumulates in LDS across steps; 0: one step per image, units write the slab
  int nitems;    // plane staging items per unit: NCG * PROWS * W / 8 (<= 512)
  unsigned o_ring, o_cel, o_red, o_plane, o_gwl, o_gal, o_st, o_g, lds;  // LDS layout (bytes)
};

template <int NB, int OBX, bool LSQ>
__global__ __launch_bounds__(512) void cim_bwd_fused_kernel(Geo g, V9 v, const uint32_t* __restrict__ st,
                                                            const v4i* __restrict__ wcy, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p,
                                                            const float* __restrict__ gout,
                                                            const uint32_t* __restrict__ xcb,
                                                            const float* __restrict__ x, float* __restrict__ gx,
                                                            float* __restrict__ gw_slab, float* __restrict__ ga_slab,
                                                            float* __restrict__ gsa_part) {
  constexpr int NKJ = NB * NB;
  constexpr int NKS = (NB * OBX + 1) / 2;
  constexpr int WPO = 4 / OBX;  // grad_w waves per 16-channel output block
  // one output block (O = 16): its four waves split the two K-steps x two row-group halves, and each
  // K-step half keeps its own grad_w accumulator in LDS; else the waves of a block split the row groups
  constexpr int KSP = OBX == 1 ? 2 : 1;
  constexpr int RGS = WPO / KSP;  // row-group stride of one wave
  constexpr int NGW = 8 / RGS;    // 16-row groups per grad_w wave and tile (xbar <= 128)
  constexpr int O = 16 * OBX;   // v9_plan: O is a multiple of 16
  constexpr int PST = (16 * O + 511) / 512;  // 16-B pieces of a unit's state words / grad_out per thread
  constexpr int GP = 68;        // grad_out LDS row pitch (floats): 16-B reads of 16 channels hit distinct banks
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = (int)blockIdx.x;
  float* ring = reinterpret_cast<float*>(smem + v.o_ring);
  float* cel = reinterpret_cast<float*>(smem + v.o_cel);  // [0, NKJ): cE (grad_x); [NKJ, 2 NKJ): cD (grad_w)
  float* red = reinterpret_cast<float*>(smem + v.o_red);
  __bf16* pl = reinterpret_cast<__bf16*>(smem + v.o_plane);
  float* gwl = reinterpret_cast<float*>(smem + v.o_gwl);   // [NGRP * 16][O]
  float* gal = reinterpret_cast<float*>(smem + v.o_gal);   // [4 gw waves][T][NKJ][16]
  uint32_t* stl = reinterpret_cast<uint32_t*>(smem + v.o_st);  // the unit's state words [64 pixels][O]
  float* gl = reinterpret_cast<float*>(smem + v.o_g);          // the step's grad_out [O][GP]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const bool gxw = wave < 4;
  const int W = 1 << v.lw;
  const int CPP = g.C * 3;
  const int RE = v.SWD + 2;
  const int rrow = v.NSEG * CPP * RE;  // floats per ring row
  const int lsw = v.lw < 4 ? v.lw : 4;
  const int zoff = v.CPITCH - 8;       // zero pad of plane (j, kw = 0), channel 0
  const float sw = *sw_p, sa = *sa_p;
  const float scale = sw / (float)NB;
  const float inv_sa = 1.f / sa;
  const size_t P = (size_t)g.P;
  const size_t img0 = (size_t)b * P;  // first pixel of the image

  for (int t = threadIdx.x; t < NKJ; t += blockDim.x) {
    cel[t] = pp.ckj[NKJ + t];
    cel[NKJ + t] = pp.ckj[2 * NKJ + t];
  }
  if (threadIdx.x < NB) *reinterpret_cast<uint4*>(pl + (size_t)threadIdx.x * 3 * v.KWP + zoff) = make_uint4(0u, 0u, 0u, 0u);
  if (v.gwl)
    for (int t = threadIdx.x; t < KSP * v.NGRP * 16 * O; t += blockDim.x) gwl[t] = 0.f;
  for (int t = threadIdx.x; t < 4 * g.T * NKJ * 16; t += blockDim.x) gal[t] = 0.f;
  __syncthreads();
  // standard binary masks (_quan_base.py:207-214): cE_kj = 2^(bsw*k), cD_kj = 2^(bsa*j) for every pair;
  // then E_k / D_j are powers of two times pass-bit popcounts (else the per-pair sums)
  bool std_mask;
  {
    const int kl = lane < NKJ ? lane / NB : 0, jl = lane < NKJ ? lane - kl * NB : 0;
    const bool bad = lane < NKJ && (cel[lane < NKJ ? lane : 0] != ldexpf(1.f, g.bsw * kl) ||
                                    cel[NKJ + (lane < NKJ ? lane : 0)] != ldexpf(1.f, g.bsa * jl));
    std_mask = __builtin_amdgcn_ballot_w64(bad) == 0ull;
  }

  // ---- per-lane geometry of the two roles ----
  // grad_x: this lane's pixel q in the step (MFMA column), its segment / column of the ring
  const int gq = 16 * (wave & 3) + r16;
  const int gq_row = gq >> v.lw, gq_ow = gq & (W - 1);
  const int seg = gq_ow >> lsw, col = gq_ow & (v.SWD - 1);
  // grad_w: output block and share of the row groups
  const int gwi = wave - 4;
  const int gob = gxw ? 0 : gwi / WPO, within = gxw ? 0 : gwi % WPO;
  const int ksel = KSP == 2 ? (within & 1) : 0;                  // KSP 2: this wave's K-step
  const int wpart = KSP == 2 ? (within >> 1) : within;            // its row groups: wpart + RGS * n
  float* gwk = gwl + (size_t)(KSP == 2 ? ksel : 0) * v.NGRP * 16 * O;  // its grad_w accumulator
  const int go = gob * 16 + r16;  // this lane's output channel (B column)

  // ---- the unit's global loads, issued one unit ahead into registers, staged into LDS at its start ----
  // state words of (tile i, the step's 64 pixels) and the step's grad_out: 16 * O pieces of 16 B each
  auto load_st = [&](int s, int i, uint4 (&sv)[PST]) {
    const uint4* src = reinterpret_cast<const uint4*>(st + ((size_t)i * g.M + img0 + (size_t)s * 64) * O);
#pragma unroll
    for (int u = 0; u < PST; ++u) {
      const int t = threadIdx.x + 512 * u;
      sv[u] = t < 16 * O ? src[t] : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto load_g = [&](int s, float4 (&gv)[PST]) {
#pragma unroll
    for (int u = 0; u < PST; ++u) {
      const int t = threadIdx.x + 512 * u;
      gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t < 16 * O) {
        const int o = t >> 4, q4 = (t & 15) * 4;
        if (g.onchw) {
          gv[u] = *reinterpret_cast<const float4*>(gout + ((size_t)b * O + o) * P + (size_t)s * 64 + q4);
        } else {
          const float* src = gout + (img0 + (size_t)s * 64 + q4) * O + o;
          gv[u] = make_float4(src[0], src[O], src[2 * O], src[3 * O]);
        }
      }
    }
  };
  // plane staging item (channel cl of the tile, staged row slot, 8-column group c8): the 8 words and
  // their two neighbours (zero outside the image)
  const int it = threadIdx.x;
  const int ng8 = W >> 3;
  const int it_c8 = it % ng8, it_rs = it / ng8;
  const int it_slot = it_rs % v.PROWS, it_cl = it_rs / v.PROWS;
  auto load_item = [&](int s, int i, uint32_t (&w)[10]) {
#pragma unroll
    for (int u = 0; u < 10; ++u) w[u] = 0u;
    if (it < v.nitems) {
      const int c0 = (i * g.xbar) / 9;
      const int c = c0 + it_cl;
      const int ih = s * v.R - 1 + it_slot;
      if (c < g.C && ih >= 0 && ih < g.H) {
        const uint32_t* src = xcb + (((size_t)b * g.C + c) * g.H + ih) * W + it_c8 * 8;
        const uint4 a0 = reinterpret_cast<const uint4*>(src)[0], a1 = reinterpret_cast<const uint4*>(src)[1];
        w[1] = a0.x; w[2] = a0.y; w[3] = a0.z; w[4] = a0.w;
        w[5] = a1.x; w[6] = a1.y; w[7] = a1.z; w[8] = a1.w;
        if (it_c8 > 0) w[0] = src[-1];
        if (it_c8 + 1 < ng8) w[9] = src[8];
      }
    }
  };

  uint4 svc[PST];
  float4 gvc[PST];
  uint32_t itc[10];
  load_st(0, 0, svc);
  load_g(0, gvc);
  load_item(0, 0, itc);

  float gsum = 0.f;  // act-LSQ d sa partial (lsq.py:549)
  int done = -1;     // last folded input row
  const int nunits = v.nsteps * g.T;
  for (int u = 0; u < nunits; ++u) {
    const int s = u / g.T, i = u - s * g.T;
    const int oh_s = s * v.R, oh_e = oh_s + v.R - 1;
    // ---- stage the unit (all waves); the previous unit's readers are done ----
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PST; ++q) {
      const int t = threadIdx.x + 512 * q;
      if (t < 16 * O) {
        reinterpret_cast<uint4*>(stl)[t] = svc[q];
        if (i == 0) *reinterpret_cast<float4*>(gl + (t >> 4) * GP + (t & 15) * 4) = gvc[q];
      }
    }
#ifndef CIMQ_EXP_F_NOSTAGE  // attribution builds only (tools/kernel_experiment.py): skip a part of the kernel
    if (it < v.nitems) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          uint32_t pk[4];
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const float f0 = (float)(int8_t)xbyte(itc[2 * e2 + kw], j);
            const float f1 = (float)(int8_t)xbyte(itc[2 * e2 + 1 + kw], j);
            pk[e2] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);  // exact bf16
          }
          __bf16* dst = pl + (size_t)(j * 3 + kw) * v.KWP + it_cl * v.CPITCH + it_slot * W + it_c8 * 8;
          *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
      }
    }
#endif
    // the next unit's loads go out now, behind this unit's work
    if (u + 1 < nunits) {
      const int s_n = (u + 1) / g.T, i_n = (u + 1) - s_n * g.T;
      load_st(s_n, i_n, svc);
      if (i_n == 0) load_g(s_n, gvc);
      load_item(s_n, i_n, itc);
    }
    __syncthreads();  // the unit is in LDS

    // the unit's two roles, compiled once per mask kind (SMC: the standard binary mask, E_k / D_j as
    // pass-bit popcounts) so no per-element uniform branch separates their VALU and MFMA work
    auto unit_roles = [&](auto smc) {
      constexpr bool SMC = decltype(smc)::value;
    if (gxw) {
#ifndef CIMQ_EXP_F_NOGX
      // ================= grad_x: G from the state words, MFMA against wcy, ring =================
      v8bf Gh[NKS], Gm[NKS], Gl[NKS];
      uint4 sq[OBX];
      float gq4[OBX][4];
#pragma unroll
      for (int ob = 0; ob < OBX; ++ob) {
        sq[ob] = *reinterpret_cast<const uint4*>(stl + gq * O + ob * 16 + 4 * g4);
#pragma unroll
        for (int r = 0; r < 4; ++r) gq4[ob][r] = gl[(ob * 16 + 4 * g4 + r) * GP + gq];
      }
#pragma unroll
      for (int sk = 0; sk < NKS; ++sk) {
        float Gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int kb = 2 * sk + (e >> 2), r = e & 3;
          Gv[e] = 0.f;
          if (kb < NB * OBX) {
            const int k = kb / OBX, ob = kb - k * OBX;
            const uint32_t sv = r == 0 ? sq[ob].x : r == 1 ? sq[ob].y : r == 2 ? sq[ob].z : sq[ob].w;
            float E;
            if constexpr (SMC) {
              E = ldexpf((float)__popc(sv & pass_mask_k(k, NB)), g.bsw * k);
            } else {
              E = 0.f;
#pragma unroll
              for (int j = 0; j < NB; ++j) E += ((sv >> (3 * (k * NB + j))) & 1u) ? cel[k * NB + j] : 0.f;
            }
            Gv[e] = gq4[ob][r] * E;
          }
        }
        split3x8(Gv, Gh[sk], Gm[sk], Gl[sk]);
      }
      const int cp_lo = (i * g.xbar) / 3, cp_hi = (min(g.K, (i + 1) * g.xbar) - 1) / 3;
      const int cpb_lo = cp_lo >> 2, ncb = (cp_hi >> 2) - cpb_lo + 1;
      const bool shared_first = i > 0 && cpb_lo == (((i * g.xbar - 1) / 3) >> 2);
      const v4i* wt = wcy + (size_t)i * v.NCPBT * NKS * 64 + lane;
      const int oh = oh_s + gq_row;
      float* rr = ring + (size_t)(oh % v.RSLOT) * rrow + seg * CPP * RE;
      v4i anx[NKS];
#pragma unroll
      for (int sk = 0; sk < NKS; ++sk) anx[sk] = wt[sk * 64];
#ifdef CIMQ_EXP_F_PF2  // experiment: the weight blocks two (c, kh)-blocks ahead
      v4i anx2[NKS];
      if (ncb > 1) {
#pragma unroll
        for (int sk = 0; sk < NKS; ++sk) anx2[sk] = wt[(NKS + sk) * 64];
      }
#endif
#pragma unroll 1
      for (int cb = 0; cb < ncb; ++cb) {
        v4i acur[NKS];
#pragma unroll
        for (int sk = 0; sk < NKS; ++sk) acur[sk] = anx[sk];
#ifdef CIMQ_EXP_F_PF2
#pragma unroll
        for (int sk = 0; sk < NKS; ++sk) anx[sk] = anx2[sk];
        if (cb + 2 < ncb) {
#pragma unroll
          for (int sk = 0; sk < NKS; ++sk) anx2[sk] = wt[((cb + 2) * NKS + sk) * 64];
        }
#else
        if (cb + 1 < ncb) {
#pragma unroll
          for (int sk = 0; sk < NKS; ++sk) anx[sk] = wt[((cb + 1) * NKS + sk) * 64];
        }
#endif
        v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sk = 0; sk < NKS; ++sk) {
          const v8bf a = as_v8bf(acur[sk]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gh[sk], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gm[sk], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gl[sk], acc, 0, 0, 0);
        }
        // acc[kw] = gx_unf[(cp, kw)][this lane's pixel]; pixel ow feeds input column ow + kw - 1
        float fn = dpp_from_next(acc[0]);  // kw = 0 of pixel ow + 1
        if (col == v.SWD - 1) fn = 0.f;
        float fp = dpp_from_prev(acc[2]);  // kw = 2 of pixel ow - 1
        if (col == 0) fp = 0.f;
        const float y = (acc[1] + fn) + fp;
        const int cp = (cpb_lo + cb) * 4 + g4;
        if (cp < CPP) {
          float* e = rr + cp * RE;
          if (cb == 0 && shared_first) {
            e[col + 1] += y;
            if (col == 0) e[0] += acc[0];
            if (col == v.SWD - 1) e[v.SWD + 1] += acc[2];
          } else {
            e[col + 1] = y;
            if (col == 0) e[0] = acc[0];
            if (col == v.SWD - 1) e[v.SWD + 1] = acc[2];
          }
        }
      }
#endif
    } else {
#ifndef CIMQ_EXP_F_NOGW
      // ================= grad_w (+ grad_alpha): B = g * D_j, A from the planes =================
      const int flo = i * g.xbar;
      const int ngt = (min(g.xbar, g.K - flo) + 15) >> 4;  // row groups of tile i
      const int c0 = flo / 9;
      // this wave's row groups gr = wpart + RGS * n; per lane the plane offset of its row (or -1)
      int gofs[NGW];
#pragma unroll
      for (int n = 0; n < NGW; ++n) {
        const int gr = wpart + RGS * n;
        const int f = flo + 16 * gr + r16;
        gofs[n] = -1;
        if (gr < ngt && f < min(g.K, flo + g.xbar)) {
          const int c = f / 9, tap = f - 9 * c, kh = tap / 3, kw = tap - 3 * kh;
          gofs[n] = kw * v.KWP + (c - c0) * v.CPITCH + kh * W;
        }
      }
      v4f acc[NGW];
#pragma unroll
      for (int n = 0; n < NGW; ++n) acc[n] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (KSP == 2 && ks != ksel) continue;  // uniform: the other K-step's waves
        const int q0 = 32 * ks + 8 * g4;  // first pixel of this lane's 8 (one row segment)
        uint32_t sv[8];
        float gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) sv[e] = stl[(q0 + e) * O + go];
        {
          const float4 a0 = *reinterpret_cast<const float4*>(gl + go * GP + q0);
          const float4 a1 = *reinterpret_cast<const float4*>(gl + go * GP + q0 + 4);
          gv[0] = a0.x; gv[1] = a0.y; gv[2] = a0.z; gv[3] = a0.w;
          gv[4] = a1.x; gv[5] = a1.y; gv[6] = a1.z; gv[7] = a1.w;
        }
        if (KSP == 2 ? wpart == 0 : (WPO == 1 || wpart == ks)) {  // one wave per (block, K-step)
          // grad_alpha partials (lsq.py:321-333): the code is the signed 2-bit field {nz, neg}
#pragma unroll
          for (int kj = 0; kj < NKJ; ++kj) {
            float q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int code = ((int)(sv[e] << (29 - 3 * kj))) >> 30;
              q = __builtin_fmaf((float)code, gv[e], q);
            }
            q = rows4_sum(q);
            if (g4 == 0) gal[((gwi * g.T + i) * NKJ + kj) * 16 + r16] += q;
          }
        }
        v8bf bh[NB], bm[NB], bq[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float D;
            if constexpr (SMC) {
              D = ldexpf((float)__popc(sv[e] & pass_mask_j(j, NB, NB)), g.bsa * j);
            } else {
              D = 0.f;
#pragma unroll
              for (int k = 0; k < NB; ++k) D += ((sv[e] >> (3 * (k * NB + j))) & 1u) ? cel[NKJ + k * NB + j] : 0.f;
            }
            d[e] = gv[e] * D;
          }
          split3x8(d, bh[j], bm[j], bq[j]);
        }
        // the row groups' MFMA chains; where the tile has all of this wave's groups (every tile but a short
        // last one) without the per-group uniform branch, so the chains' A reads and MFMAs interleave
        auto gw_chains = [&](auto fc) {
          constexpr bool FULL = decltype(fc)::value;
#pragma unroll
          for (int n = 0; n < NGW; ++n) {
            if (!FULL && wpart + RGS * n >= ngt) continue;  // uniform
            const int ofs = gofs[n] >= 0 ? gofs[n] + q0 : zoff;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
              const __bf16* src = pl + (size_t)j * 3 * v.KWP + ofs;
              const v8bf a = as_v8bf(*reinterpret_cast<const v4i*>(src));
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[j], acc[n], 0, 0, 0);
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm[j], acc[n], 0, 0, 0);
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[j], acc[n], 0, 0, 0);
            }
          }
        };
        if (wpart + RGS * (NGW - 1) < ngt) gw_chains(std::true_type{});
        else gw_chains(std::false_type{});
      }
      // accumulator rows 16 gr + 4 g4 + r, column o: owned by this wave alone
#pragma unroll
      for (int n = 0; n < NGW; ++n) {
        const int gr = wpart + RGS * n;
        if (gr >= ngt) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int fl = 16 * gr + 4 * g4 + r;
          if (v.gwl) {
            gwk[(size_t)(flo + fl) * O + go] += acc[n][r];
          } else {
            gw_slab[(((size_t)b * g.T + i) * (g.FBT * 16) + fl) * O + go] = acc[n][r];
          }
        }
      }
#endif
    }
    };
    if (std_mask) unit_roles(std::true_type{});
    else unit_roles(std::false_type{});

    if (i == g.T - 1) {
      // ---- end of step: fold the input rows whose three output rows are done (lsq.py:382) ----
      __syncthreads();
      const int upto = (s == v.nsteps - 1) ? g.H - 1 : oh_e - 1;
      const int f0 = done + 1, f1 = upto;
      if (f1 >= f0) {
        const int nf = (f1 - f0 + 1) * g.C * W;
        // XB elements per thread and round, their x loads issued together ahead of the sums
        auto fidx = [&](int t) {
          const int iw = t & (W - 1), rest = t >> v.lw;
          const int c = v.lcin >= 0 ? (rest & (g.C - 1)) : rest % g.C;
          const int ih = f0 + (v.lcin >= 0 ? (rest >> v.lcin) : rest / g.C);
          return (((size_t)b * g.C + c) * g.H + ih) * W + iw;
        };
        for (int t0 = threadIdx.x; t0 < nf; t0 += CIMQ_FOLD_XB * blockDim.x) {
        float xb[CIMQ_FOLD_XB];
#pragma unroll
        for (int u = 0; u < CIMQ_FOLD_XB; ++u) {
          const int t = t0 + u * (int)blockDim.x;
          xb[u] = (LSQ && t < nf) ? x[fidx(t)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < CIMQ_FOLD_XB; ++u) {
          const int t = t0 + u * (int)blockDim.x;
          if (t >= nf) break;
          const int iw = t & (W - 1), rest = t >> v.lw;
          const int c = v.lcin >= 0 ? (rest & (g.C - 1)) : rest % g.C;
          const int ih = f0 + (v.lcin >= 0 ? (rest >> v.lcin) : rest / g.C);
          const int sg = iw >> lsw, cl = iw & (v.SWD - 1);
          float a = 0.f;
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            const int oo = ih + 1 - kh;
            if (oo >= 0 && oo <= oh_e) {
              const float* e = ring + (size_t)(oo % v.RSLOT) * rrow + (c * 3 + kh) * RE;
              a += e[sg * CPP * RE + cl + 1];
              if (cl == v.SWD - 1 && sg + 1 < v.NSEG) a += e[(sg + 1) * CPP * RE];
              if (cl == 0 && sg > 0) a += e[(sg - 1) * CPP * RE + v.SWD + 1];
            }
          }
          const size_t gi = (((size_t)b * g.C + c) * g.H + ih) * W + iw;
          const float gqv = a * scale;
          if (LSQ) {
            // autograd of round_pass(clamp(x/sa, 0, Qp)) * sa (lsq.py:549), as cim_bwd_gx_v8_kernel
            const float xv = xb[u];
            const float y1 = xv / sa;
            const float clv = clamp_nan(y1, 0.f, g.lsq_qp);
            const float rr2 = rintf(clv);
            const float rp = (rr2 - clv) + clv;
            const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
            const float gy = pass ? gqv * sa : 0.f;
            gx[gi] = pass ? gqv : 0.f;
            gsum += gqv * rp;
            gsum += -(gy * (y1 * inv_sa));
          } else {
            gx[gi] = gqv;
          }
        }
        }
        done = f1;
      }
    }
  }

  // ---- block epilogue: act-LSQ partial, grad_w (LDS accumulation) and grad_alpha slabs ----
  if (LSQ) {
    for (int o = 32; o > 0; o >>= 1) gsum += __shfl_xor(gsum, o);
    if (lane == 0) red[wave] = gsum;
  }
  __syncthreads();
  if (LSQ && threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 8; ++w) t += red[w];
    gsa_part[b] = t;
  }
  if (v.gwl) {
    const int FR = g.FBT * 16;
    for (int t = threadIdx.x; t < g.K * O; t += blockDim.x) {
      const int f = t / O, o = t - f * O;
      const int i = f / g.xbar, fl = f - i * g.xbar;
      gw_slab[(((size_t)b * g.T + i) * FR + fl) * O + o] = KSP == 2 ? gwl[t] + gwl[(size_t)v.NGRP * 16 * O + t] : gwl[t];
    }
  }
  // grad_alpha: the waves of an output block that summed K-steps 0 / 1, in that order
  for (int t = threadIdx.x; t < g.T * NKJ * O; t += blockDim.x) {
    const int o = t % O, rest = t / O;
    const int kj = rest % NKJ, i = rest / NKJ;
    const int ob = o >> 4, oc = o & 15;
    float sum;
    if (WPO == 1) {
      sum = gal[((ob * g.T + i) * NKJ + kj) * 16 + oc];
    } else {
      const int w0 = ob * WPO;
      sum = gal[((w0 * g.T + i) * NKJ + kj) * 16 + oc] + gal[(((w0 + 1) * g.T + i) * NKJ + kj) * 16 + oc];
    }
    ga_slab[(((size_t)b * g.T + i) * NKJ + kj) * O + o] = sum;
  }
}

}  // namespace cimq

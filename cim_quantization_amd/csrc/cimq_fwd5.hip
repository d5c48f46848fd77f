// cimq_fwd5.hip -- the forward of the w3a3 module layers (lsq.py:141-233, the LSQ activation quantiser of
// lsq.py:544-549 fused in), rebuilt around one LDS layout that feeds the int8 MFMA straight from
// ds_read_b128:
//
//   * the activation patch of a 128-pixel m-tile is stored slice-planar and channel-innermost,
//     [image][row][16-channel block][col][slice j][16 channels], so the 16 contraction values one lane
//     of v_mfma_i32_16x16x64_i8 needs -- 16 channels at one kernel position (kh, kw) -- are 16 contiguous
//     bytes of one slice: one ds_read_b128 per (slice, K-step), no byte transposes, no index table;
//   * the contraction of a crossbar tile is ordered (16-channel block, position p = kh*3 + kw) with the
//     positions padded to 12 = 3 K-steps of 4 lane groups (lane group g4 of K-step s holds position
//     4s + g4), so a lane's patch offset is one of three per-lane constants plus a uniform offset; the
//     weight side (wf5, built by the module prologue) is zero for every (channel, position) outside the
//     tile and for the padding positions, which makes each tile's partial sums exactly the reference's
//     (lsq.py:179-185: any order of a tile's rows gives the same integer sum);
//   * 8 waves per block, one 16-pixel group each, two blocks per CU.  The crossbar tiles are processed
//     in groups whose weight fragments and activation channels fit the block's LDS budget: with one
//     group (16 / 32 input channels) the weight side is staged once and stays resident for all the
//     block's m-tiles; with more (64 channels) each group's is staged per m-tile, the output still
//     summed in registers across the groups.
// Outputs are those of cim_fwd_v3_kernel<4, KS, 3, *>: out (NCHW), the compact state words of the v7
// backward (bit 3*(k*3 + j) + {0 STE pass, 1 code != 0, 2 code < 0}), the backward ctx words of the rows
// the m-tile owns; the ADC sum runs in the same order (tiles ascending, k and j descending), so out is
// bit-identical to that kernel's.
#pragma once
#include "cimq_kernels_v3.hip"

namespace cimq {

constexpr int kF5MaxTc = 8;   // (tile, channel-block) pairs: 2 / 4 / 8 for C = 16 / 32 / 64 at xbar 128
constexpr int kF5MaxGrp = 4;  // tile groups

// host-computed plan (cimq_host.h: f5_plan)
struct F5 {
  int lwo;                 // log2(Wo)
  int lwi;                 // log2(W)
  int codes;               // 1: the ctx holds one code byte per element (ctx_codes: grad_w is cim_bwd_gw5_kernel)
  int IPM;                 // images per 128-pixel m-tile (1: the m-tile is R output rows of one image)
  int R, RH, WP;           // output rows per image slot, patch rows (R-1)*SH + 3, patch row length W + 2
  int NCBP;                // channel blocks one patch holds (the widest group's span)
  int nmt;                 // M / 128
  int ntc;                 // (tile, channel-block) pairs
  int ngrp;                // tile groups
  int tcmax;               // most pairs in one group
  // (int tables: the kernel indexes them with wave-uniform runtime indices, which scalar loads serve
  // only at dword granularity -- byte tables became per-lane global loads of the kernel arguments)
  int tc0[kF5MaxTc + 1];  // first pair of tile i (tc0[T] = ntc)
  int tcb[kF5MaxTc];      // channel block of pair t
  int gt0[kF5MaxGrp + 1]; // first tile of group q (gt0[ngrp] = T)
  int gcb0[kF5MaxGrp], gcb1[kF5MaxGrp];  // channel-block span of group q
  int gown[kF5MaxGrp];    // first channel block whose ctx words group q writes
};

// the part of the plan the weight prologue needs (kept small: it travels in every PrepJob)
struct F5W {
  int ntc;
  unsigned char tc0[kF5MaxTc + 1];
  unsigned char tcb[kF5MaxTc];
};
inline F5W f5w_of(const F5& v) {
  F5W w;
  w.ntc = v.ntc;
  for (int i = 0; i <= kF5MaxTc; ++i) w.tc0[i] = v.tc0[i];
  for (int i = 0; i < kF5MaxTc; ++i) w.tcb[i] = v.tcb[i];
  return w;
}

// the weight operand of one (ob, pair t, K-step s, w-slice k) fragment, lane l: output channel
// o = ob*16 + (l & 15), byte e = w-slice k of weight (c = cb*16 + e, position p = 4s + (l >> 4)),
// rint(slice) as int8 as in wfrag_item; zero when p > 8 or the row f = c*9 + p is outside tile i
// wf5[((ob*ntc + t)*3 + s)*3 + k][64]
template <typename WS>
__device__ inline void wf5_item(const Geo& g, const F5W& v, const WS& ws, v4i* __restrict__ wf5, int t) {
  const int lane = t & 63;
  int r = t >> 6;
  const int k = r % 3;
  r /= 3;
  const int s = r % 3;
  r /= 3;
  const int tc = r % v.ntc;
  const int ob = r / v.ntc;
  int i = 0;
  while (v.tc0[i + 1] <= tc) ++i;
  const int flo = i * g.xbar, fhi = min(flo + g.xbar, g.K);
  const int p = 4 * s + (lane >> 4);
  const int n = k * g.Opad + ob * 16 + (lane & 15);
  uint32_t wd[4] = {0, 0, 0, 0};
  if (p < 9) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = v.tcb[tc] * 16 + e;
      const int f = c * 9 + p;
      int val = 0;
      if (c < g.C && f >= flo && f < fhi) val = clamp_i8(wslice(g, ws, f, n));
      wd[e >> 2] |= ((uint32_t)(uint8_t)(int8_t)val) << (8 * (e & 3));
    }
  }
  v4i o;
  o.x = (int)wd[0]; o.y = (int)wd[1]; o.z = (int)wd[2]; o.w = (int)wd[3];
  wf5[t] = o;
}

// act_words_tab's table entry with the clamp moved after the rounding (rint(clamp(q, 0, Qp)) = clamp(rint(q),
// 0, Qp) for integer bounds): v_cvt_i32_f32 saturates +-inf and the NaN test picks the table's NaN entry
__device__ inline uint2 act_words_q5(float v, float sa, int qp, int nan_e, const uint32_t* lut, int& code) {
  const float q = v / sa;
  int e;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(e) : "v"(rintf(q)));
  e = min(max(e, 0), qp);
  e = (q == q) ? e : nan_e;
  code = e;
  return *reinterpret_cast<const uint2*>(lut + 2 * e);
}

// n / d for 0 <= n < 2^20, d < 2^10 (inv = 1 / d in fp32): exact, no correction step needed
__device__ inline int sdiv(int n, float inv) { return (int)(((float)n + 0.5f) * inv); }

// LDS byte offset of the patch element (row, channel-block slot, col) of one image slot, slice 0
// (slice j at + 16 j)
__device__ inline int f5_off(int NCB, int WP, int row, int cb, int col) { return ((row * NCB + cb) * WP + col) * 48; }

#ifdef CIMQ_TU_FWD5  // defined in its launcher's translation unit only
// NOB 16-channel output blocks per block (512 threads each): the NOB halves share the block's staged
// activation patch (f5_plan: NOB = 2 where OB16 is even, one 1024-thread block per CU)
// WST: write the backward's state words and ctx (false where the module backward recomputes the partial sums,
// cim_bwd_r6_kernel: the forward then writes only `out`, and its ADC epilogue skips the state-bit shifts)
template <int NOB, bool WST>
__global__ __attribute__((amdgpu_flat_work_group_size(512 * NOB, 512 * NOB), amdgpu_waves_per_eu(4, 4))) void cim_fwd5_kernel(
    Geo g, F5 v, const v4i* __restrict__ wf5, Params pp, const float* __restrict__ sw_p,
    const float* __restrict__ sa_p, const float* __restrict__ x, const float* __restrict__ sgn_p,
    float* __restrict__ out, uint32_t* __restrict__ st, uint32_t* __restrict__ xcb, uint32_t* __restrict__ cal) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int obl = wave >> 3, pw = wave & 7;  // this wave's output block within the block, its pixel group
  const int ob = blockIdx.y * NOB + obl;
  const int nfr = v.ntc * 9;  // one output block's fragments ([pair][s][k], 64 lanes each)
  const size_t WB = (size_t)v.tcmax * 9 * 1024;  // LDS bytes of one output block's staged fragments
  // smem: weight fragments [NOB][<= tcmax][s][k][64] (v4i), then the tables below
  int4* prm = reinterpret_cast<int4*>(smem + NOB * WB);                      // [obl][i][j][k][16] (all tiles)
  float* cfl = reinterpret_cast<float*>(prm + NOB * g.T * 9 * 16);           // same order
  uint32_t* alut = reinterpret_cast<uint32_t*>(cfl + NOB * g.T * 9 * 16);    // [Qp + 2][fwd, bwd]
  // [img][RH][NCBP][WP][3][16]: a 16-aligned byte offset from smem (an integer round trip through
  // uintptr_t would turn the LDS pointer into a generic one: flat loads that wait on vmcnt too)
  const size_t poff0 = NOB * WB + (size_t)NOB * g.T * 9 * 16 * (16 + 4) + (size_t)2 * ((int)g.lsq_qp + 2) * 4;
  uint8_t* patch = smem + ((poff0 + 15) & ~(size_t)15);
  const int IMGB = v.RH * v.NCBP * v.WP * 48;

  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const bool literal = pp.flags[0] != 0;
  const bool sgn = *sgn_p != 0.f;

  // the weight fragments of group q (pairs tc0[gt0[q]] .. tc0[gt0[q+1]])
  auto stage_b = [&](int q) {
    const int a = v.tc0[v.gt0[q]], n = (v.tc0[v.gt0[q + 1]] - a) * 9 * 64;
#pragma unroll
    for (int h = 0; h < NOB; ++h) {
      const v4i* src = wf5 + ((size_t)(blockIdx.y * NOB + h) * nfr + a * 9) * 64;
      batched_copy<4>(n, reinterpret_cast<v4i*>(smem + h * WB), [&](int idx) -> v4i { return src[idx]; });
    }
  };
  // thresholds and coefficients of every tile (small): resident ([obl][T * 9 * 16])
  const int TQ = g.T * 9 * 16;
  batched_copy<2>(NOB * TQ, prm, [&](int idx0) -> int4 {
    const int h = idx0 / TQ, idx = idx0 - h * TQ;
    const int o = (blockIdx.y * NOB + h) * 16 + (idx & 15), q = idx >> 4;  // q = i*9 + j*3 + k
    const int i = q / 9, jk = q - i * 9, j = jk / 3, k = jk - j * 3;
    const int pi = pidx(g, i, j, k, o);
    return literal ? make_int4(0, 0, 0, 0) : make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
  });
  batched_copy<2>(NOB * TQ, cfl, [&](int idx0) -> float {
    const int h = idx0 / TQ, idx = idx0 - h * TQ;
    const int o = (blockIdx.y * NOB + h) * 16 + (idx & 15), q = idx >> 4;
    const int i = q / 9, jk = q - i * 9, j = jk / 3, k = jk - j * 3;
    return literal ? 0.f : pp.coef[pidx(g, i, j, k, o)];
  });
  if (v.ngrp == 1) stage_b(0);  // resident for all the block's m-tiles
  // padding columns 0 and WP-1 of every patch row: zero once (the staging writes data columns only)
  for (int t = threadIdx.x; t < v.IPM * v.RH * v.NCBP * 2 * 12; t += blockDim.x) {
    const int q = t % 12, rc = t / 12, side = rc & 1, rcb = rc >> 1;
    reinterpret_cast<uint32_t*>(patch + (rcb * v.WP + (side ? v.WP - 1 : 0)) * 48)[q] = 0u;
  }
  act_lut_build_q<3>(g, sa, sgn, alut);  // entries 0 .. Qp + 1 (NaN), then the block barrier
  // ctx codes: the table grad_w expands them with (code e -> ctx word), written once per launch
  if (WST && v.codes && blockIdx.x == 0 && blockIdx.y == 0)
    for (int t = threadIdx.x; t <= (int)g.lsq_qp + 1; t += blockDim.x) {
      cal[t] = alut[2 * t + 1];
      if (t == 0) cal[kCalFlag] = kCodesMagic;  // the ctx holds code bytes (checked by grad_w)
    }

  // this lane's A-operand pixel (image slot, output row / col) and its three position offsets
  const int Wo = 1 << v.lwo;
  const int PI = g.P < 128 ? g.P : 128;  // pixels per image slot
  const int pl = pw * 16 + r16;
  const int slot = pl / PI, pin = pl - slot * PI;
  const int pix = slot * IMGB + f5_off(v.NCBP, v.WP, (pin >> v.lwo) * g.SH, 0, (pin & (Wo - 1)) * g.SW);
  int pat[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int p = min(4 * s + g4, 8);
    const int kh = p / 3, kw = p - kh * 3;
    pat[s] = pix + f5_off(v.NCBP, v.WP, kh, 0, kw);
  }
  const int nan_e = (int)g.lsq_qp + 1;
  const int tpi = g.P >= 128 ? g.P / 128 : 1;  // m-tiles per image
  const int HWi = g.H * g.W;

  for (int mt = blockIdx.x; mt < v.nmt; mt += gridDim.x) {
    const int b0 = g.P >= 128 ? mt / tpi : mt * v.IPM;  // first image of the m-tile
    const int p0 = g.P >= 128 ? (mt - b0 * tpi) * 128 : 0;
    const int oh0 = p0 >> v.lwo;
    const int ih0 = oh0 * g.SH - 1;  // patch row 0 (pad 1)
    // input rows whose ctx words this m-tile writes: its output rows' stride spans, to the image end
    // for its last m-tile (one output-channel block's blocks write them)
    // (the staging is block-wide: the block holding output block 0 writes them)
    const int own_lo = blockIdx.y == 0 ? oh0 * g.SH : 0;
    const int own_hi = blockIdx.y == 0 ? (p0 + PI >= g.P ? g.H : (oh0 + v.R) * g.SH) : 0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int m0 = mt * 128 + pw * 16 + 4 * g4;  // output pixel of acc[0] (flattened b*P + p)
    for (int q = 0; q < v.ngrp; ++q) {
      const int cb0 = v.gcb0[q], ncb = v.gcb1[q] - cb0 + 1;
      const int QC = ncb * 4;  // staged 4-channel groups
      // row staging: item = (image slot, row, 4-channel group, col), col fastest (coalesced fp32 loads);
      // quantise (act_words_tab: the prologue's own table), transpose 4 channels x 3 slices into the slice
      // planes, store the ctx words of owned rows and channel blocks.  SU items per thread and round; the
      // first round's reads are issued before the barrier (every stride-1 layer stages in that one round)
      // (index arithmetic in 32 bits -- f5_plan bounds Nin -- with the divisions by the runtime QC and RH
      // as exact float-reciprocal quotients, and every item's decomposition computed once)
      constexpr int SU = NOB == 2 ? 3 : 2;
      constexpr int NT = 512 * NOB;
      const int n = v.IPM * v.RH * QC * g.W;
      const float invQC = 1.f / (float)QC, invRH = 1.f / (float)v.RH;
      const int xbase = (b0 * g.C + 16 * cb0) * HWi + ih0 * g.W;  // element (image b0, channel 16 cb0, row ih0, col 0)
      float xv[SU][4];
      int dsto[SU], xo[SU], ihs[SU], qqs[SU];
      auto ldx = [&](int base) {
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int idx = base + u * NT;
          dsto[u] = -1;
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[u][e] = 0.f;
          if (idx < n) {
            const int col = idx & (g.W - 1), r1 = idx >> v.lwi;
            const int r2 = sdiv(r1, invQC), qq = r1 - r2 * QC;
            const int sl = sdiv(r2, invRH), row = r2 - sl * v.RH;
            ihs[u] = ih0 + row;
            qqs[u] = qq;
            dsto[u] = sl * IMGB + f5_off(v.NCBP, v.WP, row, qq >> 2, col + 1) + 4 * (qq & 3);
            xo[u] = xbase + (sl * g.C + 4 * qq) * HWi + row * g.W + col;
            if ((unsigned)ihs[u] < (unsigned)g.H) {
#pragma unroll
              for (int e = 0; e < 4; ++e) xv[u][e] = x[xo[u] + e * HWi];
            }
          }
        }
      };
      auto stx = [&]() {
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          if (dsto[u] < 0) continue;
          uint32_t* dst = reinterpret_cast<uint32_t*>(patch + dsto[u]);
          const int ih = ihs[u];
          if ((unsigned)ih >= (unsigned)g.H) {
            dst[0] = 0u; dst[4] = 0u; dst[8] = 0u;
            continue;
          }
          uint2 w[4];
          int code[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = act_words_q5(xv[u][e], sa, nan_e - 1, nan_e, alut, code[e]);
          uint32_t P[4];
          tr4(w[0].x, w[1].x, w[2].x, w[3].x, P);
          dst[0] = P[0]; dst[4] = P[1]; dst[8] = P[2];
          if (WST && ih >= own_lo && ih < own_hi && cb0 + (qqs[u] >> 2) >= v.gown[q]) {
            if (v.codes) {  // one byte per element: grad_w expands it through the same word table
              uint8_t* cb8 = reinterpret_cast<uint8_t*>(xcb);
#pragma unroll
              for (int e = 0; e < 4; ++e) cb8[xo[u] + e * HWi] = (uint8_t)code[e];
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) xcb[xo[u] + e * HWi] = w[e].y;
            }
          }
        }
      };
      // (one instance of each phase: the first round, which every thread runs, holds the barrier)
#ifdef CIMQ_EXP_FWD5_NOSTAGE  // attribution builds only: the patch staged for the block's first m-tile only
      if (mt != (int)blockIdx.x) {
        __syncthreads();
        if (v.ngrp > 1) stage_b(q);
      } else
#endif
      for (int base = (int)threadIdx.x, first = 1; first || base < n; base += SU * NT, first = 0) {
        ldx(base);
        if (first) {
          __syncthreads();  // the previous group's / m-tile's waves are done with the patch (and the fragments)
          if (v.ngrp > 1) stage_b(q);
        }
        stx();
      }
      __syncthreads();

      const int tbase = v.tc0[v.gt0[q]];  // first pair of the group (its fragments start bfr)
      for (int i = v.gt0[q]; i < v.gt0[q + 1]; ++i) {
        v4i ps[9];
        // the tile's (pair, K-step) MFMAs; the first K-step of its first pair starts from the inline zero
        // accumulator (no per-tile register clearing)
        auto ksteps = [&](int tc, bool first) {
          const int cbo = (v.tcb[tc] - cb0) * v.WP * 48;
          const v4i* bt = reinterpret_cast<const v4i*>(smem + obl * WB) + (tc - tbase) * 9 * 64 + lane;  // LDS
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const uint8_t* pa = patch + pat[s] + cbo;
            v4i a[3], w[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) a[j] = *reinterpret_cast<const v4i*>(pa + 16 * j);
#pragma unroll
            for (int k = 0; k < 3; ++k) w[k] = bt[(s * 3 + k) * 64];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
              for (int j = 0; j < 3; ++j)
#ifdef CIMQ_EXP_FWD5_NOMFMA  // attribution builds only (tools/kernel_experiment.py): wrong results
                ps[k * 3 + j] = (first && s == 0) ? (a[j] ^ w[k]) : (ps[k * 3 + j] + (a[j] ^ w[k]));
#else
                ps[k * 3 + j] = (first && s == 0)
                                    ? __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j], w[k], v4i{0, 0, 0, 0}, 0, 0, 0)
                                    : __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j], w[k], ps[k * 3 + j], 0, 0, 0);
#endif
          }
        };
        ksteps(v.tc0[i], true);  // f5_plan: every tile has at least one pair
        for (int tc = v.tc0[i] + 1; tc < v.tc0[i + 1]; ++tc) ksteps(tc, false);
        // ADC + state bits of tile i: pairs kj = k*3 + j in descending order (bit 3*kj + {0,1,2} after
        // the last shift), the output summed in cim_fwd_v3_kernel's order
        uint32_t stw[4] = {0u, 0u, 0u, 0u};
        if (!literal) {
#pragma unroll
          for (int k = 2; k >= 0; --k) {
#pragma unroll
            for (int j = 2; j >= 0; --j) {
              const int pc = obl * TQ + (i * 9 + j * 3 + k) * 16 + r16;
              const int4 pv = prm[pc];
              const float cf = cfl[pc];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int p = ps[k * 3 + j][r];
#ifdef CIMQ_EXP_FWD5_NOADC
                acc[r] += (float)(p ^ pv.x) * cf;
                continue;
#endif
                const uint64_t mhi = __builtin_amdgcn_ballot_w64(p >= pv.x);
                const uint64_t mlo = __builtin_amdgcn_ballot_w64(p <= pv.y);
                const uint64_t mps = WST ? __builtin_amdgcn_ballot_w64((unsigned)(p - pv.z) <= (unsigned)pv.w) : 0ull;
                acc[r] += adc3(cf, mhi, mlo);
                if (WST) stw[r] = shin(shin(shin(stw[r], mlo), mhi | mlo), mps);
              }
            }
          }
        } else {
          // degenerate alpha_q / scales (the literal-ADC flag): the per-partial-sum chain, summed in
          // cim_fwd_v3_kernel's literal order (k, then j, ascending)
          const int o = min(ob * 16 + r16, g.Opad - 1);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const float al = pp.alpha[pidx(g, i, j, k, o)];
              const float mk = pp.ckj[k * 3 + j];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                acc[r] += adc_literal_sum(ps[k * 3 + j], g.mode, sw, sa, al, g.qn, g.qp, mk, r);
                if (!WST) continue;
                const bool pass = ste_literal(ps[k * 3 + j][r], g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f;
                const float code = code_literal(ps[k * 3 + j][r], g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo);
                stw[r] |= st_bits(pass, code) << (3 * (k * 3 + j));
              }
            }
          }
        }
        const int o = ob * 16 + r16;
        if (WST && o < g.O) {
          const int s0 = (i * g.M + m0) * g.O + o;  // 32-bit: f5_plan bounds T * M * O
#pragma unroll
          for (int r = 0; r < 4; ++r) st[s0 + r * g.O] = stw[r];
        }
      }
    }
    const int o = ob * 16 + r16;
    if (o < g.O) {
      const int bb = m0 / g.P, pq = m0 - bb * g.P;
      *reinterpret_cast<float4*>(out + ((bb * g.O + o) * g.P + pq)) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
  }
}
#endif  // CIMQ_TU_FWD5

}  // namespace cimq

// cimq_c1.hip -- the backward of the w8a8 first conv (ReplaceModuleTool forces it to 8 bits,
// utils/wrapper/replace_module.py:83-95) in one kernel, from the partial sums RECOMPUTED on the
// int8 MFMA instead of stored state words (lsq.py:244-386).
//
// The first conv has K = C*9 <= 32 rows and 64 slice pairs (36 live under the int8-wrapped
// binary_mask): its forward's state words would be three 64-bit planes per (pixel, channel),
// 24 B against 4 B of output, read back twice by the v7 backward.  Here the forward writes none
// (cim_fwd_v3_kernel<8, 1, 9, 1>), and one workgroup per image walks it in steps of 128 output
// pixels; each wave recomputes its 16 pixels' partial sums with the pixels as MFMA rows (lane: channel o,
// 4 pixels: the layout of grad_w's B operand on v_mfma_f32_16x16x16_bf16 and of the grad_alpha code sums)
// and takes the STE pass bits and ADC codes from the same integer thresholds as the forward (or the
// literal ADC on degenerate alpha).
//   grad_x:  G[(k, o), m] = g[m, o] * E_k,  E_k = sum_j cE_kj * pass   (transposed to the pixel-per-lane
//            layout through LDS; bf16 hi / mid / lo, wcy operand, kw folded by DPP, kh over an LDS ring,
//            act-LSQ backward in the fold)
//   grad_w:  sum_m xhat_j[m, f] * (g * D_j)[m, o],  D_j = sum_k cD_kj * pass
//   grad_alpha: sum_m code * g per (pair, o)
// All sums are fixed-order (per-wave registers / LDS regions added in wave order): bit-identical run
// to run, no atomics.
#pragma once
#include <type_traits>

#include "cimq_fused.hip"

namespace cimq {

struct VC1 {
  int lw;       // log2(W)
  int R;        // output rows per step (128 / W)
  int nsteps;   // H / R
  int RH, WP;   // staged input rows per step ((R - 1) + 3) and their word pitch (W + 2)
  int SWD, NSEG, RSLOT;  // ring geometry (as V7)
  int NCPBT;    // wcy blocks
  int lcin;     // log2(C) or -1
  unsigned o_xp, o_hp, o_ptab, o_prm, o_cel, o_g, o_ring, o_gal, o_red, o_e, o_wk, o_wc, lds;
};

template <bool LSQ>
__global__ __launch_bounds__(512) void cim_bwd_c1_kernel(Geo g, VC1 v, const uint8_t* __restrict__ xcf,
                                                         const uint8_t* __restrict__ xcb,
                                                         const v4i* __restrict__ wfrag, const v4i* __restrict__ wcy,
                                                         Params pp, const float* __restrict__ sw_p,
                                                         const float* __restrict__ sa_p, const float* __restrict__ gout,
                                                         const float* __restrict__ x, float* __restrict__ gx,
                                                         float* __restrict__ gw_slab, float* __restrict__ ga_slab,
                                                         float* __restrict__ gsa_part) {
  constexpr int NB = 8, NKJ = 64, NKS = 4;  // w8a8, one 16-channel block: kappa = (k, o) = 128 = 4 K-steps
  constexpr int GP = 132;                   // grad_out LDS row pitch (128 pixels + 4)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = (int)blockIdx.x;
  uint8_t* xp = smem + v.o_xp;   // forward slice words of the step's rows [C][RH][WP] x 8 B
  uint8_t* hp = smem + v.o_hp;   // backward (int8 ctx) slice words, same layout
  int* ptab = reinterpret_cast<int*>(smem + v.o_ptab);   // [64] word offset of row f in a window
  int4* prm = reinterpret_cast<int4*>(smem + v.o_prm);   // [64 pairs kj][16 o] thi, tlo, mlo, mhi
  float* cel = reinterpret_cast<float*>(smem + v.o_cel); // [3][64]: mask, cE, cD
  float* gl = reinterpret_cast<float*>(smem + v.o_g);    // [16 o][GP] the step's grad_out
  float* ring = reinterpret_cast<float*>(smem + v.o_ring);
  float* gal = reinterpret_cast<float*>(smem + v.o_gal); // [8 waves][64][16] code * g sums
  float* red = reinterpret_cast<float*>(smem + v.o_red); // gw wave sums [2][16][16], act partials
  float* etl = reinterpret_cast<float*>(smem + v.o_e);   // [8 waves][k & 1][16 pixels][16 o]: E transposed

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int W = 1 << v.lw;
  const int CPP = g.C * 3;
  const int RE = v.SWD + 2;
  const int rrow = v.NSEG * CPP * RE;
  const int lsw = v.lw < 4 ? v.lw : 4;
  const float sw = *sw_p, sa = *sa_p;
  const float scale = sw / (float)NB;
  const float inv_sa = 1.f / sa;
  const bool literal = (pp.flags[0] != 0) || g.mode != ADC_TERNARY;
  const bool has_code = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  const size_t P = (size_t)g.P;

  // tables: row offsets of the window, ADC / STE thresholds, the mask and its grad_x / grad_w forms
  build_ptab(g, 0, 1, v.RH, v.WP, ptab);
  for (int t = threadIdx.x; t < NKJ * 16; t += blockDim.x) {
    const int kj = t >> 4, o = t & 15, k = kj >> 3, j = kj & 7;
    const int pi = pidx(g, 0, j, k, o);
    prm[t] = make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
  }
  for (int t = threadIdx.x; t < 3 * NKJ; t += blockDim.x) cel[t] = pp.ckj[t];
  for (int t = threadIdx.x; t < 8 * NKJ * 16; t += blockDim.x) gal[t] = 0.f;
  zero_lds(reinterpret_cast<uint32_t*>(xp), g.C * v.RH * v.WP * 2);
  zero_lds(reinterpret_cast<uint32_t*>(hp), g.C * v.RH * v.WP * 2);
  // the layer's weight operands, resident for the whole image: the partial-sum slices wk[k] (lane
  // order) and grad_x's wcy blocks -- in LDS, so the only vector-memory loads of a step are the next
  // step's rows (below) and the fold's x
  v4i* wkl = reinterpret_cast<v4i*>(smem + v.o_wk);
  v4i* wcl = reinterpret_cast<v4i*>(smem + v.o_wc);
  for (int t = threadIdx.x; t < NB * WAVE; t += blockDim.x) wkl[t] = wfrag[t];
  const int cp_hi = (g.K - 1) / 3;
  const int ncb = (cp_hi >> 2) + 1;  // (c, kh)-blocks of 4: at most 3 (K <= 32, c1_plan)
  for (int t = threadIdx.x; t < ncb * NKS * 64; t += blockDim.x) wcl[t] = wcy[t];
  __syncthreads();
  // the slice pairs with a nonzero binary_mask entry (36 of 64 under the standard int8-wrapped mask)
  const uint64_t live = __builtin_amdgcn_ballot_w64(cel[lane] != 0.f);
  // the standard int8-wrapped mask (_quan_base.py:207-214): cE_kj = s 2^k, cD_kj = s 2^j with s = 1 for
  // j + k < 7, -1 at j + k = 7, 0 beyond -- then E_k and D_j are small-integer counts of pass bits
  // (one add-with-carry per pass bit) times 2^k / 2^j
  bool stdm;
  {
    const int lk_ = lane >> 3, lj_ = lane & 7;
    const float se = (lk_ + lj_ < 7) ? 1.f : (lk_ + lj_ == 7 ? -1.f : 0.f);
    stdm = __builtin_amdgcn_ballot_w64(cel[NKJ + lane] != se * (float)(1 << lk_) ||
                                       cel[2 * NKJ + lane] != se * (float)(1 << lj_)) == 0ull;
  }

  // a step's rows -- forward / backward slice words of the RH input rows, grad_out of its 128 pixels
  // -- as at most three 16-byte items per thread (c1_plan), loaded into registers one step ahead
  const int QW = W / 2;  // 16-byte pieces of an 8-byte-per-element row
  const int nxi = g.C * v.RH * QW;
  uint4 pf[3];
  auto pf_load = [&](int stp) {
    const int ih0 = stp * v.R * g.SH - g.PH;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int t = (int)threadIdx.x + u * (int)blockDim.x;
      pf[u] = make_uint4(0u, 0u, 0u, 0u);
      if (stp >= v.nsteps) continue;
      if (t < 2 * nxi) {
        const int tt = t < nxi ? t : t - nxi;
        const int row = tt / QW, q = tt - row * QW, c = row / v.RH, ih = ih0 + (row - c * v.RH);
        const uint4* src = reinterpret_cast<const uint4*>(t < nxi ? xcf : xcb);
        if ((unsigned)ih < (unsigned)g.H) pf[u] = src[(((size_t)b * g.C + c) * g.H + ih) * QW + q];
      } else if (t < 2 * nxi + 512) {
        const int o = (t - 2 * nxi) >> 5, q4 = ((t - 2 * nxi) & 31) * 4;
        float4 gv;
        if (g.onchw) {
          gv = *reinterpret_cast<const float4*>(gout + ((size_t)b * 16 + o) * P + (size_t)stp * 128 + q4);
        } else {
          const float* src = gout + ((size_t)b * P + (size_t)stp * 128 + q4) * 16 + o;
          gv = make_float4(src[0], src[16], src[32], src[48]);
        }
        pf[u] = make_uint4(__float_as_uint(gv.x), __float_as_uint(gv.y), __float_as_uint(gv.z), __float_as_uint(gv.w));
      }
    }
  };
  auto pf_store = [&]() {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int t = (int)threadIdx.x + u * (int)blockDim.x;
      if (t < 2 * nxi) {
        const int tt = t < nxi ? t : t - nxi;
        const int row = tt / QW, q = tt - row * QW;
        uint32_t* d = reinterpret_cast<uint32_t*>((t < nxi ? xp : hp) + row * v.WP * 8 + g.PW * 8 + q * 16);
        d[0] = pf[u].x; d[1] = pf[u].y; d[2] = pf[u].z; d[3] = pf[u].w;
      } else if (t < 2 * nxi + 512) {
        const int o = (t - 2 * nxi) >> 5, q4 = ((t - 2 * nxi) & 31) * 4;
        *reinterpret_cast<uint4*>(gl + o * GP + q4) = pf[u];
      }
    }
  };
  pf_load(0);

  // this wave's 16 pixels of a step: p = 16 * wave + (0..15); the gather base of pixel p
  auto pix_base = [&](int p) { return ((p >> v.lw) * g.SH) * v.WP + (p & (W - 1)) * g.SW; };
  const int pA = 16 * wave + r16;            // the lane's pixel as an MFMA row / column
  const int rbA = pix_base(pA);
  const int gq_row = pA >> v.lw, gq_ow = pA & (W - 1);
  const int seg = gq_ow >> lsw, col = gq_ow & (v.SWD - 1);
  // grad_w A operand rows f = 16 fg + r16 (f < K), pixels 16 wave + 4 g4 + (0..3): window offsets
  int hoff[2];
#pragma unroll
  for (int fg = 0; fg < 2; ++fg) hoff[fg] = (16 * fg + r16 < g.K) ? ptab[16 * fg + r16] : -1;
  int hbase[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) hbase[r] = pix_base(16 * wave + 4 * g4 + r);
  float* et = etl + (size_t)wave * 2 * 256;  // E_k of the current slice pair (k even, k odd), [pixel][o]

  v4f gwa[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};  // grad_w rows 16 fg + 4 g4 + r, col o
  float gsum = 0.f;
  int done = -1;
  for (int s = 0; s < v.nsteps; ++s) {
    const int oh_s = s * v.R, oh_e = oh_s + v.R - 1;
    __syncthreads();  // the previous step's readers of the patches / grad_out are done
    pf_store();
    pf_load(s + 1);   // in flight through this step's compute
    __syncthreads();

    // ---- partial sums of the wave's 16 pixels (lane: channel r16, pixels 16w + 4 g4 + r) ----
    v4i xs[NB][1];
    gather_xs<8, 1>(xp, rbA, ptab, g4, xs);
    // D_j per (j, pixel 16w + 4 g4 + r) of channel r16: an integer pass count (standard mask) or the
    // bits of the float sum (any other mask)
    int D[NB][4];
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) D[a][r] = 0;
    float gA[4];  // grad_out at (pixel 16w + 4g4 + r, channel r16)
#pragma unroll
    for (int r = 0; r < 4; ++r) gA[r] = gl[r16 * GP + 16 * wave + 4 * g4 + r];
    float gB[4];  // grad_out at (pixel pA, channel 4 g4 + r)
#pragma unroll
    for (int r = 0; r < 4; ++r) gB[r] = gl[(4 * g4 + r) * GP + pA];
    // grad_x accumulators of the (c, kh)-blocks, fed one K-step (two slices k) at a time
    v4f acc[3];
#pragma unroll
    for (int cb = 0; cb < 3; ++cb) acc[cb] = v4f{0.f, 0.f, 0.f, 0.f};
    using F = std::false_type;
    using T = std::true_type;
    // one weight slice k: its live pairs' partial sums, pass counts, codes, then grad_x's K-step.  kv is k:
    // a compile-time constant on the standard-mask path (STD), whose pair selection j + k < 7 then folds
    // away -- no uniform branches between the slice's MFMAs and their VALU, so the scheduler can put the
    // partial sums of all its pairs in flight ahead of the compares; a runtime int otherwise
    auto kiter = [&](auto kv, auto stdc) {
      constexpr bool STD = decltype(stdc)::value;
      const int k = kv;
      const v4i wkk = wkl[k * WAVE + lane];
      const unsigned lk = (unsigned)(live >> (8 * k)) & 0xFFu;
      int E[4] = {0, 0, 0, 0};  // as D: a count (standard mask) or float bits
      float qs[NB];  // code * g over the lane's 4 pixels, per pair (k, j)
#pragma unroll
      for (int j = 0; j < NB; ++j) qs[j] = 0.f;
#ifndef CIMQ_EXP_C1_NOPAIRS  // attribution builds only (tools/kernel_experiment.py)
      auto addf = [](int& acc, bool pass, float c) { acc = __float_as_int(__int_as_float(acc) + (pass ? c : 0.f)); };
      // one pair: its partial sums (MFMA), STE pass bits into D_j / E_k, code * g into qs[j]; the
      // literal-ADC form (degenerate alpha, rare) and a non-standard mask take separate loops so the
      // common one has no per-element branches
      auto pair = [&](auto lit, auto sm, auto ng, auto jc) {
        constexpr bool LIT = decltype(lit)::value, SM = decltype(sm)::value, NEG = decltype(ng)::value;
        constexpr int j = decltype(jc)::value;
        const int kj = k * NB + j;
        const v4i ps = __builtin_amdgcn_mfma_i32_16x16x64_i8(xs[j][0], wkk, v4i{0, 0, 0, 0}, 0, 0, 0);
        // the pair's mask coefficients (uniform LDS broadcast reads; unused under the standard mask)
        const float cE = SM ? 0.f : cel[NKJ + kj], cD = SM ? 0.f : cel[2 * NKJ + kj];
        float q = 0.f;
        if constexpr (!LIT) {
          const int4 pv = prm[kj * 16 + r16];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = ps[r];
            const bool pass = (unsigned)(p - pv.z) <= (unsigned)pv.w;
            if constexpr (SM && NEG) {
              D[j][r] -= pass;
              E[r] -= pass;
            } else if constexpr (SM) {
              D[j][r] += pass;
              E[r] += pass;
            } else {
              addf(D[j][r], pass, cD);
              addf(E[r], pass, cE);
            }
            const float code = (p >= pv.x) ? 1.f : ((p <= pv.y) ? -1.f : 0.f);
            q = __builtin_fmaf(code, gA[r], q);
          }
        } else {
          const float al = pp.alpha[pidx(g, 0, j, k, r16)];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = ps[r];
            const bool pass = ste_literal(p, g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f;
            addf(D[j][r], pass, cD);
            addf(E[r], pass, cE);
            if (has_code)
              q = __builtin_fmaf(code_literal(p, g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo), gA[r], q);
          }
        }
        qs[j] = q;
      };
      // the live pairs (uniform branches): mask != 0; under the standard mask j + k < 7 (coefficient
      // +2^k / +2^j) and then the one pair j + k = 7 (-2^k / -2^j)
      auto pairs = [&](auto lit, auto sm) {
        constexpr bool SM = decltype(sm)::value;
        auto each = [&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if (SM) {
            if (j + k < 7) pair(lit, sm, F{}, jc);
          } else if ((lk >> j) & 1u) {
            pair(lit, sm, F{}, jc);
          }
        };
        each(std::integral_constant<int, 0>{});
        each(std::integral_constant<int, 1>{});
        each(std::integral_constant<int, 2>{});
        each(std::integral_constant<int, 3>{});
        each(std::integral_constant<int, 4>{});
        each(std::integral_constant<int, 5>{});
        each(std::integral_constant<int, 6>{});
        each(std::integral_constant<int, 7>{});
        if constexpr (SM) {
          auto negp = [&](auto jc) {
            if (decltype(jc)::value + k == 7) pair(lit, sm, T{}, jc);
          };
          negp(std::integral_constant<int, 0>{});
          negp(std::integral_constant<int, 1>{});
          negp(std::integral_constant<int, 2>{});
          negp(std::integral_constant<int, 3>{});
          negp(std::integral_constant<int, 4>{});
          negp(std::integral_constant<int, 5>{});
          negp(std::integral_constant<int, 6>{});
          negp(std::integral_constant<int, 7>{});
        }
      };
      if constexpr (STD) {
        pairs(F{}, T{});
      } else {
        if (literal) pairs(T{}, F{});
        else if (stdm) pairs(F{}, T{});
        else pairs(F{}, F{});
      }
#endif
      // grad_alpha partials of slice k's pairs, channel r16, this wave's 16 pixels: the four 16-lane
      // rows summed by two half-wave swaps (no LDS), then lane row g4 adds pairs j = g4 and g4 + 4 to
      // the wave's LDS region (one read-modify-write per lane instead of one per pair)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(qs[j]), __float_as_uint(qs[j]), false, false);
        const float h = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
        const auto r16s = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
        qs[j] = __uint_as_float(r16s[0]) + __uint_as_float(r16s[1]);
      }
      {
        const float q0 = g4 == 0 ? qs[0] : g4 == 1 ? qs[1] : g4 == 2 ? qs[2] : qs[3];
        const float q1 = g4 == 0 ? qs[4] : g4 == 1 ? qs[5] : g4 == 2 ? qs[6] : qs[7];
        float* ga = gal + ((size_t)wave * NKJ + k * NB + g4) * 16 + r16;
        ga[0] += q0;
        ga[4 * 16] += q1;
      }
      // E_k to the grad_x layout (lane: pixel 16w + r16, channels 4 g4 .. +3) through this wave's LDS slab
#pragma unroll
      for (int r = 0; r < 4; ++r)
        et[((k & 1) * 16 + 4 * g4 + r) * 16 + r16] =
            (stdm && !literal) ? (float)(E[r] * (1 << k)) : __int_as_float(E[r]);
      if (k & 1) {
        // ---- grad_x K-step sk = k / 2: G from E_{k-1}, E_k (lane: pixel pA, channels 4 g4 + r) ----
        const int sk = k >> 1;
        const float4 e0 = *reinterpret_cast<const float4*>(et + r16 * 16 + 4 * g4);
        const float4 e1 = *reinterpret_cast<const float4*>(et + (16 + r16) * 16 + 4 * g4);
        const float Ev[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
        float Gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) Gv[e] = gB[e & 3] * Ev[e];
        v8bf Gh, Gm, Gl;
        split3x8(Gv, Gh, Gm, Gl);
#pragma unroll
        for (int cb = 0; cb < 3; ++cb) {
          if (cb >= ncb) break;
          const v8bf a = as_v8bf(wcl[(cb * NKS + sk) * 64 + lane]);
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gh, acc[cb], 0, 0, 0);
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gm, acc[cb], 0, 0, 0);
          acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gl, acc[cb], 0, 0, 0);
        }
      }
    };
    if (stdm && !literal) {
      // the slices unrolled, a scheduling fence after each: the pairs of one slice in flight together (a
      // free schedule over all 36 pairs would hoist every partial sum and spill)
      using std::integral_constant;
      kiter(integral_constant<int, 0>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 1>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 2>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 3>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 4>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 5>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 6>{}, T{});
      __builtin_amdgcn_sched_barrier(0);
      kiter(integral_constant<int, 7>{}, T{});
    } else {
      // any other mask or the literal ADC (rare): k rolled
#pragma unroll 1
      for (int k = 0; k < NB; ++k) kiter(k, F{});
    }
    // ---- grad_w: B = g * D_j (lane: channel r16, pixels 4 g4 + r), A = xhat_j rows f, 16x16x16 bf16 ----
    {
      uint2 hw[2][4];  // the 8 slice bytes of the A elements (row 16 fg + r16, pixel 4 g4 + r)
#pragma unroll
      for (int fg = 0; fg < 2; ++fg)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          hw[fg][r] = hoff[fg] >= 0 ? reinterpret_cast<const uint2*>(hp)[hbase[r] + hoff[fg]] : make_uint2(0u, 0u);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
        v4bf bh, bm, bl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dv = gA[r] * ((stdm && !literal) ? (float)(D[j][r] * (1 << j)) : __int_as_float(D[j][r]));
          const __bf16 h = (__bf16)dv;
          const float r1 = dv - (float)h;
          const __bf16 m = (__bf16)r1;
          bh[r] = h;
          bm[r] = m;
          bl[r] = (__bf16)(r1 - (float)m);
        }
#pragma unroll
        for (int fg = 0; fg < 2; ++fg) {
          v4bf a;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t wv = j < 4 ? hw[fg][r].x : hw[fg][r].y;
            a[r] = (__bf16)(float)(int8_t)((wv >> (8 * (j & 3))) & 0xFF);  // exact small integer
          }
          gwa[fg] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bh, gwa[fg], 0, 0, 0);
          gwa[fg] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bm, gwa[fg], 0, 0, 0);
          gwa[fg] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bl, gwa[fg], 0, 0, 0);
        }
      }
    }

    // ---- grad_x: kw folded by DPP, the (c, kh) rows to the ring ----
    {
      const int oh = oh_s + gq_row;
      float* rr = ring + (size_t)(oh % v.RSLOT) * rrow + seg * CPP * RE;
#pragma unroll
      for (int cb = 0; cb < 3; ++cb) {
        if (cb >= ncb) break;
        const v4f ac = acc[cb];
        float fn = dpp_from_next(ac[0]);
        if (col == v.SWD - 1) fn = 0.f;
        float fp = dpp_from_prev(ac[2]);
        if (col == 0) fp = 0.f;
        const float y = (ac[1] + fn) + fp;
        const int cp = cb * 4 + g4;
        if (cp < CPP) {
          float* e = rr + cp * RE;
          e[col + 1] = y;
          if (col == 0) e[0] = ac[0];
          if (col == v.SWD - 1) e[v.SWD + 1] = ac[2];
        }
      }
    }
    // ---- fold the input rows whose three output rows are done, act-LSQ backward ----
    __syncthreads();
    const int upto = (s == v.nsteps - 1) ? g.H - 1 : oh_e - 1;
    const int f0 = done + 1, f1 = upto;
    if (f1 >= f0) {
      const int nf = (f1 - f0 + 1) * g.C * W;
      for (int t = threadIdx.x; t < nf; t += blockDim.x) {
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
          const float xv = x[gi];
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
      done = f1;
    }
  }

  // ---- epilogue: act-LSQ partial, grad_w (the eight waves in order), grad_alpha slabs ----
  float* gws = red;           // [2 fg][16 rows][16 o]
  float* apart = red + 512;   // [8]
  if (LSQ) {
    for (int o = 32; o > 0; o >>= 1) gsum += __shfl_xor(gsum, o);
    if (lane == 0) apart[wave] = gsum;
  }
  for (int w = 0; w < 8; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int fg = 0; fg < 2; ++fg)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* d = gws + (fg * 16 + 4 * g4 + r) * 16 + r16;
          *d = (w == 0 ? 0.f : *d) + gwa[fg][r];
        }
    }
  }
  __syncthreads();
  if (LSQ && threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 8; ++w) t += apart[w];
    gsa_part[b] = t;
  }
  const int FR = g.FBT * 16;
  for (int t = threadIdx.x; t < g.K * 16; t += blockDim.x) {
    const int f = t >> 4, o = t & 15;
    gw_slab[((size_t)b * FR + f) * g.Opad + o] = gws[t];
  }
  for (int t = threadIdx.x; t < NKJ * 16; t += blockDim.x) {
    float sum = 0.f;
    for (int w = 0; w < 8; ++w) sum += gal[w * NKJ * 16 + t];
    ga_slab[(size_t)b * NKJ * g.Opad + (t >> 4) * g.Opad + (t & 15)] = sum;
  }
}

}  // namespace cimq

// cimq_r6.hip -- the whole backward of the w3a3 16 -> 16-channel 32 x 32 stride-1 module layers (lsq.py:244-386
// with the fused LSQ activation backward of lsq.py:549) from RECOMPUTED partial sums: the forward
// (cim_fwd5_kernel<*, false>) writes only `out`, and this kernel rebuilds every tile's integer partial sums on
// the int8 MFMA from the activation (re-quantised from x through the forward's own code -> word table) and the
// forward's weight operand, as the reference keeps only int8 ctx.x_int and the weight slices for its operands
// (lsq.py:99,160) and SURVEY section 7 step 6a asks.  Per partial sum the STE-pass bit and the ADC code come
// from the same integer thresholds as the forward's (params_item), so the masks are the forward's exactly.
//
// One workgroup per image, walking it in m-tiles of R = 4 output rows (128 pixels, one 16-pixel group per
// wave).  Per m-tile:
//   * A / B (every crossbar tile i): the tile's 9 slice-pair partial sums of the wave's 16 pixels x 16 output
//     channels (v_mfma_i32_16x16x64_i8 on cim_fwd5_kernel's slice-planar patch and operand), the STE masks and
//     codes as wave ballots, then in registers: grad_alpha partials sum code * g (lsq.py:321-333); the gw B
//     operand g * D_j of the wave's own pixels (D_j = sum_k cD_kj pass_ijk), contracted at once against the
//     A-ready ctx-slice patch (bf16 x 3, as cim_bwd_gw5_kernel); and G_i = g * E_k (E_k = sum_j cE_kj pass_ijk)
//     written hi / mid / lo into an LDS "G patch" [plane][row][col][tile, k, o] of the m-tile's OWN rows;
//   * gx per (output row oh, kernel row kh): partial grad_x of input row oh + kh - 1 from the G patch row oh
//     shifted by kw (one ds_read_b128 per plane and K-step, shared by the three kh), both tiles in one
//     96-deep contraction against the LDS-resident gx operand (wx6) -- so no halo rows are recomputed;
//   * the three kh partials meet in an LDS exchange (fixed order), the two rows that straddle the next
//     m-tile are carried in LDS, and finished rows get the act-LSQ backward and are stored once.
// grad_w accumulates in registers over the whole image (every wave: all 9 16-row blocks, its own pixels),
// grad_alpha likewise; the block writes one slab chunk per image (the module tail sums the B chunks in
// order: deterministic, no atomics).  Reads x and g once per element (plus the two rows of overlap of the
// staging), writes gx once: the algorithmic traffic of SURVEY 8(d), no state words.
#pragma once
#include "cimq_fwd5.hip"

namespace cimq {

// host plan (cimq_host.h: r6_plan)
struct R6 {
  int tc0[3];  // first (tile, channel-block) pair of tile i in cim_fwd5_kernel's operand (f5_plan)
  int ntc;     // pairs
  int nmt;     // m-tiles per image (H / 4)
};

// geometry of the 16-channel layer (r6_plan checks it)
constexpr int kR6C = 16, kR6W = 32, kR6R = 4, kR6T = 2;
constexpr int kR6KO = 3 * kR6C;          // kappa (k, o) per tile: 48
constexpr int kR6NK = kR6T * kR6KO;      // kappa per G-patch pixel: 96 = 3 K-steps
constexpr int kR6KSG = kR6NK / 32;

// the gx operand: lane l of (position p, K-step s): input channel c = l & 15, kappa = 32 s + 8 (l >> 4) + e
// (e < 8) = (tile i, w-slice k, output channel o) = (kappa / 48, (kappa % 48) / 16, kappa % 16), the value
// int8(slice_k) of weight (o, f = 9 c + p) as bf16 (the backward's ctx slice, lsq.py:160), zero unless row f is
// in tile i: wx6[(p * 3 + s) * 64 + l]
template <typename WS>
__device__ inline void wx6_item(const Geo& g, const WS& ws, v4i* __restrict__ wx6, int t) {
  const int lane = t & 63;
  const int r = t >> 6;
  const int s = r % kR6KSG, p = r / kR6KSG;
  const int c = lane & 15;
  const int f = c * 9 + p;
  uint32_t wd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kap = 32 * s + 8 * (lane >> 4) + e;
    const int i = kap / kR6KO, rem = kap - i * kR6KO, k = rem >> 4, o = rem & 15;
    float val = 0.f;
    if (c < g.C && i < g.T && f >= i * g.xbar && f < min((i + 1) * g.xbar, g.K) && k < g.nbw)
      val = (float)to_i8_wrap(wslice(g, ws, f, k * g.Opad + o));
    wd[e >> 1] |= (uint32_t)bf16_bits(val) << (16 * (e & 1));
  }
  v4i q;
  q.x = (int)wd[0]; q.y = (int)wd[1]; q.z = (int)wd[2]; q.w = (int)wd[3];
  wx6[t] = q;
}
constexpr int kR6WxItems = 9 * kR6KSG * 64;

// LDS layout of cim_bwd_r6_kernel (bytes; 159.3 KB: one workgroup per CU)
struct R6L {
  static constexpr int RP = kR6R + 2, WP = kR6W + 2;
  static constexpr int GPX = kR6NK * 2 + 16;  // G-patch pixel pitch: 13 16-B slots, a wave's 16 pixels on distinct slots
  static constexpr int GROW = WP * GPX;       // one G-patch row of one plane
  static constexpr int GPL = kR6R * GROW;     // one plane
  static constexpr int EXP = 36;              // exchange pitch (floats per input channel): 16-B writes on distinct banks
  static constexpr int O_XP = 0;                             // forward slice patch [RP][WP][3 slices][16 ch] int8 (f5_off)
  static constexpr int O_XH = O_XP + RP * WP * 48;           // ctx slices, A-ready [C][RP][WP] x (bf16 x0|x1, x2|0)
  static constexpr int O_GP = O_XH + kR6C * RP * WP * 8;     // G patch [3 planes][R][WP][NK] bf16; exchange aliases it
  static constexpr int O_CA = O_GP + 3 * GPL;                // carried partial rows [2][C][W] fp32
  static constexpr int O_WX = O_CA + 2 * kR6C * kR6W * 4;    // gx operand [9][KSG][64] x 16 B
  static constexpr int O_PR = O_WX + kR6WxItems * 16;        // ADC / STE thresholds [T][9 kj][16 o] int4
  static constexpr int O_AL = O_PR + kR6T * 9 * 16 * 16;     // act word table [Qp + 2][fwd, bwd]
  static constexpr int O_CE = O_AL + 260 * 8;                // cE_kj [9], cD_kj [9]
  static constexpr int LDS = O_CE + 32 * 4;
};
static_assert(R6L::LDS <= 160 * 1024, "r6 LDS budget");
static_assert(9 * 8 * 64 * 16 <= 3 * R6L::GPL, "r6 gw reduction buffer");
static_assert(2 * kR6T * 9 * 8 * 16 * 4 <= 3 * R6L::GPL, "r6 grad_alpha reduction buffer");

#ifdef CIMQ_TU_R6
// STE pass bits of one tile's 9 slice pairs: bit k*3 + j
__device__ inline float r6_E(uint32_t pw, int k, bool std_mask, const float* cel) {
  if (std_mask) return (float)(__popc(pw & (7u << (3 * k))) << k);
  float e = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) e += ((pw >> (3 * k + j)) & 1u) ? cel[3 * k + j] : 0.f;
  return e;
}
__device__ inline float r6_D(uint32_t pw, int j, bool std_mask, const float* cel) {
  if (std_mask) return (float)(__popc(pw & (0x49u << j)) << j);
  float d = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) d += ((pw >> (3 * k + j)) & 1u) ? cel[9 + 3 * k + j] : 0.f;
  return d;
}

// DBG: the parity hook (cimq_debug_recompute_codes): recompute the partial sums of the image and write their
// state words (bits 3 kj + {0 pass, 1 code != 0, 2 code < 0}, decode_state_kernel's layout) to st_dbg, nothing else
template <bool DBG>
__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(2, 2))) void cim_bwd_r6_kernel(
    Geo g, R6 v, const v4i* __restrict__ wf5, const v4i* __restrict__ wx6, Params pp, const float* __restrict__ sw_p,
    const float* __restrict__ sa_p, const float* __restrict__ sgn_p, const float* __restrict__ x,
    const float* __restrict__ gout, float* __restrict__ gx, float* __restrict__ gw_slab, float* __restrict__ ga_slab,
    float* __restrict__ gsa_part, uint32_t* __restrict__ st_dbg) {
  constexpr int C = kR6C, O = kR6C, W = kR6W, R = kR6R, T = kR6T, RP = R + 2, WP = W + 2;
  constexpr int NK = kR6NK, KSG = kR6KSG;
  constexpr int GPX = R6L::GPX, GROW = R6L::GROW, GPL = R6L::GPL, EXP = R6L::EXP;
  constexpr int O_XP = R6L::O_XP, O_XH = R6L::O_XH, O_GP = R6L::O_GP, O_CA = R6L::O_CA, O_WX = R6L::O_WX,
                O_PR = R6L::O_PR, O_AL = R6L::O_AL, O_CE = R6L::O_CE;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* alut = reinterpret_cast<uint32_t*>(smem + O_AL);
  float* cel = reinterpret_cast<float*>(smem + O_CE);
  const int4* prm = reinterpret_cast<const int4*>(smem + O_PR);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b = (int)blockIdx.x;
  const int H = g.H, HW = H * W, P = H * W;
  const float sw = *sw_p, sa = *sa_p;
  const bool sgn = *sgn_p != 0.f;
  const bool literal = pp.flags[0] != 0;
  const int nan_e = (int)g.lsq_qp + 1;

  // ---- block prologue: the gx operand, the thresholds, the mask coefficients, zero pads, the word table ----
  if (!DBG) batched_copy<4>(kR6WxItems, reinterpret_cast<v4i*>(smem + O_WX), [&](int idx) -> v4i { return wx6[idx]; });
  batched_copy<2>(T * 9 * 16, reinterpret_cast<int4*>(smem + O_PR), [&](int idx) -> int4 {
    const int o = idx & 15, q = idx >> 4, i = q / 9, kj = q - 9 * i, k = kj / 3, j = kj - 3 * k;
    const int pi = pidx(g, i, j, k, o);
    return literal ? make_int4(0, 0, 0, 0) : make_int4(pp.thi[pi], pp.tlo[pi], pp.mlo[pi], pp.mhi[pi]);
  });
  for (int t = threadIdx.x; t < 18; t += blockDim.x) cel[t] = pp.ckj[9 + t];
  for (int t = threadIdx.x; t < RP * 2 * 12; t += blockDim.x) {  // forward patch: columns 0 and WP - 1
    const int q = t % 12, rc = t / 12, side = rc & 1, row = rc >> 1;
    reinterpret_cast<uint32_t*>(smem + O_XP + (row * WP + (side ? WP - 1 : 0)) * 48)[q] = 0u;
  }
  for (int t = threadIdx.x; t < C * RP * 2; t += blockDim.x) {  // ctx patch: columns 0 and WP - 1
    const int side = t & 1, cr = t >> 1;
    reinterpret_cast<uint2*>(smem + O_XH)[cr * WP + (side ? WP - 1 : 0)] = make_uint2(0u, 0u);
  }
  for (int t = threadIdx.x; t < 3 * R * 2 * (NK / 8); t += blockDim.x) {  // G patch: columns 0 and WP - 1
    const int q = t % (NK / 8), rc = t / (NK / 8), side = rc & 1, pr = rc >> 1;
    reinterpret_cast<uint4*>(smem + O_GP + pr * GROW + (side ? (WP - 1) * GPX : 0))[q] = make_uint4(0u, 0u, 0u, 0u);
  }
  act_lut_build_q<3>(g, sa, sgn, alut);  // entries 0 .. Qp + 1 (NaN), then the block barrier
  const bool std_mask = __builtin_amdgcn_ballot_w64(
                            lane < 9 && (cel[lane < 9 ? lane : 0] != (float)(1 << (lane / 3)) ||
                                         cel[9 + (lane < 9 ? lane : 0)] != (float)(1 << (lane % 3)))) == 0ull;

  // ---- per-lane geometry ----
  const int ohl = wave >> 1;           // the wave's output row within the m-tile
  const int cw0 = 16 * (wave & 1);     // first column of its 16-pixel group
  // phase A: this lane's A-operand pixel (column cw0 + r16) and its three position offsets (cim_fwd5_kernel)
  int pat[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int p = min(4 * s + g4, 8);
    const int kh = p / 3, kw = p - kh * 3;
    pat[s] = f5_off(1, WP, ohl + kh, 0, cw0 + r16 + kw);
  }
  // phase B / gw: the lane's four pixels cw0 + 4 g4 + r of row ohl, output channel r16
  const int ow0 = cw0 + 4 * g4;
  // gw A operand: row f = 16 fb + r16 = (c, kh, kw) of the ctx patch, packed uint2 offsets (< 2^16)
  uint32_t aoffp[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int fb = 0; fb < 9; ++fb) {
    const int f = 16 * fb + r16, c = f / 9, p = f - 9 * c, kh = p / 3, kw = p - 3 * kh;
    aoffp[fb >> 1] |= (uint32_t)((c * RP + kh) * WP + kw) << (16 * (fb & 1));
  }
  v4f acc[9];
#pragma unroll
  for (int fb = 0; fb < 9; ++fb) acc[fb] = v4f{0.f, 0.f, 0.f, 0.f};
  float ga[T][9];
#pragma unroll
  for (int i = 0; i < T; ++i)
#pragma unroll
    for (int kj = 0; kj < 9; ++kj) ga[i][kj] = 0.f;
  float gsum = 0.f;
  const float scale = sw / 3.f, inv_sa = 1.f / sa;

  // ---- staging of one m-tile: input rows r0 - 1 .. r0 + R (RP rows) -> forward slices + A-ready ctx slices ----
  // item = (row, 4-channel group q, column), column fastest: 768 items, <= 2 per thread
  constexpr int NSI = RP * (C / 4) * W;
  auto stage_load = [&](int r0, float (&xv)[2][4]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = (int)threadIdx.x + 512 * u;
      const int col = it & (W - 1), rq = it >> 5, q = rq & 3, row = rq >> 2;
      const int ih = r0 - 1 + row;
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[u][e] = 0.f;
      if (it < NSI && (unsigned)ih < (unsigned)H) {
        const int xo = ((b * C + 4 * q) * H + ih) * W + col;
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[u][e] = x[xo + e * HW];
      }
    }
  };
  auto stage_store = [&](int r0, const float (&xv)[2][4]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = (int)threadIdx.x + 512 * u;
      if (it >= NSI) continue;
      const int col = it & (W - 1), rq = it >> 5, q = rq & 3, row = rq >> 2;
      const int ih = r0 - 1 + row;
      uint32_t* dst = reinterpret_cast<uint32_t*>(smem + O_XP + (row * WP + col + 1) * 48 + 4 * q);
      uint2* xh = reinterpret_cast<uint2*>(smem + O_XH) + ((4 * q) * RP + row) * WP + col + 1;
      if ((unsigned)ih >= (unsigned)H) {
        dst[0] = 0u; dst[4] = 0u; dst[8] = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) xh[e * RP * WP] = make_uint2(0u, 0u);
        continue;
      }
      uint2 w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int code;
        w[e] = act_words_q5(xv[u][e], sa, nan_e - 1, nan_e, alut, code);
      }
      uint32_t Pq[4];
      tr4(w[0].x, w[1].x, w[2].x, w[3].x, Pq);
      dst[0] = Pq[0]; dst[4] = Pq[1]; dst[8] = Pq[2];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // int8 ctx slices (lsq.py:160 truncation, wrapped) -> exact bf16 (the high half of the fp32)
        const uint32_t f0 = __float_as_uint((float)(int8_t)(w[e].y & 0xFFu));
        const uint32_t f1 = __float_as_uint((float)(int8_t)((w[e].y >> 8) & 0xFFu));
        const uint32_t f2 = __float_as_uint((float)(int8_t)((w[e].y >> 16) & 0xFFu));
        xh[e * RP * WP] = make_uint2(__builtin_amdgcn_perm(f1, f0, 0x07060302u), f2 >> 16);
      }
    }
  };

  const int nmt = v.nmt;
#ifndef CIMQ_EXP_R6_NO_WFPF
  v4i wnx[9];  // the next tile's forward weight fragments, in flight one tile ahead
#pragma unroll
  for (int q = 0; q < 9; ++q) wnx[q] = wf5[(size_t)v.tc0[0] * 9 * 64 + lane + q * 64];
#endif
  float xv[2][4];
  stage_load(0, xv);
  float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!DBG) gq = *reinterpret_cast<const float4*>(gout + (size_t)(b * O + r16) * P + ohl * W + ow0);
  stage_store(0, xv);
  __syncthreads();

  for (int n = 0; n < nmt; ++n) {
    const int r0 = n * R;
    const bool more = n + 1 < nmt;
    // the next m-tile's x and g, in flight behind this one's work
    float4 gqn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (more) {
      stage_load(r0 + R, xv);
      if (!DBG) gqn = *reinterpret_cast<const float4*>(gout + (size_t)(b * O + r16) * P + (r0 + R + ohl) * W + ow0);
    }
    const float gv[4] = {gq.x, gq.y, gq.z, gq.w};

    // ================= A / B: recompute, masks, grad_alpha, gw, G =================
    // (one tile at a time, not unrolled: the tiles' operands and partial sums must not be live together)
#pragma unroll 1
    for (int i = 0; i < T; ++i) {
      // the tile's forward weight fragments [s][k] (cim_fwd5_kernel's operand, output block 0)
      v4i wfr[9];
#ifndef CIMQ_EXP_R6_NO_WFPF
      {
        const v4i* wt = wf5 + (size_t)v.tc0[i + 1 < T ? i + 1 : 0] * 9 * 64 + lane;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          wfr[q] = wnx[q];
          wnx[q] = wt[q * 64];
        }
      }
#else
      const v4i* wt = wf5 + (size_t)v.tc0[i] * 9 * 64 + lane;
#pragma unroll
      for (int q = 0; q < 9; ++q) wfr[q] = wt[q * 64];
#endif
      v4i ps[9];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        v4i a[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) a[j] = *reinterpret_cast<const v4i*>(smem + O_XP + pat[s] + 16 * j);
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            ps[k * 3 + j] = s == 0 ? __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j], wfr[s * 3 + k], v4i{0, 0, 0, 0}, 0, 0, 0)
                                   : __builtin_amdgcn_mfma_i32_16x16x64_i8(a[j], wfr[s * 3 + k], ps[k * 3 + j], 0, 0, 0);
      }
      // STE pass bits (bit kj after the shifts: pairs in descending order), grad_alpha partials
      uint32_t pw[4] = {0u, 0u, 0u, 0u};
      uint32_t stw[4] = {0u, 0u, 0u, 0u};
      float tga[9];
#pragma unroll
      for (int kj = 0; kj < 9; ++kj) tga[kj] = 0.f;
      if (!literal) {
#pragma unroll
        for (int k = 2; k >= 0; --k)
#pragma unroll
          for (int j = 2; j >= 0; --j) {
            const int4 pv = prm[(i * 9 + k * 3 + j) * 16 + r16];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int p = ps[k * 3 + j][r];
              const uint64_t mhi = __builtin_amdgcn_ballot_w64(p >= pv.x);
              const uint64_t mlo = __builtin_amdgcn_ballot_w64(p <= pv.y);
              const uint64_t mps = __builtin_amdgcn_ballot_w64((unsigned)(p - pv.z) <= (unsigned)pv.w);
              pw[r] = shin(pw[r], mps);
              if (DBG) stw[r] = shin(shin(shin(stw[r], mlo), mhi | mlo), mps);
              else tga[k * 3 + j] += adc3(gv[r], mhi, mlo);  // code * g (lsq.py:321-333)
            }
          }
      } else {
        // degenerate alpha_q / scales (the literal-ADC flag): the per-partial-sum chain
        const int o = r16;
#pragma unroll
        for (int k = 2; k >= 0; --k)
#pragma unroll
          for (int j = 2; j >= 0; --j) {
            const float al = pp.alpha[pidx(g, i, j, k, o)];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int p = ps[k * 3 + j][r];
              const bool pass = ste_literal(p, g.mode, sw, sa, al, g.thr_hi, g.thr_lo) != 0.f;
              const float code = code_literal(p, g.mode, sw, sa, al, g.qn, g.qp, g.thr_hi, g.thr_lo);
              pw[r] = (pw[r] << 1) | (pass ? 1u : 0u);
              if (DBG) stw[r] = (stw[r] << 3) | st_bits(pass, code);
              else tga[k * 3 + j] += code * gv[r];
            }
          }
      }
      if (!DBG) {
        if (i == 0) {
#pragma unroll
          for (int kj = 0; kj < 9; ++kj) ga[0][kj] += tga[kj];
        } else {
#pragma unroll
          for (int kj = 0; kj < 9; ++kj) ga[1][kj] += tga[kj];
        }
      }
      if (DBG) {
        const size_t m = (size_t)b * P + (size_t)(r0 + ohl) * W + ow0;
#pragma unroll
        for (int r = 0; r < 4; ++r) st_dbg[((size_t)i * g.M + m + r) * O + r16] = stw[r];
        continue;
      }
      // G_i = g * E_k (hi / mid / lo) into the G patch: kappa = i * 48 + k * 16 + o
      {
        uint8_t* gp = smem + O_GP + ohl * GROW + (ow0 + 1) * GPX + (i * kR6KO + r16) * 2;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float Gv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) Gv[r] = gv[r] * r6_E(pw[r], k, std_mask, cel);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            uint32_t hi, mid, lo;
            split3_pk(Gv[2 * h], Gv[2 * h + 1], hi, mid, lo);
            const uint32_t pl[3] = {hi, mid, lo};
#pragma unroll
            for (int q = 0; q < 3; ++q) {
              uint8_t* d0 = gp + q * GPL + (2 * h) * GPX + k * 32;
              *reinterpret_cast<uint16_t*>(d0) = (uint16_t)(pl[q] & 0xFFFFu);
              *reinterpret_cast<uint16_t*>(d0 + GPX) = (uint16_t)(pl[q] >> 16);
            }
          }
        }
      }
      // gw: B = g * D_j of the pixel pairs (4 g4 + 2 s, + 1), slots (j = 0, 1, 2, pad), against the ctx patch
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float d[8];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          d[j] = gv[2 * s] * r6_D(pw[2 * s], j, std_mask, cel);
          d[4 + j] = gv[2 * s + 1] * r6_D(pw[2 * s + 1], j, std_mask, cel);
        }
        d[3] = d[7] = 0.f;
        v8bf bh, bm, bl;
        split3x8(d, bh, bm, bl);
        const int poff = ohl * WP + ow0 + 2 * s;
        const uint2* xh = reinterpret_cast<const uint2*>(smem + O_XH);
        auto gw_fb = [&](auto fbc) {
          constexpr int fb = decltype(fbc)::value;
          const int ao = (int)((aoffp[fb >> 1] >> (16 * (fb & 1))) & 0xFFFFu) + poff;
          const uint2 a0 = xh[ao], a1 = xh[ao + 1];
          const v8bf a = as_v8bf(v4i{(int)a0.x, (int)a0.y, (int)a1.x, (int)a1.y});
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh, acc[fb], 0, 0, 0);
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm, acc[fb], 0, 0, 0);
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl, acc[fb], 0, 0, 0);
        };
        // (xbar 128: the 16-row blocks 0..7 are tile 0's, block 8 tile 1's)
        if (i == 0) {
          gw_fb(std::integral_constant<int, 0>{}); gw_fb(std::integral_constant<int, 1>{});
          gw_fb(std::integral_constant<int, 2>{}); gw_fb(std::integral_constant<int, 3>{});
          gw_fb(std::integral_constant<int, 4>{}); gw_fb(std::integral_constant<int, 5>{});
          gw_fb(std::integral_constant<int, 6>{}); gw_fb(std::integral_constant<int, 7>{});
        } else {
          gw_fb(std::integral_constant<int, 8>{});
        }
      }
    }
    __syncthreads();  // (B1) the G patch is complete; the patches' readers are done
    if (more) stage_store(r0 + R, xv);  // the next m-tile's patches (its phase A reads them after B4)
#ifndef CIMQ_EXP_R6_NO_XFPF
    float4 xf[2];  // the finished rows' x (act-LSQ backward), in flight behind the gx MFMAs
    {
      const int t = (int)threadIdx.x;
      const int cc = t & 127, part = t >> 7;
      const int c = cc >> 3, iw = 4 * (cc & 7);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int ih = part == 0 ? r0 - 1 + u : r0 + part;  // part 0: rows r0 - 1, r0; part p: row r0 + p
        xf[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((u == 0 || part == 0) && (unsigned)ih < (unsigned)H)
          xf[u] = *reinterpret_cast<const float4*>(x + ((b * C + c) * H + ih) * W + iw);
      }
    }
#endif
    if (DBG) {
      __syncthreads();
      gq = gqn;
      continue;
    }

    // ================= gx: partial rows per kernel row kh, G row ohl shifted by kw =================
    v4f gacc[3] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
    {
      const uint8_t* gb = smem + O_GP + ohl * GROW + (cw0 + r16 + 2) * GPX + 16 * g4;
      const v4i* wx = reinterpret_cast<const v4i*>(smem + O_WX) + lane;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        v8bf A[KSG][3];
#pragma unroll
        for (int s = 0; s < KSG; ++s)
#pragma unroll
          for (int q = 0; q < 3; ++q) A[s][q] = as_v8bf(*reinterpret_cast<const v4i*>(gb - kw * GPX + q * GPL + 64 * s));
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int p = 3 * kh + kw;
#pragma unroll
          for (int s = 0; s < KSG; ++s) {
            const v8bf bw = as_v8bf(wx[(p * KSG + s) * 64]);
#pragma unroll
            for (int q = 0; q < 3; ++q) gacc[kh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s][q], bw, gacc[kh], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // (B2) every wave is done with the G patch: the exchange reuses it
    // exchange: partial of input row r0 + ohl + kh - 1 from output row r0 + ohl, [c][iw] per (kh, ohl)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
      *reinterpret_cast<v4f*>(smem + O_GP + (kh * R + ohl) * GROW + GPX + (r16 * EXP + ow0) * 4) = gacc[kh];
    __syncthreads();  // (B3)
    {
      // finished input rows: r0 - 1 (with the carry) and r0 .. r0 + R - 2, and r0 + R - 1 on the last m-tile;
      // thread = (part, channel c, 4 columns): part 0 owns rows r0 - 1, r0 and the carry of its columns
      const int t = (int)threadIdx.x;
      const int cc = t & 127, part = t >> 7;
      const int c = cc >> 3, iw = 4 * (cc & 7);
      auto exr = [&](int kh, int rs) -> float4 {
        return *reinterpret_cast<const float4*>(smem + O_GP + (kh * R + rs) * GROW + GPX + (c * EXP + iw) * 4);
      };
      float4* ca = reinterpret_cast<float4*>(smem + O_CA);
      auto fin = [&](int ih, float4 v4, int u) {
        const int gi = ((b * C + c) * H + ih) * W + iw;
#ifndef CIMQ_EXP_R6_NO_XFPF
        const float4 xv4 = xf[u];
#else
        (void)u;
        const float4 xv4 = *reinterpret_cast<const float4*>(x + gi);
#endif
        const float xs[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
        const float vs[4] = {v4.x, v4.y, v4.z, v4.w};
        float o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gqv = vs[e] * scale;
          // autograd of round_pass(clamp(x/sa, 0, Qp)) * sa (lsq.py:549), as cim_bwd_gx5_kernel
          const float y1 = xs[e] / sa;
          const float clv = clamp_nan(y1, 0.f, g.lsq_qp);
          const float rr2 = rintf(clv);
          const float rp = (rr2 - clv) + clv;
          const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
          const float gy = pass ? gqv * sa : 0.f;
          o4[e] = pass ? gqv : 0.f;
          gsum += gqv * rp;
          gsum += -(gy * (y1 * inv_sa));
        }
        *reinterpret_cast<float4*>(gx + gi) = make_float4(o4[0], o4[1], o4[2], o4[3]);
      };
      auto add4 = [](float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); };
      if (part == 0) {
        const int ci = c * W + iw;
        if (n > 0) fin(r0 - 1, add4(exr(0, 0), ca[ci >> 2]), 0);
        float4 v0 = add4(exr(0, 1), exr(1, 0));
        if (n > 0) v0 = add4(v0, ca[(C * W + ci) >> 2]);
        fin(r0, v0, 1);
        if (more) {
          ca[ci >> 2] = add4(exr(1, R - 1), exr(2, R - 2));  // input row r0 + R - 1: kh 1 and 2
          ca[(C * W + ci) >> 2] = exr(2, R - 1);             // input row r0 + R: kh 2
        }
      } else if (part < R - 1) {
        fin(r0 + part, add4(add4(exr(0, part + 1), exr(1, part)), exr(2, part - 1)), 0);
      } else if (!more) {
        fin(r0 + R - 1, add4(exr(1, R - 1), exr(2, R - 2)), 0);
      }
    }
    __syncthreads();  // (B4) the exchange is read: the next m-tile's G writes may begin
    gq = gqn;
  }
  if (DBG) return;

  // ---- image epilogue: d sa partial, grad_w and grad_alpha slabs ----
  float* red = reinterpret_cast<float*>(smem + O_GP);
  for (int o = 32; o > 0; o >>= 1) gsum += __shfl_xor(gsum, o);
  if (lane == 0) red[wave] = gsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 8; ++w) t += red[w];
    gsa_part[b] = t;
  }
  __syncthreads();
  // grad_w: the 8 waves' partials of every 16-row block, summed in wave order
  v4f* gred = reinterpret_cast<v4f*>(smem + O_GP);  // [fb][wave][64]
#pragma unroll
  for (int fb = 0; fb < 9; ++fb) gred[(fb * 8 + wave) * 64 + lane] = acc[fb];
  __syncthreads();
  {
    const size_t rows = (size_t)g.T * g.FBT * 16;
    float* gws = gw_slab + (size_t)b * rows * g.Opad;
    for (int it = threadIdx.x; it < 9 * 64; it += blockDim.x) {
      const int fb = it >> 6, l = it & 63;
      v4f t = gred[(fb * 8) * 64 + l];
      for (int w = 1; w < 8; ++w) t += gred[(fb * 8 + w) * 64 + l];
      const int f0 = 16 * fb + 4 * (l >> 4), i = f0 / g.xbar;
      const size_t row0 = (size_t)i * g.FBT * 16 + (f0 - i * g.xbar);
#pragma unroll
      for (int r = 0; r < 4; ++r) gws[(row0 + r) * g.Opad + (l & 15)] = t[r];
    }
  }
  __syncthreads();
  // grad_alpha: the four lane groups, then the waves in order
  float* gar = reinterpret_cast<float*>(smem + O_GP);  // [wave][T][9][16]
#pragma unroll
  for (int i = 0; i < T; ++i)
#pragma unroll
    for (int kj = 0; kj < 9; ++kj) {
      float t = ga[i][kj];
      t = rows4_sum(t);
      if (g4 == 0) gar[((wave * T + i) * 9 + kj) * 16 + r16] = t;
    }
  __syncthreads();
  for (int it = threadIdx.x; it < T * 9 * 16; it += blockDim.x) {
    const int o = it & 15, q = it >> 4;  // q = i * 9 + kj
    float t = 0.f;
    for (int w = 0; w < 8; ++w) t += gar[(w * T * 9 + q) * 16 + o];
    ga_slab[((size_t)b * g.T * 9 + q) * g.Opad + o] = t;
  }
}
#endif  // CIMQ_TU_R6

}  // namespace cimq

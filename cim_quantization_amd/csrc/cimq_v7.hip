// cimq_v7.hip -- the backward of the CiM conv (lsq.py:244-386) from compact state words.
//
// The forward (cim_fwd_v3_kernel<.., CST = true>) leaves one uint32 per (tile i, output
// pixel m, channel o): for every slice pair (k, j) the STE pass bit (lsq.py:310-313) and the
// ADC code (lsq.py:321-332) of that partial sum, 3 bits at 3*(k*nba + j).  Two kernels
// consume them:
//
//  * cim_bwd_gx_v8_kernel -- grad_x as the UNFOLDED product, folded without atomics:
//      gx_unf[m, f] = sum_kappa W_i[f, kappa] * G_i[m, kappa],  kappa = (k, o),
//      G_i[m, (k, o)] = g[m, o] * sum_j cE_kj * pass_ijk[m, o]       (cE = mask * 2^-bsa*j)
//    on v_mfma_f32_16x16x32_bf16 with G split hi/mid/lo (fp32-exact products: W is a small
//    integer).  The lane that reads the state words of pixel m (its MFMA column) for four
//    consecutive channels IS the B-operand lane of (m, 8 kappa) -- G is built in registers,
//    never staged.  The rows f are ordered (c, kh, kw), so the nn.Fold adjoint along kw is
//    three DPP lane shifts in registers, and along kh a pass over an LDS ring of output rows
//    in which every value is written by exactly one lane; that pass also applies the fused
//    LSQ activation backward (lsq.py:549).
//  * cim_bwd_gw_v7_kernel -- grad_w (+ grad_alpha_cim partials) as a weight-gradient conv:
//      gw[(c, kh, kw), o] = sum_j sum_m xhat_j[c, ih(m, kh), iw(m, kw)] * g[m, o] * D_ij[m, o]
//    with D_ij = sum_k cD_kj * pass_ijk, i = tile of (c, kh, kw).  K = 32 output pixels per
//    MFMA: the lane holding channel o and 8 consecutive pixels builds g * D_j in registers
//    (B operand), and the activation slices come from LDS planes [j][kw][c][row][ow] that
//    hold the kw-shifted (and stride-decimated) input rows, so every A fragment is one
//    aligned 16-byte read.  grad_alpha partials sum code * g over the lane's 8 pixels.
//
// Both replace the state-word (16-bit per (i, k, quad, o)) kernels of cimq_kernels_v3.hip /
// cimq_gx_v6.hip on layers the v7 plan accepts (host: v7_plan in cimq_api.hip).
#pragma once
#include <type_traits>

#include "cimq_kernels_v3.hip"
#include "cimq_lsq_dev.h"

#ifndef CIMQ_FOLD_XB
#define CIMQ_FOLD_XB 1  // the grad_x folds' elements per thread and round (cimq_v7 / cimq_fused)
#endif

namespace cimq {

struct V7 {
  int lw;       // log2(Wo)
  // grad_x (v8: ring fold)
  int NCPBT;    // (c, kh)-row blocks of 4 per tile (wcy operand)
  int SWD;      // segment width: min(16, Wo) output columns per 16-lane MFMA column group
  int NSEG;     // segments per output row
  int NRS;      // output rows per step (64 pixels)
  int RSLOT;    // ring rows (NRS + 2)
  int NPART;    // waves sharing one pixel group (split over (c, kh)-blocks)
  int lwin, lcin;  // log2(W), log2(C) (the v7 path takes power-of-two W and C)
  // grad_x
  int RB;       // input rows owned by one block
  int nbands;   // bands per image
  int FBX;      // f-blocks per tile (FBT)
  // grad_w
  int NSLOT;    // staged input rows per 128-pixel stage
  int CPITCH;   // plane channel pitch (bf16 elements)
  int nstage;   // 128-pixel stages per chunk
  int nchunks;  // pixel chunks
  int whole;    // 1: a stage is 128/P whole images; 0: a stage is 128/Wo rows of one image
  int CPL;      // channels per staged plane: min(16, C)
  int NTL;      // most crossbar tiles touching one 16-channel block (grad_alpha LDS regions)
  int GSH;      // grad_x, NPART > 1, at most 2 o-blocks: the NPART waves of a pixel group build disjoint G chunks and
                // exchange them through LDS (else every wave builds all of them)
  int KWP;      // grad_w: (slice j, kw) plane pitch (bf16 elements, >= CPL * CPITCH; gw_pitches)
};

// pass-bit masks of the state word: all j of slice k / all k of slice j
__host__ __device__ constexpr uint32_t pass_mask_k(int k, int nba) {
  uint32_t m = 0;
  for (int j = 0; j < nba; ++j) m |= 1u << (3 * (k * nba + j));
  return m;
}
__host__ __device__ constexpr uint32_t pass_mask_j(int j, int nbw, int nba) {
  uint32_t m = 0;
  for (int k = 0; k < nbw; ++k) m |= 1u << (3 * (k * nba + j));
  return m;
}

// uniform (scalar-register) copies of values every lane computed identically
__device__ inline float sgpr_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ inline uint64_t sgpr_u64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

// lane l <- lane l+1 / l-1 of the same 16-lane row (0 past the row's end)
__device__ inline float dpp_from_next(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xF, 0xF, true));
}
__device__ inline float dpp_from_prev(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, true));
}

// ---------------------------------------------------------------------------------------
// grad_x, v8: unfolded product with the (c, kh, kw) rows ordered so that the nn.Fold adjoint
// along kw is three DPP lane shifts, and along kh a pass over a ring of output rows in LDS.
// stride 1, 3x3, pad 1 (v7_plan).  Block = image b, band of RB input rows; a step = 64 output
// pixels (4 MFMA column groups, one per wave), NRS output rows.  Per step and tile i:
//   y[(c, kh), iw] = sum_kw gx_unf[(c, kh, kw), ow = iw + 1 - kw]        (registers + DPP)
// goes to ring[row][segment][(c, kh)][col]; after the step, the input rows whose three
// contributing output rows are done are folded along kh, scaled, run through the LSQ act
// backward and stored -- no atomics, every value written by exactly one lane.
// ---------------------------------------------------------------------------------------
// NPART waves share one pixel group, each owning the (c, kh)-blocks cb = part (mod NPART): more
// waves per image for small images, every ring value still written by exactly one lane.
template <int NBW, int NBA, int OBX, bool LSQ, int SS, int NPART>
__global__ __launch_bounds__(256 * NPART) void cim_bwd_gx_v8_kernel(Geo g, V7 v, const uint32_t* __restrict__ st,
                                                            const v4i* __restrict__ wcy, Params pp,
                                                            const float* __restrict__ sw_p,
                                                            const float* __restrict__ sa_p,
                                                            const float* __restrict__ gout,
                                                            const float* __restrict__ x, float* __restrict__ gx,
                                                            float* __restrict__ gsa_part) {
  constexpr int NKS = (NBW * OBX + 1) / 2;
  constexpr int NKJ = NBW * NBA;
  constexpr bool PLS = NKJ > 10;  // plane state words (cim_fwd_v3_kernel PLF)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int bid = (int)blockIdx.x;
  const int b = bid / v.nbands, band = bid - b * v.nbands;
  const int r0 = band * v.RB, r1 = min(g.H, r0 + v.RB);
  // output rows whose windows touch input rows [r0, r1) (pad 1, 3 kernel rows, stride SS)
  const int oh_lo = max(0, (r0 + 1 - 2 + SS - 1) / SS), oh_hi = min(g.Ho - 1, (r1 - 1 + 1) / SS);
  const int nsteps = (oh_hi - oh_lo + v.NRS) / v.NRS;
  const int CPP = g.C * 3;
  const int RE = SS * v.SWD + 2;  // ring entry: input columns -1 .. SS*SWD (local), + pad
  // index math by shifts (SWD = min(16, Wo), a power of two) and ring rows by a multiply-shift
  // modulo (exact for the < 4096 relative rows of a band)
  const int lsw = v.lw < 4 ? v.lw : 4;
  const int rinv = (65536 + v.RSLOT - 1) / v.RSLOT;
  auto ring_row = [&](int x) { return x - ((x * rinv) >> 16) * v.RSLOT; };
  const int rrow = v.NSEG * CPP * RE;  // floats per ring row
  float* ring = reinterpret_cast<float*>(smem);
  float* cel = ring + (size_t)v.RSLOT * rrow;
  float* red = cel + 64;
  // G exchange (GSH): [pixel group][chunk s][hi, mid, lo][64 lanes] 16-byte operands
  v4i* gsh = reinterpret_cast<v4i*>(red + 64);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  const int Wo = 1 << v.lw;
  for (int t = threadIdx.x; t < NKJ; t += blockDim.x) cel[t] = pp.ckj[NKJ + t];
  __syncthreads();
  // standard binary masks (_quan_base.py:207-214), checked once per block: the plain mask
  // (cE_kj = 2^(bsw*k) for every j) gives E_k = 2^(bsw*k) * popcount(pass bits of slice k);
  // the int8-wrapped 8-bit mask (plane words) cE_kj = 2^k for j + k < 7, -2^k at j + k = 7 and
  // 0 beyond gives E_k = 2^k * (popcount(pass bits j < 7 - k) - pass bit j = 7 - k).  Both are
  // exact (small integers times a power of two); any other mask takes the per-pair sum.
  bool std_mask;
  {
    const int kl = lane < NKJ ? lane / NBA : 0, jl = lane < NKJ ? lane - kl * NBA : 0;
    const float ce = PLS ? ((kl + jl < 7) ? ldexpf(1.f, kl) : (kl + jl == 7 ? -ldexpf(1.f, kl) : 0.f))
                         : ldexpf(1.f, g.bsw * kl);
    std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cel[lane < NKJ ? lane : 0] != ce) == 0ull;
    if (PLS && (NBW != 8 || NBA != 8)) std_mask = false;
  }
  const float scale = sw / (float)NBA;
  const float inv_sa = 1.f / sa;
  float gpart = 0.f;
  int done = r0 - 1;
  for (int step = 0; step < nsteps; ++step) {
    const int oh_s = oh_lo + step * v.NRS, oh_e = min(oh_hi, oh_s + v.NRS - 1);
    const int q = 16 * (wave & 3) + r16;
    const int part = wave >> 2;
    const int oh = oh_s + (q >> v.lw), ow = q & (Wo - 1);
    const bool pv = oh <= oh_e;
    const int pimg = (oh << v.lw) + ow;
    const size_t m = (size_t)b * g.P + pimg;
    const int seg = ow >> lsw, col = ow & (v.SWD - 1);
    float* rr = ring + (size_t)ring_row(oh - oh_lo) * rrow + seg * CPP * RE;
    float gv[OBX][4];
#pragma unroll
    for (int ob = 0; ob < OBX; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = ob * 16 + 4 * g4 + r;
        gv[ob][r] = pv ? (g.onchw ? gout[((size_t)b * g.O + o) * g.P + pimg] : gout[m * g.O + o]) : 0.f;
      }
    for (int i = 0; i < g.T; ++i) {
      // state words of this lane's pixel, channels 4*g4 .. +3 of each o-block: interleaved
      // (3 bits per slice pair) or, for more than 10 pairs, the 64-bit pass plane
      uint32_t sv[OBX][4];
      uint64_t sp[OBX][4];
#pragma unroll
      for (int ob = 0; ob < OBX; ++ob) {
        if constexpr (PLS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            uint2 w2 = make_uint2(0u, 0u);
            if (pv) w2 = reinterpret_cast<const uint2*>(st)[(((size_t)i * g.M + m) * g.O + ob * 16 + 4 * g4 + r) * 3];
            sp[ob][r] = (uint64_t)w2.x | ((uint64_t)w2.y << 32);
            sv[ob][r] = 0u;
          }
        } else {
          uint4 s4 = make_uint4(0u, 0u, 0u, 0u);
          if (pv) s4 = *reinterpret_cast<const uint4*>(st + ((size_t)i * g.M + m) * g.O + ob * 16 + 4 * g4);
          sv[ob][0] = s4.x; sv[ob][1] = s4.y; sv[ob][2] = s4.z; sv[ob][3] = s4.w;
#pragma unroll
          for (int r = 0; r < 4; ++r) sp[ob][r] = 0ull;
        }
      }
      v8bf Gh[NKS], Gm[NKS], Gl[NKS];
      // (not for 4 o-blocks: its 6 chunks already fill the register budget, the exchange spills)
      const bool share = NPART > 1 && OBX <= 2 && v.GSH;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (share && s % NPART != part) continue;  // built by another wave of this pixel group
        float Gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int kb = 2 * s + (e >> 2), r = e & 3;
          Gv[e] = 0.f;
          if (kb < NBW * OBX) {
            const int k = kb / OBX, ob = kb - k * OBX;
            float E;
            if constexpr (PLS) {
              const uint32_t fld = (uint32_t)(sp[ob][r] >> (k * NBA)) & ((1u << NBA) - 1u);
              if (std_mask) {
                const int n = __popc(fld & ((1u << (7 - k)) - 1u)) - (int)((fld >> (7 - k)) & 1u);
                E = (float)(n * (1 << k));
              } else {
                E = 0.f;
#pragma unroll 1
                for (int j = 0; j < NBA; ++j) E += ((fld >> j) & 1u) ? cel[k * NBA + j] : 0.f;
              }
            } else if (std_mask) {
              E = ldexpf((float)__popc(sv[ob][r] & pass_mask_k(k, NBA)), g.bsw * k);
            } else {
              E = 0.f;
#pragma unroll
              for (int j = 0; j < NBA; ++j) E += ((sv[ob][r] >> (3 * (k * NBA + j))) & 1u) ? cel[k * NBA + j] : 0.f;
            }
            Gv[e] = gv[ob][r] * E;
          }
        }
        split3x8(Gv, Gh[s], Gm[s], Gl[s]);
      }
      if (share) {
        // every wave of the pixel group (same lanes, same pixels) publishes its chunks and
        // takes the others'; the second barrier keeps the next tile's writes behind the reads
        v4i* gq = gsh + (size_t)(wave & 3) * NKS * 3 * 64 + lane;
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
          if (s % NPART != part) continue;
          gq[(s * 3 + 0) * 64] = as_v4i(Gh[s]);
          gq[(s * 3 + 1) * 64] = as_v4i(Gm[s]);
          gq[(s * 3 + 2) * 64] = as_v4i(Gl[s]);
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
          if (s % NPART == part) continue;
          Gh[s] = as_v8bf(gq[(s * 3 + 0) * 64]);
          Gm[s] = as_v8bf(gq[(s * 3 + 1) * 64]);
          Gl[s] = as_v8bf(gq[(s * 3 + 2) * 64]);
        }
        __syncthreads();
      }
      const int cp_lo = (i * g.xbar) / 3, cp_hi = (min(g.K, (i + 1) * g.xbar) - 1) / 3;
      const int cpb_lo = cp_lo >> 2, ncb = (cp_hi >> 2) - cpb_lo + 1;
      const bool shared_first = i > 0 && cpb_lo == (((i * g.xbar - 1) / 3) >> 2);
      const v4i* wt = wcy + (size_t)i * v.NCPBT * NKS * 64 + lane;
      // this wave's (c, kh)-blocks of tile i: cb = cb0, cb0 + NPART, ...; the operand
      // fragments of the next block are loaded while the current block's MFMAs run
      const int cb0 = (NPART == 1) ? 0 : ((part - cpb_lo % NPART) + NPART) % NPART;
      v4i anx[NKS];
      if (cb0 < ncb) {
#pragma unroll
        for (int s = 0; s < NKS; ++s) anx[s] = wt[(cb0 * NKS + s) * 64];
      }
#pragma unroll 1
      for (int cb = cb0; cb < ncb; cb += NPART) {
        {
          v4i acur[NKS];
#pragma unroll
          for (int s = 0; s < NKS; ++s) acur[s] = anx[s];
          if (cb + NPART < ncb) {
#pragma unroll
            for (int s = 0; s < NKS; ++s) anx[s] = wt[((cb + NPART) * NKS + s) * 64];
          }
          v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NKS; ++s) {
            const v8bf a = as_v8bf(acur[s]);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gh[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gm[s], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, Gl[s], acc, 0, 0, 0);
          }
          // acc[kw] = gx_unf[(cp, kw)][this lane's pixel], cp = (cpb_lo + cb)*4 + g4; pixel ow
          // feeds input column SS*ow + kw - 1
          float fn = dpp_from_next(acc[0]);  // kw = 0 of pixel ow + 1
          if (col == v.SWD - 1) fn = 0.f;
          const int cp = (cpb_lo + cb) * 4 + g4;
          const bool acc_mode = cb == 0 && shared_first;
          if (SS == 1) {
            float fp = dpp_from_prev(acc[2]);  // kw = 2 of pixel ow - 1 -> iw = ow
            if (col == 0) fp = 0.f;
            const float y = (acc[1] + fn) + fp;
            if (pv && cp < CPP) {
              float* e = rr + cp * RE;
              if (acc_mode) {
                e[col + 1] += y;
                if (col == 0) e[0] += acc[0];
                if (col == v.SWD - 1) e[v.SWD + 1] += acc[2];
              } else {
                e[col + 1] = y;
                if (col == 0) e[0] = acc[0];
                if (col == v.SWD - 1) e[v.SWD + 1] = acc[2];
              }
            }
          } else {
            // stride 2: even column 2ow <- kw 1; odd column 2ow + 1 <- kw 2 of ow, kw 0 of ow + 1
            const float ye = acc[1], yo = acc[2] + fn;
            if (pv && cp < CPP) {
              float* e = rr + cp * RE;
              if (acc_mode) {
                e[2 * col + 1] += ye;
                e[2 * col + 2] += yo;
                if (col == 0) e[0] += acc[0];
              } else {
                e[2 * col + 1] = ye;
                e[2 * col + 2] = yo;
                if (col == 0) e[0] = acc[0];
              }
            }
          }
        }
      }
    }
    __syncthreads();
    // fold along kh the input rows whose contributing output rows are all in the ring
    // input row ih is complete once floor((ih + 1) / SS) <= oh_e
    const int upto = (oh_e == g.Ho - 1) ? g.H - 1 : (oh_e + 1) * SS - 2;
    const int f0 = max(done + 1, r0), f1 = min(upto, r1 - 1);
    if (f1 >= f0) {
      const int nf = (f1 - f0 + 1) * g.C * g.W;
      // CIMQ_FOLD_XB elements per thread and round, their x loads issued together ahead of the sums
      auto fidx = [&](int t) {
        const int iw = t & (g.W - 1), rest = t >> v.lwin;
        const int c = v.lcin >= 0 ? (rest & (g.C - 1)) : rest % g.C;
        const int ih = f0 + (v.lcin >= 0 ? (rest >> v.lcin) : rest / g.C);
        return (((size_t)b * g.C + c) * g.H + ih) * g.W + iw;
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
        const int iw = t & (g.W - 1), rest = t >> v.lwin;  // power-of-two W (v7_plan)
        const int c = v.lcin >= 0 ? (rest & (g.C - 1)) : rest % g.C;
        const int ih = f0 + (v.lcin >= 0 ? (rest >> v.lcin) : rest / g.C);
        const int sg = iw >> (lsw + SS - 1), cl = iw & (SS * v.SWD - 1);
        float a = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int oo2 = ih + 1 - kh;  // = SS * oh
          const int oo = oo2 / SS;
          if (oo2 >= 0 && oo * SS == oo2 && oo >= oh_lo && oo <= oh_e) {
            const float* e = ring + (size_t)ring_row(oo - oh_lo) * rrow + (c * 3 + kh) * RE;
            a += e[sg * CPP * RE + cl + 1];
            if (cl == SS * v.SWD - 1 && sg + 1 < v.NSEG) a += e[(sg + 1) * CPP * RE];
            if (SS == 1 && cl == 0 && sg > 0) a += e[(sg - 1) * CPP * RE + v.SWD + 1];
          }
        }
        const size_t gi = (((size_t)b * g.C + c) * g.H + ih) * g.W + iw;
        const float gqv = a * scale;
        if (LSQ) {
          // autograd of round_pass(clamp(x/sa, 0, Qp)) * sa (lsq.py:549), as cim_bwd_gx_v6_kernel
          const float xv = xb[u];
          const float y1 = xv / sa;
          const float clv = clamp_nan(y1, 0.f, g.lsq_qp);
          const float rr2 = rintf(clv);
          const float rp = (rr2 - clv) + clv;
          const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
          const float gy = pass ? gqv * sa : 0.f;
          // (gqv * sa) / sa and y1 / sa only feed gradients (within the 1e-5 bar, one rounding
          // apart); y1 itself stays an IEEE division: it decides the clamp mask and rint
          gx[gi] = pass ? gqv : 0.f;
          gpart += gqv * rp;
          gpart += -(gy * (y1 * inv_sa));
        } else {
          gx[gi] = gqv;
        }
      }
      }
      done = f1;
    }
    __syncthreads();
  }
  if (LSQ) {
    for (int o = 32; o > 0; o >>= 1) gpart += __shfl_xor(gpart, o);
    if (lane == 0) red[wave] = gpart;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < 4 * NPART; ++w) t += red[w];
      gsa_part[bid] = t;
    }
  }
}

// ---------------------------------------------------------------------------------------
// grad_w + grad_alpha_cim partials
// ---------------------------------------------------------------------------------------
// block = (pixel chunk, (channel block cb, output block ob)); a chunk is nstage stages of 128
// output pixels; in a stage wave w owns the 32 pixels 32w..32w+31 (one MFMA K-step).
// stride 1 (v7_plan); at most 3 crossbar tiles touch one 16-channel block.
// ctx slice bytes of one input element: NBP = 4 (uint32) or 8 (uint2) bytes, slice j in byte j
__device__ inline uint32_t xbyte(uint32_t w, int j) { return (w >> (8 * j)) & 0xFFu; }
__device__ inline uint32_t xbyte(uint2 w, int j) { return (j < 4 ? (w.x >> (8 * j)) : (w.y >> (8 * (j - 4)))) & 0xFFu; }
template <typename XW>
__device__ inline XW xzero();
template <>
__device__ inline uint32_t xzero<uint32_t>() { return 0u; }
template <>
__device__ inline uint2 xzero<uint2>() { return make_uint2(0u, 0u); }
// n consecutive elements from a 16-B aligned source by 16-B loads
template <int N>
__device__ inline void xload(const uint32_t* src, uint32_t* d) {
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const uint4 t = reinterpret_cast<const uint4*>(src)[q];
    d[4 * q] = t.x; d[4 * q + 1] = t.y; d[4 * q + 2] = t.z; d[4 * q + 3] = t.w;
  }
}
template <int N>
__device__ inline void xload(const uint2* src, uint2* d) {
#pragma unroll
  for (int q = 0; q < N / 2; ++q) {
    const uint4 t = reinterpret_cast<const uint4*>(src)[q];
    d[2 * q] = make_uint2(t.x, t.y); d[2 * q + 1] = make_uint2(t.z, t.w);
  }
}

template <int NBW, int NBA, int SS>
__global__ __launch_bounds__(256, 2) void cim_bwd_gw_v7_kernel(Geo g, V7 v, const uint32_t* __restrict__ st,
                                                            const uint8_t* __restrict__ xcb, Params pp,
                                                            const float* __restrict__ gout,
                                                            float* __restrict__ gw_slab,
                                                            float* __restrict__ ga_slab) {
  constexpr int NKJ = NBW * NBA;
  constexpr bool PLS = NKJ > 10;  // plane state words (cim_fwd_v3_kernel PLF)
  constexpr int NGR = PLS ? 2 : 9;  // row groups of 16 per channel block (w8a8 plan: C*KHW <= 32)
  typedef typename std::conditional<(NBA > 4), uint2, uint32_t>::type XW;  // ctx slice bytes (NBP)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int chunk = blockIdx.x, pair = blockIdx.y;
  const int CPL = v.CPL, NTL = v.NTL;
  const int cb = pair / g.OB16, ob = pair - cb * g.OB16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int Wo = 1 << v.lw;
  const int KHW = g.KHW;
  const int o = ob * 16 + r16;   // this lane's output channel (B column)
  const int ca = cb * 16 + r16;  // this lane's input channel (A row)
  // tiles touching this channel block; grad_alpha of tile i is owned by the block of the
  // channel block holding the tile's first row
  const int i_lo = (cb * 16 * KHW) / g.xbar;
  const int i_hi = (min(g.C, cb * 16 + 16) * KHW - 1) / g.xbar;
  const int ntl = i_hi - i_lo + 1;

  const size_t plane = (size_t)v.KWP;  // one (j, kw) plane, bf16 elements (padded: gw_pitches)
  uint8_t* cur = smem;
  __bf16* pl = reinterpret_cast<__bf16*>(cur); { const size_t pb = (size_t)NBA * 3 * plane * 2; cur += al16(pb > 36864 ? pb : (size_t)36864); }
  float* cdl = reinterpret_cast<float*>(cur); cur += 64 * 4;
  float* red = reinterpret_cast<float*>(cur);  // [4 waves][NTL][NKJ][16] grad_alpha partials
  for (int t = threadIdx.x; t < NKJ; t += blockDim.x) cdl[t] = pp.ckj[2 * NKJ + t];
  // the 8-element pad after the staged rows of each slice j's first plane (kw 0, channel 0) stays
  // zero: A fragments of rows past C or of kernel rows outside the image read it, so one address
  // select per row group replaces a select per fragment register
  const int zoff = v.CPITCH - 8;
  if (threadIdx.x < NBA)
    *reinterpret_cast<uint4*>(pl + (size_t)threadIdx.x * 3 * plane + zoff) = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  // standard binary masks, as cim_bwd_gx_v8_kernel, now summed over k for each a-slice j: the
  // plain mask (cD_kj = 2^(bsa*j)) gives D_j = 2^(bsa*j) * popcount(pass bits of slice j); the
  // int8-wrapped 8-bit mask (cD_kj = 2^j for k < 7 - j, -2^j at k = 7 - j, 0 beyond) gives
  // D_j = 2^j * (popcount(pass bits k < 7 - j) - pass bit k = 7 - j).  Else the per-pair sum.
  bool std_mask;
  {
    const int kl = lane < NKJ ? lane / NBA : 0, jl = lane < NKJ ? lane - kl * NBA : 0;
    const float ce = PLS ? ((kl + jl < 7) ? ldexpf(1.f, jl) : (kl + jl == 7 ? -ldexpf(1.f, jl) : 0.f))
                         : ldexpf(1.f, g.bsa * jl);
    std_mask = __builtin_amdgcn_ballot_w64(lane < NKJ && cdl[lane < NKJ ? lane : 0] != ce) == 0ull;
    if (PLS && (NBW != 8 || NBA != 8)) std_mask = false;
  }
  // pairs with a nonzero mask (grad_alpha of the others is 0 * sum = 0)
  const uint64_t live = __builtin_amdgcn_ballot_w64(lane < NKJ && cdl[lane < NKJ ? lane : 0] != 0.f);

  // A rows: 16 consecutive weight rows f per MFMA row group -- f = cb*16*KHW + 16*gr + (lane & 15),
  // f = (c, kh, kw) -- so a crossbar tile's rows of this channel block take ceil(rows / 16) groups
  // (tile boundaries are multiples of 16 here: xbar and 16*KHW are).  Per lane and group: the
  // plane offset of its row's (kw, channel) times 4 plus kh, or -1 past C; per group: its tile.
  int gpk[NGR], gtile[NGR];
#pragma unroll
  for (int gr = 0; gr < NGR; ++gr) {
    const int f0 = cb * 16 * KHW + 16 * gr, f = f0 + r16;
    const int c = f / KHW, tap = f - c * KHW, kh = tap / 3, kw = tap - 3 * kh;
    gpk[gr] = (c < g.C) ? ((kw * v.KWP + (c - cb * 16) * v.CPITCH) << 2) | kh : -1;
    gtile[gr] = (f0 < g.C * KHW) ? f0 / g.xbar : -1;
  }
  (void)ca;

  v4f acc[NGR];
#pragma unroll
  for (int tp = 0; tp < NGR; ++tp) acc[tp] = v4f{0.f, 0.f, 0.f, 0.f};
  // grad_alpha partials accumulate in LDS, one region per wave: red[wave][tl][kj][16 o]
  for (int t = threadIdx.x; t < 4 * NTL * NKJ * 16; t += blockDim.x) red[t] = 0.f;

  // Software pipeline over the chunk's stages: the global loads of stage n+1 (source words of
  // the staged rows, state words and grad_out of this lane's K-step) are issued before the
  // MFMA work of stage n, so their latency hides behind it.
  const int ng8 = Wo >> 3;
  const int nit = CPL * v.NSLOT * ng8;  // staging items (<= 2 per thread, v7_plan)
  struct Pref {
    XW w[2][10];
  };
  // a stage's first pixel m0 = 128 s (M < 2^31): image b0 and, when a stage is part of one image,
  // its first staged input row; per-thread staging items are stage-invariant (decomposed once)
  auto stage_geom = [&](int stg, int& b0, int& ih_first) {
    const unsigned m0 = (unsigned)(chunk * v.nstage + stg) * 128u;
    b0 = (int)(m0 / (unsigned)g.P);
    const int pim0 = (int)(m0 - (unsigned)b0 * (unsigned)g.P);
    ih_first = v.whole ? 0 : (pim0 >> v.lw) * SS - g.PH;
  };
  int it_cl[2], it_db[2], it_ih[2], it_c8[2];
#pragma unroll
  for (int u2 = 0; u2 < 2; ++u2) {
    const int it = threadIdx.x + u2 * 256;
    const int cl = it / (v.NSLOT * ng8), rem = it - cl * (v.NSLOT * ng8);
    const int slot = rem >> (v.lw - 3), c8 = rem & (ng8 - 1);
    it_cl[u2] = cl;
    it_c8[u2] = c8;
    it_db[u2] = v.whole ? slot / g.H : 0;
    it_ih[u2] = v.whole ? slot - it_db[u2] * g.H : slot;
  }
  auto load = [&](int stg, Pref& pf) {
    if (SS != 1) return;  // stride 2 stages without prefetch (17 source words per item)
    int b0, ih_first;
    stage_geom(stg, b0, ih_first);
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2) {
      const int it = threadIdx.x + u2 * 256;
#pragma unroll
      for (int u = 0; u < 10; ++u) pf.w[u2][u] = xzero<XW>();
      if (it < nit) {
        const int cl = it_cl[u2], c8 = it_c8[u2];
        const int b = b0 + it_db[u2], ih = ih_first + it_ih[u2];
        const int c = cb * 16 + cl;
        if (c < g.C && ih >= 0 && ih < g.H && b < g.B) {
          const XW* src = reinterpret_cast<const XW*>(xcb) + (((size_t)b * g.C + c) * g.H + ih) * g.W + c8 * 8;
          xload<8>(src, &pf.w[u2][1]);
          if (c8 > 0) pf.w[u2][0] = src[-1];
          if (c8 * 8 + 8 < g.W) pf.w[u2][9] = src[8];
        }
      }
    }
  };

  // stride 2 keeps the per-stage LDS reduction: the registers would cost it a wave per SIMD
  constexpr bool RGQ = !PLS && SS == 1;
  constexpr int NGQ = RGQ ? NKJ : 1;
  float gq0[NGQ], gq1[NGQ];  // grad_alpha partials of tiles i_lo, i_lo + 1 (this lane's pixels)
#pragma unroll
  for (int kj = 0; kj < NGQ; ++kj) gq0[kj] = gq1[kj] = 0.f;
  Pref pf;
  load(0, pf);
  for (int stg = 0; stg < v.nstage; ++stg) {
    int b0, ih_first;
    stage_geom(stg, b0, ih_first);
    // this wave's K-step: pixels mk .. mk+31; this lane's 8 pixels mk8 .. mk8+7 (one row).  Its
    // grad_out and the state words of the first two tiles are loaded here, ahead of the staging,
    // so that their latency hides behind it
    const size_t mk8 = ((size_t)chunk * v.nstage + stg) * 128 + 32 * wave + 8 * g4;
    const bool kvalid = mk8 < (size_t)g.M;
    // image and in-image pixel: a stage lies in one image, or (whole) spans 128 / P images of a
    // power-of-two P
    int b = b0, pimg;
    {
      const int moff = 32 * wave + 8 * g4;
      if (v.whole) {
        const int lp = __builtin_ctz(g.P);
        b = b0 + (moff >> lp);
        pimg = moff & (g.P - 1);
      } else {
        pimg = (int)((unsigned)(chunk * v.nstage + stg) * 128u - (unsigned)b0 * (unsigned)g.P) + moff;
      }
    }
    const int oh = pimg >> v.lw, ow0 = pimg & (Wo - 1);
    float gv[8];
    uint32_t sv0[8], sv1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { gv[e] = 0.f; sv0[e] = sv1[e] = 0u; }
    if (kvalid) {
      if (g.onchw) {
        const float4* gp = reinterpret_cast<const float4*>(gout + ((size_t)b * g.O + o) * g.P + pimg);
        const float4 a0 = gp[0], a1 = gp[1];
        gv[0] = a0.x; gv[1] = a0.y; gv[2] = a0.z; gv[3] = a0.w;
        gv[4] = a1.x; gv[5] = a1.y; gv[6] = a1.z; gv[7] = a1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = gout[(mk8 + e) * g.O + o];
      }
      if (!PLS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sv0[e] = st[((size_t)i_lo * g.M + mk8 + e) * g.O + o];
        if (ntl > 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sv1[e] = st[((size_t)(i_lo + 1) * g.M + mk8 + e) * g.O + o];
        }
      }
    }
    __syncthreads();
    if (SS == 2) {
      // stride 2: output column ow reads input column 2 ow + kw - 1 -> 17 words per 8 columns
      for (int it = threadIdx.x; it < nit; it += blockDim.x) {
        const int cl = it / (v.NSLOT * ng8), rem = it - cl * (v.NSLOT * ng8);
        const int slot = rem / ng8, c8 = rem - slot * ng8;
        int b = b0, ih = ih_first + slot;
        if (v.whole) { b = b0 + slot / g.H; ih = slot - (slot / g.H) * g.H; }
        const int c = cb * 16 + cl;
        XW wv[17];
#pragma unroll
        for (int u = 0; u < 17; ++u) wv[u] = xzero<XW>();
        if (c < g.C && ih >= 0 && ih < g.H && b < g.B) {
          const XW* src = reinterpret_cast<const XW*>(xcb) + (((size_t)b * g.C + c) * g.H + ih) * g.W + c8 * 16;
          xload<16>(src, &wv[1]);
          if (c8 > 0) wv[0] = src[-1];
        }
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
          for (int j = 0; j < NBA; ++j) {
            uint32_t pk[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const float f0 = (float)(int8_t)xbyte(wv[4 * e2 + kw], j);
              const float f1 = (float)(int8_t)xbyte(wv[4 * e2 + 2 + kw], j);
              pk[e2] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
            }
            __bf16* dst = pl + (size_t)(j * 3 + kw) * plane + cl * v.CPITCH + slot * Wo + c8 * 8;
            *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          }
        }
      }
    }
    // bf16 planes of the staged rows: item (channel cl, slot, 8-column group), kw shifts
#pragma unroll
    for (int u2 = 0; u2 < 2; ++u2) {
      if (SS != 1) break;
      const int it = threadIdx.x + u2 * 256;
      if (it < nit) {
        const int cl = it_cl[u2], c8 = it_c8[u2];
        const int slot = v.whole ? it_db[u2] * g.H + it_ih[u2] : it_ih[u2];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
          for (int j = 0; j < NBA; ++j) {
            uint32_t pk[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
              const float f0 = (float)(int8_t)xbyte(pf.w[u2][2 * e2 + kw], j);
              const float f1 = (float)(int8_t)xbyte(pf.w[u2][2 * e2 + 1 + kw], j);
              pk[e2] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);  // exact bf16
            }
            __bf16* dst = pl + (size_t)(j * 3 + kw) * plane + cl * v.CPITCH + slot * Wo + c8 * 8;
            *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          }
        }
      }
    }
    __syncthreads();
    if (stg + 1 < v.nstage) load(stg + 1, pf);
    if (!kvalid) continue;
    // row slot of each kernel row for this lane's output row (-1: outside the image)
    int slot_kh[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * SS - g.PH + kh;
      int sl = -1;
      if (ih >= 0 && ih < g.H) sl = v.whole ? (b - b0) * g.H + ih : ih - ih_first;
      slot_kh[kh] = sl;
    }
#pragma unroll 1
    for (int tl = 0; tl < 3; ++tl) {
      if (PLS && tl < ntl) {
        // plane state words: grad_alpha from the code planes, then one slice j at a time
        const int i = i_lo + tl;
        const uint2* s2 = reinterpret_cast<const uint2*>(st) + ((size_t)i * g.M + mk8) * g.O * 3 + (size_t)o * 3;
        const size_t es = (size_t)g.O * 3;
        if (((i * g.xbar) / KHW) / 16 == cb) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            uint32_t nzw[8], ngw[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint2 a = s2[e * es + 1], c2 = s2[e * es + 2];
              nzw[e] = h ? a.y : a.x;
              ngw[e] = h ? c2.y : c2.x;
            }
            // the live pairs of this half, lowest first (a uniform loop: runtime bit offsets)
            uint32_t lv = (uint32_t)(live >> (32 * h));
            while (lv != 0u) {
              const int kk = __builtin_ctz(lv);
              lv &= lv - 1u;
              const int kj = 32 * h + kk;
              float q = 0.f;
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const uint32_t nzm = (uint32_t)(((int)(nzw[e] << (31 - kk))) >> 31);
                const uint32_t sgn = (ngw[e] << (31 - kk)) & 0x80000000u;
                q += __uint_as_float((__float_as_uint(gv[e]) ^ sgn) & nzm);
              }
              q = rows4_sum(q);
              if (g4 == 0) red[((wave * NTL + tl) * NKJ + kj) * 16 + r16] += q;
            }
          }
        }
        uint64_t ps[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint2 a = s2[e * es];
          ps[e] = (uint64_t)a.x | ((uint64_t)a.y << 32);
        }
#pragma unroll 1
        for (int j = 0; j < NBA; ++j) {
          // pass bits k*8 + j of the k < 7 - j pairs, and of the k = 7 - j pair (uniform)
          const uint64_t m1 = (0x0101010101010101ull & ((1ull << (8 * (7 - j))) - 1ull)) << j;
          const int nb = 56 - 7 * j;
          if (!std_mask) {
            bool any = false;
            for (int k = 0; k < NBW; ++k) any = any || cdl[k * NBA + j] != 0.f;
            if (!any) continue;  // every pair of slice j masked out
          }
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float D;
            if (std_mask) {
              const int n = __popcll(ps[e] & m1) - (int)((ps[e] >> nb) & 1ull);
              D = (float)(n * (1 << j));
            } else {
              D = 0.f;
#pragma unroll 1
              for (int k = 0; k < NBW; ++k) D += ((ps[e] >> (k * NBA + j)) & 1ull) ? cdl[k * NBA + j] : 0.f;
            }
            d[e] = gv[e] * D;
          }
          v8bf bh, bm, bq;
          split3x8(d, bh, bm, bq);
#pragma unroll
          for (int gr = 0; gr < NGR; ++gr) {
            if (gtile[gr] != i) continue;  // uniform: the row groups of tile i
            const int kh = gpk[gr] & 3;
            const int sl = kh == 0 ? slot_kh[0] : (kh == 1 ? slot_kh[1] : slot_kh[2]);
            const bool ok = gpk[gr] >= 0 && sl >= 0;
            const __bf16* src = pl + (size_t)j * 3 * plane + (ok ? (gpk[gr] >> 2) + sl * Wo + ow0 : zoff);
            const v8bf a = as_v8bf(*reinterpret_cast<const v4i*>(src));
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh, acc[gr], 0, 0, 0);
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm, acc[gr], 0, 0, 0);
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq, acc[gr], 0, 0, 0);
          }
        }
      } else if (!PLS && tl < ntl) {
        const int i = i_lo + tl;
        uint32_t sv[8];
        if (tl < 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sv[e] = tl == 0 ? sv0[e] : sv1[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) sv[e] = st[((size_t)i * g.M + mk8 + e) * g.O + o];
        }
        // grad_alpha partials (lsq.py:321-333): sum over the pixels of code * g
        if (((i * g.xbar) / KHW) / 16 == cb) {
          float qv[NKJ];
#pragma unroll
          for (int kj = 0; kj < NKJ; ++kj) {
            float q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              // the code itself is the signed 2-bit field at bits 3kj+1 .. 3kj+2 ({nz, neg}: 01 = +1,
              // 11 = -1, 00 = 0): one v_bfe_i32, a convert and an fma (code * g is exact)
              const int code = ((int)(sv[e] << (29 - 3 * kj))) >> 30;
              q = __builtin_fmaf((float)code, gv[e], q);
            }
            qv[kj] = q;
          }
          // the first two tiles accumulate per lane in registers over the chunk (one cross-lane
          // reduction at the end); a third takes the per-stage reduction into LDS
          if (RGQ && tl == 0) {
#pragma unroll
            for (int kj = 0; kj < NGQ; ++kj) gq0[kj] += qv[kj];
          } else if (RGQ && tl == 1) {
#pragma unroll
            for (int kj = 0; kj < NGQ; ++kj) gq1[kj] += qv[kj];
          } else {
#pragma unroll
            for (int kj = 0; kj < NKJ; ++kj) {
              float q = qv[kj];
              q = rows4_sum(q);
              if (g4 == 0) red[((wave * NTL + tl) * NKJ + kj) * 16 + r16] += q;
            }
          }
        }
        // B operands: g * D_j, D_j = sum_k cD_kj * pass_ijk, split into bf16 hi / mid / lo
        v8bf bh[NBA], bm[NBA], bq[NBA];
#pragma unroll
        for (int j = 0; j < NBA; ++j) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float D;
            if (std_mask) {
              D = ldexpf((float)__popc(sv[e] & pass_mask_j(j, NBW, NBA)), g.bsa * j);
            } else {
              D = 0.f;
#pragma unroll
              for (int k = 0; k < NBW; ++k) D += ((sv[e] >> (3 * (k * NBA + j))) & 1u) ? cdl[k * NBA + j] : 0.f;
            }
            d[e] = gv[e] * D;
          }
          split3x8(d, bh[j], bm[j], bq[j]);
        }
        // A fragments of a row group (rows past C and kernel rows outside the image read the
        // zero pad: one address select, no branch)
        auto read_group = [&](int gr, v4i (&dst)[NBA]) {
          const int kh = gpk[gr] & 3;
          const int sl = kh == 0 ? slot_kh[0] : (kh == 1 ? slot_kh[1] : slot_kh[2]);
          const bool ok = gpk[gr] >= 0 && sl >= 0;
          const __bf16* src = pl + (ok ? (gpk[gr] >> 2) + sl * Wo + ow0 : zoff);
#pragma unroll
          for (int j = 0; j < NBA; ++j) dst[j] = *reinterpret_cast<const v4i*>(src + (size_t)j * 3 * plane);
        };
#pragma unroll
        for (int gr = 0; gr < NGR; ++gr) {
          if (gtile[gr] != i) continue;  // uniform: the row groups of tile i
          v4i acur[NBA];
          read_group(gr, acur);
#pragma unroll
          for (int j = 0; j < NBA; ++j) {
            const v8bf a = as_v8bf(acur[j]);
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[j], acc[gr], 0, 0, 0);
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm[j], acc[gr], 0, 0, 0);
            acc[gr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[j], acc[gr], 0, 0, 0);
          }
        }
      }
    }
  }
  if (RGQ) {
    // the register grad_alpha partials of the first two tiles into this wave's LDS region
#pragma unroll
    for (int tl = 0; tl < 2; ++tl) {
      const int i = i_lo + tl;
      if (tl < ntl && ((i * g.xbar) / KHW) / 16 == cb) {
#pragma unroll
        for (int kj = 0; kj < NGQ; ++kj) {
          float q = tl == 0 ? gq0[kj] : gq1[kj];
          q = rows4_sum(q);
          if (g4 == 0) red[((wave * NTL + tl) * NKJ + kj) * 16 + r16] += q;
        }
      }
    }
  }
  // reduce the four waves' partials through LDS (the planes are free now; plain stores, one
  // region per wave -- LDS float atomics are slow), then write the slabs
  __syncthreads();
  float* gred = reinterpret_cast<float*>(pl);  // [4 waves][NGR row groups][16 rows f][16 o]
#pragma unroll
  for (int gr = 0; gr < NGR; ++gr)
#pragma unroll
    for (int r = 0; r < 4; ++r) gred[((wave * NGR + gr) * 16 + 4 * g4 + r) * 16 + r16] = acc[gr][r];
  __syncthreads();
  const int FR = g.FBT * 16;
  for (int t = threadIdx.x; t < NGR * 256; t += blockDim.x) {
    const int oc = t & 15;
    const int f = cb * 16 * KHW + (t >> 4);  // row group t >> 8, row (t >> 4) & 15
    if (f < g.C * KHW) {
      const int i = f / g.xbar, fl = f - i * g.xbar;
      const float sum = (gred[t] + gred[NGR * 256 + t]) + (gred[2 * NGR * 256 + t] + gred[3 * NGR * 256 + t]);
      gw_slab[(((size_t)chunk * g.T + i) * FR + fl) * g.Opad + ob * 16 + oc] = sum;
    }
  }
  for (int t = threadIdx.x; t < ntl * NKJ * 16; t += blockDim.x) {
    const int tl = t / (NKJ * 16), rem = t - tl * NKJ * 16, kj = rem >> 4, oc = rem & 15;
    const int i = i_lo + tl;
    if (((i * g.xbar) / KHW) / 16 == cb) {
      const int w1 = NTL * NKJ * 16;
      const float sum = (red[t] + red[w1 + t]) + (red[2 * w1 + t] + red[3 * w1 + t]);
      ga_slab[(((size_t)chunk * g.T + i) * NKJ + kj) * g.Opad + ob * 16 + oc] = sum;
    }
  }
}

}  // namespace cimq

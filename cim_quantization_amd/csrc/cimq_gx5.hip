// cimq_gx5.hip -- grad_x of the w3a3 stride-1 module layers 16 -> 16 channels at 32 x 32 and 32 -> 32 at
// 16 x 16 (lsq.py:336-386 with the fused LSQ activation backward of lsq.py:549), from the forward's compact state
// words (cimq_v7.hip), computed per INPUT pixel so that the nn.Fold adjoint is part of the contraction:
//
//   gx[c, ih, iw] = sw/nba * sum_i sum_{kh,kw} sum_{k,o} G_i[(ih+1-kh, iw+1-kw), (k, o)] * What_k[o, (c, kh, kw)]
//   G_i[m, (k, o)] = g[m, o] * E_ik[m, o],   E_ik = sum_j cE_kj * pass_ijk   (tile i of row (c, kh, kw))
//
// on v_mfma_f32_16x16x32_bf16 (rows: 16 input pixels of one row; columns: 16 channels; K: the 48 (k, o)
// of one kernel position and 16-channel output half, two 32-deep steps), G split hi / mid / lo
// (fp32-accurate: What is a small integer).  Per m-tile of 4 input rows, crossbar tile i and output half
// h the block builds G_i of the six output rows those input rows read into an LDS "G patch" -- three
// bf16 planes [row][col][k][o of the half] -- once; a wave then reads its A operand for kernel position
// (kh, kw) at the patch position shifted by (kh, kw): one ds_read_b128 per plane and K-step, the shift an
// address offset.  The weight operand of (tile i, half h) is staged per step (zero for the rows of other
// tiles).  Waves: (16-pixel group, 16-channel input block); a wave whose channel block tile i does not
// touch skips its MFMAs.  Every grad_x value is produced by one lane, stored once after the LSQ
// backward: no fold pass, no ring, no atomics.
#pragma once
#include "cimq_v7.hip"

namespace cimq {

struct X5 {
  int nmt;     // H / 4 * B: m-tiles of four input rows
  int tpi;     // m-tiles per image
  int CBN;     // 16-channel input blocks (1 or 2) = 16-channel output halves
  int NPG;     // 16-pixel groups per m-tile: W / 4 (8 or 4); waves = NPG * CBN = 8
  int lw;      // log2(W)
};

// weight operand of (tile i, output half h, position p, K-step s, input block cb), lane l: channel
// c = 16 cb + (l & 15), K values kappa = 32 s + 8 (l >> 4) + e (e < 8) = (k, o) = (kappa / 16, 16 h + kappa % 16),
// int8(slice_k) of weight (o, f = 9 c + p) as bf16 (wcy_item's values), zero for kappa >= 48 or f outside
// tile i: wg5[((((i * CBN + h) * 9 + p) * 2 + s) * CBN + cb) * 64 + l]
template <typename WS>
__device__ inline void wg5_item(const Geo& g, const WS& ws, v4i* __restrict__ wg5, int t) {
  const int CBN = g.C / 16;
  const int lane = t & 63;
  int r = t >> 6;
  const int cb = r % CBN;
  r /= CBN;
  const int s = r & 1;
  r >>= 1;
  const int p = r % 9;
  r /= 9;
  const int h = r % CBN, i = r / CBN;
  const int c = 16 * cb + (lane & 15);
  const int f = c * 9 + p;
  const int flo = i * g.xbar, fhi = min(flo + g.xbar, g.K);
  const bool ok = c < g.C && f >= flo && f < fhi;
  uint32_t wd[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kap = 32 * s + 8 * (lane >> 4) + e;
    const int k = kap >> 4, o = 16 * h + (kap & 15);
    float val = 0.f;
    if (ok && k < g.nbw) val = (float)to_i8_wrap(wslice(g, ws, f, k * g.Opad + o));
    wd[e >> 1] |= (uint32_t)bf16_bits(val) << (16 * (e & 1));
  }
  v4i q;
  q.x = (int)wd[0]; q.y = (int)wd[1]; q.z = (int)wd[2]; q.w = (int)wd[3];
  wg5[t] = q;
}

#ifdef CIMQ_TU_GX5
// the Function entry points' prologue (prep_all: w_q already quantised) builds the same operand
__global__ void prep_wg5_kernel(Geo g, const float* __restrict__ w_q, const float* __restrict__ sw_p, int total,
                                v4i* __restrict__ wg5) {
  const WSrc ws{w_q, *sw_p, 0, 0.f, 0.f};
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) wg5_item(g, ws, wg5, t);
}
#endif  // CIMQ_TU_GX5

#if defined(CIMQ_TU_GX5) || defined(CIMQ_TU_GXW5)
// the kernel body for workgroup bid of nblk (cim_bwd_gx5_kernel, and the first part of the grid of
// cim_bwd_gxw5_kernel, which runs grad_w's workgroups behind it in the same launch)
template <int CBN>  // 16-channel input blocks = output halves (X5::CBN)
__device__ __forceinline__ void gx5_body(int bid, int nblk, const Geo& g, const X5& v, const uint32_t* __restrict__ st,
                                         const v4i* __restrict__ wg5, const Params& pp, const float* __restrict__ sw_p,
                                         const float* __restrict__ sa_p, const float* __restrict__ gout,
                                         const float* __restrict__ x, float* __restrict__ gx,
                                         float* __restrict__ gsa_part) {
  // LDS: G patch, three planes [6 rows][W + 2 cols][48 (k, o)] bf16 (96 B per pixel; 32 B of slack after
  // the last plane: the padded K-step reads past a pixel's 48 values), then the tile's weight operand
  // [9 p][2 s][64 lanes] (16 B each), then the mask coefficients and the partials
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int WP = g.W + 2;
  const int PLANE = 6 * WP * 96;                        // bytes per plane
  const int OW5 = 3 * PLANE + 32;                       // weight operand offset
  constexpr int NW5 = 9 * 2 * CBN * 64;                 // weight fragments per (tile, half)
  constexpr int NWI = (NW5 + 511) / 512;                // ... per thread
  float* cel = reinterpret_cast<float*>(smem + OW5 + NW5 * 16);  // cE_kj
  float* red = cel + 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sw = *sw_p, sa = *sa_p;
  for (int t = threadIdx.x; t < 9; t += blockDim.x) cel[t] = pp.ckj[9 + t];
  // zero padding columns 0 and W + 1 of every plane row (output columns -1 and W) and the slack after the
  // last plane (read by the padded K-step of the last pixel, times a zero weight): written once
  if (threadIdx.x < 2) reinterpret_cast<uint4*>(smem + 3 * PLANE)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
  for (int t = threadIdx.x; t < 3 * 6 * 2 * 6; t += blockDim.x) {
    const int q = t % 6, rc = t / 6, side = rc & 1, pr = rc >> 1;  // pr = plane * 6 + row
    reinterpret_cast<uint4*>(smem + (size_t)pr * WP * 96 + (side ? (WP - 1) * 96 : 0))[q] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  // standard mask (cE_kj = 2^k): E_k = 2^k * popcount(pass bits of slice k); else the per-pair sum
  const bool std_mask =
      __builtin_amdgcn_ballot_w64(lane < 9 && cel[lane < 9 ? lane : 0] != (float)(1 << (lane / 3))) == 0ull;
  const float scale = sw / 3.f;
  const float inv_sa = 1.f / sa;
  float gpart = 0.f;
  // this wave: input block cb, 16 input pixels: row 4 mt + rl, columns iw0 .. iw0 + 15
  const int cb = wave / v.NPG, pg = wave - cb * v.NPG;
  const int gpr = g.W >> 4;  // pixel groups per row
  const int rl = pg / gpr, iw0 = 16 * (pg - rl * gpr);
  const int c_lo = 16 * cb, c_hi = 16 * cb + 15;
  const int gstride = g.onchw ? g.P : 1;  // grad_out element stride between output channels

  const int NG = 6 * g.W * 4;  // G patch items (row, col, 4 channels): <= 2 per thread (x5_plan)
  for (int mt = bid; mt < v.nmt; mt += nblk) {
    const int b = mt / v.tpi, r0 = (mt - b * v.tpi) * 4;  // input rows r0 .. r0 + 3
    v4f acc = v4f{0.f, 0.f, 0.f, 0.f};
#ifdef CIMQ_EXP_GX5_CHAINS
    v4f acc1 = v4f{0.f, 0.f, 0.f, 0.f};
#endif
    // grad_out of the m-tile's G-patch items, both output halves: read once here, used by every tile's step
    // (it was re-read per tile)
    float gvr[2][2][4];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int it = threadIdx.x + k * (int)blockDim.x;
        const int oq = (it & 3) + 4 * hh, rc = it >> 2, col = rc & (g.W - 1), row = rc >> v.lw;
        const int oh = r0 - 1 + row;
#pragma unroll
        for (int e = 0; e < 4; ++e) gvr[hh][k][e] = 0.f;
        if (hh < CBN && it < NG && (unsigned)oh < (unsigned)g.Ho) {
          const int pimg = oh * g.Wo + col;
          const int go = g.onchw ? (b * g.O + 4 * oq) * g.P + pimg : (b * g.P + pimg) * g.O + 4 * oq;
#pragma unroll
          for (int e = 0; e < 4; ++e) gvr[hh][k][e] = gout[go + e * gstride];
        }
      }
    for (int i = 0; i < g.T; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h >= CBN) break;
      const int ih2 = i * CBN + h;  // step: tile i, output half h
      // the step's global reads, all issued before the barrier and the first wait: its weight operand and
      // the state words of its G-patch items (a copy loop and then the build's loads were 2-4 dependent
      // round trips per step)
      v4i wv[NWI];
#pragma unroll
      for (int u = 0; u < NWI; ++u) {
        const int idx = threadIdx.x + u * 512;
#ifdef CIMQ_EXP_GX5_NOLOAD  // attribution builds only: no global reads in the step (wrong results)
        if (idx < NW5) wv[u] = v4i{idx, ih2, u, 1};
#else
        if (idx < NW5) wv[u] = wg5[ih2 * NW5 + idx];
#endif
      }
      uint4 s4r[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int it = threadIdx.x + kk * 512;
        const int rc = it >> 2, col = rc & (g.W - 1), row = rc >> v.lw;
        const int oh = r0 - 1 + row;
        s4r[kk] = make_uint4(0u, 0u, 0u, 0u);
        if (it < NG && (unsigned)oh < (unsigned)g.Ho) {
          const int m = b * g.P + oh * g.Wo + col;
#ifdef CIMQ_EXP_GX5_NOLOAD
          s4r[kk] = make_uint4((uint32_t)m, (uint32_t)it, 7u, (uint32_t)i);
#else
          s4r[kk] = *reinterpret_cast<const uint4*>(st + ((i * g.M + m) * g.O + 4 * ((it & 3) + 4 * h)));
#endif
        }
      }
      __syncthreads();  // the previous step's (or m-tile's) MFMAs are done with the patch and weights
#pragma unroll
      for (int u = 0; u < NWI; ++u) {
        const int idx = threadIdx.x + u * 512;
        if (idx < NW5) reinterpret_cast<v4i*>(smem + OW5)[idx] = wv[u];
      }
      // G patch of output rows r0 - 1 .. r0 + 4, output channels 16 h .. 16 h + 15: item = (row, col,
      // 4 channels), channels fastest
      // (32-bit offsets -- x5_plan bounds T * M * O -- W a power of two, the grad_out layout's element stride
      // chosen once)
      auto build = [&](auto stdc) {
        constexpr bool STD = decltype(stdc)::value;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int it = threadIdx.x + kk * (int)blockDim.x;
          if (it >= NG) continue;
          const int oq = (it & 3) + 4 * h, rc = it >> 2, col = rc & (g.W - 1), row = rc >> v.lw;
          const float* gv = gvr[h][kk];
          const uint4 s4 = s4r[kk];
          const uint32_t sv[4] = {s4.x, s4.y, s4.z, s4.w};
          uint8_t* px = smem + (row * WP + col + 1) * 96 + 8 * (oq - 4 * h);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            float Gv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float E;
              if constexpr (STD) {
                E = (float)(__popc(sv[e] & pass_mask_k(k, 3)) << k);
              } else {
                E = 0.f;
#pragma unroll
                for (int j = 0; j < 3; ++j) E += ((sv[e] >> (3 * (k * 3 + j))) & 1u) ? cel[k * 3 + j] : 0.f;
              }
              Gv[e] = gv[e] * E;
            }
            // hi / mid / lo bf16 parts (split3x8's arithmetic), two values per conversion
            uint32_t ph[2], pm[2], plo[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) split3_pk(Gv[2 * u], Gv[2 * u + 1], ph[u], pm[u], plo[u]);
            *reinterpret_cast<uint2*>(px + 32 * k) = make_uint2(ph[0], ph[1]);
            *reinterpret_cast<uint2*>(px + PLANE + 32 * k) = make_uint2(pm[0], pm[1]);
            *reinterpret_cast<uint2*>(px + 2 * PLANE + 32 * k) = make_uint2(plo[0], plo[1]);
          }
        }
      };
#ifndef CIMQ_EXP_GX5_NOBUILD  // attribution builds only: the G patch left as the first step built it
      if (std_mask) build(std::true_type{});
      else build(std::false_type{});
#else
      if (mt == bid && i == 0) {
        if (std_mask) build(std::true_type{});
        else build(std::false_type{});
      }
#endif
      __syncthreads();
      // the wave's 16 input pixels x 16 channels: 9 positions x 2 K-steps x 3 planes, unless tile i holds
      // none of the block's rows (f = 9 c + p for c in c_lo .. c_hi)
      if (9 * c_hi + 8 < i * g.xbar || 9 * c_lo >= (i + 1) * g.xbar) continue;
      const v4i* wb = reinterpret_cast<const v4i*>(smem + OW5) + cb * 64 + lane;
#ifdef CIMQ_EXP_GX5_DPP
      // (tried, round 6: 5 us per launch SLOWER than the nine reads below) per kernel row kh the wave reads only
      // the kw = 1 window; kw = 0 / 2 are its pixels shifted by one lane within each 16-lane row (DPP row_shl /
      // row_shr: the pixels of a row are consecutive columns), the row's edge lane (r16 = 15 for kw = 0, r16 = 0
      // for kw = 2) reading its one column outside the window by itself
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const uint8_t* pc = smem + (size_t)((rl + 2 - kh) * WP + iw0 + r16 + 1) * 96 + 16 * g4;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4i c[3];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) c[pl] = *reinterpret_cast<const v4i*>(pc + pl * PLANE + 64 * s);
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int p = kh * 3 + kw;
            const v8bf w = as_v8bf(wb[(p * 2 + s) * CBN * 64]);
            v4i a[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
              if (kw == 1) {
                a[pl] = c[pl];
              } else {
                // kw = 0: lane r16 takes pixel r16 + 1 (row_shl:1); kw = 2: pixel r16 - 1 (row_shr:1)
#pragma unroll
                for (int d = 0; d < 4; ++d)
                  a[pl][d] = kw == 0 ? __builtin_amdgcn_update_dpp(0, c[pl][d], 0x101, 0xF, 0xF, true)
                                     : __builtin_amdgcn_update_dpp(0, c[pl][d], 0x111, 0xF, 0xF, true);
                if (r16 == (kw == 0 ? 15 : 0))
                  a[pl] = *reinterpret_cast<const v4i*>(pc + (kw == 0 ? 96 : -96) + pl * PLANE + 64 * s);
              }
            }
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_v8bf(a[0]), w, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_v8bf(a[1]), w, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_v8bf(a[2]), w, acc, 0, 0, 0);
          }
        }
      }
#else
#pragma unroll
      for (int p = 0; p < 9; ++p) {
        const int kh = p / 3, kw = p - 3 * kh;
        // output pixel (oh, ow) = (ih + 1 - kh, iw + 1 - kw): patch row rl + 2 - kh, column iw + 2 - kw
        const uint8_t* pa = smem + (size_t)((rl + 2 - kh) * WP + iw0 + r16 + 2 - kw) * 96 + 16 * g4;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const v8bf ah = as_v8bf(*reinterpret_cast<const v4i*>(pa + 64 * s));
          const v8bf am = as_v8bf(*reinterpret_cast<const v4i*>(pa + PLANE + 64 * s));
          const v8bf al = as_v8bf(*reinterpret_cast<const v4i*>(pa + 2 * PLANE + 64 * s));
          const v8bf w = as_v8bf(wb[(p * 2 + s) * CBN * 64]);
#ifdef CIMQ_EXP_GX5_NOMFMA
          acc[0] += (float)ah[0] + (float)am[1] + (float)al[2] + (float)w[3];
          continue;
#endif
#ifdef CIMQ_EXP_GX5_CHAINS  // attribution builds: the two K-steps into separate accumulators (two MFMA chains)
          v4f& a2 = s == 0 ? acc : acc1;
          a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, w, a2, 0, 0, 0);
          a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, w, a2, 0, 0, 0);
          a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, w, a2, 0, 0, 0);
#else
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, w, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, w, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, w, acc, 0, 0, 0);
#endif
        }
      }
#endif
    }
#ifdef CIMQ_EXP_GX5_CHAINS
    acc += acc1;
#endif
    // acc[r]: input pixel (r0 + rl, iw0 + 4 g4 + r), channel c_lo + r16: scale, LSQ activation backward, store
    const int ih = r0 + rl, iw = iw0 + 4 * g4;
    const int gi = ((b * g.C + c_lo + r16) * g.H + ih) * g.W + iw;
    const float4 xv4 = *reinterpret_cast<const float4*>(x + gi);
    const float xv[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
    float o4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float gqv = acc[r] * scale;
      // autograd of round_pass(clamp(x/sa, 0, Qp)) * sa (lsq.py:549), as cim_bwd_gx_v8_kernel
      const float y1 = xv[r] / sa;
      const float clv = clamp_nan(y1, 0.f, g.lsq_qp);
      const float rr2 = rintf(clv);
      const float rp = (rr2 - clv) + clv;
      const bool pass = (y1 >= 0.f) && (y1 <= g.lsq_qp);
      const float gy = pass ? gqv * sa : 0.f;
      o4[r] = pass ? gqv : 0.f;
      gpart += gqv * rp;
      gpart += -(gy * (y1 * inv_sa));
    }
    *reinterpret_cast<float4*>(gx + gi) = make_float4(o4[0], o4[1], o4[2], o4[3]);
  }
  // the block's d sa partial (fixed order: lanes, then waves)
  for (int o = 32; o > 0; o >>= 1) gpart += __shfl_xor(gpart, o);
  __syncthreads();
  if (lane == 0) red[wave] = gpart;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 8; ++w) t += red[w];
    gsa_part[bid] = t;
  }
}
#endif  // CIMQ_TU_GX5 || CIMQ_TU_GXW5

#ifdef CIMQ_TU_GX5
template <int CBN>
__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 8)))
void cim_bwd_gx5_kernel(Geo g, X5 v, const uint32_t* __restrict__ st, const v4i* __restrict__ wg5, Params pp,
                        const float* __restrict__ sw_p, const float* __restrict__ sa_p,
                        const float* __restrict__ gout, const float* __restrict__ x, float* __restrict__ gx,
                        float* __restrict__ gsa_part) {
  gx5_body<CBN>((int)blockIdx.x, (int)gridDim.x, g, v, st, wg5, pp, sw_p, sa_p, gout, x, gx, gsa_part);
}
#endif  // CIMQ_TU_GX5

}  // namespace cimq

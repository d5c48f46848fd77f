// cimq_gw5.hip -- grad_w and the grad_alpha_cim partials of the w3a3 stride-1 module layers with 16 or 32
// input channels (lsq.py:321-356), from the forward's compact state words (cimq_v7.hip) and ctx words:
//
//   gw[f, o]  = sum_j sum_m xhat_j[m, f] * g[m, o] * D_j[m, o],   D_j = sum_k cD_kj * pass_ijk  (i = tile of f)
//   ga[i, kj, o] = sum_m code_ijk[m, o] * g[m, o]
//
// as one v_mfma_f32_16x16x32_bf16 contraction over (pixel, slice) per 16 weight rows f:
//   * K is ordered (pixel pair, slot) with slots (j = 0, 1, 2, pad): one lane of the A operand holds the
//     three ctx slices of two pixels of its row f, one lane of the B operand g * D_j of the same two
//     pixels for its output channel, split hi / mid / lo (three MFMAs, fp32-accurate products: xhat is a
//     small integer);
//   * the block's input rows are staged once per 128-pixel m-tile into an "A-ready" LDS patch: per
//     element the four bf16 (xhat_0, xhat_1, xhat_2, 0), so an A fragment is two ds_read_b64 at a lane
//     offset fixed per 16-row block -- no per-element conversion in the MFMA loop;
//   * block = (pixel chunk, 16-channel input block, 16-channel output block), as cim_bwd_gw_v7_kernel
//     splits its pairs: the block's 144 weight rows are 9 16-row blocks in at most two tiles, its patch
//     holds 16 channels; wave = 16 pixels of the m-tile, building the B operands of its own pixels and
//     keeping its grad_w / grad_alpha sums in registers across the block's m-tiles.  At the end the 8
//     waves are summed in LDS in wave order and the block writes its part of the chunk's slab (the
//     module epilogue sums the slabs in chunk order: deterministic).
#pragma once
#include <type_traits>

#include "cimq_v7.hip"

namespace cimq {

// n / d for 0 <= n < 2^20, d < 2^10 (inv = 1 / d in fp32): exact
__device__ inline int sdiv5(int n, float inv) { return (int)(((float)n + 0.5f) * inv); }

// the code -> ctx word table's entry for out-of-image elements (a zero word; codes are <= 256)
constexpr int kZeroCode = 259;

struct G5 {
  int lwo;     // log2(Wo)
  int lwi;     // log2(W)
  int codes;   // 1: the ctx holds one activation code byte per element (the forward was cim_fwd5_kernel with
               // ctx_codes): expanded through the act word table, as the forward's staging does
  int IPM;     // images per 128-pixel m-tile (1: the m-tile is R output rows of one image)
  int R, RH, WP;  // output rows per image slot, staged input rows R + 2, patch row length W + 2
  int nmt;     // M / 128
  int nst;     // m-tiles per block (chunk)
  int nchunks; // blocks = slab chunks
};

#if defined(CIMQ_TU_GW5) || defined(CIMQ_TU_GXW5)
// SS: the conv stride (1 or 2): a compile-time constant, so the pixel-pair offsets stay immediates
// SP: the row blocks of the block's two tiles split at fb = 8 - (cb mod 8) (its first 144 cb mod 128 rows lie in the
// first tile), compiled in so that the MFMA chains of consecutive row blocks are not separated by branches and
// their A reads issue ahead: 8 when every block has cb = 0 (16 input channels), 78 for cb 0 / 1 (32 input
// channels: two m-tile loops); 0: a uniform per-block table
template <int SS, bool CODES, int SP>  // CODES: G5::codes, a compile-time choice of the staging's load width
// the kernel body for workgroup (bx, by) (cim_bwd_gw5_kernel, and the second part of the grid of
// cim_bwd_gxw5_kernel, behind grad_x's workgroups)
__device__ __forceinline__ void gw5_body(int bx, int by, const Geo& g, const G5& v, const uint32_t* __restrict__ st,
                                         const uint32_t* __restrict__ xcb, const Params& pp,
                                         const float* __restrict__ gout, const uint32_t* __restrict__ cal,
                                         float* __restrict__ gw_slab, float* __restrict__ ga_slab) {
  // block = (pixel chunk, input-channel block cb, output block ob): the 9 16-row blocks of rows
  // f = 144 cb .. 144 cb + 143 (the 16 channels of cb at every (kh, kw)), which touch at most two tiles
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint2* pat = reinterpret_cast<uint2*>(smem);  // [16 channels][IPM][RH][WP] of (xhat_0 | xhat_1 << 16, xhat_2)
  const int CH = v.IPM * v.RH;  // patch rows per channel
  float* cdl = reinterpret_cast<float*>(smem + (size_t)16 * CH * v.WP * 8);  // cD_kj
  // code -> ctx word (v.codes), addressed as a byte offset from smem (LDS loads, not generic ones)
  const int alut_off = 16 * CH * v.WP * 8 + 16 * 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int cb = by / g.OB16, ob = by - cb * g.OB16;
  const int o = ob * 16 + r16;
  const int i_lo = (144 * cb) / 128, i_hi = (144 * cb + 143) / 128;  // tiles of the block's rows (xbar 128)
  const int ntl = i_hi - i_lo + 1;
  for (int t = threadIdx.x; t < 9; t += blockDim.x) cdl[t] = pp.ckj[18 + t];
  // the forward's backward-word table (ctx, written by cim_fwd5_kernel): code e -> ctx word
  // (entry kZeroCode: 0, the code of the staging's out-of-image elements)
  if (CODES) {
    for (int t = threadIdx.x; t <= (int)g.lsq_qp + 1; t += blockDim.x)
      *reinterpret_cast<uint32_t*>(smem + alut_off + 4 * t) = cal[t];
    if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(smem + alut_off + 4 * kZeroCode) = 0u;
  }
  // the ctx format the forward wrote (kCalFlag): code bytes expected; a mismatch poisons the outputs
  const bool fmt_ok = !CODES || cal[kCalFlag] == kCodesMagic;
  // padding columns 0 and WP-1: zero once
  for (int t = threadIdx.x; t < 16 * CH * 2; t += blockDim.x) {
    const int side = t & 1, cr = t >> 1;
    pat[cr * v.WP + (side ? v.WP - 1 : 0)] = make_uint2(0u, 0u);
  }
  __syncthreads();
  // standard binary mask (cD_kj = 2^j): D_j = 2^j * popcount(pass bits of slice j); else the per-pair sum
  const bool std_mask =
      __builtin_amdgcn_ballot_w64(lane < 9 && cdl[lane < 9 ? lane : 0] != (float)(1 << (lane % 3))) == 0ull;
  // grad_alpha of tile i belongs to the block of the channel block holding the tile's first row
  // (as cim_bwd_gw_v7_kernel): each (tile, pair, channel) is summed by one block per chunk
  bool own[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) own[q] = q < ntl && ((i_lo + q) * 128) / 144 == cb;

  // per 16-row block fb: this lane's row f = 144 cb + 16 fb + r16 = (c, kh, kw) -> patch offset (uint2
  // units, c relative to the block), and its tile (slot 0 or 1 of the block's tiles)
  // (two 16-bit offsets per register, unpacked per use: g5_plan's one-round staging bound keeps the patch
  // below 2^16 uint2)
  uint32_t aoffp[5] = {0u, 0u, 0u, 0u, 0u};
  int atl[9];
#pragma unroll
  for (int fb = 0; fb < 9; ++fb) {
    const int f = 16 * fb + r16, c = f / 9, p = f - 9 * c, kh = p / 3, kw = p - 3 * kh;
    aoffp[fb >> 1] |= (uint32_t)((c * CH + kh) * v.WP + kw) << (16 * (fb & 1));
    atl[fb] = (144 * cb + 16 * fb) / 128 - i_lo;  // uniform
  }
  v4f acc[9];
#pragma unroll
  for (int fb = 0; fb < 9; ++fb) acc[fb] = v4f{0.f, 0.f, 0.f, 0.f};
  float ga[2][9];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int kj = 0; kj < 9; ++kj) ga[q][kj] = 0.f;

  const int Wo = 1 << v.lwo;
  const int PI = g.P < 128 ? g.P : 128;  // pixels per image slot
  const int HWi = g.H * g.W;
  const float invRH = 1.f / (float)v.RH, invIPM = 1.f / (float)v.IPM;
  const int tpi = g.P >= 128 ? g.P / 128 : 1;
#ifdef CIMQ_EXP_GW5_EMPTY  // attribution builds only: the prologue and the slab epilogue without any m-tile
  const int mt_lo = bx * v.nst, mt_hi = mt_lo;
#else
  const int mt_lo = bx * v.nst, mt_hi = min(mt_lo + v.nst, v.nmt);
#endif
  // the m-tile loop with the block's row-block split SPL compiled in (0: the per-block table)
  auto mtiles = [&](auto spc) __attribute__((always_inline)) {
    constexpr int SPL = decltype(spc)::value;
  for (int mt = mt_lo; mt < mt_hi; ++mt) {
#pragma unroll
    for (int k = 0; k < 5; ++k) asm volatile("" : "+v"(aoffp[k]));
    const int b0 = g.P >= 128 ? mt / tpi : mt * v.IPM;  // first image of the m-tile
    const int p0 = g.P >= 128 ? (mt - b0 * tpi) * 128 : 0;
    const int oh0 = p0 >> v.lwo;
    // this lane's four pixels 16 wave + 4 g4 .. +3 of the m-tile (one image slot): grad_out and the state
    // words of the block's tiles, loaded ahead of the staging
    const int pw = 16 * wave + 4 * g4;  // within the m-tile
    const int sl = pw / PI, pin0 = pw - sl * PI;  // image slot, pixel within the slot
    const int b = b0 + sl;
    float4 gq;
#ifdef CIMQ_EXP_GW5_NOLOAD  // attribution builds only: no global reads in the m-tile loop (wrong results)
    gq = make_float4(1e-3f * o, 2e-3f, 3e-3f * mt, 4e-3f);
    if (false) {
#else
    if (g.onchw) {
#endif
      gq = *reinterpret_cast<const float4*>(gout + ((size_t)b * g.O + o) * g.P + p0 + pin0);
    } else {  // the Function path's [B, P, O]
      const float* gp = gout + ((size_t)b * g.P + p0 + pin0) * g.O + o;
      gq = make_float4(gp[0], gp[g.O], gp[2 * g.O], gp[3 * g.O]);
    }
    uint32_t sq[2][4];
    {
      const size_t m = (size_t)b * g.P + p0 + pin0;
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#ifdef CIMQ_EXP_GW5_NOLOAD
          sq[q][e] = (uint32_t)(m * 2654435761u + e * 40503u + o) & 0x7FFFFFFu;
#else
          sq[q][e] = q < ntl ? st[((size_t)(i_lo + q) * g.M + m + e) * g.O + o] : 0u;
#endif
    }
    // A-ready patch: input rows oh0 * SH - 1 .. (oh0 + R - 1) * SH + 1 of each image slot, the block's 16
    // channels; item = (c, slot, row, col) (W a power of two; the divisions by RH and CH as exact
    // float-reciprocal quotients; 32-bit offsets: g5_plan bounds Nin).  SU items per thread and round: the
    // first round's reads are issued with grad_out's and the state words', before the barrier (the stride-1
    // layers stage in that one round)
    constexpr int SU = 6;
    const int n = 16 * CH * g.W;
    const int ih0 = oh0 * SS - 1;  // patch row 0 (pad 1)
    const int xb = (b0 * g.C + 16 * cb) * HWi + ih0 * g.W;  // (image b0, channel 16 cb, row ih0)
    // (branch-free: every item loads -- out-of-patch and out-of-image items from element 0 -- and selects, so the
    // SU reads are in flight together; a branch around each load made hipcc wait for each before the next)
    auto ld = [&](int base, uint32_t (&wv)[SU]) {
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int idx = base + u * 512;
        const int col = idx & (g.W - 1), cr = idx >> v.lwi;
        const int rr = sdiv5(cr, invRH), row = cr - rr * v.RH;  // rr = c * IPM + slot
        const int c = sdiv5(rr, invIPM), slt = rr - c * v.IPM;
        const int ih = ih0 + row;
        const bool ok = idx < n && (unsigned)ih < (unsigned)g.H;
        // (a code byte, expanded below through the LDS table, or the word itself)
        // (unsigned offsets: the loads take the scalar base + 32-bit offset form)
        const uint32_t xi = ok ? (uint32_t)(xb + (slt * g.C + c) * HWi + row * g.W + col) : 0u;
#ifdef CIMQ_EXP_GW5_NOLOAD
        const uint32_t w = CODES ? (xi & 7u) : xi * 0x010203u;
#else
        const uint32_t w = CODES ? (uint32_t)reinterpret_cast<const uint8_t*>(xcb)[xi] : xcb[xi];
#endif
        wv[u] = ok ? w : (CODES ? (uint32_t)kZeroCode : 0u);
      }
    };
    auto stv = [&](int base, uint32_t (&wv)[SU]) {
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int idx = base + u * 512;
        if (idx >= n) continue;
        if (CODES) wv[u] = *reinterpret_cast<const uint32_t*>(smem + alut_off + 4 * (int)wv[u]);
        // int8 ctx slices (lsq.py:160 truncation, wrapped) -> exact bf16 (the high half of the fp32)
        const uint32_t f0 = __float_as_uint((float)(int8_t)(wv[u] & 0xFFu));
        const uint32_t f1 = __float_as_uint((float)(int8_t)((wv[u] >> 8) & 0xFFu));
        const uint32_t f2 = __float_as_uint((float)(int8_t)((wv[u] >> 16) & 0xFFu));
        pat[(idx >> v.lwi) * v.WP + (idx & (g.W - 1)) + 1] = make_uint2(__builtin_amdgcn_perm(f1, f0, 0x07060302u), f2 >> 16);
      }
    };
    if constexpr (SS == 1) {  // one round (g5_plan: 16 * CH * W <= SU * 512 at stride 1)
      uint32_t wv[SU];
      ld((int)threadIdx.x, wv);
      __syncthreads();  // the previous m-tile's waves are done with the patch
      stv((int)threadIdx.x, wv);
    } else {  // stride 2: further rounds after the barrier
      for (int base = (int)threadIdx.x, first = 1; first || base < n; base += SU * 512, first = 0) {
        uint32_t wv[SU];
        ld(base, wv);
        if (first) __syncthreads();
        stv(base, wv);
      }
    }
    __syncthreads();

    {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int e0 = 2 * s;  // pixels e0, e0 + 1 of this lane's four (same output row: Wo % 4 == 0)
        const float gv0 = (&gq.x)[e0], gv1 = (&gq.x)[e0 + 1];
        const int pin = pin0 + e0;  // within the image slot
        const int poff = (sl * v.RH + (pin >> v.lwo) * SS) * v.WP + (pin & (Wo - 1)) * SS;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (q >= ntl) break;
          const uint32_t s0 = sq[q][e0], s1 = sq[q][e0 + 1];
#ifdef CIMQ_EXP_GW5_NOGA
          if (false) {
#else
          if (own[q]) {
#endif
            // grad_alpha partials (lsq.py:321-333): code * g, the code the signed 2-bit field at bit 3kj + 1
#pragma unroll
            for (int kj = 0; kj < 9; ++kj) {
              const int c0 = ((int)(s0 << (29 - 3 * kj))) >> 30, c1 = ((int)(s1 << (29 - 3 * kj))) >> 30;
              ga[q][kj] = __builtin_fmaf((float)c1, gv1, __builtin_fmaf((float)c0, gv0, ga[q][kj]));
            }
          }
          // B operand: g * D_j of the two pixels, slots (j = 0, 1, 2, 0), split hi / mid / lo
          float d[8];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            float D0, D1;
            if (std_mask) {
              D0 = (float)(__popc(s0 & pass_mask_j(j, 3, 3)) << j);
              D1 = (float)(__popc(s1 & pass_mask_j(j, 3, 3)) << j);
            } else {
              D0 = D1 = 0.f;
#pragma unroll
              for (int k = 0; k < 3; ++k) {
                const int bit = 3 * (k * 3 + j);
                D0 += ((s0 >> bit) & 1u) ? cdl[k * 3 + j] : 0.f;
                D1 += ((s1 >> bit) & 1u) ? cdl[k * 3 + j] : 0.f;
              }
            }
            d[j] = gv0 * D0;
            d[4 + j] = gv1 * D1;
          }
          d[3] = d[7] = 0.f;
          v8bf bh, bm, bl;
          split3x8(d, bh, bm, bl);
#pragma unroll
          for (int fb = 0; fb < 9; ++fb) {
            // the 16-row blocks of this tile: fb < SP in the block's first tile, the rest in its second (compile
            // time: the MFMA chains of consecutive row blocks are not separated by branches, so their A reads
            // issue ahead); SP 0: the uniform per-block table
            if constexpr (SPL > 0) {
              if (q == 0 ? fb >= SPL : fb < SPL) continue;
            } else {
              if (atl[fb] != q) continue;
            }
            const int ao = (int)((aoffp[fb >> 1] >> (16 * (fb & 1))) & 0xFFFFu);
            const uint2 a0 = pat[ao + poff], a1 = pat[ao + poff + SS];
            const v8bf a = as_v8bf(v4i{(int)a0.x, (int)a0.y, (int)a1.x, (int)a1.y});
#ifdef CIMQ_EXP_GW5_NOMFMA
            acc[fb][0] += (float)a[0] + (float)bh[0] + (float)bm[1] + (float)bl[2];
            continue;
#endif
            acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh, acc[fb], 0, 0, 0);
            acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm, acc[fb], 0, 0, 0);
            acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl, acc[fb], 0, 0, 0);
          }
        }
      }
    }
  }
  };
  if constexpr (SP == 78) {  // 32 input channels: input-channel block 0 splits at 8, block 1 at 7
    if (cb == 0) mtiles(std::integral_constant<int, 8>{});
    else mtiles(std::integral_constant<int, 7>{});
  } else {
    mtiles(std::integral_constant<int, SP>{});
  }

  // the block's part of its chunk's slab: the 8 waves summed in LDS in wave order
#ifdef CIMQ_EXP_GW5_NOEPI
  {
    float* gws = gw_slab + (size_t)bx * g.T * g.FBT * 16 * g.Opad;
    float t = 0.f;
#pragma unroll
    for (int fb = 0; fb < 9; ++fb) t += acc[fb][0] + acc[fb][1] + acc[fb][2] + acc[fb][3];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int kj = 0; kj < 9; ++kj) t += ga[q][kj];
    gws[threadIdx.x] = t;
    return;
  }
#endif
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [8 waves][FC row blocks][64 lanes][4] (g5_plan: >= 24 KB)
  const size_t rows = (size_t)g.T * g.FBT * 16;
  float* gws = gw_slab + (size_t)bx * rows * g.Opad;
  // three 16-row blocks at a time: every wave stores its accumulators, then all 512 threads sum the 8 waves
  // (in wave order, from 0: the sums of the one-wave reduction before, bit for bit) and store 16 consecutive
  // channels per 16 threads
  constexpr int FC = 3;
#pragma unroll
  for (int c0 = 0; c0 < 9; c0 += FC) {
#pragma unroll
    for (int fl = 0; fl < FC; ++fl)
      reinterpret_cast<float4*>(red)[(wave * FC + fl) * 64 + lane] =
          make_float4(acc[c0 + fl][0], acc[c0 + fl][1], acc[c0 + fl][2], acc[c0 + fl][3]);
    __syncthreads();
    for (int t = threadIdx.x; t < FC * 256; t += 512) {
      const int oc = t & 15, r = (t >> 4) & 3, gq = (t >> 6) & 3, fl = t >> 8;
      const int ln = gq * 16 + oc;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum += red[((w * FC + fl) * 64 + ln) * 4 + r];
      const int f0 = 144 * cb + 16 * (c0 + fl) + 4 * gq, i = f0 / g.xbar;
      const size_t row0 = (size_t)i * g.FBT * 16 + (f0 - i * g.xbar);
      gws[(row0 + r) * g.Opad + ob * 16 + oc] = fmt_ok ? sum : __builtin_nanf("");
    }
    __syncthreads();
  }
  // grad_alpha of the owned tiles: the four lane groups, then the 8 waves
  float* gas = ga_slab + (size_t)bx * g.T * 9 * g.Opad;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (!own[q]) continue;  // uniform
#pragma unroll
    for (int kj = 0; kj < 9; ++kj) {
      float t = ga[q][kj];
      t = rows4_sum(t);
      if (g4 == 0) red[(wave * 9 + kj) * 16 + r16] = t;
    }
    __syncthreads();
    if ((int)threadIdx.x < 9 * 16) {
      const int kj = threadIdx.x >> 4, oc = threadIdx.x & 15;
      float t = 0.f;
      for (int w = 0; w < 8; ++w) t += red[(w * 9 + kj) * 16 + oc];
      gas[((size_t)(i_lo + q) * 9 + kj) * g.Opad + ob * 16 + oc] = fmt_ok ? t : __builtin_nanf("");
    }
    __syncthreads();
  }
}
#endif  // CIMQ_TU_GW5 || CIMQ_TU_GXW5

#ifdef CIMQ_TU_GW5
template <int SS, bool CODES, int SP>
__global__ __attribute__((amdgpu_flat_work_group_size(512, 512), amdgpu_waves_per_eu(4, 4)))
void cim_bwd_gw5_kernel(Geo g, G5 v, const uint32_t* __restrict__ st, const uint32_t* __restrict__ xcb, Params pp,
                        const float* __restrict__ gout, const uint32_t* __restrict__ cal, float* __restrict__ gw_slab,
                        float* __restrict__ ga_slab) {
  gw5_body<SS, CODES, SP>((int)blockIdx.x, (int)blockIdx.y, g, v, st, xcb, pp, gout, cal, gw_slab, ga_slab);
}
#endif  // CIMQ_TU_GW5

}  // namespace cimq

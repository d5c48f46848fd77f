// cimq_lsq_dev.h -- device side of the LSQ quantiser backward: the module epilogue kernels
// (cimq_lsq.hip), one layer per launch or packed over a chain of layers (cimq_pending_flush).
#pragma once
#include "cimq_kernels_v3.hip"

namespace cimq {

struct LsqArgs {
  float qn_w, qp_w;      // weight clamp range
  float gs_a, gs_w;      // grad_scale factors
  int nbits_alpha;       // 0: no alpha_cim
  int nalpha;            // numel(alpha_cim) = T*nbw*nba*O
};

// block-wide reductions: across the wave with lane shuffles, then across the (<= 16) waves
// through LDS with one barrier.  red needs 4 * 16 floats.
__device__ inline float nan_max(float a, float b) { return (a != a || b != b) ? (a + b) : fmaxf(a, b); }
__device__ inline float nan_min(float a, float b) { return (a != a || b != b) ? (a + b) : fminf(a, b); }

// (max, min) with torch.max / torch.min's NaN propagation
__device__ inline float2 block_max_min(float mx, float mn, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = nan_max(mx, __shfl_xor(mx, o));
    mn = nan_min(mn, __shfl_xor(mn, o));
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = mx;
    red[2 * w + 1] = mn;
  }
  __syncthreads();
  float2 r = make_float2(red[0], red[1]);
  for (int i = 1; i < nw; ++i) {
    r.x = nan_max(r.x, red[2 * i]);
    r.y = nan_min(r.y, red[2 * i + 1]);
  }
  __syncthreads();
  return r;
}

__device__ inline float4 block_sum4(float4 v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o);
    v.y += __shfl_xor(v.y, o);
    v.z += __shfl_xor(v.z, o);
    v.w += __shfl_xor(v.w, o);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) reinterpret_cast<float4*>(red)[w] = v;
  __syncthreads();
  float4 r = reinterpret_cast<const float4*>(red)[0];
  for (int i = 1; i < nw; ++i) {
    const float4 t = reinterpret_cast<const float4*>(red)[i];
    r.x += t.x;
    r.y += t.y;
    r.z += t.z;
    r.w += t.w;
  }
  __syncthreads();
  return r;
}

// =========================================================================================
// backward epilogue of the module entry points: two launches.  Blocks [0, nwb) reduce the
// grad_w slabs and run the weight quantiser's backward; blocks [nwb, nwb + nga) reduce the
// grad_alpha slabs into d loss / d alpha_q; then one block runs alpha_cim's quantiser
// backward and the two step-size gradients.  With accum set, every parameter gradient is
// added into its output buffer (torch's AccumulateGrad: grad = grad + new).
// =========================================================================================
struct ModuleTail {
  const float* gw_slab;
  const float* ga_slab;
  const float* scal;
  const float* weight;
  const float* alpha_cim;
  const float* apart;  // act-LSQ partials of the grad_x kernel
  float* wpart;        // [2 * nwb] weight-LSQ partials
  float* gaq;          // d loss / d alpha_q
  float* grad_weight;
  float* grad_alpha_act;
  float* grad_alpha_w;
  float* grad_alpha_cim;
  const float* ckj;  // Params::ckj of the layer
  float* gapart;     // wide alpha_cim (> kFinishInReg elements): [nga][4] first-sweep partials, else null
  float cgrad;       // 1 / sqrt(numel(ps) Qp_adc) (lsq.py:323,330)
  int nchunks, nwb, nga, napart;
  uint8_t accum;
  uint8_t gaq_ready;  // d loss / d alpha_q already in gaq (the shift ADC's statistics kernel): no slab sums
  uint8_t wide;       // few chunks, many outputs (the dense path): one output per thread of a 1024-thread
                      // block (nwb / nga count such blocks), the chunks summed in order by that thread
  uint8_t lpr;        // not wide: float4 slab reads, lpr lanes (16 or 64) x 4 outputs per block and
                      // 1024 / lpr chunk groups (reduce_chunks4); 0: one output per lane, 64 per
                      // block, 16 chunk groups (reduce_chunks); nwb / nga count such blocks
};
// alpha_cim sizes the one-block epilogue keeps in registers (module_finish_block); larger ones
// (the QuantLinear layers: T * nbw * nba * O = 131072 at 1024 -> 1024 w4a4) take the wide path:
// the first sweep's partials per tail block, then a grid-wide second sweep.
constexpr int kFinishInReg = 8 * 1024;

// grad_w slab sum -> G = d loss / d w_q, then through w_q = rp * sw, rp = round_pass(clamp(w / sw)):
//   grad_weight = mask * (G * sw) / sw; per block the partial sums of G * rp (MulBackward,
//   d/d sw) and of -grad_t1 * ((w / sw) / sw) (DivBackward wrt the divisor) -> wpart[2*blk].
// the slab sum of one output over few chunks, in chunk order, up to 8 loads in flight
__device__ inline float sum_chunks_serial(const float* __restrict__ slab, size_t stride, int nchunks, size_t idx) {
  float v = 0.f;
  int c = 0;
  for (; c + 8 <= nchunks; c += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = slab[(size_t)(c + u) * stride + idx];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; c < nchunks; ++c) v += slab[(size_t)c * stride + idx];
  return v;
}

// The slab sum of four consecutive outputs per lane: the block's lpr-lane rows (lpr = 16 or 64)
// each take every nsub-th chunk, then the first row sums the rows in
// order through LDS.  lpr 16 (64 chunk rows: one batch of loads per lane on the 256-512-chunk
// slabs, 4x the blocks) measured slower than 64 for the packed tail.  red: blockDim float4s.
__device__ inline float4 reduce_chunks4(const float* __restrict__ slab, size_t chunk_stride, int nchunks, size_t idx,
                                        int lpr, float4* red) {
  const int sub = (int)threadIdx.x / lpr, nsub = (int)blockDim.x / lpr;
  // 4 accumulators, 4 float4 loads in flight: the kernel stays within 64 VGPRs (two 1024-thread
  // blocks per CU)
  float4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  int c = sub;
  for (; c + 3 * nsub < nchunks; c += 4 * nsub) {
    float4 t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(slab + (size_t)(c + u * nsub) * chunk_stride + idx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u].x += t[u].x;
      a[u].y += t[u].y;
      a[u].z += t[u].z;
      a[u].w += t[u].w;
    }
  }
  for (; c < nchunks; c += nsub) {
    const float4 t = *reinterpret_cast<const float4*>(slab + (size_t)c * chunk_stride + idx);
    a[0].x += t.x;
    a[0].y += t.y;
    a[0].z += t.z;
    a[0].w += t.w;
  }
  float4 r;
  r.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  r.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  r.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  r.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  red[threadIdx.x] = r;
  __syncthreads();
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sub == 0)
#pragma unroll 8
    for (int t = 0; t < nsub; ++t) {
      const float4 u = red[threadIdx.x + lpr * t];
      v.x += u.x;
      v.y += u.y;
      v.z += u.z;
      v.w += u.w;
    }
  return v;
}

// one output's weight-quantiser backward (below), in two halves: its loads (gw_pre, issued before
// the slab sums so their latency overlaps them), then grad_weight and the two d / d sw terms
struct GwPre {
  int e;  // weight element (O * K < 2^31), -1: a padding row / channel
  float w, old;
};

__device__ inline GwPre gw_pre(const Geo& g, const ModuleTail& a, size_t idx) {
  GwPre p;
  const int o = (int)(idx % g.Opad);
  const size_t row = idx / g.Opad;
  const int i = (int)(row / (g.FBT * 16)), fl = (int)(row - (size_t)i * g.FBT * 16);
  const int f = i * g.xbar + fl;
  const bool ok = o < g.O && fl < g.xbar && f < g.K;
  p.e = ok ? o * g.K + f : -1;
  p.w = ok ? a.weight[p.e] : 0.f;
  p.old = (ok && a.accum) ? a.grad_weight[p.e] : 0.f;
  return p;
}

__device__ inline void gw_fin(const LsqArgs& q, const ModuleTail& a, const GwPre& p, float vsum, float nbw,
                              float& p_mul, float& p_div) {
  if (p.e < 0) return;
  const float sa = a.scal[0], sw = a.scal[1];
  const float G = vsum * (sa / nbw);  // d loss / d w_q (as reduce_gw_v3)
  const float t1 = p.w / sw;
  const float c = clamp_nan(t1, q.qn_w, q.qp_w);
  const float rp = round_pass_value(c);
  const float grad_rp = G * sw;
  const bool pass = (t1 >= q.qn_w) && (t1 <= q.qp_w);
  const float grad_t1 = pass ? grad_rp : 0.f;
  const float gwv = grad_t1 / sw;
  a.grad_weight[p.e] = a.accum ? p.old + gwv : gwv;
  p_mul += G * rp;
  p_div += -grad_t1 * (t1 / sw);
}

__device__ inline void gw_lsq_role(const Geo& g, const LsqArgs& q, const ModuleTail& a, int blk, float* red) {
  const size_t rows = (size_t)g.T * g.FBT * 16;
  const size_t nout = rows * g.Opad;
  if (!a.wide && a.lpr == 0) {  // scalar: one output per lane of the first wave, 64 per block (reduce_chunks)
    const size_t idx = (size_t)blk * 64 + (threadIdx.x & 63);
    const GwPre pre = (threadIdx.x < 64 && idx < nout) ? gw_pre(g, a, idx) : GwPre{-1, 0.f, 0.f};
    const float vsum = reduce_chunks(a.gw_slab, nout, a.nchunks, idx < nout ? idx : 0, red);
    if (threadIdx.x >= 64) return;
    float p_mul = 0.f, p_div = 0.f;
    gw_fin(q, a, pre, vsum, (float)g.nbw, p_mul, p_div);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      p_mul += __shfl_xor(p_mul, o);
      p_div += __shfl_xor(p_div, o);
    }
    if (threadIdx.x == 0) {
      a.wpart[2 * blk] = p_mul;
      a.wpart[2 * blk + 1] = p_div;
    }
    return;
  }
  if (!a.wide) {  // nout % 16 == 0 (Opad)
    {
      // a block whose rows are all padding rows of one tile (rows xbar .. FBT*16 - 1 of a tile, or past K
      // in the last one: gw_pre's e = -1) has nothing to sum: its slab reads skipped (the 16-channel layers'
      // second tile holds 16 rows of 128)
      const size_t r0 = (size_t)blk * a.lpr * 4 / g.Opad, r1 = ((size_t)(blk + 1) * a.lpr * 4 - 1) / g.Opad;
      const size_t tr = (size_t)g.FBT * 16;
      const int i = (int)(r0 / tr), fl = (int)(r0 - (size_t)i * tr);
      if (r1 / tr == (size_t)i && (fl >= g.xbar || i * g.xbar + fl >= g.K)) {
        if (threadIdx.x == 0) {
          a.wpart[2 * blk] = 0.f;
          a.wpart[2 * blk + 1] = 0.f;
        }
        return;
      }
    }
    const size_t i0 = ((size_t)blk * a.lpr + (threadIdx.x & (a.lpr - 1))) * 4;
    const bool mine = (int)threadIdx.x < a.lpr && i0 < nout;
    GwPre pre[4];
#ifdef CIMQ_EXP_TAIL_NOEPI  // attribution builds only (tools/kernel_experiment.py)
#pragma unroll
    for (int u = 0; u < 4; ++u) pre[u] = GwPre{-1, 0.f, 0.f};
#else
#pragma unroll
    for (int u = 0; u < 4; ++u) pre[u] = mine ? gw_pre(g, a, i0 + u) : GwPre{-1, 0.f, 0.f};
#endif
#ifdef CIMQ_EXP_TAIL_NOSLAB
    const float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#else
    const float4 v = reduce_chunks4(a.gw_slab, nout, a.nchunks, i0 < nout ? i0 : 0, a.lpr,
                                    reinterpret_cast<float4*>(red));
#endif
    if (threadIdx.x >= 64) return;
    float p_mul = 0.f, p_div = 0.f;
    const float nbw = (float)g.nbw;
    gw_fin(q, a, pre[0], v.x, nbw, p_mul, p_div);
    gw_fin(q, a, pre[1], v.y, nbw, p_mul, p_div);
    gw_fin(q, a, pre[2], v.z, nbw, p_mul, p_div);
    gw_fin(q, a, pre[3], v.w, nbw, p_mul, p_div);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      p_mul += __shfl_xor(p_mul, o);
      p_div += __shfl_xor(p_div, o);
    }
    if (threadIdx.x == 0) {
      a.wpart[2 * blk] = p_mul;
      a.wpart[2 * blk + 1] = p_div;
    }
    return;
  }
  // wide: every thread holds an output, a block reduction
  const size_t idx = (size_t)blk * blockDim.x + threadIdx.x;
  const float vsum = idx < nout ? sum_chunks_serial(a.gw_slab, nout, a.nchunks, idx) : 0.f;
  float p_mul = 0.f, p_div = 0.f;
  if (idx < nout) gw_fin(q, a, gw_pre(g, a, idx), vsum, (float)g.nbw, p_mul, p_div);
  const float4 r = block_sum4(make_float4(p_mul, p_div, 0.f, 0.f), red);
  if (threadIdx.x == 0) {
    a.wpart[2 * blk] = r.x;
    a.wpart[2 * blk + 1] = r.y;
  }
}

// one output of the grad_alpha slab: G = d loss / d alpha_q into gaq; with gapart set, its terms of
// alpha_cim_bwd_block's first sweep.  Loads first (ga_pre, ahead of the slab sums), as gw_pre.
struct GaPre {
  int e;       // alpha_cim element (i, k, j, o), -1: a padding channel
  float g, v;  // gaq (gaq_ready), alpha_cim (gapart)
};

__device__ inline GaPre ga_pre(const Geo& g, const ModuleTail& a, size_t idx) {
  GaPre p;
  const int nkj = g.nbw * g.nba;
  const int o = (int)(idx % g.Opad);
  const int qq = (int)(idx / g.Opad);  // (i, k, j)
  const int kj = qq % nkj, i = qq / nkj;
  const int k = kj / g.nba, j = kj - k * g.nba;
  p.e = o < g.O ? ((i * g.nbw + k) * g.nba + j) * g.O + o : -1;
  p.g = (p.e >= 0 && a.gaq_ready) ? a.gaq[p.e] : 0.f;
  p.v = (p.e >= 0 && a.gapart) ? a.alpha_cim[p.e] : 0.f;
  return p;
}

__device__ inline float4 ga_fin(const Geo& g, const LsqArgs& q, const ModuleTail& a, const GaPre& p, size_t idx,
                                float s) {
  float4 part = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.e < 0) return part;
  float G;
  if (a.gaq_ready) {
    G = p.g;
  } else {
    const int kj = (int)((idx / g.Opad) % (size_t)(g.nbw * g.nba));
    G = (a.cgrad * a.ckj[kj]) * s;  // lsq.py:323-334
    a.gaq[p.e] = G;
  }
  if (a.gapart) {  // alpha_cim_bwd_block's first sweep, this element
    const float scale = a.scal[2], mx = a.scal[3], mn = a.scal[4];
    const float qp_al = (float)((1 << q.nbits_alpha) - 1);
    const float v = p.v;
    const float t = v / scale;
    const float rp = round_pass_value(t);
    const float c = clamp_nan(rp, 1.f, qp_al);
    const bool pass = (rp >= 1.f) && (rp <= qp_al);
    const float gt = pass ? G * scale : 0.f;
    part = make_float4(G * c, -gt * (t / scale), ((mx != mx) ? (v != v) : (v == mx)) ? 1.f : 0.f,
                       ((mn != mn) ? (v != v) : (v == mn)) ? 1.f : 0.f);
  }
  return part;
}

__device__ inline void galpha_role(const Geo& g, const LsqArgs& q, const ModuleTail& a, int blk, float* red) {
  const size_t nout = (size_t)g.T * g.nbw * g.nba * g.Opad;
  if (a.wide) {
    const size_t idx = (size_t)blk * blockDim.x + threadIdx.x;
    const float s = (a.gaq_ready || idx >= nout) ? 0.f : sum_chunks_serial(a.ga_slab, nout, a.nchunks, idx);
    const float4 part = idx < nout ? ga_fin(g, q, a, ga_pre(g, a, idx), idx, s) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.gapart) {
      const float4 r = block_sum4(part, red);
      if (threadIdx.x == 0) reinterpret_cast<float4*>(a.gapart)[blk] = r;
    }
    return;
  }
  if (a.lpr == 0) {  // scalar, as gw_lsq_role
    const size_t idx = (size_t)blk * 64 + (threadIdx.x & 63);
    const GaPre pre = (threadIdx.x < 64 && idx < nout) ? ga_pre(g, a, idx) : GaPre{-1, 0.f, 0.f};
    const float sv = a.gaq_ready ? 0.f : reduce_chunks(a.ga_slab, nout, a.nchunks, idx < nout ? idx : 0, red);
    if (threadIdx.x >= 64) return;
    float4 part = ga_fin(g, q, a, pre, idx, sv);
    if (a.gapart) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        part.x += __shfl_xor(part.x, off);
        part.y += __shfl_xor(part.y, off);
        part.z += __shfl_xor(part.z, off);
        part.w += __shfl_xor(part.w, off);
      }
      if (threadIdx.x == 0) reinterpret_cast<float4*>(a.gapart)[blk] = part;
    }
    return;
  }
  const size_t i0 = ((size_t)blk * a.lpr + (threadIdx.x & (a.lpr - 1))) * 4;
  const bool mine = (int)threadIdx.x < a.lpr && i0 < nout;
  GaPre pre[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) pre[u] = mine ? ga_pre(g, a, i0 + u) : GaPre{-1, 0.f, 0.f};
  const float4 s = a.gaq_ready ? make_float4(0.f, 0.f, 0.f, 0.f)
                               : reduce_chunks4(a.ga_slab, nout, a.nchunks, i0 < nout ? i0 : 0, a.lpr,
                                                reinterpret_cast<float4*>(red));
  if (threadIdx.x >= 64) return;
  float4 part = make_float4(0.f, 0.f, 0.f, 0.f);
  if (mine) {
    const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 t = ga_fin(g, q, a, pre[u], i0 + u, sv[u]);
      part.x += t.x;
      part.y += t.y;
      part.z += t.z;
      part.w += t.w;
    }
  }
  if (a.gapart) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      part.x += __shfl_xor(part.x, off);
      part.y += __shfl_xor(part.y, off);
      part.z += __shfl_xor(part.z, off);
      part.w += __shfl_xor(part.w, off);
    }
    if (threadIdx.x == 0) reinterpret_cast<float4*>(a.gapart)[blk] = part;
  }
}

// Backward of alpha_q = clamp(round_pass(a / scale), 1, qp) * scale, scale = (max - min) / N,
// from G = d loss / d alpha_q, as torch's engine runs it: DivBackward wrt a, then the scale's
// MulBackward / DivBackward sums -> (max - min) / N -> MinBackward, then MaxBackward, each
// spread evenly over ties.
__device__ inline void alpha_cim_bwd_block(const LsqArgs& q, const ModuleTail& a, float* red) {
  const float scale = a.scal[2], mx = a.scal[3], mn = a.scal[4];
  const float qp_al = (float)((1 << q.nbits_alpha) - 1);
  const float N = (float)((1 << q.nbits_alpha) - 2);
  const float* G = a.gaq;
  float s_mul = 0.f, s_div = 0.f, cmax = 0.f, cmin = 0.f;
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float v = a.alpha_cim[e];
    const float t = v / scale;
    const float rp = round_pass_value(t);
    const float c = clamp_nan(rp, 1.f, qp_al);
    const bool pass = (rp >= 1.f) && (rp <= qp_al);
    const float gt = pass ? G[e] * scale : 0.f;
    s_mul += G[e] * c;
    s_div += -gt * (t / scale);
    cmax += ((mx != mx) ? (v != v) : (v == mx)) ? 1.f : 0.f;
    cmin += ((mn != mn) ? (v != v) : (v == mn)) ? 1.f : 0.f;
  }
  const float4 r = block_sum4(make_float4(s_mul, s_div, cmax, cmin), red);
  s_mul = r.x;
  s_div = r.y;
  cmax = r.z;
  cmin = r.w;
  const float gscale = s_mul + s_div;  // d loss / d scale
  const float gdiff = gscale / N;      // DivBackward of (max - min) / N
  const float pmax = gdiff / cmax, pmin = -gdiff / cmin;
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float v = a.alpha_cim[e];
    const float t = v / scale;
    const float rp = round_pass_value(t);
    const bool pass = (rp >= 1.f) && (rp <= qp_al);
    const float gt = pass ? G[e] * scale : 0.f;
    const bool ismin = (mn != mn) ? (v != v) : (v == mn);
    const bool ismax = (mx != mx) ? (v != v) : (v == mx);
    float r = gt / scale;          // DivBackward wrt a
    r = r + (ismin ? pmin : 0.f);  // MinBackward reaches alpha_cim before MaxBackward
    r = r + (ismax ? pmax : 0.f);
    a.grad_alpha_cim[e] = a.accum ? a.grad_alpha_cim[e] + r : r;
  }
}

// d loss / d alpha_weight = (sum G*rp + sum div-term) * gs_w  (GradScale's MulBackward);
// d loss / d alpha_act = (sum of the act-LSQ partials) * gs_a.
__device__ inline void lsq_finish_block(const LsqArgs& q, const ModuleTail& a, float* red) {
  float m = 0.f, d = 0.f, s = 0.f;
  for (int t = threadIdx.x; t < a.nwb; t += blockDim.x) {
    m += a.wpart[2 * t];
    d += a.wpart[2 * t + 1];
  }
  for (int t = threadIdx.x; t < a.napart; t += blockDim.x) s += a.apart[t];
  const float4 r = block_sum4(make_float4(m, d, s, 0.f), red);
  m = r.x;
  d = r.y;
  s = r.z;
  if (threadIdx.x == 0) {
    const float gw = (m + d) * q.gs_w;  // MulBackward's contribution reaches sw first, then DivBackward's
    const float ga = s * q.gs_a;
    a.grad_alpha_w[0] = a.accum ? a.grad_alpha_w[0] + gw : gw;
    a.grad_alpha_act[0] = a.accum ? a.grad_alpha_act[0] + ga : ga;
  }
}

// The epilogue's last step (module_bwd_finish_kernel): alpha_cim's quantiser backward and the
// two step-size gradients from the partials module_bwd_tail_kernel left.  It is a chain of
// dependent memory round trips, so with nalpha <= 8 * 1024 every load is issued up front
// (alpha_cim, d loss / d alpha_q, the accumulated gradient, both partial sets), the two
// reductions share one pass, and the second sweep runs from registers.  Same per-thread
// order, same sums as the two-sweep form (alpha_cim_bwd_block + lsq_finish_block).
template <int N>
__device__ inline void block_sumn(float (&v)[N], float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], o);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int i = 0; i < N; ++i) red[w * N + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = red[i];
  for (int k = 1; k < nw; ++k)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += red[k * N + i];
  __syncthreads();
}

__device__ inline void module_finish_block(const LsqArgs& q, const ModuleTail& a, float* red) {
  constexpr int PER = 8;
  if (q.nbits_alpha > 0 && q.nalpha > PER * (int)blockDim.x) {  // large alpha_cim: two sweeps
    alpha_cim_bwd_block(q, a, red);
    lsq_finish_block(q, a, red);
    return;
  }
  const bool has_a = q.nbits_alpha > 0;
  float av[PER], gv[PER], old[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + u * (int)blockDim.x;
    const bool in = has_a && e < q.nalpha;
    av[u] = in ? a.alpha_cim[e] : 0.f;
    gv[u] = in ? a.gaq[e] : 0.f;
    old[u] = (in && a.accum) ? a.grad_alpha_cim[e] : 0.f;
  }
  float m = 0.f, d = 0.f, sp = 0.f;
  for (int t = threadIdx.x; t < a.nwb; t += blockDim.x) {
    m += a.wpart[2 * t];
    d += a.wpart[2 * t + 1];
  }
  for (int t = threadIdx.x; t < a.napart; t += blockDim.x) sp += a.apart[t];
  const float scale = has_a ? a.scal[2] : 1.f, mx = has_a ? a.scal[3] : 0.f, mn = has_a ? a.scal[4] : 0.f;
  const float qp_al = (float)((1 << q.nbits_alpha) - 1);
  const float N = (float)((1 << q.nbits_alpha) - 2);
  float s_mul = 0.f, s_div = 0.f, cmax = 0.f, cmin = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + u * (int)blockDim.x;
    if (has_a && e < q.nalpha) {  // as alpha_cim_bwd_block's first sweep
      const float v = av[u];
      const float t = v / scale;
      const float rp = round_pass_value(t);
      const float c = clamp_nan(rp, 1.f, qp_al);
      const bool pass = (rp >= 1.f) && (rp <= qp_al);
      const float gt = pass ? gv[u] * scale : 0.f;
      s_mul += gv[u] * c;
      s_div += -gt * (t / scale);
      cmax += ((mx != mx) ? (v != v) : (v == mx)) ? 1.f : 0.f;
      cmin += ((mn != mn) ? (v != v) : (v == mn)) ? 1.f : 0.f;
    }
  }
  float r[8] = {s_mul, s_div, cmax, cmin, m, d, sp, 0.f};
  block_sumn<8>(r, red);
  if (has_a) {
    const float gdiff = (r[0] + r[1]) / N;  // d loss / d scale, then DivBackward of (max - min) / N
    const float pmax = gdiff / r[2], pmin = -gdiff / r[3];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = threadIdx.x + u * (int)blockDim.x;
      if (e < q.nalpha) {
        const float v = av[u];
        const float t = v / scale;
        const float rp = round_pass_value(t);
        const bool pass = (rp >= 1.f) && (rp <= qp_al);
        const float gt = pass ? gv[u] * scale : 0.f;
        const bool ismin = (mn != mn) ? (v != v) : (v == mn);
        const bool ismax = (mx != mx) ? (v != v) : (v == mx);
        float rr = gt / scale;
        rr = rr + (ismin ? pmin : 0.f);
        rr = rr + (ismax ? pmax : 0.f);
        a.grad_alpha_cim[e] = a.accum ? old[u] + rr : rr;
      }
    }
  }
  if (threadIdx.x == 0) {  // as lsq_finish_block
    const float gw = (r[4] + r[5]) * q.gs_w;
    const float ga = r[6] * q.gs_a;
    a.grad_alpha_w[0] = a.accum ? a.grad_alpha_w[0] + gw : gw;
    a.grad_alpha_act[0] = a.accum ? a.grad_alpha_act[0] + ga : ga;
  }
}

// The wide epilogue's last step (module_bwd_finish_wide_kernel, a.gapart set): every block sums
// the tail blocks' first-sweep partials in the same order, then runs the second sweep of
// alpha_cim_bwd_block over its 1024-element slice; block 0 also finishes the step sizes.
__device__ inline void module_finish_wide_block(const LsqArgs& q, const ModuleTail& a, float* red, int blk) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int t = threadIdx.x; t < a.nga; t += blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(a.gapart)[t];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  const float4 r = block_sum4(acc, red);
  const float scale = a.scal[2], mx = a.scal[3], mn = a.scal[4];
  const float qp_al = (float)((1 << q.nbits_alpha) - 1);
  const float N = (float)((1 << q.nbits_alpha) - 2);
  const float gdiff = (r.x + r.y) / N;  // d loss / d scale, then DivBackward of (max - min) / N
  const float pmax = gdiff / r.z, pmin = -gdiff / r.w;
  const int e = blk * blockDim.x + threadIdx.x;
  if (e < q.nalpha) {
    const float v = a.alpha_cim[e];
    const float t = v / scale;
    const float rp = round_pass_value(t);
    const bool pass = (rp >= 1.f) && (rp <= qp_al);
    const float gt = pass ? a.gaq[e] * scale : 0.f;
    const bool ismin = (mn != mn) ? (v != v) : (v == mn);
    const bool ismax = (mx != mx) ? (v != v) : (v == mx);
    float rr = gt / scale;
    rr = rr + (ismin ? pmin : 0.f);
    rr = rr + (ismax ? pmax : 0.f);
    a.grad_alpha_cim[e] = a.accum ? a.grad_alpha_cim[e] + rr : rr;
  }
  if (blk == 0) lsq_finish_block(q, a, red);
}

}  // namespace cimq

// cimq_lsq.hip -- the LSQ quantisers of Conv2dLSQCiM.forward (lsq.py:544-571) fused around
// the CiM kernels for the module entry points (cimq_module_forward / _backward):
//   sa = grad_scale(alpha_act, 1/sqrt(numel(x) Qp_a)), sw = grad_scale(alpha_weight, ...),
//   w_q = round_pass(clamp(w / sw, Qn_w, Qp_w)) * sw,
//   alpha_q = clamp(round_pass(alpha_cim / scale), 1, 2^b - 1) * scale,
//   scale = (max(alpha_cim) - min(alpha_cim)) / (2^b - 2),
// each value with the reference's fp32 op sequence, and their autograd backward with the
// order in which torch's engine accumulates the contributions.
#pragma once
#include "cimq_lsq_dev.h"

namespace cimq {

// =========================================================================================
// forward prologue of the module entry points: one launch does the activation quantiser and
// its slicing (the last nact_blocks blocks) and, in the first blocks, the weight quantiser
// feeding every weight operand layout, alpha_cim's quantiser feeding the ADC thresholds, and
// the scalars the later kernels read (one designated block).  Nothing is materialised in
// between: each thread evaluates w_q / alpha_q for the elements it packs.
// =========================================================================================
struct ModulePrep {
  const float* x;
  const float* alpha_act;
  const float* alpha_w;
  const float* weight;
  const float* alpha_cim;
  const float* signed_act;
  const int8_t* bmask;
  const float* beta;  // beta_cim of the shift ADC module entry points (null otherwise)
  uint8_t* xcf;
  uint8_t* xcb;
  v4i* wfrag;
  v4i* wgx;   // general / dense grad_x operand (nwg == 0 on the v7 path)
  v4i* wcy;   // v8 grad_x operand (nwc == 0 unless the v7 backward applies)
  v4i* wf5;   // cim_fwd5_kernel's weight operand (nw5 == 0 unless f5_plan applies)
  F5W f5;
  v4i* wg5;   // cim_bwd_gx5_kernel's weight operand (nwx5 == 0 unless x5_plan applies)
  v4i* wx6;   // cim_bwd_r6_kernel's gx operand (nwx6 == 0 unless r6_plan applies)
  int ncpbt;
  Params pp;
  float* scal;  // [0] sa, [1] sw, [2] alpha scale, [3] max(alpha_cim), [4] min(alpha_cim)
  int nact_blocks;
  int nwf, nwg, nwc, npp, nw5, nwx5, nwx6;  // items of the weight-side roles
  const float* amm;             // wide alpha_cim: [namm][2] per-block (max, min) of alpha_minmax_kernel
  int namm;                     // 0: every weight block reduces alpha_cim itself
};

// the weight side of the prologue: block wb of nwblk (quantised weight operands, alpha_cim's
// quantiser into the ADC thresholds, and in block 0 the step sizes / literal-ADC flag)
__device__ inline void module_prep_weights(const Geo& g, const LsqArgs& q, const ModulePrep& a, int wb, int nwblk,
                                           float* red) {
  const float sa = grad_scale_value(a.alpha_act[0], q.gs_a);  // lsq.py:547-548
  const float sw = grad_scale_value(a.alpha_w[0], q.gs_w);  // lsq.py:553-554
  ASrc as{nullptr, 1, 0.f, 0.f};
  float mx = 0.f, mn = 0.f;
  // alpha_cim is read once into registers when it fits (<= AP per thread): every load in
  // flight together, not one dependent round trip per loop iteration
  constexpr int AP = 16;
  float av[AP];
  const bool inreg = q.nalpha <= AP * (int)blockDim.x;
  if (q.nbits_alpha > 0) {  // lsq.py:566-571
    mx = -INFINITY;
    mn = INFINITY;
    if (a.namm > 0) {
      for (int t = threadIdx.x; t < a.namm; t += blockDim.x) {
        mx = nan_max(mx, a.amm[2 * t]);
        mn = nan_min(mn, a.amm[2 * t + 1]);
      }
    } else if (inreg) {
#pragma unroll
      for (int u = 0; u < AP; ++u) {
        const int e = threadIdx.x + u * (int)blockDim.x;
        av[u] = e < q.nalpha ? a.alpha_cim[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < AP; ++u) {
        if ((int)threadIdx.x + u * (int)blockDim.x < q.nalpha) {
          const float v = av[u];
          mx = (v != v || mx != mx) ? v + mx : fmaxf(mx, v);
          mn = (v != v || mn != mn) ? v + mn : fminf(mn, v);
        }
      }
    } else {
      for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
        const float v = a.alpha_cim[e];
        mx = (v != v || mx != mx) ? v + mx : fmaxf(mx, v);
        mn = (v != v || mn != mn) ? v + mn : fminf(mn, v);
      }
    }
    const float2 r = block_max_min(mx, mn, red);
    mx = r.x;
    mn = r.y;
    as.a = a.alpha_cim;
    as.scale = (mx - mn) / (float)((1 << q.nbits_alpha) - 2);
    as.qp_al = (float)((1 << q.nbits_alpha) - 1);
  }
  const WSrc ws{a.weight, sw, 1, q.qn_w, q.qp_w};  // lsq.py:555
  if (wb == 0) {
    // literal-ADC flag: any entry whose alpha_q / scales break the threshold search
    bool lit = false;
    if (g.mode == ADC_SIGN || g.mode == ADC_TERNARY) {
      lit = !scales_ok(sw, sa);
      if (as.a && a.namm > 0) {
        // alpha_q is monotone in alpha_cim for a positive finite scale (and 0 / NaN / inf for
        // every entry otherwise), so its extremes decide: the entries at max and min
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float v = clamp_nan(round_pass_value((u ? mn : mx) / as.scale), 1.f, as.qp_al) * as.scale;
          lit = lit || !(v > 0.f && isfinite(v));
        }
      } else if (as.a && inreg) {
#pragma unroll
        for (int u = 0; u < AP; ++u) {
          if ((int)threadIdx.x + u * (int)blockDim.x < q.nalpha) {  // as ASrc::get on the loaded value
            const float v = clamp_nan(round_pass_value(av[u] / as.scale), 1.f, as.qp_al) * as.scale;
            lit = lit || !(v > 0.f && isfinite(v));
          }
        }
      } else if (as.a) {
        for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
          const float v = as.get(e);
          lit = lit || !(v > 0.f && isfinite(v));
        }
      }
    }
    if (a.beta)  // the shift ADC's thresholds need a finite beta everywhere (params_item)
      for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) lit = lit || !isfinite(a.beta[e]);
    lit = __syncthreads_or(lit);
    if (threadIdx.x == 0) {
      a.scal[0] = sa;
      a.scal[1] = sw;
      a.scal[2] = as.scale;
      a.scal[3] = mx;
      a.scal[4] = mn;
      a.pp.flags[0] = lit ? 1 : 0;
      a.pp.flags[1] = a.pp.flags[2] = a.pp.flags[3] = 0;
    }
  }
  const int e1 = a.nwf, e2 = e1 + a.nwg, e3 = e2 + a.nwc, e4 = e3 + a.nw5, e5 = e4 + a.nwx5, e6 = e5 + a.nwx6,
            total = e6 + a.npp;
  for (int t = wb * blockDim.x + threadIdx.x; t < total; t += nwblk * blockDim.x) {
    if (t < e1) wfrag_item(g, ws, a.wfrag, t);
    else if (t < e2) wgx_item(g, ws, a.wgx, t - e1);
    else if (t < e3) wcy_item(g, ws, a.ncpbt, a.wcy, t - e2);
    else if (t < e4) wf5_item(g, a.f5, ws, a.wf5, t - e3);
    else if (t < e5) wg5_item(g, ws, a.wg5, t - e4);
    else if (t < e6) wx6_item(g, ws, a.wx6, t - e5);
    else (void)params_item(g, as, sw, sa, a.bmask, a.pp, t - e6, a.beta);
  }
}

__global__ __launch_bounds__(256) void prep_module_kernel(Geo g, LsqArgs q, ModulePrep a) {
  __shared__ float4 red4[16];
  float* red = reinterpret_cast<float*>(red4);
  // the few weight-side blocks go first so their latency-bound work overlaps the act stream
  // (none when the weight side was prepared beforehand: cimq_module_prepare)
  const int nwblk = (int)gridDim.x - a.nact_blocks;
  if ((int)blockIdx.x >= nwblk) {
    const float sa = grad_scale_value(a.alpha_act[0], q.gs_a);  // lsq.py:547-548
    const int ab = (int)blockIdx.x - nwblk;
    const bool sgn = a.signed_act[0] != 0.f;
    __shared__ __attribute__((aligned(16))) uint32_t lut[kActLutMax * 4];  // the RAW_LSQ word table (act_range)
    act_range(g, a.x, sa, sgn, a.xcf, a.xcb, (long long)ab * blockDim.x + threadIdx.x,
              (long long)a.nact_blocks * blockDim.x, lut);
    return;
  }
  module_prep_weights(g, q, a, (int)blockIdx.x, nwblk, red);
}

// The job of block b in a packed launch: the number of job starts blk0[1 .. n-1] at or below b, counted
// over the whole (fixed-size) table -- independent scalar loads of the kernel arguments and a compare
// chain, instead of a search loop whose every step waits on the previous step's argument load
template <int NJ>
__device__ inline int job_of(const int (&blk0)[NJ + 1], int n, int b) {
  int j = 0;
#pragma unroll
  for (int t = 1; t < NJ; ++t) j += (t < n && b >= blk0[t]) ? 1 : 0;
  return j;
}

// The weight side of several layers' prologues in one launch (cimq_module_prepare): a layer's
// weight work is a few latency-bound blocks, so packing the layers of a network into one grid
// pays that latency once instead of once per layer.  The jobs travel as kernel arguments.
struct PrepJob {
  Geo g;
  LsqArgs q;
  ModulePrep a;
  int nwblk;
};
constexpr int kPrepJobs = 7;
struct PrepPack {
  int n;
  int blk0[kPrepJobs + 1];  // first block of each job, blk0[n] = grid
  PrepJob job[kPrepJobs];
};
static_assert(sizeof(PrepPack) <= 4000, "PrepPack exceeds the kernel-argument budget");

__global__ __launch_bounds__(256) void prep_weights_many_kernel(PrepPack p) {
  __shared__ float4 red4[16];
  const int j = job_of<kPrepJobs>(p.blk0, p.n, (int)blockIdx.x);
  module_prep_weights(p.job[j].g, p.job[j].q, p.job[j].a, (int)blockIdx.x - p.blk0[j], p.job[j].nwblk,
                      reinterpret_cast<float*>(red4));
}

__global__ __launch_bounds__(1024, 8) void module_bwd_tail_kernel(Geo g, LsqArgs q, ModuleTail a) {
  __shared__ __attribute__((aligned(16))) float red[4 * 1024];
  const int b = (int)blockIdx.x;
  if (b < a.nwb) gw_lsq_role(g, q, a, b, red);
  else galpha_role(g, q, a, b - a.nwb, red);
}

// One block: the epilogue's last step after the kernel boundary (which orders the partials
// across the XCDs' L2s).  Fusing it into module_bwd_tail_kernel behind a last-block ticket
// measured slower: 18.3 us per layer for the fused launch against 5.8 + 7.5 us for the two
// (the per-block agent-scope release costs more than the boundary it replaces).
__global__ __launch_bounds__(1024) void module_bwd_finish_kernel(LsqArgs q, ModuleTail a) {
  __shared__ __attribute__((aligned(16))) float red[16 * 8];
  module_finish_block(q, a, red);
}

__global__ __launch_bounds__(1024) void module_bwd_finish_wide_kernel(LsqArgs q, ModuleTail a) {
  __shared__ __attribute__((aligned(16))) float red[16 * 8];
  module_finish_wide_block(q, a, red, (int)blockIdx.x);
}

// The epilogues of several chained layers in two launches (cimq_pending_flush): a layer's tail is
// a few microseconds of slab sums, mostly launch ramp and drain at the small layers, so the
// chained backward packs every layer's tail blocks into one grid and every finish into another.
// The jobs travel as kernel arguments, with only the geometry fields the two roles read.
struct TailGeo {
  int T, FBT, Opad, O, xbar, K, nbw, nba;
};
struct TailJob {
  TailGeo t;
  LsqArgs q;
  ModuleTail a;
};
constexpr int kTailJobs = 20;
struct TailPack {
  int n;
  int blk0[kTailJobs + 1];  // first block of each job, blk0[n] = grid
  TailJob job[kTailJobs];
};
static_assert(sizeof(TailPack) <= 4000, "TailPack exceeds the kernel-argument budget");

__device__ inline Geo geo_of(const TailGeo& t) {
  Geo g{};
  g.T = t.T;
  g.FBT = t.FBT;
  g.Opad = t.Opad;
  g.O = t.O;
  g.xbar = t.xbar;
  g.K = t.K;
  g.nbw = t.nbw;
  g.nba = t.nba;
  return g;
}

__global__ __launch_bounds__(1024, 8) void module_tail_many_kernel(TailPack p) {
  __shared__ __attribute__((aligned(16))) float red[4 * 1024];
  const int j = job_of<kTailJobs>(p.blk0, p.n, (int)blockIdx.x);
  const TailJob& jb = p.job[j];
  const Geo g = geo_of(jb.t);
  const int b = (int)blockIdx.x - p.blk0[j];
  if (b < jb.a.nwb) gw_lsq_role(g, jb.q, jb.a, b, red);
  else galpha_role(g, jb.q, jb.a, b - jb.a.nwb, red);
}

struct FinishJob {
  LsqArgs q;
  ModuleTail a;
};
constexpr int kFinishJobs = 24;
struct FinishPack {
  int n;
  int blk0[kFinishJobs + 1];
  FinishJob job[kFinishJobs];
};
static_assert(sizeof(FinishPack) <= 4000, "FinishPack exceeds the kernel-argument budget");

// one block per job, cdiv(nalpha, 1024) for a wide alpha_cim (module_finish_wide_block)
__global__ __launch_bounds__(1024) void module_finish_many_kernel(FinishPack p) {
  __shared__ __attribute__((aligned(16))) float red[16 * 8];
  const int j = job_of<kFinishJobs>(p.blk0, p.n, (int)blockIdx.x);
  const FinishJob& jb = p.job[j];
  if (jb.a.gapart) module_finish_wide_block(jb.q, jb.a, red, (int)blockIdx.x - p.blk0[j]);
  else module_finish_block(jb.q, jb.a, red);
}

// max / min of a wide alpha_cim (> kFinishInReg elements) per block, for the prologue's weight
// blocks to combine (module_prep_weights) instead of each re-reading all of alpha_cim
__global__ __launch_bounds__(256) void alpha_minmax_kernel(const float* __restrict__ alpha_cim, int n,
                                                           float* __restrict__ part) {
  __shared__ float red[4 * 16];
  float mx = -INFINITY, mn = INFINITY;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const float v = alpha_cim[e];
    mx = nan_max(mx, v);
    mn = nan_min(mn, v);
  }
  const float2 r = block_max_min(mx, mn, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = r.x;
    part[2 * blockIdx.x + 1] = r.y;
  }
}

// layout changes for the general (non-fast-path) kernels in module mode
// Parity hook: the ADC code and STE-pass bit of every partial sum, decoded from the state
// words cim_fwd_v3_kernel<.., CST> wrote (compact: bits 3*(k*nba + j) + {0 pass, 1 code != 0,
// 2 code < 0} of st32[(i*M + m)*O + o]; planes: bit k*nba + j of st64[((i*M + m)*O + o)*3 + q]),
// in the reference's [B, T, nbw, nba, P, O] order.
__global__ void decode_state_kernel(Geo g, int planes, const uint8_t* __restrict__ st, int8_t* __restrict__ code,
                                    uint8_t* __restrict__ pass) {
  const size_t n = (size_t)g.T * g.M * g.O;
  const int nkj = g.nbw * g.nba;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int o = (int)(e % g.O);
    const size_t im = e / g.O;
    const int m = (int)(im % g.M), i = (int)(im / g.M);
    const int b = m / g.P, p = m - b * g.P;
    uint64_t ps = 0, nz = 0, ng = 0;
    uint32_t w32 = 0;
    if (planes) {
      const uint64_t* s64 = reinterpret_cast<const uint64_t*>(st) + e * 3;
      ps = s64[0]; nz = s64[1]; ng = s64[2];
    } else {
      w32 = reinterpret_cast<const uint32_t*>(st)[e];
    }
    for (int kj = 0; kj < nkj; ++kj) {
      const int k = kj / g.nba, j = kj - k * g.nba;
      int bp, bz, bn;
      if (planes) {
        bp = (int)((ps >> kj) & 1u); bz = (int)((nz >> kj) & 1u); bn = (int)((ng >> kj) & 1u);
      } else {
        bp = (w32 >> (3 * kj)) & 1; bz = (w32 >> (3 * kj + 1)) & 1; bn = (w32 >> (3 * kj + 2)) & 1;
      }
      const size_t di = ((((size_t)b * g.T + i) * g.nbw + k) * g.nba + j) * g.P * g.O + (size_t)p * g.O + o;
      code[di] = (int8_t)(bz ? (bn ? -1 : 1) : 0);
      pass[di] = (uint8_t)bp;
    }
  }
}

__global__ void bpo_to_nchw_kernel(Geo g, const float* __restrict__ src, float* __restrict__ dst) {
  const size_t n = (size_t)g.M * g.O;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e % g.P, bo = e / g.P;
    const size_t o = bo % g.O, b = bo / g.O;
    dst[e] = src[(b * g.P + p) * g.O + o];
  }
}
__global__ void nchw_to_bpo_kernel(Geo g, const float* __restrict__ src, float* __restrict__ dst) {
  const size_t n = (size_t)g.M * g.O;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t o = e % g.O, m = e / g.O;
    const size_t p = m % g.P, b = m / g.P;
    dst[e] = src[(b * g.O + o) * g.P + p];
  }
}

}  // namespace cimq

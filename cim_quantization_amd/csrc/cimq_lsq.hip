// cimq_lsq.hip -- the LSQ quantisers of Conv2dLSQCiM.forward (lsq.py:544-571) fused around
// the CiM kernels for the module entry points (cimq_module_forward / _backward):
//   sa = grad_scale(alpha_act, 1/sqrt(numel(x) Qp_a)), sw = grad_scale(alpha_weight, ...),
//   w_q = round_pass(clamp(w / sw, Qn_w, Qp_w)) * sw,
//   alpha_q = clamp(round_pass(alpha_cim / scale), 1, 2^b - 1) * scale,
//   scale = (max(alpha_cim) - min(alpha_cim)) / (2^b - 2),
// each value with the reference's fp32 op sequence, and their autograd backward with the
// order in which torch's engine accumulates the contributions.
#pragma once
#include "cimq_device.h"

namespace cimq {

struct LsqArgs {
  float qn_w, qp_w;      // weight clamp range
  float gs_a, gs_w;      // grad_scale factors
  int nbits_alpha;       // 0: no alpha_cim
  int nalpha;            // numel(alpha_cim) = T*nbw*nba*O
};

// grad_scale(x, s) forward value: (x - x*s).detach() + x*s  (_quan_base.py grad_scale)
__device__ inline float grad_scale_value(float x, float s) {
  const float yg = x * s;
  const float d = x - yg;
  return d + yg;
}

// round_pass(v) forward value: (v.round() - v).detach() + v
__device__ inline float round_pass_value(float v) {
  const float r = rintf(v);
  return (r - v) + v;
}

// block-wide (1024 threads) reductions
__device__ inline float block_reduce_max(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = blockDim.x >> 1; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      const float a = red[threadIdx.x], b = red[threadIdx.x + s];
      red[threadIdx.x] = (a != a || b != b) ? (a + b) : fmaxf(a, b);  // torch.max propagates NaN
    }
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}
__device__ inline float block_reduce_min(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = blockDim.x >> 1; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      const float a = red[threadIdx.x], b = red[threadIdx.x + s];
      red[threadIdx.x] = (a != a || b != b) ? (a + b) : fminf(a, b);
    }
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}
__device__ inline float block_reduce_sum(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = blockDim.x >> 1; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// One block of 1024 threads.  scal[0] = sa, scal[1] = sw, scal[2] = alpha scale,
// scal[3] = max(alpha_cim), scal[4] = min(alpha_cim).
__global__ __launch_bounds__(1024) void prep_lsq_kernel(Geo g, LsqArgs q, const float* __restrict__ alpha_act,
                                                        const float* __restrict__ alpha_w,
                                                        const float* __restrict__ weight,
                                                        const float* __restrict__ alpha_cim,
                                                        float* __restrict__ scal, float* __restrict__ wq,
                                                        float* __restrict__ alpha_q) {
  __shared__ float red[1024];
  const float sa = grad_scale_value(alpha_act[0], q.gs_a);  // lsq.py:547-548
  const float sw = grad_scale_value(alpha_w[0], q.gs_w);    // lsq.py:553-554
  const int nw = g.O * g.K;
  for (int e = threadIdx.x; e < nw; e += blockDim.x) {  // lsq.py:555
    const float t = weight[e] / sw;
    const float c = clamp_nan(t, q.qn_w, q.qp_w);
    wq[e] = round_pass_value(c) * sw;
  }
  if (threadIdx.x == 0) {
    scal[0] = sa;
    scal[1] = sw;
  }
  if (q.nbits_alpha <= 0) return;
  // lsq.py:566-571
  float mx = -INFINITY, mn = INFINITY;
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float a = alpha_cim[e];
    mx = (a != a || mx != mx) ? a + mx : fmaxf(mx, a);
    mn = (a != a || mn != mn) ? a + mn : fminf(mn, a);
  }
  mx = block_reduce_max(mx, red);
  mn = block_reduce_min(mn, red);
  const float qp_al = (float)((1 << q.nbits_alpha) - 1);
  const float scale = (mx - mn) / (float)((1 << q.nbits_alpha) - 2);
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float t = alpha_cim[e] / scale;
    const float c = clamp_nan(round_pass_value(t), 1.f, qp_al);
    alpha_q[e] = c * scale;
  }
  if (threadIdx.x == 0) {
    scal[2] = scale;
    scal[3] = mx;
    scal[4] = mn;
  }
}

// grad_w reducer fused with the weight quantiser's backward: slab sum -> G = d loss / d w_q,
// then through w_q = rp * sw, rp = round_pass(clamp(w / sw)):
//   grad_weight = mask * (G * sw) / sw; partial sums of G * rp (MulBackward, d/d sw) and of
//   -grad_t1 * ((w / sw) / sw) (DivBackward wrt the divisor) per block -> wpart[2*block].
__global__ __launch_bounds__(1024) void reduce_gw_lsq_kernel(Geo g, LsqArgs q, int nchunks,
                                                             const float* __restrict__ gw_slab,
                                                             const float* __restrict__ scal,
                                                             const float* __restrict__ weight,
                                                             float* __restrict__ grad_weight,
                                                             float* __restrict__ wpart) {
  __shared__ float red[1024];
  const size_t rows = (size_t)g.T * g.FBT * 16;
  const size_t nout = rows * g.Opad;
  const size_t idx = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int sub = threadIdx.x >> 6;
  const float vsum = reduce_chunks(gw_slab, nout, nchunks, idx < nout ? idx : 0, red);
  float p_mul = 0.f, p_div = 0.f;
  if (sub == 0 && idx < nout) {
    const float v = vsum;
    const int o = (int)(idx % g.Opad);
    const size_t row = idx / g.Opad;
    const int i = (int)(row / (g.FBT * 16)), fl = (int)(row - (size_t)i * g.FBT * 16);
    const int f = i * g.xbar + fl;
    if (o < g.O && fl < g.xbar && f < g.K) {
      const float sa = scal[0], sw = scal[1];
      const float G = v * (sa / (float)g.nbw);  // d loss / d w_q (as reduce_gw_v3)
      const float w = weight[(size_t)o * g.K + f];
      const float t1 = w / sw;
      const float c = clamp_nan(t1, q.qn_w, q.qp_w);
      const float rp = round_pass_value(c);
      const float grad_rp = G * sw;
      const bool pass = (t1 >= q.qn_w) && (t1 <= q.qp_w);
      const float grad_t1 = pass ? grad_rp : 0.f;
      grad_weight[(size_t)o * g.K + f] = grad_t1 / sw;
      p_mul = G * rp;
      p_div = -grad_t1 * (t1 / sw);
    }
  }
  __syncthreads();
  red[threadIdx.x] = p_mul;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int t = 0; t < 64; ++t) a += red[t];
    wpart[2 * blockIdx.x] = a;
  }
  __syncthreads();
  red[threadIdx.x] = p_div;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int t = 0; t < 64; ++t) a += red[t];
    wpart[2 * blockIdx.x + 1] = a;
  }
}

// d loss / d alpha_weight = (sum G*rp + sum div-term) * gs_w  (GradScale's MulBackward);
// d loss / d alpha_act = (sum of the act-LSQ partials) * gs_a.  One block of 1024 threads.
__global__ __launch_bounds__(1024) void lsq_scalars_finish_kernel(LsqArgs q, int nw, const float* __restrict__ wpart,
                                                                  int na, const float* __restrict__ apart,
                                                                  float* __restrict__ grad_alpha_w,
                                                                  float* __restrict__ grad_alpha_act) {
  __shared__ float red[1024];
  float m = 0.f, d = 0.f, a = 0.f;
  for (int t = threadIdx.x; t < nw; t += blockDim.x) {
    m += wpart[2 * t];
    d += wpart[2 * t + 1];
  }
  for (int t = threadIdx.x; t < na; t += blockDim.x) a += apart[t];
  m = block_reduce_sum(m, red);
  d = block_reduce_sum(d, red);
  a = block_reduce_sum(a, red);
  if (threadIdx.x == 0) {
    const float gsw = m + d;  // MulBackward's contribution reaches sw first, then DivBackward's
    grad_alpha_w[0] = gsw * q.gs_w;
    grad_alpha_act[0] = a * q.gs_a;
  }
}

// Backward of alpha_q = clamp(round_pass(a / scale), 1, qp) * scale, scale = (max - min) / N,
// from G = d loss / d alpha_q.  One block of 1024 threads; ga[] = d loss / d alpha_cim.
__global__ __launch_bounds__(1024) void alpha_cim_bwd_kernel(LsqArgs q, const float* __restrict__ alpha_cim,
                                                             const float* __restrict__ scal,
                                                             const float* __restrict__ G,
                                                             float* __restrict__ ga) {
  __shared__ float red[1024];
  const float scale = scal[2], mx = scal[3], mn = scal[4];
  const float qp_al = (float)((1 << q.nbits_alpha) - 1);
  const float N = (float)((1 << q.nbits_alpha) - 2);
  float s_mul = 0.f, s_div = 0.f, cmax = 0.f, cmin = 0.f;
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float a = alpha_cim[e];
    const float t = a / scale;
    const float rp = round_pass_value(t);
    const float c = clamp_nan(rp, 1.f, qp_al);
    const float gc = G[e] * scale;
    const bool pass = (rp >= 1.f) && (rp <= qp_al);
    const float gt = pass ? gc : 0.f;
    ga[e] = gt / scale;  // DivBackward wrt a
    s_mul += G[e] * c;
    s_div += -gt * (t / scale);
    cmax += ((mx != mx) ? (a != a) : (a == mx)) ? 1.f : 0.f;
    cmin += ((mn != mn) ? (a != a) : (a == mn)) ? 1.f : 0.f;
  }
  s_mul = block_reduce_sum(s_mul, red);
  s_div = block_reduce_sum(s_div, red);
  cmax = block_reduce_sum(cmax, red);
  cmin = block_reduce_sum(cmin, red);
  const float gscale = s_mul + s_div;  // d loss / d scale
  const float gdiff = gscale / N;      // DivBackward of (max - min) / N
  const float gmax = gdiff, gmin = -gdiff;
  const float pmax = gmax / cmax, pmin = gmin / cmin;  // evenly distributed over ties
  for (int e = threadIdx.x; e < q.nalpha; e += blockDim.x) {
    const float a = alpha_cim[e];
    const bool ismin = (mn != mn) ? (a != a) : (a == mn);
    const bool ismax = (mx != mx) ? (a != a) : (a == mx);
    float v = ga[e];
    v = v + (ismin ? pmin : 0.f);  // MinBackward reaches alpha_cim before MaxBackward
    v = v + (ismax ? pmax : 0.f);
    ga[e] = v;
  }
}

// layout changes for the general (non-fast-path) kernels in module mode
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

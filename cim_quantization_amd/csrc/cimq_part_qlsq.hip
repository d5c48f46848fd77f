// cimq_part_qlsq.hip -- the plain LSQ modules of models/_modules/lsq.py on MI355X:
//   ActLSQ (lsq.py:620-662) and the weight quantisers of Conv2dLSQ (:389-436) / LinearLSQ
//   (:591-617): x_q = round_pass(clamp(x / s, Qn, Qp)) [* s], s = grad_scale(alpha, g), and
//   its autograd backward (STE through round_pass, clamp mask, the two DivBackward / MulBackward
//   sums for s), one elementwise launch + one partial-sum launch each way;
//   Conv2dLSQ's conv of integer codes, conv2d(x_q, w_q) * act_scale * w_scale, as an
//   implicit-GEMM int8 conv on v_mfma_i32_16x16x64_i8 (exact int32 sums, so the fp32 result
//   is the reference's conv of integer-valued fp32 tensors while |sum| < 2^24), and the
//   elementwise part of its backward.
// Own translation unit of libcimq.so (extern "C" entry points declared in include/cimq.h).
#define CIMQ_TU_QLSQ
#include "cimq_host.h"

namespace cimq {

// ---------------------------------------------------------------------------------------
// LSQ quantiser
// ---------------------------------------------------------------------------------------
struct LsqQ {
  long long n;
  float qn, qp;
  int scaled;  // LinearLSQ: the quantised value times s (lsq.py:611); else the integer code
  int vec;     // x and out 16-byte aligned: float4 loads / stores (else element-wise: a parameter
               // view inside a flat buffer, a batch slice, sits at any 4-byte offset)
};

__device__ inline float lsq_code(float x, float s, float qn, float qp) {
  return round_pass_value(clamp_nan(x / s, qn, qp));  // lsq.py:412 / :611 / :656
}

__global__ __launch_bounds__(256) void lsq_quant_fwd_kernel(LsqQ q, const float* __restrict__ x,
                                                            const float* __restrict__ s_p, float* __restrict__ out) {
  const float s = *s_p;
  const long long n4 = q.vec ? q.n >> 2 : 0;
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += step) {
    const float4 v = reinterpret_cast<const float4*>(x)[t];
    float4 r;
    r.x = lsq_code(v.x, s, q.qn, q.qp);
    r.y = lsq_code(v.y, s, q.qn, q.qp);
    r.z = lsq_code(v.z, s, q.qn, q.qp);
    r.w = lsq_code(v.w, s, q.qn, q.qp);
    if (q.scaled) { r.x *= s; r.y *= s; r.z *= s; r.w *= s; }
    reinterpret_cast<float4*>(out)[t] = r;
  }
  for (long long e = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; e < q.n; e += step) {
    const float r = lsq_code(x[e], s, q.qn, q.qp);
    out[e] = q.scaled ? r * s : r;
  }
}

// block sums of two values -> part[2 * block] (wave butterfly, then the waves in order)
__device__ inline void block_sum2_store(float a, float b, float* part) {
  __shared__ float red[2 * 16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sa = red[0], sb = red[1];
    for (int i = 1; i < nw; ++i) {
      sa += red[2 * i];
      sb += red[2 * i + 1];
    }
    part[2 * blockIdx.x] = sa;
    part[2 * blockIdx.x + 1] = sb;
  }
}

// autograd of out = round_pass(clamp(x / s, Qn, Qp)) [* s]:
//   grad_r = g [* s] (MulBackward), STE through round_pass, clamp passes Qn <= t <= Qp,
//   grad_x = grad_t / s (DivBackward wrt x); per block: sum g * r (MulBackward wrt s, scaled
//   only) and sum -grad_t * ((x / s) / s) (DivBackward wrt s, torch's div_tensor_other_backward)
__global__ __launch_bounds__(256) void lsq_quant_bwd_kernel(LsqQ q, const float* __restrict__ x,
                                                            const float* __restrict__ s_p,
                                                            const float* __restrict__ gout, float* __restrict__ gx,
                                                            float* __restrict__ part) {
  const float s = *s_p;
  float pm = 0.f, pd = 0.f;
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < q.n; e += step) {
    const float g = gout[e];
    const float t = x[e] / s;
    const float c = clamp_nan(t, q.qn, q.qp);
    const float r = round_pass_value(c);
    const float grad_r = q.scaled ? g * s : g;
    const bool pass = (t >= q.qn) && (t <= q.qp);
    const float grad_t = pass ? grad_r : 0.f;
    gx[e] = grad_t / s;
    if (q.scaled) pm += g * r;
    pd += -grad_t * (t / s);
  }
  block_sum2_store(pm, pd, part);
}

// one block: grad_s = sum(mul partials) + sum(div partials) (MulBackward's contribution
// reaches s before DivBackward's, as torch's engine orders them), or, with two = 1, the two
// sums separately (out[0], out[1])
__global__ __launch_bounds__(256) void lsq_partials_finish_kernel(int nblk, const float* __restrict__ part,
                                                                  int two, float* __restrict__ out) {
  __shared__ float red[2 * 16];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sa = red[0], sb = red[1];
    for (int i = 1; i < nw; ++i) {
      sa += red[2 * i];
      sb += red[2 * i + 1];
    }
    if (two) {
      out[0] = sa;
      out[1] = sb;
    } else {
      out[0] = sa + sb;
    }
  }
}

// ---------------------------------------------------------------------------------------
// int8 conv of integer codes (Conv2dLSQ, lsq.py:436): y0 = conv2d(x_q, w_q) (+ bias),
// y = y0 * act_scale * w_scale.  Implicit GEMM D[o][pixel] = sum_k W[o][k] X[k][pixel] with
// the contraction ordered k = (kh, kw, c), channels fastest (integer sums: any order is exact):
// a pre-pass writes the codes as int8 NHWC with channels padded to 16, so one lane's 16
// consecutive k -- 16 channels of one tap -- are ONE 16-byte load.  A = packed weight codes
// (rows o), B = those loads (column = pixel): a lane's four results are four channels of one
// pixel and each store instruction writes 16 consecutive pixels of four channels (NCHW rows).
// ---------------------------------------------------------------------------------------
struct QConv {
  int B, C, H, W, O, KH, KW, SH, SW, PH, PW, DH, DW, Ho, Wo;
  int Cp;          // channels padded to 16
  int K, KS, NOB;  // contraction KH*KW*Cp, its 64-steps, 16-channel output blocks
  long long M;     // B*Ho*Wo
  int has_bias;
};

// xq8[((b*H + h)*W + w)*Cp + c] = int8 code (0 past C); one thread per 16 channels of a pixel
__global__ __launch_bounds__(256) void qconv_nhwc_kernel(QConv q, const float* __restrict__ x,
                                                         uint4* __restrict__ xq8) {
  const int g16 = q.Cp >> 4;
  const long long total = (long long)q.B * q.H * q.W * g16;
  const long long HW = (long long)q.H * q.W;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % g16);
    const long long pix = t / g16;  // b*H*W + h*W + w
    const long long b = pix / HW, hw = pix - b * HW;
    uint32_t wd[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = cg * 16 + e;
      int v = 0;
      if (c < q.C) v = __float2int_rn(x[((size_t)b * q.C + c) * HW + hw]);
      wd[e >> 2] |= ((uint32_t)(uint8_t)(int8_t)v) << (8 * (e & 3));
    }
    xq8[t] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
  }
}

// wpk[(ks * NOB + ob) * 64 + lane]: 16 int8 codes, row o = ob*16 + (lane & 15),
// k = ks*64 + 16*(lane >> 4) + e = (kh*KW + kw)*Cp + c; zero past C / the taps / O
__global__ void qconv_pack_w_kernel(QConv q, const float* __restrict__ w, v4i* __restrict__ wpk) {
  const int total = q.KS * q.NOB * 64;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int lane = t & 63, r = t >> 6;
    const int ob = r % q.NOB, ks = r / q.NOB;
    const int o = ob * 16 + (lane & 15);
    uint32_t wd[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int k = ks * 64 + 16 * (lane >> 4) + e;
      const int tap = k / q.Cp, c = k - tap * q.Cp;
      int v = 0;
      if (o < q.O && c < q.C && tap < q.KH * q.KW) {
        const int kh = tap / q.KW, kw = tap - kh * q.KW;
        v = __float2int_rn(w[(((size_t)o * q.C + c) * q.KH + kh) * q.KW + kw]);
      }
      wd[e >> 2] |= ((uint32_t)(uint8_t)(int8_t)v) << (8 * (e & 3));
    }
    wpk[t] = v4i{(int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]};
  }
}

// SPLIT: codes in [0, 255] (unsigned 8-bit activations) go through two MFMAs, x = 16 hi + lo
template <int NB, bool SPLIT>
__global__ __launch_bounds__(256) void qconv_fwd_kernel(QConv q, const uint4* __restrict__ xq8,
                                                        const v4i* __restrict__ wpk, const float* __restrict__ sa_p,
                                                        const float* __restrict__ sw_p, const float* __restrict__ bias,
                                                        float* __restrict__ y, float* __restrict__ y0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const long long p = (long long)blockIdx.x * 64 + wave * 16 + r16;  // this lane's pixel (B column)
  const bool valid = p < q.M;
  const int P = q.Ho * q.Wo;
  const int b = valid ? (int)(p / P) : 0;
  const int pimg = valid ? (int)(p - (long long)b * P) : 0;
  const int oh = pimg / q.Wo, ow = pimg - oh * q.Wo;
  const int ih0 = oh * q.SH - q.PH, iw0 = ow * q.SW - q.PW;
  const int g16 = q.Cp >> 4, ntap = q.KH * q.KW;
  const uint4* xb = xq8 + (size_t)b * q.H * q.W * g16;
  const int ob0 = blockIdx.y * NB;
  v4i acc[NB], acch[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    acc[nb] = v4i{0, 0, 0, 0};
    acch[nb] = v4i{0, 0, 0, 0};
  }
  for (int ks = 0; ks < q.KS; ++ks) {
    const int kc = ks * 4 + g4;  // this lane's 16-channel chunk of the contraction
    const int tap = kc / g16, cg = kc - tap * g16;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (tap < ntap && valid) {
      const int kh = tap / q.KW, kw = tap - kh * q.KW;
      const int ih = ih0 + kh * q.DH, iw = iw0 + kw * q.DW;
      if (ih >= 0 && ih < q.H && iw >= 0 && iw < q.W) v = xb[((size_t)ih * q.W + iw) * g16 + cg];
    }
    v4i bl, bh;
    if (SPLIT) {
      bl = v4i{(int)(v.x & 0x0F0F0F0Fu), (int)(v.y & 0x0F0F0F0Fu), (int)(v.z & 0x0F0F0F0Fu), (int)(v.w & 0x0F0F0F0Fu)};
      bh = v4i{(int)((v.x >> 4) & 0x0F0F0F0Fu), (int)((v.y >> 4) & 0x0F0F0F0Fu), (int)((v.z >> 4) & 0x0F0F0F0Fu),
               (int)((v.w >> 4) & 0x0F0F0F0Fu)};
    } else {
      bl = v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      bh = bl;
    }
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if (ob0 + nb < q.NOB) {
        const v4i a = wpk[((size_t)ks * q.NOB + ob0 + nb) * 64 + lane];
        acc[nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bl, acc[nb], 0, 0, 0);
        if (SPLIT) acch[nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bh, acch[nb], 0, 0, 0);
      }
    }
  }
  if (!valid) return;
  const float sa = *sa_p, sw = *sw_p;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = (ob0 + nb) * 16 + 4 * g4 + r;
      if (o < q.O) {
        const int iv = SPLIT ? acc[nb][r] + 16 * acch[nb][r] : acc[nb][r];
        float v0 = (float)iv;
        if (q.has_bias) v0 = v0 + bias[o];
        const size_t di = ((size_t)b * q.O + o) * P + pimg;
        y0[di] = v0;
        y[di] = (v0 * sa) * sw;  // lsq.py:436: conv(...) * act_scaling_factor * weight_scaling_factor
      }
    }
  }
}

// elementwise backward of y = (y0 * a) * s: grad_y0 = (g * s) * a; per block the sums
// g * (y0 * a) (MulBackward wrt s) and (g * s) * y0 (MulBackward wrt a)
__global__ __launch_bounds__(256) void qconv_bwd_ew_kernel(long long n, const float* __restrict__ gout,
                                                           const float* __restrict__ y0, const float* __restrict__ sa_p,
                                                           const float* __restrict__ sw_p, float* __restrict__ gy0,
                                                           float* __restrict__ part) {
  const float a = *sa_p, s = *sw_p;
  float ps = 0.f, pa = 0.f;
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += step) {
    const float g = gout[e], v0 = y0[e];
    const float y1 = v0 * a;
    const float g1 = g * s;
    gy0[e] = g1 * a;
    ps += g * y1;
    pa += g1 * v0;
  }
  block_sum2_store(ps, pa, part);
}

inline int ew_blocks(long long n) { return (int)std::max(1LL, std::min<long long>((n + 1023) / 1024, 2048)); }

}  // namespace cimq

using namespace cimq;

static size_t qconv_xq8_offset(const QConv& q) { return align256((size_t)q.KS * q.NOB * 64 * 16); }

static int qconv_geo(const cimq_qconv_desc* d, QConv* q) {
  if (!d) return fail(CIMQ_EINVAL, "null qconv descriptor");
  QConv g;
  memset(&g, 0, sizeof(g));
  g.B = d->batch; g.C = d->in_channels; g.H = d->in_h; g.W = d->in_w; g.O = d->out_channels;
  g.KH = d->kernel_h; g.KW = d->kernel_w; g.SH = d->stride_h; g.SW = d->stride_w;
  g.PH = d->pad_h; g.PW = d->pad_w; g.DH = d->dilation_h; g.DW = d->dilation_w;
  if (g.B < 1 || g.C < 1 || g.H < 1 || g.W < 1 || g.O < 1 || g.KH < 1 || g.KW < 1 || g.SH < 1 || g.SW < 1 ||
      g.PH < 0 || g.PW < 0 || g.DH < 1 || g.DW < 1)
    return fail(CIMQ_EINVAL, "qconv: bad geometry");
  if (d->groups != 1) return fail(CIMQ_EUNSUPPORTED, "qconv: groups != 1");
  if (g.C >= 32768 || g.KH > 255 || g.KW > 255) return fail(CIMQ_EUNSUPPORTED, "qconv: C >= 32768 or kernel > 255");
  if (d->code_min < -128 || d->code_max > 255 || (d->code_min < 0 && d->code_max > 127))
    return fail(CIMQ_EUNSUPPORTED, "qconv: activation codes outside [-128, 127] / [0, 255]");
  g.Ho = (g.H + 2 * g.PH - g.DH * (g.KH - 1) - 1) / g.SH + 1;
  g.Wo = (g.W + 2 * g.PW - g.DW * (g.KW - 1) - 1) / g.SW + 1;
  if (g.Ho < 1 || g.Wo < 1) return fail(CIMQ_EINVAL, "qconv: empty output");
  g.Cp = (g.C + 15) / 16 * 16;
  g.K = g.KH * g.KW * g.Cp;
  g.KS = (g.K + 63) / 64;
  g.NOB = (g.O + 15) / 16;
  g.M = (long long)g.B * g.Ho * g.Wo;
  g.has_bias = d->has_bias ? 1 : 0;
  *q = g;
  return CIMQ_OK;
}

extern "C" {

size_t cimq_lsq_quantize_workspace_bytes(long long n) { return (size_t)2 * sizeof(float) * ew_blocks(n); }

int cimq_lsq_quantize_forward(const float* x, long long n, const float* s, float qn, float qp, int scaled,
                              float* out, void* stream) {
  if (n < 0 || (n > 0 && (!x || !s || !out))) return fail(CIMQ_EINVAL, "lsq_quantize_forward: bad arguments");
  if (n == 0) return CIMQ_OK;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 3)
    return fail(CIMQ_EINVAL, "lsq_quantize_forward: x / out must be float-aligned");
  const int vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) ? 0 : 1;
  LsqQ q{n, qn, qp, scaled ? 1 : 0, vec};
  hipLaunchKernelGGL(lsq_quant_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, q, x, s, out);
  return check_hip("lsq_quant_fwd");
}

int cimq_lsq_quantize_backward(const float* x, long long n, const float* s, float qn, float qp, int scaled,
                               const float* grad_out, float* grad_x, float* grad_s, void* ws, void* stream) {
  if (n < 0 || (n > 0 && (!x || !s || !grad_out || !grad_x || !grad_s || !ws)))
    return fail(CIMQ_EINVAL, "lsq_quantize_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int nb = ew_blocks(n);
  float* part = reinterpret_cast<float*>(ws);
  LsqQ q{n, qn, qp, scaled ? 1 : 0, 0};
  if (n > 0) {
    hipLaunchKernelGGL(lsq_quant_bwd_kernel, dim3(nb), dim3(256), 0, st, q, x, s, grad_out, grad_x, part);
    CIMQ_TRY(check_hip("lsq_quant_bwd"));
  }
  hipLaunchKernelGGL(lsq_partials_finish_kernel, dim3(1), dim3(256), 0, st, n > 0 ? nb : 0, part, 0, grad_s);
  return check_hip("lsq_partials_finish");
}

int cimq_qconv_sizes(const cimq_qconv_desc* d, size_t* fwd_workspace_bytes, size_t* bwd_workspace_bytes) {
  QConv q;
  CIMQ_TRY(qconv_geo(d, &q));
  if (fwd_workspace_bytes) *fwd_workspace_bytes = qconv_xq8_offset(q) + (size_t)q.B * q.H * q.W * q.Cp;
  if (bwd_workspace_bytes) *bwd_workspace_bytes = (size_t)2 * sizeof(float) * ew_blocks(q.M * q.O);
  return CIMQ_OK;
}

int cimq_qconv_forward(const cimq_qconv_desc* d, const float* x_codes, const float* w_codes, const float* act_scale,
                       const float* w_scale, const float* bias, float* y, float* y0, void* ws, void* stream) {
  QConv q;
  CIMQ_TRY(qconv_geo(d, &q));
  if (!x_codes || !w_codes || !act_scale || !w_scale || !y || !y0 || !ws || (q.has_bias && !bias))
    return fail(CIMQ_EINVAL, "qconv_forward: null pointer");
  hipStream_t st = (hipStream_t)stream;
  v4i* wpk = reinterpret_cast<v4i*>(ws);
  const int npk = q.KS * q.NOB * 64;
  hipLaunchKernelGGL(qconv_pack_w_kernel, dim3((npk + 255) / 256), dim3(256), 0, st, q, w_codes, wpk);
  CIMQ_TRY(check_hip("qconv_pack_w"));
  uint4* xq8 = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(ws) + qconv_xq8_offset(q));
  const long long nx = (long long)q.B * q.H * q.W * (q.Cp / 16);
  hipLaunchKernelGGL(qconv_nhwc_kernel, dim3((unsigned)std::min<long long>((nx + 255) / 256, 65536)), dim3(256), 0, st,
                     q, x_codes, xq8);
  CIMQ_TRY(check_hip("qconv_nhwc"));
  const bool split = d->code_max > 127;
  const int NB = q.NOB >= 4 ? 4 : (q.NOB >= 2 ? 2 : 1);
  dim3 grid((unsigned)((q.M + 63) / 64), (unsigned)((q.NOB + NB - 1) / NB));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, q, xq8, wpk, act_scale, w_scale, bias, y, y0);
    return check_hip("qconv_fwd");
  };
  if (NB == 4) return split ? launch(qconv_fwd_kernel<4, true>) : launch(qconv_fwd_kernel<4, false>);
  if (NB == 2) return split ? launch(qconv_fwd_kernel<2, true>) : launch(qconv_fwd_kernel<2, false>);
  return split ? launch(qconv_fwd_kernel<1, true>) : launch(qconv_fwd_kernel<1, false>);
}

int cimq_qconv_backward_scales(const cimq_qconv_desc* d, const float* grad_y, const float* y0, const float* act_scale,
                               const float* w_scale, float* grad_y0, float* grad_scales, void* ws, void* stream) {
  QConv q;
  CIMQ_TRY(qconv_geo(d, &q));
  if (!grad_y || !y0 || !act_scale || !w_scale || !grad_y0 || !grad_scales || !ws)
    return fail(CIMQ_EINVAL, "qconv_backward_scales: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const long long n = q.M * q.O;
  const int nb = ew_blocks(n);
  float* part = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(qconv_bwd_ew_kernel, dim3(nb), dim3(256), 0, st, n, grad_y, y0, act_scale, w_scale, grad_y0, part);
  CIMQ_TRY(check_hip("qconv_bwd_ew"));
  hipLaunchKernelGGL(lsq_partials_finish_kernel, dim3(1), dim3(256), 0, st, nb, part, 1, grad_scales);
  return check_hip("qconv_bwd_finish");
}

}  // extern "C"

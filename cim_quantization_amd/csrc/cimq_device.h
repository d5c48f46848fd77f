// cimq_device.h -- geometry, parameter tables and exact-fp32 device helpers shared by the
// libcimq kernels.  Compiled only for gfx950 (CDNA4): 64-lane waves, MFMA int8/bf16.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

// every kernel's lane math (16-lane MFMA rows, xor-32 butterflies, threadIdx >> 6 wave ids)
// assumes 64-lane wavefronts (CDNA)
#if defined(__HIP_DEVICE_COMPILE__) && defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "libcimq assumes 64-lane wavefronts (gfx9 CDNA targets)"
#endif
#include <stdint.h>

// The kernels assume 64-lane waves (shuffle butterflies over 32..1, threadIdx >> 6 as the
// wave id): build.py accepts only gfx9 (wave64-only) targets.
namespace cimq {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

enum AdcMode { ADC_FP = 0, ADC_SIGN = 1, ADC_TERNARY = 2, ADC_MULTI = 3 };
// cimq_conv_desc.adc_variant & 0xFF (include/cimq.h CIMQ_ADC_*)
enum AdcVariant { VAR_LIBRARY = 0, VAR_STOCHASTIC = 1, VAR_SHIFT_ROUND = 2, VAR_SHIFT_SIGN = 3 };

// Problem geometry, computed once on the host (cimq_api.hip) and passed by value.
struct Geo {
  int B, C, H, W, O, KH, KW, SH, SW, PH, PW, Ho, Wo;
  int P, M, K, KHW, HW;
  int xbar, T, KS, KTP;    // KS: 64-deep int8 K-steps per tile, KTP: LDS row pitch (bytes)
  int FBT;                 // 16-wide f-blocks per tile (ceil(xbar/16))
  int nbw, nba, bsw, bsa, NBP;  // NBP: bytes per input element in the packed act-code array
  int Opad, OB16, NBLK, NKS;    // Opad=roundup(O,16); NBLK = nbw*Opad/16; NKS = ceil(NBLK/2)
  int mode;
  float qn, qp, thr_hi, thr_lo;  // ADC range; backward clamp thresholds fl32(Qp+1e-5), fl32(Qn-1e-5)
  int input_kind;
  float lsq_qp;
  int psmax;               // bound on |partial sum| used by the threshold search
  long long Nin;           // B*C*H*W
  int onchw;               // out / grad_out layout: 0 = [B, P, O] (the Function's), 1 = NCHW (the module's)
  int variant;             // AdcVariant; anything but VAR_LIBRARY runs the literal (general) kernels
  int ps_int8;             // partial sums pass an int8 buffer before the ADC (scale_shift.py:401)
  int recompute;           // cimq_conv_desc.options & CIMQ_OPT_RECOMPUTE: the module backward recomputes partial sums
  uint32_t seed_lo, seed_hi;  // VAR_STOCHASTIC: Philox key
  const unsigned char* wbase;  // host side: the weight-side ctx regions (cimq_lsq_desc.wprep); null: inside ctx
};

// Per-(tile i, a-slice j, w-slice k, out-channel o) ADC / STE parameters, SoA.
// index: ((i*nba + j)*nbw + k)*Opad + o
struct Params {
  int* thi;     // forward: ps >= thi -> code +1   (ternary mode)
  int* tlo;     // forward: ps <= tlo -> code -1
  int* mlo;     // backward: STE passes iff (unsigned)(ps - mlo) <= (unsigned)mhi (lsq.py:310-313)
  int* mhi;     //   ... mhi holds the interval span
  float* coef;  // alpha_q * binary_mask  (ternary / sign)
  float* alpha; // alpha_q (literal paths)
  float* ckj;   // [3][nbw*nba]: mask as float, cE = 2^-(bsa*j)*mask, cD = 2^-(bsw*k)*mask
  int* flags;   // [0]: literal ADC (degenerate alpha / scales), [1..3] reserved
  float* beta;  // shift of the scale + shift ADC variants (0 otherwise)
  float* bsum;  // [Opad]: sum over (i, k, j) of beta * binary_mask (shift_fast forward)
};

__host__ __device__ inline int pidx(const Geo& g, int i, int j, int k, int o) {
  return ((i * g.nba + j) * g.nbw + k) * g.Opad + o;
}

// ---------------------------------------------------------------------------------------
// exact fp32 emulation of the reference's torch op sequence (compiled with -ffp-contract=off)
// ---------------------------------------------------------------------------------------
__device__ inline float pow2f(int e) { return __int_as_float((127 + e) << 23); }  // |e| < 127

// torch.remainder(t, 2^bs) for float t: floor-mod, result has the divisor's sign.
__device__ inline float rem_pow2(float t, int bs) {
  const float b = (float)(1 << bs);
  return t - b * floorf(t * pow2f(-bs));
}

// Plane k of the reference's slicing of a non-negative magnitude v (lsq.py:454-457 / 475-478):
// floor(v / (2^bs)^k) for k >= 1, then remainder 2^bs.
__device__ inline float slice_mag(float v, int k, int bs) {
  float t = (k == 0) ? v : floorf(v * pow2f(-bs * k));
  return rem_pow2(t, bs);
}

// slicing_act (unsigned, lsq.py:466-480): the same digit extraction on the raw value.
__device__ inline float slice_unsigned(float v, int k, int bs) { return slice_mag(v, k, bs); }

// slicing_weights_signed / slicing_act_signed (lsq.py:438-464, 483-509): slice the positive
// part and the negated negative part separately and subtract.
__device__ inline float slice_signed(float v, int k, int bs) {
  float pos = (v <= 0.f) ? 0.f : v;
  float neg = (v >= 0.f) ? 0.f : v;
  neg = -1.f * neg;
  return slice_mag(pos, k, bs) - slice_mag(neg, k, bs);
}

// tensor.type(torch.int8): truncate toward zero, keep the low byte (wraps).  NaN -> 0.
__device__ inline int to_i8_wrap(float v) {
  if (!(fabsf(v) < 2147483520.f)) return 0;
  int t = (int)v;
  return (int)(int8_t)(t & 0xFF);
}

__device__ inline int clamp_i8(float v) {
  v = rintf(v);
  v = fminf(fmaxf(v, -127.f), 127.f);
  return (int)v;
}

// torch.clamp: NaN propagates.
__device__ inline float clamp_nan(float v, float lo, float hi) {
  return (v != v) ? v : fminf(fmaxf(v, lo), hi);
}

// The fp16 store of the partial sums (lsq.py:169,177): an integer ps rounded to half.
// grad_scale(x, s) forward value: (x - x*s).detach() + x*s  (_quan_base.py grad_scale)
__device__ inline float grad_scale_value(float x, float s) {
  const float yg = x * s;
  const float d = x - yg;
  return d + yg;
}

// round_pass(v) forward value: (v.round() - v).detach() + v  (lsq.py:29-32)
__device__ inline float round_pass_value(float v) {
  const float r = rintf(v);
  return (r - v) + v;
}

__device__ inline float ps_half(int p) { return __half2float(__float2half_rn((float)p)); }

// u = ps * sw * sa in fp32, in the reference's order (lsq.py:195).
__device__ inline float u_of(int p, float sw, float sa) {
  float ps = ps_half(p);
  float t = ps * sw;
  return t * sa;
}

// The ADC of lsq.py:197-230 evaluated literally for one partial sum (no threshold shortcut).
__device__ inline float adc_literal(int p, int mode, float sw, float sa, float alpha, float qn,
                                    float qp) {
  float u = u_of(p, sw, sa);
  if (mode == ADC_FP) return u;
  if (mode == ADC_SIGN) {
    float s = (u > 0.f) ? 1.f : ((u < 0.f) ? -1.f : ((u != u) ? u : 0.f));
    return s * alpha;
  }
  if (mode == ADC_TERNARY) {
    float v = u / alpha;
    float q = clamp_nan(rintf(v), qn, qp);
    return q * alpha;
  }
  float d = sw * sa;
  float v = u / d;
  float q = clamp_nan(rintf(v), qn, qp);
  float t = q * sw;
  return t * sa;
}

// The backward's rescaled partial sum (lsq.py:257-267).
__device__ inline float psb_literal(int p, int mode, float sw, float sa, float alpha) {
  if (mode == ADC_SIGN || mode == ADC_TERNARY) return u_of(p, sw, sa) / alpha;
  return ps_half(p);
}

// STE mask (lsq.py:310-313): gradient passes unless clamped.
__device__ inline bool ste_pass(float psb, float thr_hi, float thr_lo) {
  return !(psb >= thr_hi || psb <= thr_lo);
}

// ADC code used by grad_alpha (lsq.py:321-332), literal form.
__device__ inline float alpha_code_literal(float psb, int mode, float qn, float qp, float thr_hi,
                                           float thr_lo) {
  if (mode == ADC_SIGN) return (psb > 0.f) ? 1.f : ((psb < 0.f) ? -1.f : ((psb != psb) ? psb : 0.f));
  float q = rintf(psb);
  if (psb >= thr_hi) q = qp;
  if (psb <= thr_lo) q = qn;
  return q;
}

// ---------------------------------------------------------------------------------------
// ADC variants (cimq_conv_desc.adc_variant), evaluated literally per partial sum
// ---------------------------------------------------------------------------------------
__device__ inline bool has_alpha(const Geo& g) {
  return g.mode == ADC_SIGN || g.mode == ADC_TERNARY || g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN;
}
__device__ inline bool is_shift(const Geo& g) { return g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN; }
// The scale / shift "round" ADC of Conv2dLSQCiM(adc_shift=True) on the threshold fast path: 1.5 bits
// with the library's range (codes -1, 0, 1), the library's fp16 partial sums (no int8 buffer), every
// |ps| exact in fp16.  v = (u - beta) / alpha is then a monotone step function of the integer ps,
// captured by integer thresholds like the library ADC; the output gains sum beta * mask per channel.
__host__ __device__ inline bool shift_fast(const Geo& g) {
  return g.variant == VAR_SHIFT_ROUND && g.mode == ADC_TERNARY && !g.ps_int8 && g.qp == 1.f && g.qn == -1.f &&
         g.psmax <= 2048;
}

// torch.sign: NaN propagates
__device__ inline float sign_nan(float v) { return (v > 0.f) ? 1.f : ((v < 0.f) ? -1.f : ((v != v) ? v : 0.f)); }

// the partial sum as the ADC input sees it, times sw * sa (lsq.py:195): the fp16 store of the
// library (lsq.py:169) or the int8 buffer of the scale/shift ver2 Function (scale_shift.py:401)
__device__ inline float u_var(const Geo& g, int p, float sw, float sa) {
  float ps = ps_half(p);
  if (g.ps_int8) ps = (float)(int8_t)(((int)ps) & 0xFF);
  const float t = ps * sw;
  return t * sa;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based, so a draw depends only on (key, counter)
__device__ inline void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// number of draws U ~ [0,1) (24-bit) with ceil(s - U) == 1, i.e. U < s, out of 50 (lsq.py:214-217);
// draws d = 0..49 of stream `which` of element `eid`
__device__ inline float bernoulli50(float s, uint64_t eid, uint32_t which, uint32_t k0, uint32_t k1) {
  if (s <= 0.f) return 0.f;   // ceil(0 - U) = 0 for every U in [0, 1)
  if (s >= 1.f) return 50.f;  // ceil(1 - U) = 1
  float n = 0.f;
  for (uint32_t blk = 0; blk < 13; ++blk) {
    uint32_t c[4] = {(uint32_t)eid, (uint32_t)(eid >> 32), which, blk};
    philox4x32(c, k0, k1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (blk * 4 + e < 50) {
        const float u = (float)(c[e] >> 8) * 5.9604644775390625e-8f;  // 2^-24
        n += (s - u > 0.f) ? 1.f : 0.f;                                // ceil(s - u) with s - u in (-1, 1)
      }
    }
  }
  return n;
}

// stochastic 1.5-bit ADC of lsq.py:205-221 for one partial sum (u = ps*sw*sa)
__device__ inline float adc_stochastic(const Geo& g, float u, float alpha, uint64_t eid) {
  const float h = 0.5f * alpha;
  const float z1 = (u - h) / 0.01f, z2 = (u + h) / 0.01f;
  const float s1 = 1.f / (1.f + expf(-z1)), s2 = 1.f / (1.f + expf(-z2));  // torch.sigmoid
  const float n1 = bernoulli50(s1, eid, 0u, g.seed_lo, g.seed_hi);
  const float n2 = bernoulli50(s2, eid, 1u, g.seed_lo, g.seed_hi);
  const float a = n1 / 50.f, b = n2 / 50.f;
  const float v = (a + b) - 1.f;
  return clamp_nan(rintf(v), g.qn, g.qp) * alpha;
}

// ADC output (before the shift-and-add mask) of one partial sum, every variant
__device__ inline float adc_value(const Geo& g, int p, float sw, float sa, float alpha, float beta, uint64_t eid) {
  if (g.variant == VAR_SHIFT_ROUND) {
    const float v = (u_var(g, p, sw, sa) - beta) / alpha;  // scale_shift.py:421
    const float t = clamp_nan(rintf(v), g.qn, g.qp) * alpha;  // :424-425
    return t + beta;
  }
  if (g.variant == VAR_SHIFT_SIGN) {
    const float v = (u_var(g, p, sw, sa) - beta) / alpha;  // scale_shift.py:202
    const float t = sign_nan(v) * alpha;                    // :209-211
    return t + beta;
  }
  if (g.variant == VAR_STOCHASTIC) return adc_stochastic(g, u_of(p, sw, sa), alpha, eid);
  return adc_literal(p, g.mode, sw, sa, alpha, g.qn, g.qp);
}

// the backward's rescaled partial sum (lsq.py:257-267; scale_shift.py:469 / :202)
__device__ inline float psb_value(const Geo& g, int p, float sw, float sa, float alpha, float beta) {
  if (is_shift(g)) return (u_var(g, p, sw, sa) - beta) / alpha;
  return psb_literal(p, g.mode, sw, sa, alpha);
}

// per-partial-sum factor of grad_alpha (times g, summed over the batch and pixels)
__device__ inline float alpha_term(const Geo& g, float b) {
  if (g.variant == VAR_SHIFT_ROUND) {  // scale_shift.py:488-495: round(ps) - ps, Qp / Qn where clamped
    if (b >= g.thr_hi) return g.qp;
    if (b <= g.thr_lo) return g.qn;
    return rintf(b) - b;
  }
  if (g.variant == VAR_SHIFT_SIGN) return sign_nan(b);  // scale_shift.py:281
  return alpha_code_literal(b, g.mode, g.qn, g.qp, g.thr_hi, g.thr_lo);
}

// per-partial-sum factor of grad_beta: the clamped region (ver2, :496-501) or 1 (adcless, :287)
__device__ inline float beta_term(const Geo& g, float b) {
  if (g.variant == VAR_SHIFT_SIGN) return 1.f;
  return (b >= g.thr_hi || b <= g.thr_lo) ? 1.f : 0.f;
}

// fp32 -> bf16 round-to-nearest-even (finite inputs) and back
__device__ inline uint16_t bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  uint32_t r = u + 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(r >> 16);
}
__device__ inline float bf16_to_f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Split a float into hi + mid + lo bf16 parts (24 significant bits): the three-term
// decomposition that gives fp32-accurate products on the bf16 MFMA when the other operand
// is a small integer (exact in bf16).
__device__ inline void split3(float a, uint16_t& hi, uint16_t& mid, uint16_t& lo) {
  hi = bf16_bits(a);
  float r1 = a - bf16_to_f(hi);
  mid = bf16_bits(r1);
  float r2 = r1 - bf16_to_f(mid);
  lo = bf16_bits(r2);
}

__device__ inline v8bf as_v8bf(v4i x) { return __builtin_bit_cast(v8bf, x); }
__device__ inline v4i as_v4i(v8bf x) { return __builtin_bit_cast(v4i, x); }

// (v_l + v_{l^16}) + (v_{l^32} + v_{l^48}) in every lane: the sum over the four 16-lane rows of a wave,
// in __shfl_xor(16)-then-(32)'s order and rounding (each add is commutative, so bit-identical to it), on
// the gfx950 row-swap permutes (VALU) instead of two LDS-crossbar ds_bpermute round trips
__device__ inline float rows4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float h = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(h), __float_as_uint(h), false, false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}

}  // namespace cimq

// cimq_host.h -- host-side plans, layouts, error state and the kernel timer shared by the
// translation units of libcimq.so (cimq_api.hip and the cimq_part_*.hip launchers, which are
// compiled in parallel).
#pragma once
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <string>

#include "../../include/cimq.h"
#include "cimq_c1.hip"
#include "cimq_fwd5.hip"
#include "cimq_gw5.hip"
#include "cimq_gx5.hip"
#include "cimq_r6.hip"


namespace cimq {

inline thread_local std::string g_last_error;

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

inline int check_hip(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CIMQ_EHIP, "%s: %s", where, hipGetErrorString(e));
  return CIMQ_OK;
}

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// tuning knobs for experiments (tools/, built with -DCIMQ_TUNING): CIMQ_TUNE_<name>=<int>
// overrides a launch shape; the shipped library compiles them to the defaults
#ifdef CIMQ_TUNING
inline int tune(const char* name, int dflt) {
  char key[64];
  snprintf(key, sizeof(key), "CIMQ_TUNE_%s", name);
  const char* v = getenv(key);
  return v ? atoi(v) : dflt;
}
#else
constexpr int tune(const char*, int dflt) { return dflt; }
#endif
// Host plans and layouts memoised per geometry (the launch paths ask for the same ones several times per call):
// a few recent Geo values per thread, compared bytewise with the fields no plan reads (the prepared-weight
// pointer, the stochastic-ADC key) cleared.  Padding can only cause a miss, never a wrong hit.
template <class T, T (*F)(const Geo&)>
inline T memo_geo(const Geo& g) {
  struct Entry {
    Geo k;
    T v;
    bool used;
  };
  thread_local Entry e[4] = {};
  thread_local int next = 0;
  Geo k = g;
  k.wbase = nullptr;
  k.seed_lo = k.seed_hi = 0;
  for (Entry& x : e)
    if (x.used && memcmp(&x.k, &k, sizeof(Geo)) == 0) return x.v;
  Entry& d = e[next];
  next = (next + 1) & 3;
  d.v = F(g);
  d.k = k;
  d.used = true;
  return d.v;
}
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

inline int make_geo(const cimq_conv_desc* d, Geo* out) {
  if (!d || !out) return fail(CIMQ_EINVAL, "null descriptor");
  Geo g;
  memset(&g, 0, sizeof(g));
  g.B = d->batch; g.C = d->in_channels; g.H = d->in_h; g.W = d->in_w;
  g.O = d->out_channels; g.KH = d->kernel_h; g.KW = d->kernel_w;
  g.SH = d->stride_h; g.SW = d->stride_w; g.PH = d->pad_h; g.PW = d->pad_w;
  if (g.B <= 0 || g.C <= 0 || g.H <= 0 || g.W <= 0 || g.O <= 0 || g.KH <= 0 || g.KW <= 0 ||
      g.SH <= 0 || g.SW <= 0 || g.PH < 0 || g.PW < 0)
    return fail(CIMQ_EINVAL, "bad conv geometry");
  g.Ho = (g.H + 2 * g.PH - g.KH) / g.SH + 1;
  g.Wo = (g.W + 2 * g.PW - g.KW) / g.SW + 1;
  if (g.Ho <= 0 || g.Wo <= 0) return fail(CIMQ_EINVAL, "empty output");
  g.P = g.Ho * g.Wo;
  long long M = (long long)g.B * g.P;
  g.KHW = g.KH * g.KW;
  g.HW = g.H * g.W;
  g.K = g.C * g.KHW;
  long long nin = (long long)g.B * g.C * g.H * g.W;
  if (M >= (1LL << 31) || nin >= (1LL << 31) || (long long)g.O * g.K >= (1LL << 31))
    return fail(CIMQ_EUNSUPPORTED, "tensor too large for 32-bit indexing");
  g.M = (int)M;
  g.Nin = nin;
  g.xbar = d->xbar;
  if (g.xbar <= 0 || g.xbar % 16 != 0 || g.xbar > 128)
    return fail(CIMQ_EUNSUPPORTED, "xbar must be a positive multiple of 16 and <= 128 (got %d)", g.xbar);
  g.T = (g.K + g.xbar - 1) / g.xbar;
  const int tmax = g.K < g.xbar ? g.K : g.xbar;
  g.KS = (tmax + 63) / 64;
  g.KTP = g.KS * 64 + 16;
  g.FBT = (tmax + 15) / 16;
  if (d->bs_w <= 0 || d->bs_a <= 0 || d->bits_w <= 0 || d->bits_a <= 0)
    return fail(CIMQ_EINVAL, "bad bit widths");
  g.bsw = d->bs_w; g.bsa = d->bs_a;
  g.nbw = d->bits_w / d->bs_w;  // int(bits/bit_slice), lsq.py:115-117
  g.nba = d->bits_a / d->bs_a;
  if (g.nbw < 1 || g.nba < 1 || g.nbw > 8 || g.nba > 8)
    return fail(CIMQ_EUNSUPPORTED, "1..8 bit slices supported (nbw=%d nba=%d)", g.nbw, g.nba);
  if (g.bsw > 5 || g.bsa > 5) return fail(CIMQ_EUNSUPPORTED, "bit slices wider than 5 bits");
  if (g.nbw * g.nba > 64) return fail(CIMQ_EUNSUPPORTED, "too many slice pairs");
  g.NBP = g.nba <= 4 ? 4 : 8;
  g.Opad = (g.O + 15) / 16 * 16;
  g.OB16 = g.Opad / 16;
  g.NBLK = g.nbw * g.OB16;
  g.NKS = (g.NBLK + 1) / 2;
  const float ab = d->adc_bits;
  double qp, qn;
  if (ab == 0.f) g.mode = ADC_FP;
  else if (ab == 1.f) g.mode = ADC_SIGN;
  else if (ab == 1.5f) g.mode = ADC_TERNARY;
  else if (ab > 1.5f) g.mode = ADC_MULTI;
  else return fail(CIMQ_EINVAL, "adc_bits %g not one of 0, 1, 1.5 or > 1.5", (double)ab);
  if (g.mode == ADC_SIGN || g.mode == ADC_TERNARY) { qp = 1.0; qn = -1.0; }
  else { qp = pow(2.0, (double)ab - 1.0) - 1.0; qn = -pow(2.0, (double)ab - 1.0); }  // lsq.py:125-126
  g.qp = (float)qp; g.qn = (float)qn;
  g.thr_hi = (float)(qp + 1e-5);  // ps.ge(Qp_adc+1e-5): scalar rounded to fp32
  g.thr_lo = (float)(qn - 1e-5);
  g.input_kind = d->input_kind;
  if (g.input_kind != CIMQ_INPUT_XQ && g.input_kind != CIMQ_INPUT_RAW_LSQ)
    return fail(CIMQ_EINVAL, "bad input_kind");
  g.lsq_qp = d->lsq_qp;
  g.variant = d->adc_variant & 0xFF;
  if (d->adc_variant & ~(0xFF | CIMQ_ADC_F_PS_INT8 | CIMQ_ADC_F_SHIFT_RANGE))
    return fail(CIMQ_EINVAL, "unknown adc_variant flags 0x%x", d->adc_variant);
  g.ps_int8 = (d->adc_variant & CIMQ_ADC_F_PS_INT8) ? 1 : 0;
  g.seed_lo = d->seed_lo;
  g.seed_hi = d->seed_hi;
  if (d->options & ~CIMQ_OPT_RECOMPUTE) return fail(CIMQ_EINVAL, "unknown options 0x%x", d->options);
  g.recompute = (d->options & CIMQ_OPT_RECOMPUTE) ? 1 : 0;
  switch (g.variant) {
    case VAR_LIBRARY: break;
    case VAR_STOCHASTIC:  // lsq.py:136-137: the stochastic ADC is the 1.5-bit one
      if (g.mode != ADC_TERNARY) return fail(CIMQ_EINVAL, "the stochastic ADC needs adc_bits 1.5");
      break;
    case VAR_SHIFT_SIGN:
      if (ab != 1.f) return fail(CIMQ_EINVAL, "the scale/shift sign ADC needs adc_bits 1");
      break;
    case VAR_SHIFT_ROUND:
      if (g.mode == ADC_FP) return fail(CIMQ_EINVAL, "the scale/shift ADC needs adc_bits >= 1");
      break;
    default: return fail(CIMQ_EINVAL, "unknown adc_variant %d", g.variant);
  }
  if ((d->adc_variant & CIMQ_ADC_F_SHIFT_RANGE) && ab != 1.f) {
    // scale_shift.py:369-375: Qp = 2^(b-1) - 1, Qn = -2^(b-1) (also for 1.5 bits)
    qp = pow(2.0, (double)ab - 1.0) - 1.0;
    qn = -pow(2.0, (double)ab - 1.0);
    g.qp = (float)qp; g.qn = (float)qn;
    g.thr_hi = (float)(qp + 1e-5);
    g.thr_lo = (float)(qn - 1e-5);
  }
  long long psmax = (long long)tmax * (1LL << g.bsa) * (1LL << g.bsw);
  g.psmax = (int)(psmax > (1 << 24) ? (1 << 24) : psmax);
  *out = g;
  return CIMQ_OK;
}

// ctx: the weight-side regions first ([0, wbytes): weight operand fragments, ADC / STE
// parameters, the module's step sizes -- functions of the parameters only, so a prepared
// buffer (cimq_module_prepare, cimq_lsq_desc.wprep) can hold them instead), then the
// activation-side regions (slice words, state words) of one forward.
inline bool dense_plan(const Geo& g);

struct CtxLayout {
  size_t xcode, xhat, alut, wfrag, wf5, wg5, wx6, wgx, wcy, thi, tlo, mlo, mhi, coef, alpha, beta, bsum, ckj, flags, st;
  size_t lsq_scal;  // module entry points: sa, sw, alpha scale, max, min
  size_t wbytes;    // end of the weight-side regions
  size_t total;
};

inline size_t f5_frag_bytes(const Geo& g);  // after f5_plan
inline size_t x5_frag_bytes(const Geo& g);  // after x5_plan
inline size_t r6_frag_bytes(const Geo& g);  // after r6_plan
inline bool r6_bwd(const Geo& g);           // after r6_plan

inline CtxLayout ctx_layout_compute(const Geo& g) {
  CtxLayout L;
  size_t o = 0;
  const size_t npar = (size_t)g.T * g.nba * g.nbw * g.Opad;
  L.wfrag = o; o = align256(o + (size_t)g.T * g.KS * g.NBLK * 64 * 16);
  L.wf5 = o; o = align256(o + f5_frag_bytes(g));  // cim_fwd5_kernel's weight operand
  L.wg5 = o; o = align256(o + x5_frag_bytes(g));  // cim_bwd_gx5_kernel's weight operand
  L.wx6 = o; o = align256(o + r6_frag_bytes(g));  // cim_bwd_r6_kernel's gx operand
  L.wgx = o; o = align256(o + (size_t)g.T * g.FBT * g.NKS * 64 * 16);
  L.wcy = o; o = align256(o + (size_t)g.T * 12 * g.NKS * 64 * 16);  // v8 grad_x operand (<= 12 blocks / tile)
  L.thi = o; o = align256(o + npar * 4);
  L.tlo = o; o = align256(o + npar * 4);
  L.mlo = o; o = align256(o + npar * 4);
  L.mhi = o; o = align256(o + npar * 4);
  L.coef = o; o = align256(o + npar * 4);
  L.alpha = o; o = align256(o + npar * 4);
  L.beta = o; o = align256(o + npar * 4);
  L.bsum = o; o = align256(o + (size_t)g.Opad * 4);
  L.ckj = o; o = align256(o + 3 * 64 * 4);
  L.flags = o; o = align256(o + 16);
  L.lsq_scal = o; o = align256(o + 16 * 4);
  L.wbytes = o;
  L.xcode = o; o = align256(o + (size_t)g.Nin * g.NBP);  // forward slice bytes
  L.xhat = o; o = align256(o + (size_t)g.Nin * g.NBP);   // backward (int8 ctx) slice bytes
  L.alut = o; o = align256(o + (size_t)4 * 301);         // ctx codes: code -> ctx word (ctx_codes), format word 300
  // per-partial-sum state words written by the fast forward (cimq_kernels_v3.hip: StWord)
  // (v7: one uint32 per (i, m, o) -- never larger for nbw >= 2; the max covers nbw == 1)
  // state words: per-(k) words of the v3-v6 kernels, or the v7 compact words (4 B, or three
  // 64-bit planes for w8a8) per (tile, pixel, channel)
  // (the dense path, cimq_part_dense.hip: a uint2 of three 16-bit planes per (i, m, o))
  // (none where the module backward recomputes the partial sums, cim_bwd_r6_kernel: the region is last, so
  // the module path's smaller ctx -- cimq_sizes.module_ctx_bytes -- keeps every other offset)
  L.st = o; o = align256(o + (r6_bwd(g) ? (size_t)0
                                        : std::max({(size_t)g.T * g.nbw * g.M * g.O * (g.NBP == 4 ? 2 : 4),
                                                    (size_t)g.T * g.M * g.O * (g.NBP == 4 ? 4 : 24),
                                                    dense_plan(g) ? (size_t)g.T * g.M * g.O * 8 : (size_t)0})));
  L.total = o;
  return L;
}
inline CtxLayout ctx_layout(const Geo& g) { return memo_geo<CtxLayout, ctx_layout_compute>(g); }

// base of the weight-side regions of a ctx: the prepared buffer when the call has one
inline uint8_t* wreg(const Geo& g, const uint8_t* ctx) {
  return const_cast<uint8_t*>(g.wbase ? g.wbase : ctx);
}

inline Params params_of(const Geo& g, uint8_t* ctx) {
  CtxLayout L = ctx_layout(g);
  uint8_t* base = wreg(g, ctx);
  Params p;
  p.thi = reinterpret_cast<int*>(base + L.thi);
  p.tlo = reinterpret_cast<int*>(base + L.tlo);
  p.mlo = reinterpret_cast<int*>(base + L.mlo);
  p.mhi = reinterpret_cast<int*>(base + L.mhi);
  p.coef = reinterpret_cast<float*>(base + L.coef);
  p.alpha = reinterpret_cast<float*>(base + L.alpha);
  p.beta = reinterpret_cast<float*>(base + L.beta);
  p.bsum = reinterpret_cast<float*>(base + L.bsum);
  p.ckj = reinterpret_cast<float*>(base + L.ckj);
  p.flags = reinterpret_cast<int*>(base + L.flags);
  return p;
}

// pixel chunking of the gw / init kernel: ~1024 blocks over (chunks x tiles x 32-col groups)
inline void gw_chunks(const Geo& g, int* rows_per_chunk, int* nchunks) {
  const int og = (g.OB16 + 1) / 2;
  long long want = 1024 / ((long long)g.T * og);
  if (want < 1) want = 1;
  long long rows = ((g.M + want - 1) / want + 63) / 64 * 64;
  if (rows < 64) rows = 64;
  *rows_per_chunk = (int)rows;
  *nchunks = cdiv(g.M, rows);
}

const int kLsqParts = 1024;

inline size_t lds_tile(const Geo& g) {
  return align256((size_t)g.nba * 64 * g.KTP + 2 * sizeof(int) * g.KS * 64 + sizeof(int4) * 64);
}
// general grad_w (one 16-channel output block per workgroup): the tile (later the grad_w block sum),
// per-wave code * g sums [4 waves][nkj][16] (and the beta-term sums for the shift variants), the
// backward slices
inline size_t lds_gw(const Geo& g) {
  const bool shift = g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN;
  return std::max(lds_tile(g), sizeof(float) * g.FBT * 16 * 16) + (shift ? 2 : 1) * 4 * sizeof(float) * g.nbw * g.nba * 16 +
         (size_t)g.nba * g.KS * 64 * 64;
}
const size_t kLdsMax = 160 * 1024;

// ---- v3 fast path (whole-row 64-pixel tiles): patch geometry and LDS budgets ----
struct Plan3 {
  bool ok;
  V3 v;
  size_t lds_fwd;
};

inline size_t a16(size_t v) { return (v + 15) & ~(size_t)15; }

// activation-prep blocks (grid-stride over 4-element items)
inline int act_blocks() { return tune("ACT_BLOCKS", 8192); }

inline Plan3 v3_plan(const Geo& g) {
  Plan3 p;
  memset(&p, 0, sizeof(p));
  if (tune("V3", 1) == 0) return p;  // experiments: force the general kernels
  // ADC variants: literal per-partial-sum evaluation on the general kernels, except the shift ADC
  // whose thresholds the params kernel finds like the library's (shift_fast)
  if (g.variant != VAR_LIBRARY && !shift_fast(g)) return p;
  if (g.P % 64 != 0 || g.Wo > 64 || 64 % g.Wo != 0 || g.Wo < 4) return p;
  if (g.O > 256 || 256 % g.O != 0) return p;  // grad_alpha reducer: one thread per channel
  if ((g.W * g.NBP) % 16 != 0 || g.KS > 2 || g.FBT > 8) return p;
  if (g.M >= (1 << 24)) return p;  // float-reciprocal index division (fdiv) in the kernels
  V3& v = p.v;
  v.lw = 0;
  while ((1 << v.lw) < g.Wo) ++v.lw;
  v.RH = (64 / g.Wo - 1) * g.SH + g.KH;
  v.WP = g.W + 2 * g.PW;
  v.RI = std::min(g.H, 8);
  v.nbands = (g.H + v.RI - 1) / v.RI;
  v.RHB = 0;
  v.NPB = 0;
  for (int band = 0; band < v.nbands; ++band) {
    const int r0 = band * v.RI, r1 = std::min(g.H, r0 + v.RI);
    int oh_lo = r0 + g.PH - (g.KH - 1);
    oh_lo = oh_lo <= 0 ? 0 : (oh_lo + g.SH - 1) / g.SH;
    const int oh_hi = std::min(g.Ho - 1, (r1 - 1 + g.PH) / g.SH);
    const int nro = oh_hi - oh_lo + 1;
    if (nro <= 0) return p;
    v.RHB = std::max(v.RHB, (nro - 1) * g.SH + g.KH);
    v.NPB = std::max(v.NPB, nro * g.Wo);
  }
  v.CB = (g.C + 15) / 16;
  v.NT = (v.RI * g.W + 15) / 16 * v.CB;
  if (v.NT > 8 * 4 || g.KH > 3 || g.KW > 3) return p;
  v.nmt = g.M / 64;
  const int nkj = g.nbw * g.nba;
  const size_t ckl = a16((size_t)3 * nkj * 4);
  const size_t patch = a16((size_t)g.C * v.RH * v.WP * g.NBP);
  v.obm = tune("FWD_OBM", 2);  // two o-blocks per block (measured best for O = 32 / 64)
  if (v.obm != 1 && v.obm != 2 && v.obm != 4) v.obm = 4;
  const int nof = std::min(v.obm, g.OB16);
  const size_t fwd_common = patch + (size_t)g.T * g.KS * 64 * 4 + ckl;
  const size_t fwd_w1 = (size_t)g.nbw * nof * g.KS * 1024 + (size_t)nkj * nof * 16 * (16 + 4);
  const size_t fwd_res = fwd_common + (size_t)g.T * fwd_w1;
  v.fwd_res = fwd_res <= (size_t)tune("FWD_RES_KB", 52) * 1024 ? 1 : 0;
  v.pf = tune("FWD_PF", 1);
  p.lds_fwd = v.fwd_res ? fwd_res : fwd_common + fwd_w1;
  const size_t lim = kLdsMax - 512;
  p.ok = p.lds_fwd <= lim;
  return p;
}

// ---- v7 backward (compact state words, unfolded grad_x, conv-style grad_w) ----
struct Plan7 {
  bool ok;
  V7 v;
  size_t lds_gx, lds_gw;
  int pairs;
};

// grad_w LDS plane pitches.  A row group's A fragment: lane l reads 16 B (8 bf16) at plane
// kw*KWP + channel c*CPITCH + staged row (oh*SH + kh)*Wo + ow0, for row f = 16*gr + (l & 15) =
// (c, kh, kw) and pixels 32*wave + 8*(l >> 4) of the stage.  ds_read_b128 serves a wave in 4 fixed
// groups of 16 lanes, one LDS cycle per distinct address on a busy 16-B slot of the 256-B bank row
// (MI355X_MICROARCH.md, LDS).  The unpadded pitches (CPITCH = NSLOT*Wo + 8, KWP = CPL*CPITCH) put
// the three kw planes of a row on one slot: 140 cycles per stage-wave where 36 is the floor.
inline int gw_read_cycles(const Geo& g, const V7& v, int cp, int kwp) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  int cyc = 0;
  for (int wave = 0; wave < 4; ++wave)
    for (int gr = 0; gr * 16 < v.CPL * g.KHW; ++gr)
      for (int q = 0; q < 4; ++q) {
        int addr[16], slot[16];
        for (int t = 0; t < 16; ++t) {
          const int l = grp[q][t], f = 16 * gr + (l & 15);
          const int c = f / g.KHW, tap = f - c * g.KHW, kh = tap / g.KW, kw = tap - kh * g.KW;
          const int moff = 32 * wave + 8 * (l >> 4);
          const int img = v.whole ? moff / g.P : 0, pim = v.whole ? moff % g.P : moff;
          addr[t] = c < v.CPL ? kw * kwp + c * cp + (img * g.H + (pim / g.Wo) * g.SH + kh) * g.Wo + pim % g.Wo : -1;
          slot[t] = addr[t] < 0 ? -1 : (addr[t] / 8) % 16;  // rows past CPL read one zero pad (broadcast)
        }
        int worst = 1;
        for (int s = 0; s < 16; ++s) {
          int n = 0;
          for (int t = 0; t < 16; ++t) {
            if (slot[t] != s) continue;
            bool dup = false;
            for (int u = 0; u < t; ++u) dup = dup || addr[u] == addr[t];
            n += dup ? 0 : 1;
          }
          worst = std::max(worst, n);
        }
        cyc += worst;
      }
  return cyc;
}
// pads in 8-element (16-B) steps -- CPITCH by up to 24, KWP by up to 120 elements (<= 10 % more LDS) --
// with the fewest read cycles, then the smallest planes; cached per geometry
inline void gw_pitches(const Geo& g, V7& v) {
  static std::mutex mu;
  static std::map<std::array<int, 8>, std::pair<int, int>> memo;
  const std::array<int, 8> key = {g.C, g.H, g.Wo, g.P, g.SH, g.KHW, v.NSLOT, v.whole};
  std::lock_guard<std::mutex> lk(mu);
  auto it = memo.find(key);
  if (it == memo.end()) {
    const int cp0 = v.NSLOT * g.Wo + 8;
    int best = -1, bcp = cp0, bkwp = v.CPL * cp0;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 16; ++b) {
        const int cp = cp0 + 8 * a, kwp = v.CPL * cp + 8 * b;
        const int c = tune("GW_PAD", 1) ? gw_read_cycles(g, v, cp, kwp) : (a + b == 0 ? 0 : 1);
        if (best < 0 || c < best || (c == best && kwp < bkwp)) { best = c; bcp = cp; bkwp = kwp; }
      }
    it = memo.emplace(key, std::make_pair(bcp, bkwp)).first;
  }
  v.CPITCH = it->second.first;
  v.KWP = it->second.second;
}

inline Plan7 v7_plan_compute(const Geo& g) {
  Plan7 p;
  memset(&p, 0, sizeof(p));
#ifdef CIMQ_NO_V7
  return p;
#endif
  const Plan3 p3 = v3_plan(g);
  if (!p3.ok) return p;
  // instantiated slice pairs: w3a3 / w2a2 (interleaved state words) and w8a8 (plane state words)
  if (g.NBP == 4 && !((g.nbw == 3 && g.nba == 3) || (g.nbw == 2 && g.nba == 2))) return p;
  // w8a8: one 16-channel output block (the first conv of the CIFAR ResNets; wider blocks spill)
  // plane words: the w8a8 first layer only (grad_w: at most two 16-row groups, C*KHW <= 32)
  if (g.NBP == 8 && !(g.nbw == 8 && g.nba == 8 && g.OB16 == 1 && g.C * g.KHW <= 32)) return p;
  if (g.O % 16 != 0 || !(g.OB16 == 1 || g.OB16 == 2 || g.OB16 == 4)) return p;
  // 3x3, stride 1, pad 1 ("same" conv: every CiM conv of the CIFAR ResNets but the downsampling ones)
  if (g.KH != 3 || g.KW != 3 || g.SH != g.SW || g.SH > 2 || g.PH != 1 || g.PW != 1) return p;
  if (g.Wo % 8 != 0 || (g.Wo & (g.Wo - 1)) != 0 || g.Wo > 64 || g.M % 128 != 0 || g.FBT > 8) return p;
  V7& v = p.v;
  if (g.P % 128 == 0) v.whole = 0;
  else if (128 % g.P == 0) v.whole = 1;
  else return p;
  v.lw = p3.v.lw;
  // input rows per band, per shape: 16 at stride 2 (round 5: 105.7 -> 80.6 us/step for ResNet-20's two
  // downsampling layers; 8 and 32 slower, gpurun_out/r05_sw7, r05_sw8), 8 at stride 1 (the w2a2 ResNet-56
  // layers and the xbar-64 single conv: 16-row bands made them 6-33 % slower), halved while the grid has fewer
  // blocks than the chip has CUs (cfg1, B = 4: 16 -> 128 bands, 0.138 / 0.107 -> 0.108 / 0.077 ms per fwd+bwd,
  // gpurun_out/r06_rb)
  int rb = g.SH == 2 ? 16 : 8;
  while (rb > 1 && (long long)g.B * cdiv(g.H, rb) < 256) rb /= 2;
  v.RB = std::min(g.H, tune("GX_RB", rb));
  v.nbands = (g.H + v.RB - 1) / v.RB;
  v.FBX = g.FBT;
  // grad_x v8: (c, kh)-row blocks per tile, ring of output rows
  v.NCPBT = 0;
  for (int i = 0; i < g.T; ++i) {
    const int cplo = (i * g.xbar) / 3, cphi = (std::min(g.K, (i + 1) * g.xbar) - 1) / 3;
    v.NCPBT = std::max(v.NCPBT, (cphi >> 2) - (cplo >> 2) + 1);
  }
  if (v.NCPBT > 12) return p;
  v.SWD = std::min(16, g.Wo);
  v.NSEG = g.Wo / v.SWD;
  v.NRS = 64 / g.Wo;
  if (v.NRS < 1) return p;
  v.RSLOT = v.NRS + 2;
  // grad_x fold pass: power-of-two W (index math by shifts); C by shifts when a power of two
  if ((g.W & (g.W - 1)) != 0) return p;
  v.lwin = 0;
  while ((1 << v.lwin) < g.W) ++v.lwin;
  v.lcin = 0;
  while ((1 << v.lcin) < g.C) ++v.lcin;
  if ((1 << v.lcin) != g.C) v.lcin = -1;
  // waves per pixel group: more parallelism where an image has few pixel groups
  v.NPART = tune("GX_NPART", g.Wo >= 32 ? 1 : 2);
  if (v.NPART != 1 && v.NPART != 2 && v.NPART != 4) return p;
  if (g.NBP == 8 && v.NPART == 4) v.NPART = 2;  // 128-VGPR cap of 1024-thread blocks spills w8a8
  // ring, mask coefficients (64 floats), per-wave partials (64 floats), and with NPART > 1 the G
  // exchange [4 pixel groups][NKS][3][64 lanes][16 B] when it fits (GSH)
  p.lds_gx = a16((size_t)v.RSLOT * v.NSEG * g.C * 3 * (g.SH * v.SWD + 2) * 4) + 64 * 4 + 64 * 4;
  {
    const size_t gsh = (size_t)4 * g.NKS * 3 * 64 * 16;
    v.GSH = (v.NPART > 1 && g.OB16 <= 2 && tune("GX_GSH", 1) && p.lds_gx + gsh <= kLdsMax - 512) ? 1 : 0;
    if (v.GSH) p.lds_gx += gsh;
  }
  // grad_w
  v.NSLOT = v.whole ? (128 / g.P) * g.H : ((128 / g.Wo) - 1) * g.SH + g.KH;
  v.CPL = std::min(16, g.C);
  gw_pitches(g, v);
  // tiles touching one channel block (the kernel's loop takes at most 3)
  v.NTL = 1;
  for (int cb = 0; cb * 16 < g.C; ++cb) {
    const int ilo = (cb * 16 * g.KHW) / g.xbar, ihi = (std::min(g.C, cb * 16 + 16) * g.KHW - 1) / g.xbar;
    v.NTL = std::max(v.NTL, ihi - ilo + 1);
  }
  if (v.NTL > 3) return p;
  const size_t planes = (size_t)g.nba * g.KW * v.KWP * 2;
  p.lds_gw = std::max(a16(planes), (size_t)4 * 9 * 256 * 4) + 64 * 4 + (size_t)4 * v.NTL * g.nbw * g.nba * 16 * 4;
  if (g.SH == 1 && v.CPL * v.NSLOT * (g.Wo / 8) > 512) return p;  // grad_w staging: <= 2 items per thread
  p.pairs = ((g.C + 15) / 16) * g.OB16;
  const int stages = g.M / 128;
  const int want = std::max(1, tune("GW_BLOCKS", 512) / p.pairs);
  v.nstage = std::max(1, (stages + want - 1) / want);
  v.nchunks = (stages + v.nstage - 1) / v.nstage;
  const size_t lim = kLdsMax - 512;
  p.ok = p.lds_gx <= lim && p.lds_gw <= lim;
  return p;
}
inline Plan7 v7_plan(const Geo& g) { return memo_geo<Plan7, v7_plan_compute>(g); }

// ---- the fused backward (cimq_fused.hip): one kernel per stride-1 3x3 w2a2 / w3a3 layer ----
struct Plan9 {
  bool ok;
  V9 v;
};

// LDS read cycles of the fused kernel's grad_w A fragments (ds_read_b128, four fixed groups of 16 lanes,
// one cycle per distinct address on a busy 16-B slot of the 256-B bank row; MI355X_MICROARCH.md, LDS) for
// plane pitches cp (channel) and kwp (kw plane), over every row group of tile 0: lane l reads row
// f = 16 gr + (l & 15) = (c, kh, kw) at kw*kwp + c*cp + kh*W + 8 (l >> 4); rows past the tile read one
// zero pad (a broadcast)
inline int fused_read_cycles(const Geo& g, int cp, int kwp) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int flen = std::min(g.K, g.xbar);
  int cyc = 0;
  for (int gr = 0; gr * 16 < flen; ++gr)
    for (int q = 0; q < 4; ++q) {
      int addr[16], slot[16];
      for (int t = 0; t < 16; ++t) {
        const int l = grp[q][t], f = 16 * gr + (l & 15);
        const int c = f / 9, tap = f - 9 * c, kh = tap / 3, kw = tap - 3 * kh;
        addr[t] = f < flen ? kw * kwp + c * cp + kh * g.W + 8 * (l >> 4) : cp - 8;
        slot[t] = (addr[t] / 8) % 16;
      }
      int worst = 1;
      for (int sl = 0; sl < 16; ++sl) {
        int n = 0;
        for (int t = 0; t < 16; ++t) {
          if (slot[t] != sl) continue;
          bool dup = false;
          for (int u = 0; u < t; ++u) dup = dup || addr[u] == addr[t];
          n += dup ? 0 : 1;
        }
        worst = std::max(worst, n);
      }
      cyc += worst;
    }
  return cyc;
}
// plane pitches: CPITCH = PROWS*W + 8 (+ 8a), KWP = NCG*CPITCH (+ 8b), the fewest read cycles, then the
// smallest planes; cached per geometry
inline void fused_pitches(const Geo& g, V9& v) {
  static std::mutex mu;
  static std::map<std::array<int, 6>, std::pair<int, int>> memo;
  const std::array<int, 6> key = {g.W, g.K, g.xbar, v.PROWS, v.NCG, 0};
  std::lock_guard<std::mutex> lk(mu);
  auto it = memo.find(key);
  if (it == memo.end()) {
    const int cp0 = v.PROWS * g.W + 8;
    int best = -1, bcp = cp0, bkwp = v.NCG * cp0;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 16; ++b) {
        const int cp = cp0 + 8 * a, kwp = v.NCG * cp + 8 * b;
        const int c = tune("FUSED_PAD", 1) ? fused_read_cycles(g, cp, kwp) : (a + b == 0 ? 0 : 1);
        if (best < 0 || c < best || (c == best && kwp < bkwp)) { best = c; bcp = cp; bkwp = kwp; }
      }
    it = memo.emplace(key, std::make_pair(bcp, bkwp)).first;
  }
  v.CPITCH = it->second.first;
  v.KWP = it->second.second;
}

inline Plan9 v9_plan_compute(const Geo& g) {
  Plan9 p;
  memset(&p, 0, sizeof(p));
  if (tune("FUSED", 1) == 0) return p;
  const Plan7 p7 = v7_plan(g);
  if (!p7.ok) return p;
  if (g.NBP != 4 || g.nbw != g.nba || (g.nbw != 2 && g.nbw != 3)) return p;
  if (g.SH != 1 || g.SW != 1 || g.KHW != 9) return p;
  if (g.W < 8 || g.W > 64 || (g.W & (g.W - 1)) != 0 || g.Wo != g.W) return p;
  // four 16-channel blocks only: on ResNet-20's layers the fused kernel measured 200 / 110 / 77 us per
  // launch at 16 / 32 / 64 channels against 107 / 95 / 85 us for the v8 grad_x + v7 grad_w pair
  // (DESIGN.md section 4): below four blocks a step has too little MFMA work to hide its staging
  if (g.O != g.Opad || g.O != 64) return p;
  V9& v = p.v;
  v.lw = 0;
  while ((1 << v.lw) < g.W) ++v.lw;
  v.R = 64 / g.W;
  if (g.H % v.R != 0 || g.Ho != g.H) return p;
  v.nsteps = g.H / v.R;
  v.SWD = std::min(16, g.W);
  v.NSEG = g.W / v.SWD;
  v.RSLOT = v.nsteps == 1 ? g.H : v.R + 2;
  v.NCPBT = p7.v.NCPBT;
  v.lcin = p7.v.lcin;
  v.NCG = 0;
  for (int i = 0; i < g.T; ++i) {
    const int c0 = (i * g.xbar) / 9, c1 = (std::min(g.K, (i + 1) * g.xbar) - 1) / 9;
    v.NCG = std::max(v.NCG, c1 - c0 + 1);
  }
  if (v.NCG > 16) return p;
  v.PROWS = v.R + 2;
  fused_pitches(g, v);
  v.nitems = v.NCG * v.PROWS * (g.W / 8);
  if (v.nitems > 512) return p;
  v.NGRP = (g.K + 15) / 16;
  // grad_w in LDS across the steps (and, for one 16-channel output block, one accumulator per K-step)
  v.gwl = (v.nsteps > 1 || g.OB16 == 1) ? 1 : 0;
  const int nkj = g.nbw * g.nba;
  size_t o = 0;
  v.o_ring = (unsigned)o; o += a16((size_t)v.RSLOT * v.NSEG * 3 * g.C * (v.SWD + 2) * 4);
  v.o_cel = (unsigned)o; o += a16((size_t)2 * nkj * 4);
  v.o_red = (unsigned)o; o += 64;
  v.o_plane = (unsigned)o; o += a16((size_t)g.nba * 3 * v.KWP * 2);
  v.o_gwl = (unsigned)o; o += v.gwl ? a16((size_t)(g.OB16 == 1 ? 2 : 1) * v.NGRP * 16 * g.Opad * 4) : 0;
  v.o_gal = (unsigned)o; o += a16((size_t)4 * g.T * nkj * 16 * 4);
  v.o_st = (unsigned)o; o += a16((size_t)64 * g.O * 4);
  v.o_g = (unsigned)o; o += a16((size_t)g.O * 68 * 4);
  v.lds = (unsigned)o;
  p.ok = o <= kLdsMax - 512;
  return p;
}
inline Plan9 v9_plan(const Geo& g) { return memo_geo<Plan9, v9_plan_compute>(g); }

// ---- the first conv's backward from recomputed partial sums (cimq_c1.hip) ----
struct PlanC1 {
  bool ok;
  VC1 v;
};

inline PlanC1 c1_plan(const Geo& g) {
  PlanC1 p;
  memset(&p, 0, sizeof(p));
  if (tune("C1", 1) == 0) return p;
  const Plan7 p7 = v7_plan(g);
  if (!p7.ok || g.variant != VAR_LIBRARY) return p;
  if (g.NBP != 8 || g.nbw != 8 || g.nba != 8 || g.bsw != 1 || g.bsa != 1 || g.O != 16 || g.K > 32) return p;
  if (g.SH != 1 || g.SW != 1 || g.KHW != 9 || g.T != 1) return p;
  if (g.W < 8 || g.W > 64 || (g.W & (g.W - 1)) != 0 || g.Wo != g.W || g.Ho != g.H) return p;
  VC1& v = p.v;
  v.lw = 0;
  while ((1 << v.lw) < g.W) ++v.lw;
  v.R = 128 / g.W;
  if (g.H % v.R != 0) return p;
  v.nsteps = g.H / v.R;
  v.RH = (v.R - 1) + 3;
  v.WP = g.W + 2;
  v.SWD = std::min(16, g.W);
  v.NSEG = g.W / v.SWD;
  v.RSLOT = v.nsteps == 1 ? g.H : v.R + 2;
  v.NCPBT = p7.v.NCPBT;
  v.lcin = p7.v.lcin;
  size_t o = 0;
  const size_t patch = a16((size_t)g.C * v.RH * v.WP * 8);
  v.o_xp = (unsigned)o; o += patch;
  v.o_hp = (unsigned)o; o += patch;
  v.o_ptab = (unsigned)o; o += 64 * 4;
  v.o_prm = (unsigned)o; o += 64 * 16 * 16;
  v.o_cel = (unsigned)o; o += a16(3 * 64 * 4);
  v.o_g = (unsigned)o; o += 16 * 132 * 4;
  v.o_ring = (unsigned)o; o += a16((size_t)v.RSLOT * v.NSEG * 3 * g.C * (v.SWD + 2) * 4);
  v.o_gal = (unsigned)o; o += 8 * 64 * 16 * 4;
  v.o_red = (unsigned)o; o += a16((2 * 16 * 16 + 8) * 4);
  v.o_e = (unsigned)o; o += 8 * 2 * 256 * 4;
  v.o_wk = (unsigned)o; o += 8 * 64 * 16;
  v.o_wc = (unsigned)o; o += (size_t)3 * 4 * 64 * 16;
  v.lds = (unsigned)o;
  // the kernel's one-step-ahead staging: at most three 16-byte items per thread of 512
  if (2 * g.C * v.RH * (g.W / 2) + 512 > 3 * 512 || (g.K - 1) / 3 / 4 + 1 > 3) return p;
  p.ok = o <= kLdsMax - 512;
  return p;
}

// ---- the dense path (cimq_part_dense.hip): 1x1 kernels on 1x1 images, a [B][C] x [C][O] GEMM ----
// (BASELINE cfg5, QuantLinear as Conv2dLSQCiM(k=1) on [B, C, 1, 1]); the library ternary ADC, equal
// weight / activation slice counts up to 4 (the uint2 state word holds 16 slice pairs per plane)
inline bool dense_plan(const Geo& g) {
  if (tune("DENSE", 1) == 0) return false;
  if (g.KH != 1 || g.KW != 1 || g.SH != 1 || g.SW != 1 || g.PH != 0 || g.PW != 0 || g.H != 1 || g.W != 1) return false;
  if (g.variant != VAR_LIBRARY || g.mode != ADC_TERNARY || g.NBP != 4 || g.nbw != g.nba || g.nbw > 4) return false;
  if (g.xbar % 64 != 0 || g.xbar > 128 || g.C % 16 != 0 || g.O % 64 != 0 || g.M % 128 != 0) return false;
  return true;
}
// grad_w row chunks: about 512 workgroups over (chunks x tiles x 128-channel groups), 32-row multiples
inline int dense_chunks(const Geo& g) {
  const int per = std::max(1, 512 / (g.T * ((g.O + 127) / 128)));
  return std::max(1, std::min(per, g.M / 256));
}
// the dense grad_x kernel's MFMA waves (8 per block), each leaving one act-LSQ partial when it runs
// the quantiser's backward (0: that does not fit the partial buffer, the separate pass runs)
inline int dense_lsq_parts(const Geo& g) {
  const int n = (g.M / 128) * g.T * 8;
  return n <= std::max(kLsqParts, g.B * g.H) ? n : 0;
}
inline int dense_rows_per_chunk(const Geo& g) {
  const int n = dense_chunks(g);
  return ((g.M + n - 1) / n + 31) / 32 * 32;
}

// the shift ADC's statistics kernel (cimq_part_shift.hip) applies: interleaved 3-bit state words of
// w2a2 / w3a3 on a v7 shape (other shift layers take the general backward)
inline bool shift_stats_ok(const Geo& g) {
  if (!shift_fast(g)) return false;
  if (g.NBP == 8)  // the w8a8 first conv: one K-step, one crossbar tile (shift_stats8_kernel)
    return g.nbw == 8 && g.nba == 8 && g.KS == 1 && g.T == 1 && g.bsw == 1 && g.bsa == 1;
  return g.NBP == 4 && g.nbw == g.nba && (g.nbw == 2 || g.nbw == 3);
}
// half-range of its q tables: the largest |ps| of 0 .. 2^bs - 1 slices over one tile (the sign slice of
// the weights included); larger partial sums (slice artifacts) take the direct evaluation
inline int shift_table_range(const Geo& g) {
  const int tmax = std::min(g.K, g.xbar);
  return tmax * ((1 << g.bsa) - 1) * ((1 << g.bsw) - 1);
}
inline bool shift_table_fits(const Geo& g) {
  return (size_t)g.nbw * g.nba * 16 * (2 * shift_table_range(g) + 1) * 4 <= 48 * 1024;
}

// the backward runs on the v7 plan's state words (v7 / fused / first-conv kernels): the library ADC, or
// the shift ADC where the statistics kernel takes it; every other layer runs the general kernels
// the module forward with the LSQ activation quantiser fused into the forward's row staging: the
// v3 fast path with v7 state words (so no later kernel reads the forward slice words), 4-byte slice
// words, the prologue's word table applicable, and not the first conv (whose backward re-reads the
// forward words) or a shift layer (its statistics kernel does)
struct ActQ {
  const float* x;
  const float* signed_act;
};
inline bool v7_bwd(const Geo& g);
inline bool fwd_actq_ok(const Geo& g);

inline bool v7_bwd(const Geo& g) {
  return v7_plan(g).ok && (g.variant == VAR_LIBRARY || shift_stats_ok(g));
}

inline bool fwd_actq_ok(const Geo& g) {
  if (tune("ACTQ", 1) == 0) return false;
  return g.input_kind == CIMQ_INPUT_RAW_LSQ && g.NBP == 4 && g.variant == VAR_LIBRARY && g.W % 4 == 0 &&
         g.P % 64 == 0 && g.lsq_qp >= 0.f && g.lsq_qp < 255.f && v3_plan(g).ok && v7_bwd(g) && !c1_plan(g).ok;
}

// ---- the w3a3 forward on the slice-planar patch (cimq_fwd5.hip) ----
struct Plan5 {
  bool ok;
  F5 v;
  size_t lds;
  int nob;  // 16-channel output blocks per workgroup (the kernel's template argument)
};

inline Plan5 f5_plan_compute(const Geo& g) {
  Plan5 p;
  memset(&p, 0, sizeof(p));
  if (tune("FWD5", 1) == 0) return p;
  // the module forward with the fused activation quantiser, w3a3 1-bit slices, the ternary library ADC,
  // 3x3 / pad 1 / stride 1 or 2, whole 16-pixel groups, 128-pixel m-tiles of R rows of one image or of
  // 128 / P whole images
  if (!fwd_actq_ok(g) || g.mode != ADC_TERNARY || g.variant != VAR_LIBRARY) return p;
  if (g.nbw != 3 || g.nba != 3 || g.bsw != 1 || g.bsa != 1) return p;
  if (g.KH != 3 || g.KW != 3 || g.PH != 1 || g.PW != 1 || g.SH != g.SW || (g.SH != 1 && g.SH != 2)) return p;
  if (g.C % 16 != 0 || g.O % 16 != 0 || g.W % 4 != 0 || g.P % 16 != 0) return p;
  if (g.P >= 128 ? g.P % 128 != 0 : 128 % g.P != 0) return p;
  if (g.M % 128 != 0) return p;  // whole 128-pixel m-tiles (B * P: whole images per m-tile when P < 128)
  if (g.Wo % 16 != 0 && 16 % g.Wo != 0) return p;
  F5& v = p.v;
  v.lwo = 0;
  while ((1 << v.lwo) < g.Wo) ++v.lwo;
  if ((1 << v.lwo) != g.Wo) return p;
  v.lwi = 0;
  while ((1 << v.lwi) < g.W) ++v.lwi;
  if ((1 << v.lwi) != g.W) return p;
  // the kernel's element, state-word and output offsets are 32-bit
  if ((long long)g.Nin >= (1LL << 31) || (long long)g.T * g.M * g.O >= (1LL << 31) || (long long)g.M * g.O >= (1LL << 31))
    return p;
  const int PI = std::min(g.P, 128);
  v.IPM = 128 / PI;
  v.R = PI / g.Wo;
  v.RH = (v.R - 1) * g.SH + 3;
  v.WP = g.W + 2;
  v.nmt = g.M / 128;
  v.ntc = 0;
  for (int i = 0; i < g.T; ++i) {
    v.tc0[i] = (unsigned char)v.ntc;
    const int flo = i * g.xbar, fhi = std::min(flo + g.xbar, g.K);
    const int cblo = (flo / 9) / 16, cbhi = ((fhi - 1) / 9) / 16;
    for (int cb = cblo; cb <= cbhi; ++cb) {
      if (v.ntc >= kF5MaxTc) return p;
      v.tcb[v.ntc++] = (unsigned char)cb;
    }
  }
  v.tc0[g.T] = (unsigned char)v.ntc;
  // output blocks per workgroup: two (a 1024-thread block per CU, sharing the activation patch) where
  // OB16 is even, else one (two 512-thread blocks per CU)
  p.nob = (g.OB16 % 2 == 0 && tune("FWD5_NOB2", 1)) ? 2 : 1;
  // tile groups: greedy, while the block's LDS (the widest group's fragments and channel span) fits
  const size_t fixed = (size_t)p.nob * g.T * 9 * 16 * (16 + 4) + a16((size_t)2 * ((int)g.lsq_qp + 2) * 4) + 16;
  const size_t budget = (size_t)(p.nob == 2 ? tune("FWD5_LDS2_KB", 150) : tune("FWD5_LDS_KB", 80)) * 1024;
  auto need = [&](int tcm, int ncb) {
    return fixed + (size_t)p.nob * tcm * 9 * 1024 + (size_t)v.IPM * v.RH * ncb * v.WP * 48;
  };
  v.ngrp = 0;
  v.tcmax = 0;
  v.NCBP = 0;
  for (int i = 0; i < g.T;) {
    if (v.ngrp >= kF5MaxGrp) return p;
    int e = i + 1;
    auto span = [&](int a, int b) { return v.tcb[v.tc0[b] - 1] - v.tcb[v.tc0[a]] + 1; };
    auto pairs = [&](int a, int b) { return v.tc0[b] - v.tc0[a]; };
    if (need(std::max(v.tcmax, pairs(i, e)), std::max(v.NCBP, span(i, e))) > budget) return p;
    while (e < g.T && need(std::max(v.tcmax, pairs(i, e + 1)), std::max(v.NCBP, span(i, e + 1))) <= budget) ++e;
    const int q = v.ngrp++;
    v.gt0[q] = (unsigned char)i;
    v.gcb0[q] = v.tcb[v.tc0[i]];
    v.gcb1[q] = v.tcb[v.tc0[e] - 1];
    v.gown[q] = (unsigned char)(q == 0 ? v.gcb0[0] : v.gcb1[q - 1] + 1);
    v.tcmax = std::max(v.tcmax, pairs(i, e));
    v.NCBP = std::max(v.NCBP, span(i, e));
    i = e;
  }
  v.gt0[v.ngrp] = (unsigned char)g.T;
  p.lds = need(v.tcmax, v.NCBP);
  p.ok = p.lds <= budget;
  return p;
}
inline Plan5 f5_plan(const Geo& g) { return memo_geo<Plan5, f5_plan_compute>(g); }
// wf5 fragments of a layer (all output-channel blocks)
inline size_t f5_frag_items(const Geo& g, const Plan5& p) { return p.ok ? (size_t)g.OB16 * p.v.ntc * 9 * 64 : 0; }
inline size_t f5_frag_bytes(const Geo& g) { return f5_frag_items(g, f5_plan(g)) * 16; }

// ---- grad_w + grad_alpha partials of the w3a3 stride-1 16 / 32-channel layers (cimq_gw5.hip) ----
struct PlanG5 {
  bool ok;
  G5 v;
  size_t lds;
  int pairs;  // (input, output) 16-channel block pairs: grid y
};

inline PlanG5 g5_plan_compute(const Geo& g) {
  PlanG5 p;
  memset(&p, 0, sizeof(p));
  if (tune("GW5", 1) == 0) return p;
  if (!v7_bwd(g) || g.variant != VAR_LIBRARY || g.NBP != 4 || g.nbw != 3 || g.nba != 3 || g.bsa != 1) return p;
  if (g.KH != 3 || g.KW != 3 || g.SH != g.SW || (g.SH != 1 && g.SH != 2) || g.PH != 1 || g.PW != 1 ||
      g.xbar != 128)
    return p;
  if (g.W != g.Wo * g.SH || g.H != g.Ho * g.SH) return p;  // (stride 2: even input sides)
  // stride 2 (17 staged rows for 8 output rows): 65.8 vs cim_bwd_gw_v7_kernel's 87.4 us/step on ResNet-20's
  // two transition layers once the staging's first round went before the barrier (51.5 vs 43 us per
  // launch before: gpurun_out/r05_sw11)
  if (g.SH == 2 && tune("GW5_S2", 1) == 0) return p;
  if (g.C % 16 != 0 || g.O % 16 != 0 || g.Wo % 4 != 0) return p;
  if (g.P >= 128 ? g.P % 128 != 0 : (128 % g.P != 0 || g.P % 16 != 0)) return p;
  if (g.M % 128 != 0) return p;  // whole 128-pixel m-tiles
  // (no dependence on g.onchw: the ctx / workspace layouts are computed from the same Geo at query, prologue
  // and launch time, and the module backward sets onchw only at launch; the kernel reads both layouts)
  if (g.T != (9 * g.C + 127) / 128) return p;
  G5& v = p.v;
  v.lwo = 0;
  while ((1 << v.lwo) < g.Wo) ++v.lwo;
  if ((1 << v.lwo) != g.Wo || 128 % g.Wo != 0) return p;
  v.lwi = v.lwo + (g.SH == 2 ? 1 : 0);  // W = Wo * SH
  if ((long long)g.Nin >= (1LL << 31)) return p;  // 32-bit element offsets in the staging
  v.IPM = 128 / std::min(g.P, 128);
  v.R = std::min(g.P, 128) / g.Wo;
  v.RH = (v.R - 1) * g.SH + 3;
  v.WP = g.W + 2;
  // the kernel stages an m-tile's patch in rounds of six items per thread, the first round's reads issued
  // before the barrier (the stride-1 16 / 32-channel layers: 3072 / 2560 items, one round; stride 2 stages
  // 17 rows, three rounds); the packed row offsets need the patch below 2^16 uint2
  if ((long long)16 * v.IPM * v.RH * v.WP >= (1LL << 16)) return p;
  if (g.SH == 1 && 16 * v.IPM * v.RH * g.W > 6 * 512) return p;
  v.nmt = g.M / 128;
  p.pairs = (g.C / 16) * g.OB16;
  // blocks: about two per CU; chunks (slabs) = blocks / pairs
  const int want = std::max(1, tune("GW5_BLOCKS", 512) / p.pairs);
  v.nst = std::max(1, (v.nmt + want - 1) / want);
  v.nchunks = (v.nmt + v.nst - 1) / v.nst;
  // the A-ready patch (or the epilogue's wave-sum buffer, three 16-row blocks of 8 waves), then cD_kj (16
  // floats) and the code -> word table (260)
  p.lds = std::max((size_t)16 * v.IPM * v.RH * v.WP * 8, (size_t)3 * 8 * 64 * 16) + 64 + 4 * 260;
  p.ok = p.lds <= (size_t)80 * 1024;
  return p;
}
inline PlanG5 g5_plan(const Geo& g) { return memo_geo<PlanG5, g5_plan_compute>(g); }

// ---- grad_x of the w3a3 stride-1 16 -> 16 (32 x 32) / 32 -> 32 (16 x 16) layers, per input pixel (cimq_gx5.hip) ----
struct PlanX5 {
  bool ok;
  X5 v;
  size_t lds;
  int nblk;  // grid = the d sa partials it leaves
};

inline PlanX5 x5_plan_compute(const Geo& g) {
  PlanX5 p;
  memset(&p, 0, sizeof(p));
  if (tune("GX5", 1) == 0) return p;
  if (!v7_bwd(g) || g.variant != VAR_LIBRARY || g.NBP != 4 || g.nbw != 3 || g.nba != 3 || g.bsw != 1) return p;
  if (g.input_kind != CIMQ_INPUT_RAW_LSQ) return p;  // (not g.onchw: see g5_plan)
  if (g.KH != 3 || g.KW != 3 || g.SH != 1 || g.SW != 1 || g.PH != 1 || g.PW != 1 || g.xbar != 128) return p;
  // 16 -> 16 at 32 x 32 (8 pixel groups x 1 channel block) or 32 -> 32 at 16 x 16 (4 x 2)
  const bool c16 = g.C == 16 && g.O == 16 && g.W == 32, c32 = g.C == 32 && g.O == 32 && g.W == 16;
  if (!(c16 || c32) || g.H % 4 != 0 || g.Wo != g.W || g.Ho != g.H || g.T != (9 * g.C + 127) / 128) return p;
  p.v.tpi = g.H / 4;
  p.v.nmt = g.B * p.v.tpi;
  p.v.CBN = g.C / 16;
  p.v.NPG = g.W / 4;
  if (p.v.NPG * p.v.CBN != 8) return p;
  p.v.lw = g.W == 32 ? 5 : 4;  // (c16: W 32, c32: W 16)
  if (6 * g.W * 4 > 2 * 512) return p;  // the kernel keeps <= 2 G-patch items' grad_out per thread
  // 32-bit element / state-word offsets in the kernel
  if ((long long)g.T * g.M * g.O >= (1LL << 31) || (long long)g.Nin >= (1LL << 31) || (long long)g.M * g.O >= (1LL << 31))
    return p;
  // 256 workgroups (one per CU) since grad_x and grad_w share a launch: grad_w's workgroups then start beside
  // grad_x's instead of behind them (whole step 2.30 -> 2.28 ms, 4 of 4 A/B pairs; 512 was best for gx5
  // alone; 128 / 192 / 320 / 384 / 768 / 1024 slower: profiles/r06_final/extra/gxw5_grid_sweep.txt)
  p.nblk = std::min(p.v.nmt, tune("GX5_GRID", 256));
  p.lds = (size_t)3 * 6 * (g.W + 2) * 96 + 32 + (size_t)9 * 2 * p.v.CBN * 1024 + 32 * 4;
  p.ok = p.lds <= (size_t)80 * 1024;
  return p;
}
inline PlanX5 x5_plan(const Geo& g) { return memo_geo<PlanX5, x5_plan_compute>(g); }
inline size_t x5_frag_bytes(const Geo& g) {
  const PlanX5 p = x5_plan(g);
  return p.ok ? (size_t)g.T * p.v.CBN * 9 * 2 * p.v.CBN * 64 * 16 : 0;
}

// ---- the whole backward of the w3a3 16 -> 16 stride-1 layers from recomputed partial sums (cimq_r6.hip) ----
struct PlanR6 {
  bool ok;
  R6 v;
  size_t lds;
};

inline PlanR6 r6_plan_compute(const Geo& g) {
  PlanR6 p;
  memset(&p, 0, sizeof(p));
  if (!g.recompute || tune("R6", 1) == 0) return p;  // the caller's choice (CIMQ_OPT_RECOMPUTE)
  // the module forward is cim_fwd5_kernel (its weight operand wf5 and activation word table are the recompute's),
  // the library ternary ADC, w3a3 1-bit slices, 3x3 / stride 1 / pad 1, xbar 128, 16 -> 16 channels, 32 wide
  const Plan5 p5 = f5_plan(g);
  if (!p5.ok || !v7_bwd(g) || g.variant != VAR_LIBRARY || g.mode != ADC_TERNARY) return p;
  if (g.input_kind != CIMQ_INPUT_RAW_LSQ || g.nbw != 3 || g.nba != 3 || g.bsw != 1 || g.bsa != 1) return p;
  if (g.KH != 3 || g.KW != 3 || g.SH != 1 || g.SW != 1 || g.PH != 1 || g.PW != 1 || g.xbar != 128) return p;
  if (g.C != kR6C || g.O != kR6C || g.W != kR6W || g.Wo != g.W || g.Ho != g.H || g.H % kR6R != 0) return p;
  if (g.T != kR6T || g.lsq_qp >= 255.f || (long long)g.Nin >= (1LL << 31)) return p;
  // one (tile, channel-block) pair per tile in the forward's operand
  if (p5.v.ntc != kR6T || p5.v.tc0[0] != 0 || p5.v.tc0[1] != 1 || p5.v.tc0[2] != 2) return p;
  for (int i = 0; i <= kR6T; ++i) p.v.tc0[i] = p5.v.tc0[i];
  p.v.ntc = p5.v.ntc;
  p.v.nmt = g.H / kR6R;
  p.lds = R6L::LDS;
  p.ok = true;
  return p;
}
inline PlanR6 r6_plan(const Geo& g) { return memo_geo<PlanR6, r6_plan_compute>(g); }
inline size_t r6_frag_bytes(const Geo& g) { return r6_plan(g).ok ? (size_t)kR6WxItems * 16 : 0; }
// decided at launch: the module entry points (g.onchw) run cim_fwd5_kernel, whose operand the recompute needs; the
// Function path's forward writes state words and keeps the state-word backward
inline bool r6_bwd(const Geo& g) { return g.onchw && r6_plan(g).ok; }

// The module path's ctx as ONE activation-code byte per element (instead of the 4-byte backward word):
// where the forward is cim_fwd5_kernel (which quantises the activation itself) and the layer's grad_w
// is cim_bwd_gw5_kernel (dispatch_bwd_any's order: c1, fused, then the v7 pair), the only ctx reader.
// Decided at launch: g.onchw is the module entry points' flag (the Function path's prologue writes words).
// (c1_plan / v9_plan are declared above ws_layout.)
inline bool ctx_codes(const Geo& g) {
  return g.onchw && fwd_actq_ok(g) && f5_plan(g).ok && v7_bwd(g) && !c1_plan(g).ok && !v9_plan(g).ok &&
         g5_plan(g).ok && !r6_bwd(g);
}

struct WsLayout {
  size_t gw_slab, ga_slab, gb_slab, ss_slab, qtab, lsq_part, gaq, gapart, wpart, bpo, gxu, total;
  int rows, nchunks, nchunks_bwd;
};

// pixel chunks of the shift-ADC statistics kernel: about 1024 blocks over (chunks x tiles x o-blocks)
inline int shift_chunks(const Geo& g) {
  const int per = std::max(1, 1024 / (g.T * g.OB16));
  return std::max(1, std::min(per, g.M / 64));
}

inline WsLayout ws_layout_compute(const Geo& g) {
  WsLayout W;
  gw_chunks(g, &W.rows, &W.nchunks);
  // backward slabs: the v7 grad_w kernel's pixel chunks when it applies (the alpha_cim init
  // kernel keeps gw_chunks' split: W.nchunks / W.rows)
  // (the one-kernel backwards: one chunk per image; the v7 plan also covers shift-ADC layers that the
  // statistics kernel does not take -- those run the general backward)
  const Plan7 p7 = v7_plan(g);
  const bool v7b = v7_bwd(g);
  const PlanG5 pg5 = g5_plan(g);
  W.nchunks_bwd = (v9_plan(g).ok || c1_plan(g).ok || r6_bwd(g)) ? g.B : pg5.ok ? pg5.v.nchunks : v7b ? p7.v.nchunks
                : dense_plan(g) ? cdiv(g.M, dense_rows_per_chunk(g)) : W.nchunks;
  // (sizes for either backward of a layer: the module path's recompute backward has one chunk per image)
  const size_t nch = (size_t)std::max({W.nchunks, W.nchunks_bwd, r6_plan(g).ok ? g.B : 0});
  size_t o = 0;
  W.gw_slab = o; o = align256(o + sizeof(float) * nch * g.T * g.FBT * 16 * g.Opad);
  W.ga_slab = o; o = align256(o + sizeof(float) * nch * g.T * g.nbw * g.nba * g.Opad);
  W.gb_slab = o; o = align256(o + (g.variant == VAR_SHIFT_ROUND || g.variant == VAR_SHIFT_SIGN
                                       ? sizeof(float) * nch * g.T * g.nbw * g.nba * g.Opad : 0));
  // shift ADC on the fast path: per pixel chunk, tile, pair and channel the grad_alpha / grad_beta partials
  // shift ADC statistics (v7 shapes, shift_stats_ok): per pixel chunk, tile, pair and channel the
  // grad_alpha / grad_beta partials, and the q tables [T][OB16][nbw * nba][16][2R + 1] when they fit
  const bool stats = p7.ok && shift_stats_ok(g);
  W.ss_slab = o; o = align256(o + (stats ? sizeof(float) * shift_chunks(g) * g.T * 2 * g.nbw * g.nba * g.Opad : 0));
  W.qtab = o; o = align256(o + ((stats && shift_table_fits(g)) ? sizeof(float) * (size_t)g.T * g.OB16 * g.nbw * g.nba *
                                                                    16 * (2 * shift_table_range(g) + 1)
                                                              : 0));
  W.lsq_part = o; o = align256(o + sizeof(float) * std::max(kLsqParts, g.B * g.H));  // >= B * bands
  // module entry points: d loss / d alpha_q, weight-LSQ partials of the grad_w reducer, and
  // a [B, P, O] staging copy of out / grad_out for the general kernels
  W.gaq = o; o = align256(o + sizeof(float) * (size_t)g.T * g.nbw * g.nba * g.O);
  W.gapart = o; o = align256(o + sizeof(float) * 4 * (size_t)cdiv((long long)g.T * g.nbw * g.nba * g.Opad, 64));
  W.wpart = o; o = align256(o + sizeof(float) * 2 * (size_t)cdiv((long long)g.T * g.FBT * 16 * g.Opad, 64));
  W.bpo = o; o = align256(o + sizeof(float) * (size_t)g.M * g.O);
  // the general backward's unfolded grad_x [M][K] (folded by fold_gx_kernel)
  W.gxu = o; o = align256(o + ((v7b || dense_plan(g)) ? 0 : sizeof(float) * (size_t)g.M * g.K));
  W.total = o;
  return W;
}
inline WsLayout ws_layout(const Geo& g) { return memo_geo<WsLayout, ws_layout_compute>(g); }

template <typename K>
inline int set_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024) {
    if (bytes > kLdsMax) return fail(CIMQ_EUNSUPPORTED, "needs %zu bytes of LDS", bytes);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return fail(CIMQ_EHIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
  }
  return CIMQ_OK;
}

#define CIMQ_TRY(x)        \
  do {                     \
    int _rc = (x);         \
    if (_rc) return _rc;   \
  } while (0)

// ---------------------------------------------------------------------------------------
// diagnostic kernel timer (cimq_profile_start / _stop): a hipEvent pair around every launch of
// one kernel id, recorded on the launch stream; algorithmic bytes / flops per launch follow
// SURVEY.md section 8(d) (fp32 tensors the kernel must read or write once).
// ---------------------------------------------------------------------------------------
// 1-4: every launch of that role (all kernel variants); 5-7: only the v7-path kernels
// (cim_fwd_v3_kernel<4, KS, true>, cim_bwd_gx_v8_kernel, cim_bwd_gw_v7_kernel), so that one
// id maps to the launches of one rocprof kernel symbol family
// (8: the fused backward, cimq_fused.hip -- grad_x and grad_w in one launch, role grad_x)
enum KernelId {
  KID_NONE = 0, KID_FWD = 1, KID_BWD_GX = 2, KID_BWD_GW = 3, KID_PREP_ACT = 4,
  KID_FWD_V7 = 5, KID_GX_V8 = 6, KID_GW_V7 = 7, KID_FUSED = 8, KID_LAST = 8
};

struct Profiler {
  std::mutex mu;
  int kid = KID_NONE;
  int cap = 0, n = 0;
  hipEvent_t* ev = nullptr;  // 2*cap
  double bytes = 0, flops = 0;
  // per launch: algorithmic bytes, logical flops, MFMA operations as issued (cimq_profile_read)
  double *lb = nullptr, *lf = nullptr, *lm = nullptr;
};
inline Profiler& prof() {
  static Profiler p;
  return p;
}

// slice pairs whose binary_mask entry is nonzero: 2^(bsa*j + bsw*k) wraps to 0 in int8 at >= 2^8
// (_quan_base.py:207-214), so the w8a8 first layer has 36 live pairs of 64
inline int live_pairs(const Geo& g) {
  int n = 0;
  for (int k = 0; k < g.nbw; ++k)
    for (int j = 0; j < g.nba; ++j) n += (g.bsa * j + g.bsw * k <= 7) ? 1 : 0;
  return n;
}

// SURVEY 8(d) per launch: *bytes = the fp32 tensors the kernel must read or write once, *flops = the
// logical 2*MAC (times the slice count the contraction runs over), *mops = the MFMA operations as the
// algorithm issues them: int8 bit-slice products of the live pairs (forward), three bf16 products per
// fp32-accurate backward MAC
inline void algo_counts(const Geo& g, int kid, double* bytes, double* flops, double* mops) {
  const double x4 = 4.0 * (double)g.Nin, y4 = 4.0 * (double)g.M * g.O;
  const double mac = (double)g.M * g.O * g.K;
  switch (kid) {
    case KID_FWD_V7:
    case KID_FWD: *bytes = x4 + y4; *flops = 2.0 * mac; *mops = 2.0 * mac * live_pairs(g); break;  // read x, write y
    case KID_GX_V8:
    case KID_BWD_GX: *bytes = 2.0 * x4 + y4; *flops = 2.0 * mac * g.nbw; *mops = 3.0 * *flops; break;  // read gy, x; write gx
    case KID_GW_V7:
    case KID_BWD_GW: *bytes = x4 + y4; *flops = 2.0 * mac * g.nba; *mops = 3.0 * *flops; break;  // read gy, x
    case KID_PREP_ACT: *bytes = x4 + (double)g.Nin * (g.NBP + 1); *flops = 0; *mops = 0; break;
    case KID_FUSED: *bytes = 2.0 * x4 + y4; *flops = 2.0 * mac * (g.nbw + g.nba); *mops = 3.0 * *flops; break;  // read gy, x; write gx
    default: *bytes = 0; *flops = 0; *mops = 0;
  }
}

// returns the event slot to close after the launch (-1: not profiling this kernel)
inline int prof_begin(int kid, const Geo& g, hipStream_t s) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.n >= p.cap) return -1;
  const int role = kid == KID_FWD_V7 ? KID_FWD : (kid == KID_GX_V8 || kid == KID_FUSED) ? KID_BWD_GX
                 : kid == KID_GW_V7 ? KID_BWD_GW : kid;
  if (p.kid != kid && p.kid != role) return -1;
  const int slot = p.n++;
  double b, f, mo;
  algo_counts(g, kid, &b, &f, &mo);
  p.bytes += b;
  p.flops += f;
  p.lb[slot] = b;
  p.lf[slot] = f;
  p.lm[slot] = mo;
  (void)hipEventRecord(p.ev[2 * slot], s);
  return slot;
}
inline void prof_end(int slot, hipStream_t s) {
  if (slot < 0) return;
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  (void)hipEventRecord(p.ev[2 * slot + 1], s);
}

// ---- launchers defined in the cimq_part_*.hip translation units (compiled in parallel) ----
// cimq_part_fwd.hip: the forward partial-sum kernels (v3 fast path or the general kernel;
// the general kernel with ps_dbg / adc_dbg also writes every partial sum and ADC output)
int launch_fwd_any(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, int* ps_dbg,
                   float* adc_dbg, hipStream_t s,
                   const ActQ* aq = nullptr);
// cimq_part_fwd5.hip: the w3a3 module forward on the slice-planar patch (f5_plan)
int launch_fwd5(const Geo& g, const Plan5& p, uint8_t* ctx, const float* sw, const float* sa, float* out,
                hipStream_t s, const ActQ* aq);
// cimq_part_gx5.hip: grad_x (+ the fused act-LSQ backward) of the 16 -> 16-channel 32-wide layers (x5_plan)
int launch_gx5(const Geo& g, const PlanX5& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
               const float* x, float* gx, uint8_t* ws, hipStream_t s);
// ... and its weight operand from a quantised w_q (the Function entry points' prologue, prep_all)
int launch_prep_wg5(const Geo& g, const float* w_q, const float* sw, uint8_t* ctx, hipStream_t s);
// cimq_part_gw5.hip: grad_w + grad_alpha slabs of the w3a3 stride-1 16 / 32-channel layers (g5_plan)
int launch_gw5(const Geo& g, const PlanG5& p, const uint8_t* ctx, const float* gout, uint8_t* ws, hipStream_t s);
// cimq_part_gxw5.hip: both in one launch (grad_x's workgroups, then grad_w's)
int launch_gxw5(const Geo& g, const PlanX5& px, const PlanG5& pw, const uint8_t* ctx, const float* sw, const float* sa,
                const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s);
// cimq_part_dense.hip: the dense path (dense_plan) -- forward, and grad_x + grad_w / grad_alpha slabs
int launch_dense_fwd(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, hipStream_t s);
// shift ADC on the fast path (cimq_part_shift.hip): grad_alpha / grad_beta from the forward's state words
// (shift_stats_ok, above ws_layout; other layers take the general backward)
int launch_shift_stats(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
                       const int8_t* bmask, uint8_t* ws, float* grad_alpha, float* grad_beta, hipStream_t s,
                       int accum_beta = 0);
int launch_dense_bwd(const Geo& g, const uint8_t* ctx, const float* sw, const float* gout, float* gx, uint8_t* ws,
                     hipStream_t s,
                     const float* x = nullptr, const float* sa = nullptr);
// cimq_part_bwd.hip: backward of layers outside the v7 / dense plans (the general kernels)
int launch_bwd_general(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
                       const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused);
// cimq_part_bwd.hip: per-chunk sums of |ps * sw * sa| for the alpha_cim initialisation
int launch_alpha_init_sums(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                           const float* signed_act, uint8_t* ws, hipStream_t s);
// cimq_part_v7_*.hip: the v7 backward (grad_x v8 + grad_w v7) for one slice-pair shape
template <int NBW, int NBA>
int launch_v7_n(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa,
                const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq,
                int parts);
#define CIMQ_V7_SIG(NBW, NBA)                                                                              \
  int launch_v7_n<NBW, NBA>(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa, \
                            const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq, \
                            int parts)
// cimq_part_fused.hip: the fused backward (v9_plan)
int launch_fused(const Geo& g, const Plan9& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
                 const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq);
int launch_c1(const Geo& g, const PlanC1& p, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
              const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq);
// cimq_part_r6.hip: the recompute backward (r6_bwd); dbg: the parity hook's state words into st_dbg instead
int launch_r6(const Geo& g, const PlanR6& p, const uint8_t* ctx, const float* sw, const float* sa, const float* sgn,
              const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, uint32_t* st_dbg = nullptr);
extern template CIMQ_V7_SIG(2, 2);
extern template CIMQ_V7_SIG(3, 3);
extern template CIMQ_V7_SIG(8, 8);

}  // namespace cimq

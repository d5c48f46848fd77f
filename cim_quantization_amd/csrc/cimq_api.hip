// cimq_api.hip -- the extern "C" boundary of libcimq.so (declared in include/cimq.h).
// Host-side geometry validation, ctx / workspace carving and the kernel launch sequences
// that replace get_cim_output_signed.forward / backward (models/_modules/lsq.py:92-386).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "../../include/cimq.h"
#include "cimq_kernels_v3.hip"
#include "cimq_gx_v6.hip"
#include "cimq_v7.hip"
#include "cimq_lsq.hip"

using namespace cimq;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int check_hip(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CIMQ_EHIP, "%s: %s", where, hipGetErrorString(e));
  return CIMQ_OK;
}

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// tuning knobs for experiments (tools/, built with -DCIMQ_TUNING): CIMQ_TUNE_<name>=<int>
// overrides a launch shape; the shipped library compiles them to the defaults
#ifdef CIMQ_TUNING
int tune(const char* name, int dflt) {
  char key[64];
  snprintf(key, sizeof(key), "CIMQ_TUNE_%s", name);
  const char* v = getenv(key);
  return v ? atoi(v) : dflt;
}
#else
constexpr int tune(const char*, int dflt) { return dflt; }
#endif
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

int make_geo(const cimq_conv_desc* d, Geo* out) {
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
  long long psmax = (long long)tmax * (1LL << g.bsa) * (1LL << g.bsw);
  g.psmax = (int)(psmax > (1 << 24) ? (1 << 24) : psmax);
  *out = g;
  return CIMQ_OK;
}

struct CtxLayout {
  size_t xcode, xhat, wfrag, wgx, wtc, wcy, thi, tlo, mlo, mhi, coef, alpha, ckj, flags, st;
  size_t lsq_scal;  // module entry points: sa, sw, alpha scale, max, min
  size_t total;
};

CtxLayout ctx_layout(const Geo& g) {
  CtxLayout L;
  size_t o = 0;
  const size_t npar = (size_t)g.T * g.nba * g.nbw * g.Opad;
  L.xcode = o; o = align256(o + (size_t)g.Nin * g.NBP);  // forward slice bytes
  L.xhat = o; o = align256(o + (size_t)g.Nin * g.NBP);   // backward (int8 ctx) slice bytes
  L.wfrag = o; o = align256(o + (size_t)g.T * g.KS * g.NBLK * 64 * 16);
  L.wgx = o; o = align256(o + (size_t)g.T * g.FBT * g.NKS * 64 * 16);
  L.wtc = o; o = align256(o + (size_t)g.T * g.KHW * ((g.C + 15) / 16 * 16) * g.NKS * 32 * 2);
  L.wcy = o; o = align256(o + (size_t)g.T * 12 * g.NKS * 64 * 16);  // v8 grad_x operand (<= 12 blocks / tile)
  L.thi = o; o = align256(o + npar * 4);
  L.tlo = o; o = align256(o + npar * 4);
  L.mlo = o; o = align256(o + npar * 4);
  L.mhi = o; o = align256(o + npar * 4);
  L.coef = o; o = align256(o + npar * 4);
  L.alpha = o; o = align256(o + npar * 4);
  L.ckj = o; o = align256(o + 3 * 64 * 4);
  L.flags = o; o = align256(o + 16);
  // per-partial-sum state words written by the fast forward (cimq_kernels_v3.hip: StWord)
  // (v7: one uint32 per (i, m, o) -- never larger for nbw >= 2; the max covers nbw == 1)
  // state words: per-(k) words of the v3-v6 kernels, or the v7 compact words (4 B, or three
  // 64-bit planes for w8a8) per (tile, pixel, channel)
  L.st = o; o = align256(o + std::max((size_t)g.T * g.nbw * g.M * g.O * (g.NBP == 4 ? 2 : 4), (size_t)g.T * g.M * g.O * (g.NBP == 4 ? 4 : 24)));
  L.lsq_scal = o; o = align256(o + 16 * 4);
  L.total = o;
  return L;
}

Params params_of(const Geo& g, uint8_t* base) {
  CtxLayout L = ctx_layout(g);
  Params p;
  p.thi = reinterpret_cast<int*>(base + L.thi);
  p.tlo = reinterpret_cast<int*>(base + L.tlo);
  p.mlo = reinterpret_cast<int*>(base + L.mlo);
  p.mhi = reinterpret_cast<int*>(base + L.mhi);
  p.coef = reinterpret_cast<float*>(base + L.coef);
  p.alpha = reinterpret_cast<float*>(base + L.alpha);
  p.ckj = reinterpret_cast<float*>(base + L.ckj);
  p.flags = reinterpret_cast<int*>(base + L.flags);
  return p;
}

// pixel chunking of the gw / init kernel: ~1024 blocks over (chunks x tiles x 32-col groups)
void gw_chunks(const Geo& g, int* rows_per_chunk, int* nchunks) {
  const int og = (g.OB16 + 1) / 2;
  long long want = 1024 / ((long long)g.T * og);
  if (want < 1) want = 1;
  long long rows = ((g.M + want - 1) / want + 63) / 64 * 64;
  if (rows < 64) rows = 64;
  *rows_per_chunk = (int)rows;
  *nchunks = cdiv(g.M, rows);
}

const int kLsqParts = 1024;

size_t lds_tile(const Geo& g) {
  return align256((size_t)g.nba * 64 * g.KTP + 2 * sizeof(int) * g.KS * 64 + sizeof(int4) * 64);
}
size_t lds_gw(const Geo& g) {
  return lds_tile(g) + sizeof(float) * g.nbw * g.nba * 32 + sizeof(float) * g.FBT * 16 * 32 +
         (size_t)g.nba * g.KS * 64 * 64;
}
const size_t kLdsMax = 160 * 1024;

bool gx_lds_ok(const Geo& g) { return lds_tile(g) + sizeof(float) * g.C * g.HW <= kLdsMax - 1024; }

// ---- v3 fast path (whole-row 64-pixel tiles): patch geometry and LDS budgets ----
struct Plan3 {
  bool ok;
  V3 v;
  size_t lds_fwd, lds_gx, lds_gw, lds_init;
  size_t lds_gx6;  // 0: cim_bwd_gx_v6_kernel does not apply
};

inline size_t a16(size_t v) { return (v + 15) & ~(size_t)15; }

// activation-prep blocks (grid-stride over 4-element items)
static int act_blocks() { return tune("ACT_BLOCKS", 8192); }

Plan3 v3_plan(const Geo& g) {
  Plan3 p;
  memset(&p, 0, sizeof(p));
  if (tune("V3", 1) == 0) return p;  // experiments: force the general kernels
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
  const int nof = std::min(v.obm, g.OB16), nog = std::min(2, g.OB16);
  const size_t fwd_common = patch + (size_t)g.T * g.KS * 64 * 4 + ckl;
  const size_t fwd_w1 = (size_t)g.nbw * nof * g.KS * 1024 + (size_t)nkj * nof * 16 * (16 + 4);
  const size_t fwd_res = fwd_common + (size_t)g.T * fwd_w1;
  v.fwd_res = fwd_res <= 80 * 1024 ? 1 : 0;
  p.lds_fwd = v.fwd_res ? fwd_res : fwd_common + fwd_w1;
  p.lds_gx = a16((size_t)3 * (v.NPB + 1) * 32 * 2) + a16((size_t)g.KHW * v.CB * 16 * 40 * 2) + ckl + 64;
  {
    // v6: G rows at pitch 40, two W buffers of the tile's channel blocks, the band's grad_out
    // slab, two state buffers
    v.NCBT = 0;
    for (int i = 0; i < g.T; ++i) {
      const int c0 = (i * g.xbar) / g.KHW, c1 = (std::min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
      v.NCBT = std::max(v.NCBT, c1 / 16 - c0 / 16 + 1);
    }
    const size_t pq = (size_t)64 * (g.NBP == 4 ? 2 : 4);
    const size_t l6 = a16((size_t)3 * (v.NPB + 1) * 40 * 2) + 2 * a16((size_t)g.KHW * v.NCBT * 16 * 64) +
                      a16((size_t)g.O * v.NPB * 4) + 2 * a16((size_t)2 * (v.NPB / 4) * pq) + ckl + 64;
    p.lds_gx6 = (g.O % 16 == 0 && l6 <= kLdsMax - 512) ? l6 : 0;
#ifdef CIMQ_GX_V5
    p.lds_gx6 = 0;
#endif
  }
  v.NCG = 0;
  for (int i = 0; i < g.T; ++i) {
    const int c0 = (i * g.xbar) / g.KHW, c1 = (std::min(g.K, (i + 1) * g.xbar) - 1) / g.KHW;
    v.NCG = std::max(v.NCG, c1 - c0 + 1);
  }
  const size_t pg = a16((size_t)v.NCG * v.RH * v.WP * g.NBP);
  const size_t gw_tail = (size_t)g.KS * 64 * 4 + (size_t)g.nbw * nog * g.KS * 1024 + (size_t)nkj * nog * 16 * 16 +
                         a16((size_t)nkj * 32 * 4 * 4) + ckl;  // init: per-wave |u| rows
  p.lds_gw = std::max(a16(2 * (size_t)v.NCG * v.RH * v.WP * g.NBP), (size_t)g.FBT * 16 * 32 * 4) + 128 * 4 +
             a16((size_t)nkj * 16 * 4) + ckl;
  p.lds_init = pg + gw_tail;
  const size_t lim = kLdsMax - 512;
  p.ok = p.lds_fwd <= lim && p.lds_gx <= lim && p.lds_gw <= lim;
  return p;
}

// ---- v7 backward (compact state words, unfolded grad_x, conv-style grad_w) ----
struct Plan7 {
  bool ok;
  V7 v;
  size_t lds_gx, lds_gw;
  int pairs;
};

Plan7 v7_plan(const Geo& g) {
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
  if (g.NBP == 8 && !(g.nbw == 8 && g.nba == 8 && g.OB16 == 1)) return p;
  if (g.O % 16 != 0 || !(g.OB16 == 1 || g.OB16 == 2 || g.OB16 == 4)) return p;
  // 3x3, stride 1, pad 1 ("same" conv: every CiM conv of the CIFAR ResNets but the downsampling ones)
  if (g.KH != 3 || g.KW != 3 || g.SH != g.SW || g.SH > 2 || g.PH != 1 || g.PW != 1) return p;
  if (g.Wo % 8 != 0 || (g.Wo & (g.Wo - 1)) != 0 || g.Wo > 64 || g.M % 128 != 0 || g.FBT > 8) return p;
  V7& v = p.v;
  if (g.P % 128 == 0) v.whole = 0;
  else if (128 % g.P == 0) v.whole = 1;
  else return p;
  v.lw = p3.v.lw;
  v.RB = std::min(g.H, tune("GX_RB", 8));
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
  p.lds_gx = a16((size_t)v.RSLOT * v.NSEG * g.C * 3 * (g.SH * v.SWD + 2) * 4) + 64 * 4 + 64;
  // grad_w
  v.NSLOT = v.whole ? (128 / g.P) * g.H : ((128 / g.Wo) - 1) * g.SH + g.KH;
  v.CPITCH = v.NSLOT * g.Wo + 8;
  v.CPL = std::min(16, g.C);
  // tiles touching one channel block (the kernel's loop takes at most 3)
  v.NTL = 1;
  for (int cb = 0; cb * 16 < g.C; ++cb) {
    const int ilo = (cb * 16 * g.KHW) / g.xbar, ihi = (std::min(g.C, cb * 16 + 16) * g.KHW - 1) / g.xbar;
    v.NTL = std::max(v.NTL, ihi - ilo + 1);
  }
  if (v.NTL > 3) return p;
  const size_t planes = (size_t)g.nba * g.KW * v.CPL * v.CPITCH * 2;
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

struct WsLayout {
  size_t gw_slab, ga_slab, lsq_part, gaq, wpart, bpo, total;
  int rows, nchunks, nchunks_bwd;
};

WsLayout ws_layout(const Geo& g) {
  WsLayout W;
  gw_chunks(g, &W.rows, &W.nchunks);
  // backward slabs: the v7 grad_w kernel's pixel chunks when it applies (the alpha_cim init
  // kernel keeps gw_chunks' split: W.nchunks / W.rows)
  const Plan7 p7 = v7_plan(g);
  W.nchunks_bwd = p7.ok ? p7.v.nchunks : W.nchunks;
  const size_t nch = (size_t)std::max(W.nchunks, W.nchunks_bwd);
  size_t o = 0;
  W.gw_slab = o; o = align256(o + sizeof(float) * nch * g.T * g.FBT * 16 * g.Opad);
  W.ga_slab = o; o = align256(o + sizeof(float) * nch * g.T * g.nbw * g.nba * g.Opad);
  W.lsq_part = o; o = align256(o + sizeof(float) * std::max(kLsqParts, g.B * g.H));  // >= B * bands
  // module entry points: d loss / d alpha_q, weight-LSQ partials of the grad_w reducer, and
  // a [B, P, O] staging copy of out / grad_out for the general kernels
  W.gaq = o; o = align256(o + sizeof(float) * (size_t)g.T * g.nbw * g.nba * g.O);
  W.wpart = o; o = align256(o + sizeof(float) * 2 * (size_t)cdiv((long long)g.T * g.FBT * 16 * g.Opad, 64));
  W.bpo = o; o = align256(o + sizeof(float) * (size_t)g.M * g.O);
  W.total = o;
  return W;
}

template <typename K>
int set_lds(K kernel, size_t bytes) {
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
enum KernelId {
  KID_NONE = 0, KID_FWD = 1, KID_BWD_GX = 2, KID_BWD_GW = 3, KID_PREP_ACT = 4,
  KID_FWD_V7 = 5, KID_GX_V8 = 6, KID_GW_V7 = 7, KID_LAST = 7
};

struct Profiler {
  std::mutex mu;
  int kid = KID_NONE;
  int cap = 0, n = 0;
  hipEvent_t* ev = nullptr;  // 2*cap
  double bytes = 0, flops = 0;
};
Profiler& prof() {
  static Profiler p;
  return p;
}

void algo_counts(const Geo& g, int kid, double* bytes, double* flops) {
  const double x4 = 4.0 * (double)g.Nin, y4 = 4.0 * (double)g.M * g.O;
  const double mac = (double)g.M * g.O * g.K;
  switch (kid) {
    case KID_FWD_V7:
    case KID_FWD: *bytes = x4 + y4; *flops = 2.0 * mac; break;             // read x, write y
    case KID_GX_V8:
    case KID_BWD_GX: *bytes = 2.0 * x4 + y4; *flops = 2.0 * mac * g.nbw; break;  // read gy, x; write gx
    case KID_GW_V7:
    case KID_BWD_GW: *bytes = x4 + y4; *flops = 2.0 * mac * g.nba; break;  // read gy, x
    case KID_PREP_ACT: *bytes = x4 + (double)g.Nin * (g.NBP + 1); *flops = 0; break;
    default: *bytes = 0; *flops = 0;
  }
}

// returns the event slot to close after the launch (-1: not profiling this kernel)
int prof_begin(int kid, const Geo& g, hipStream_t s) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.n >= p.cap) return -1;
  const int role = kid == KID_FWD_V7 ? KID_FWD : kid == KID_GX_V8 ? KID_BWD_GX : kid == KID_GW_V7 ? KID_BWD_GW : kid;
  if (p.kid != kid && p.kid != role) return -1;
  const int slot = p.n++;
  double b, f;
  algo_counts(g, kid, &b, &f);
  p.bytes += b;
  p.flops += f;
  (void)hipEventRecord(p.ev[2 * slot], s);
  return slot;
}
void prof_end(int slot, hipStream_t s) {
  if (slot < 0) return;
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  (void)hipEventRecord(p.ev[2 * slot + 1], s);
}

int prep_all(const Geo& g, const float* x, const float* w_q, const float* sa, const float* sw,
             const float* alpha_q, const int8_t* bmask, const float* signed_act, uint8_t* ctx,
             hipStream_t s, bool need_params, bool need_wgx) {
  CtxLayout L = ctx_layout(g);
  const int blk = 256;
  {
    // one 4-element item per thread up to 8192 blocks (fewer, fatter blocks measured slower)
    int grid = cdiv(g.Nin, 4 * blk);
    if (grid > act_blocks()) grid = act_blocks();
    const int slot = prof_begin(KID_PREP_ACT, g, s);
    hipLaunchKernelGGL(prep_act_kernel, dim3(grid), dim3(blk), 0, s, g, x, sa, signed_act,
                       ctx + L.xcode, ctx + L.xhat);
    prof_end(slot, s);
    CIMQ_TRY(check_hip("prep_act"));
  }
  {
    int total = g.T * g.KS * g.NBLK * 64;
    hipLaunchKernelGGL(prep_wfrag_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, w_q, sw,
                       reinterpret_cast<v4i*>(ctx + L.wfrag));
    CIMQ_TRY(check_hip("prep_wfrag"));
  }
  if (need_wgx) {
    int total = g.T * g.FBT * g.NKS * 64;
    hipLaunchKernelGGL(prep_wgx_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, w_q, sw,
                       reinterpret_cast<v4i*>(ctx + L.wgx));
    const int Cp = (g.C + 15) / 16 * 16;
    const int tw = g.T * g.KHW * Cp * g.NKS * 4;
    hipLaunchKernelGGL(prep_wtc_kernel, dim3(cdiv(tw, blk)), dim3(blk), 0, s, g, w_q, sw, Cp,
                       reinterpret_cast<uint4*>(ctx + L.wtc));
    CIMQ_TRY(check_hip("prep_wgx"));
    const Plan7 p7 = v7_plan(g);
    if (p7.ok) {
      const int tc = g.T * p7.v.NCPBT * g.NKS * 64;
      hipLaunchKernelGGL(prep_wcy_kernel, dim3(cdiv(tc, blk)), dim3(blk), 0, s, g, w_q, sw, p7.v.NCPBT,
                         reinterpret_cast<v4i*>(ctx + L.wcy));
      CIMQ_TRY(check_hip("prep_wcy"));
    }
  }
  Params pp = params_of(g, ctx);
  if (need_params) {
    if (hipMemsetAsync(pp.flags, 0, 16, s) != hipSuccess) return fail(CIMQ_EHIP, "memset flags");
    int total = g.T * g.nba * g.nbw * g.Opad + g.nbw * g.nba;
    hipLaunchKernelGGL(prep_params_kernel, dim3(cdiv(total, blk)), dim3(blk), 0, s, g, alpha_q, sw, sa,
                       bmask, pp);
    CIMQ_TRY(check_hip("prep_params"));
  }
  return CIMQ_OK;
}

template <int NBP, int KS>
int launch_fwd_v3(const Geo& g, const Plan3& p, uint8_t* ctx, const float* sw, const float* sa, float* out,
                  hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  // compact state words when the v7 backward will read them
  const bool cst = v7_plan(g).ok;
  // OBM: 16-channel output blocks per block (register arrays sized for exactly that)
  const int obm = std::min(p.v.obm, g.OB16 <= 2 ? g.OB16 : 4);
  // CST: compact state words with nbw = nba = CST fixed at compile time (v7_plan's slice pairs)
  void (*kern)(Geo, V3, const uint8_t*, const v4i*, Params, const float*, const float*, float*, uint8_t*);
  if (!cst) {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 0, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 0, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 0, 4>;
  } else if constexpr (NBP == 8) {
    kern = cim_fwd_v3_kernel<8, KS, 8, 1>;  // v7_plan: w8a8 with one 16-channel block
  } else if (g.nbw == 2) {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 2, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 2, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 2, 4>;
  } else {
    kern = obm == 1 ? cim_fwd_v3_kernel<NBP, KS, 3, 1> : obm == 2 ? cim_fwd_v3_kernel<NBP, KS, 3, 2>
                                                       : cim_fwd_v3_kernel<NBP, KS, 3, 4>;
  }
  CIMQ_TRY(set_lds(kern, p.lds_fwd));
  // grid: about three resident 256-thread blocks per CU (measured: 768 blocks for w3a3, 1024
  // for the 236-VGPR w8a8 instance)
  dim3 grid(std::min(p.v.nmt, tune("FWD_GRID", NBP == 8 ? 1024 : 768)), cdiv(g.OB16, obm));
  const int slot = prof_begin(cst ? KID_FWD_V7 : KID_FWD, g, s);
  hipLaunchKernelGGL(kern, grid, dim3(256), p.lds_fwd, s, g, p.v, ctx + L.xcode,
                     reinterpret_cast<const v4i*>(ctx + L.wfrag), params_of(g, ctx), sw, sa, out, ctx + L.st);
  prof_end(slot, s);
  return check_hip("cim_fwd_v3");
}

template <int NBP, bool DBG>
int launch_fwd(const Geo& g, uint8_t* ctx, const float* sw, const float* sa, float* out, int* ps_dbg,
               float* adc_dbg, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  const Plan3 p = v3_plan(g);
  if (p.ok && !DBG) {
    if (g.KS == 1) return launch_fwd_v3<NBP, 1>(g, p, ctx, sw, sa, out, s);
    return launch_fwd_v3<NBP, 2>(g, p, ctx, sw, sa, out, s);
  }
  if (p.ok) {
    // the debug forward is the general kernel; the fast one still fills the state words the
    // fast backward reads (same out values)
    if (g.KS == 1) CIMQ_TRY((launch_fwd_v3<NBP, 1>(g, p, ctx, sw, sa, out, s)));
    else CIMQ_TRY((launch_fwd_v3<NBP, 2>(g, p, ctx, sw, sa, out, s)));
  }
  dim3 grid(cdiv(g.M, 64), cdiv(g.OB16, 4));
  const size_t lds = lds_tile(g);
  auto kern = cim_fwd_kernel<NBP, DBG>;
  CIMQ_TRY(set_lds(kern, lds));
  const int slot = DBG ? -1 : prof_begin(KID_FWD, g, s);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, reinterpret_cast<const int8_t*>(ctx + L.xcode),
                     reinterpret_cast<const v4i*>(ctx + L.wfrag), params_of(g, ctx), sw, sa, out, ps_dbg,
                     adc_dbg);
  prof_end(slot, s);
  return check_hip("cim_fwd");
}

template <int NBP, int FBMAX, bool INIT>
int launch_gw(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
              const float* gout, uint8_t* ws, hipStream_t s) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const Plan3 p = v3_plan(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  dim3 grid(W.nchunks, g.T, (g.OB16 + 1) / 2);
  const int slot = INIT ? -1 : prof_begin(KID_BWD_GW, g, s);
  if (p.ok && !INIT) {
    auto kern = g.nbw <= 4 ? cim_bwd_gw_v5_kernel<NBP, FBMAX, 4> : cim_bwd_gw_v5_kernel<NBP, FBMAX, 8>;
    CIMQ_TRY(set_lds(kern, p.lds_gw));
    dim3 grid16(W.nchunks, g.T, g.OB16);
    hipLaunchKernelGGL(kern, grid16, dim3(256), p.lds_gw, s, g, p.v, ctx + L.st, ctx + L.xhat, pp, gout, W.rows,
                       reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
    prof_end(slot, s);
    return check_hip("cim_bwd_gw_v5");
  }
  if constexpr (INIT) {
    // alpha_cim init sums (the v3 kernel runs only in this mode)
    if (p.ok && p.lds_init <= kLdsMax - 512) {
      const size_t lds = p.lds_init;
      auto kern = g.KS == 1 ? cim_bwd_gw_v3_kernel<NBP, 1, FBMAX, true> : cim_bwd_gw_v3_kernel<NBP, 2, FBMAX, true>;
      CIMQ_TRY(set_lds(kern, lds));
      hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, p.v, ctx + L.xcode, ctx + L.xhat,
                         reinterpret_cast<const v4i*>(ctx + L.wfrag), pp, sw, sa, gout, W.rows,
                         reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
      return check_hip("cim_bwd_gw_v3(init)");
    }
  }
  {
    const size_t lds = lds_gw(g);
    auto kern = cim_bwd_gw_kernel<NBP, FBMAX, INIT>;
    CIMQ_TRY(set_lds(kern, lds));
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, reinterpret_cast<const int8_t*>(ctx + L.xcode),
                       reinterpret_cast<const int8_t*>(ctx + L.xhat), reinterpret_cast<const v4i*>(ctx + L.wfrag),
                       pp, sw, sa, signed_act, gout, W.rows, reinterpret_cast<float*>(ws + W.gw_slab),
                       reinterpret_cast<float*>(ws + W.ga_slab));
  }
  prof_end(slot, s);
  return check_hip("cim_bwd_gw");
}

// grad_x; returns through *lsq_fused whether the LSQ activation backward was applied
template <int NBP, int FBMAX>
int launch_gx(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* gout,
              const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const Plan3 p = v3_plan(g);
  const v4i* wf = reinterpret_cast<const v4i*>(ctx + L.wfrag);
  const v4i* wg = reinterpret_cast<const v4i*>(ctx + L.wgx);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  *lsq_fused = false;
  if (p.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    float* part = reinterpret_cast<float*>(ws + W.lsq_part);
    dim3 grid(g.B * p.v.nbands);
    const bool two = p.v.NT <= 16;
    if (p.lds_gx6) {
      auto kern = two ? (lsq ? cim_bwd_gx_v6_kernel<NBP, 2, true> : cim_bwd_gx_v6_kernel<NBP, 2, false>)
                      : (lsq ? cim_bwd_gx_v6_kernel<NBP, 4, true> : cim_bwd_gx_v6_kernel<NBP, 4, false>);
      CIMQ_TRY(set_lds(kern, p.lds_gx6));
      const int slot = prof_begin(KID_BWD_GX, g, s);
      hipLaunchKernelGGL(kern, grid, dim3(512), p.lds_gx6, s, g, p.v, ctx + L.st,
                         reinterpret_cast<const uint4*>(ctx + L.wtc), pp, sw, sa, gout, x, gx, part);
      prof_end(slot, s);
      *lsq_fused = lsq;
      return check_hip("cim_bwd_gx_v6");
    }
    auto kern = two ? (lsq ? cim_bwd_gx_v5_kernel<NBP, 2, true> : cim_bwd_gx_v5_kernel<NBP, 2, false>)
                    : (lsq ? cim_bwd_gx_v5_kernel<NBP, 4, true> : cim_bwd_gx_v5_kernel<NBP, 4, false>);
    CIMQ_TRY(set_lds(kern, p.lds_gx));
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL(kern, grid, dim3(512), p.lds_gx, s, g, p.v, ctx + L.st,
                       reinterpret_cast<const uint4*>(ctx + L.wtc), pp, sw, sa, gout, x, gx, part);
    prof_end(slot, s);
    *lsq_fused = lsq;
    return check_hip("cim_bwd_gx_v5");
  }
  const int8_t* xc = reinterpret_cast<const int8_t*>(ctx + L.xcode);
  if (gx_lds_ok(g)) {
    const size_t lds = lds_tile(g) + sizeof(float) * g.C * g.HW;
    auto kern = cim_bwd_gx_kernel<NBP, FBMAX, true>;
    CIMQ_TRY(set_lds(kern, lds));
    const int slot = prof_begin(KID_BWD_GX, g, s);
    hipLaunchKernelGGL(kern, dim3(g.B), dim3(256), lds, s, g, xc, wf, wg, pp, sw, sa, gout, gx);
    prof_end(slot, s);
    return check_hip("cim_bwd_gx(lds)");
  }
  if (hipMemsetAsync(gx, 0, sizeof(float) * g.Nin, s) != hipSuccess) return fail(CIMQ_EHIP, "memset gx");
  const size_t lds = lds_tile(g);
  auto kern = cim_bwd_gx_kernel<NBP, FBMAX, false>;
  CIMQ_TRY(set_lds(kern, lds));
  const int slot = prof_begin(KID_BWD_GX, g, s);
  hipLaunchKernelGGL(kern, dim3(cdiv(g.M, 64)), dim3(256), lds, s, g, xc, wf, wg, pp, sw, sa, gout, gx);
  prof_end(slot, s);
  CIMQ_TRY(check_hip("cim_bwd_gx(global)"));
  int grid = cdiv(g.Nin, 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(scale_kernel, dim3(grid), dim3(256), 0, s, gx, g.Nin, sw, g.nba);
  return check_hip("scale");
}

template <int NBW, int NBA, int OBX>
int launch_v7_nb(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa,
                 const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  Params pp = params_of(g, const_cast<uint8_t*>(ctx));
  const uint32_t* st = reinterpret_cast<const uint32_t*>(ctx + L.st);
  {
    const int np = p.v.NPART;
#define CIMQ_GX8(L, S, N) cim_bwd_gx_v8_kernel<NBW, NBA, OBX, L, S, N>
#define CIMQ_GX8N(L, S) (np == 1 ? CIMQ_GX8(L, S, 1) : np == 2 ? CIMQ_GX8(L, S, 2) : CIMQ_GX8(L, S, 4))
    auto kern = g.SH == 1 ? (lsq ? CIMQ_GX8N(true, 1) : CIMQ_GX8N(false, 1)) : (lsq ? CIMQ_GX8N(true, 2) : CIMQ_GX8N(false, 2));
#undef CIMQ_GX8N
#undef CIMQ_GX8
    CIMQ_TRY(set_lds(kern, p.lds_gx));
    const int slot = prof_begin(KID_GX_V8, g, s);
    hipLaunchKernelGGL(kern, dim3(g.B * p.v.nbands), dim3(256 * np), p.lds_gx, s, g, p.v, st,
                       reinterpret_cast<const v4i*>(ctx + L.wcy), pp, sw, sa, gout, x, gx,
                       reinterpret_cast<float*>(ws + W.lsq_part));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("cim_bwd_gx_v8"));
  }
  {
    auto kern = g.SH == 1 ? cim_bwd_gw_v7_kernel<NBW, NBA, 1> : cim_bwd_gw_v7_kernel<NBW, NBA, 2>;
    CIMQ_TRY(set_lds(kern, p.lds_gw));
    const int slot = prof_begin(KID_GW_V7, g, s);
    hipLaunchKernelGGL(kern, dim3(p.v.nchunks, p.pairs), dim3(256), p.lds_gw, s, g, p.v, st, ctx + L.xhat, pp,
                       gout, reinterpret_cast<float*>(ws + W.gw_slab), reinterpret_cast<float*>(ws + W.ga_slab));
    prof_end(slot, s);
    CIMQ_TRY(check_hip("cim_bwd_gw_v7"));
  }
  return CIMQ_OK;
}

template <int NBW, int NBA>
int launch_v7_n(const Geo& g, const Plan7& p, const uint8_t* ctx, const float* sw, const float* sa,
                const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool lsq) {
  if constexpr (NBW * NBA > 10) {
    return launch_v7_nb<NBW, NBA, 1>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);  // v7_plan: OB16 == 1
  } else {
    if (g.OB16 == 1) return launch_v7_nb<NBW, NBA, 1>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
    if (g.OB16 == 2) return launch_v7_nb<NBW, NBA, 2>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
    return launch_v7_nb<NBW, NBA, 4>(g, p, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  }
}

template <int NBP, int FBMAX>
int launch_bwd_all(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                   const float* signed_act, const float* gout, const float* x, float* gx, uint8_t* ws,
                   hipStream_t s, bool* lsq_fused) {
  const Plan7 p7 = v7_plan(g);
  if (p7.ok) {
    const bool lsq = g.input_kind == CIMQ_INPUT_RAW_LSQ;
    *lsq_fused = lsq;
    if (NBP == 8) return launch_v7_n<8, 8>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq);
    if (g.nbw == 2) return launch_v7_n<2, 2>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq);
    return launch_v7_n<3, 3>(g, p7, ctx, sw, sa, gout, x, gx, ws, s, lsq);
  }
  CIMQ_TRY((launch_gx<NBP, FBMAX>(g, ctx, sw, sa, gout, x, gx, ws, s, lsq_fused)));
  CIMQ_TRY((launch_gw<NBP, FBMAX, false>(g, ctx, sw, sa, signed_act, gout, ws, s)));
  return CIMQ_OK;
}

template <int NBP>
int dispatch_bwd(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa, const float* signed_act,
                 const float* gout, const float* x, float* gx, uint8_t* ws, hipStream_t s, bool* lsq_fused) {
  if (g.FBT <= 4) return launch_bwd_all<NBP, 4>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
  return launch_bwd_all<NBP, 8>(g, ctx, sw, sa, signed_act, gout, x, gx, ws, s, lsq_fused);
}

template <int NBP>
int dispatch_init(const Geo& g, const uint8_t* ctx, const float* sw, const float* sa,
                  const float* signed_act, uint8_t* ws, hipStream_t s) {
  if (g.FBT <= 4) return launch_gw<NBP, 4, true>(g, ctx, sw, sa, signed_act, nullptr, ws, s);
  return launch_gw<NBP, 8, true>(g, ctx, sw, sa, signed_act, nullptr, ws, s);
}

int launch_reduce_galpha(const Geo& g, const uint8_t* ctx, uint8_t* ws, float cgrad, int init, const float* sw,
                         const float* sa, float* out, hipStream_t s) {
  WsLayout W = ws_layout(g);
  const long long nout = (long long)g.T * g.nbw * g.nba * g.Opad;
  hipLaunchKernelGGL(reduce_galpha_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, init ? W.nchunks : W.nchunks_bwd,
                     reinterpret_cast<const float*>(ws + W.ga_slab), params_of(g, const_cast<uint8_t*>(ctx)),
                     cgrad, init, sw, sa, (float)((double)g.B * g.P), (float)sqrt((double)g.qp), out);
  return check_hip("reduce_galpha");
}

}  // namespace

extern "C" {

int cimq_abi_version(void) { return CIMQ_ABI_VERSION; }

const char* cimq_last_error(void) { return g_last_error.c_str(); }

int cimq_query_sizes(const cimq_conv_desc* d, cimq_sizes* out) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!out) return fail(CIMQ_EINVAL, "null output");
  out->ctx_bytes = ctx_layout(g).total;
  WsLayout W = ws_layout(g);
  out->fwd_workspace_bytes = W.total;
  out->bwd_workspace_bytes = W.total;
  return CIMQ_OK;
}

int cimq_forward(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                 const float* sw, const float* alpha_q, const int8_t* binary_mask,
                 const float* signed_act, float* out, void* ctx, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !out || !ctx)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && !alpha_q)
    return fail(CIMQ_EINVAL, "adc_bits 1 / 1.5 need alpha_q");
  (void)ws;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, alpha_q, binary_mask, signed_act, c, s, true, true));
  if (g.NBP == 4) return launch_fwd<4, false>(g, c, sw, sa, out, nullptr, nullptr, s);
  return launch_fwd<8, false>(g, c, sw, sa, out, nullptr, nullptr, s);
}

int cimq_debug_partial_sums(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                            const float* sw, const float* alpha_q, const int8_t* binary_mask,
                            const float* signed_act, float* out, int32_t* ps_out, float* adc_out, void* ctx,
                            void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !out || !ps_out || !adc_out || !ctx)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && !alpha_q)
    return fail(CIMQ_EINVAL, "adc_bits 1 / 1.5 need alpha_q");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, alpha_q, binary_mask, signed_act, c, s, true, true));
  if (g.NBP == 4) return launch_fwd<4, true>(g, c, sw, sa, out, ps_out, adc_out, s);
  return launch_fwd<8, true>(g, c, sw, sa, out, ps_out, adc_out, s);
}

int cimq_backward(const cimq_conv_desc* d, const float* grad_out, const float* x, const float* sa,
                  const float* sw, const float* alpha_q, const int8_t* binary_mask,
                  const float* signed_act, const void* ctx, float* grad_x, float* grad_w,
                  float* grad_alpha, float* grad_sa, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  (void)alpha_q; (void)binary_mask;
  if (!grad_out || !sa || !sw || !signed_act || !ctx || !grad_x || !grad_w || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ && (!x || !grad_sa))
    return fail(CIMQ_EINVAL, "RAW_LSQ backward needs x and grad_sa");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  bool lsq_fused = false;
  if (g.NBP == 4) CIMQ_TRY(dispatch_bwd<4>(g, c, sw, sa, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
  else CIMQ_TRY(dispatch_bwd<8>(g, c, sw, sa, signed_act, grad_out, x, grad_x, w, s, &lsq_fused));
  WsLayout W = ws_layout(g);
  {
    const long long nout = (long long)g.T * g.FBT * 16 * g.Opad;
    hipLaunchKernelGGL(reduce_gw_v3_kernel, dim3(cdiv(nout, 64)), dim3(1024), 0, s, g, W.nchunks_bwd,
                       reinterpret_cast<const float*>(w + W.gw_slab), sa, grad_w);
    CIMQ_TRY(check_hip("reduce_gw"));
  }
  if ((g.mode == ADC_SIGN || g.mode == ADC_TERNARY) && grad_alpha) {
    const double numel = (double)g.B * g.T * g.nbw * g.nba * g.P * g.O;
    const float cgrad = (float)(1.0 / sqrt(numel * (double)g.qp));  // lsq.py:323,330
    CIMQ_TRY(launch_reduce_galpha(g, c, w, cgrad, 0, sw, sa, grad_alpha, s));
  }
  if (g.input_kind == CIMQ_INPUT_RAW_LSQ) {
    float* part = reinterpret_cast<float*>(w + W.lsq_part);
    int nparts;
    if (lsq_fused) {
      const Plan7 p7 = v7_plan(g);
      nparts = g.B * (p7.ok ? p7.v.nbands : v3_plan(g).v.nbands);
    } else {
      int grid = cdiv(g.Nin, 256);
      if (grid > kLsqParts) grid = kLsqParts;
      hipLaunchKernelGGL(lsq_act_bwd_kernel, dim3(grid), dim3(256), 0, s, g.Nin, x, sa, g.lsq_qp, grad_x, part);
      CIMQ_TRY(check_hip("lsq_act_bwd"));
      nparts = grid;
    }
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, nparts, part, grad_sa);
    CIMQ_TRY(check_hip("sum_partials"));
  }
  return CIMQ_OK;
}

static int lsq_args(const Geo& g, const cimq_lsq_desc* q, LsqArgs* a) {
  if (!q) return fail(CIMQ_EINVAL, "null LSQ descriptor");
  if (!(q->qn_w < q->qp_w) || !(q->gscale_a > 0.f) || !(q->gscale_w > 0.f))
    return fail(CIMQ_EINVAL, "bad LSQ descriptor");
  if (q->nbits_alpha < 0 || q->nbits_alpha > 16 || q->nbits_alpha == 1)
    return fail(CIMQ_EINVAL, "nbits_alpha must be 0 (no alpha_cim) or 2..16");
  a->qn_w = q->qn_w;
  a->qp_w = q->qp_w;
  a->gs_a = q->gscale_a;
  a->gs_w = q->gscale_w;
  a->nbits_alpha = q->nbits_alpha;
  a->nalpha = g.T * g.nbw * g.nba * g.O;
  if (q->flags & ~CIMQ_LSQ_ACCUMULATE_GRADS) return fail(CIMQ_EINVAL, "unknown LSQ flags 0x%x", q->flags);
  return CIMQ_OK;
}

int cimq_module_forward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* x, const float* weight,
                        const float* alpha_act, const float* alpha_weight, const float* alpha_cim,
                        const int8_t* binary_mask, const float* signed_act, float* out, void* ctx, void* ws,
                        void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (g.input_kind != CIMQ_INPUT_RAW_LSQ) return fail(CIMQ_EINVAL, "module entry points take the raw activation");
  LsqArgs la;
  CIMQ_TRY(lsq_args(g, q, &la));
  if (!x || !weight || !alpha_act || !alpha_weight || !binary_mask || !signed_act || !out || !ctx || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || la.nbits_alpha == 0)) return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  CtxLayout L = ctx_layout(g);
  float* scal = reinterpret_cast<float*>(c + L.lsq_scal);
  {
    const bool fast = v3_plan(g).ok;
    ModulePrep a;
    a.x = x;
    a.alpha_act = alpha_act;
    a.alpha_w = alpha_weight;
    a.weight = weight;
    a.alpha_cim = has_alpha ? alpha_cim : nullptr;
    a.signed_act = signed_act;
    a.bmask = binary_mask;
    a.xcf = c + L.xcode;
    a.xcb = c + L.xhat;
    a.wfrag = reinterpret_cast<v4i*>(c + L.wfrag);
    a.wgx = reinterpret_cast<v4i*>(c + L.wgx);
    a.wtc = reinterpret_cast<uint4*>(c + L.wtc);
    a.Cp = (g.C + 15) / 16 * 16;
    a.pp = params_of(g, c);
    a.scal = scal;
    a.nact_blocks = (int)std::min<long long>(cdiv(g.Nin, 4 * 256), act_blocks());
    a.nwf = g.T * g.KS * g.NBLK * 64;
    const Plan7 p7 = v7_plan(g);
    a.nwg = fast ? 0 : g.T * g.FBT * g.NKS * 64;                   // general grad_x operand
    a.nwt = (fast && !p7.ok) ? g.T * g.KHW * a.Cp * g.NKS * 4 : 0;  // v5 / v6 grad_x operand
    a.wcy = reinterpret_cast<v4i*>(c + L.wcy);
    a.ncpbt = p7.ok ? p7.v.NCPBT : 1;
    a.nwc = p7.ok ? g.T * p7.v.NCPBT * g.NKS * 64 : 0;              // v8 grad_x operand
    a.npp = g.T * g.nba * g.nbw * g.Opad + g.nbw * g.nba;
    const int nwblk = std::max(1, std::min(cdiv(a.nwf + a.nwg + a.nwt + a.nwc + a.npp, 256), 1024));
    const int slot = prof_begin(KID_PREP_ACT, g, s);
    hipLaunchKernelGGL(prep_module_kernel, dim3(a.nact_blocks + nwblk), dim3(256), 0, s, g, la, a);
    prof_end(slot, s);
    CIMQ_TRY(check_hip("prep_module"));
  }
  const Plan3 p = v3_plan(g);
  if (p.ok) {
    g.onchw = 1;
    if (g.NBP == 4) return launch_fwd<4, false>(g, c, scal + 1, scal, out, nullptr, nullptr, s);
    return launch_fwd<8, false>(g, c, scal + 1, scal, out, nullptr, nullptr, s);
  }
  // general kernels write [B, P, O]; the module returns NCHW
  WsLayout W = ws_layout(g);
  float* bpo = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) + W.bpo);
  if (g.NBP == 4) CIMQ_TRY((launch_fwd<4, false>(g, c, scal + 1, scal, bpo, nullptr, nullptr, s)));
  else CIMQ_TRY((launch_fwd<8, false>(g, c, scal + 1, scal, bpo, nullptr, nullptr, s)));
  hipLaunchKernelGGL(bpo_to_nchw_kernel, dim3(std::min(cdiv((long long)g.M * g.O, 256), 8192)), dim3(256), 0, s,
                     g, bpo, out);
  return check_hip("bpo_to_nchw");
}

int cimq_module_backward(const cimq_conv_desc* d, const cimq_lsq_desc* q, const float* grad_out, const float* x,
                         const float* weight, const float* alpha_act, const float* alpha_weight,
                         const float* alpha_cim, const int8_t* binary_mask, const float* signed_act,
                         const void* ctx, float* grad_x, float* grad_weight, float* grad_alpha_act,
                         float* grad_alpha_weight, float* grad_alpha_cim, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (g.input_kind != CIMQ_INPUT_RAW_LSQ) return fail(CIMQ_EINVAL, "module entry points take the raw activation");
  LsqArgs la;
  CIMQ_TRY(lsq_args(g, q, &la));
  (void)alpha_act; (void)alpha_weight; (void)binary_mask;
  if (!grad_out || !x || !weight || !signed_act || !ctx || !grad_x || !grad_weight || !grad_alpha_act ||
      !grad_alpha_weight || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  const bool has_alpha = g.mode == ADC_SIGN || g.mode == ADC_TERNARY;
  if (has_alpha && (!alpha_cim || !grad_alpha_cim || la.nbits_alpha == 0))
    return fail(CIMQ_EINVAL, "adc 1 / 1.5 need alpha_cim and grad_alpha_cim");
  if (!has_alpha) la.nbits_alpha = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  CtxLayout L = ctx_layout(g);
  WsLayout W = ws_layout(g);
  const float* scal = reinterpret_cast<const float*>(c + L.lsq_scal);
  const float* sa = scal;
  const float* sw = scal + 1;
  const Plan3 p = v3_plan(g);
  const float* gsrc = grad_out;
  if (p.ok) {
    g.onchw = 1;
  } else {
    float* bpo = reinterpret_cast<float*>(w + W.bpo);
    hipLaunchKernelGGL(nchw_to_bpo_kernel, dim3(std::min(cdiv((long long)g.M * g.O, 256), 8192)), dim3(256), 0, s,
                       g, grad_out, bpo);
    CIMQ_TRY(check_hip("nchw_to_bpo"));
    gsrc = bpo;
  }
  bool lsq_fused = false;
  if (g.NBP == 4) CIMQ_TRY(dispatch_bwd<4>(g, c, sw, sa, signed_act, gsrc, x, grad_x, w, s, &lsq_fused));
  else CIMQ_TRY(dispatch_bwd<8>(g, c, sw, sa, signed_act, gsrc, x, grad_x, w, s, &lsq_fused));
  // the act-LSQ partials: fused into the fast grad_x kernel, a separate pass otherwise
  float* part = reinterpret_cast<float*>(w + W.lsq_part);
  int nparts;
  if (lsq_fused) {
    const Plan7 p7 = v7_plan(g);
    nparts = g.B * (p7.ok ? p7.v.nbands : p.v.nbands);
  } else {
    int grid = cdiv(g.Nin, 256);
    if (grid > kLsqParts) grid = kLsqParts;
    hipLaunchKernelGGL(lsq_act_bwd_kernel, dim3(grid), dim3(256), 0, s, g.Nin, x, sa, g.lsq_qp, grad_x, part);
    CIMQ_TRY(check_hip("lsq_act_bwd"));
    nparts = grid;
  }
  // one epilogue launch: grad_w + weight-LSQ backward, grad_alpha_cim, the step-size grads
  ModuleTail a;
  a.gw_slab = reinterpret_cast<const float*>(w + W.gw_slab);
  a.ga_slab = reinterpret_cast<const float*>(w + W.ga_slab);
  a.scal = scal;
  a.weight = weight;
  a.alpha_cim = alpha_cim;
  a.apart = part;
  a.wpart = reinterpret_cast<float*>(w + W.wpart);
  a.gaq = reinterpret_cast<float*>(w + W.gaq);
  a.grad_weight = grad_weight;
  a.grad_alpha_act = grad_alpha_act;
  a.grad_alpha_w = grad_alpha_weight;
  a.grad_alpha_cim = grad_alpha_cim;
  a.pp = params_of(g, const_cast<uint8_t*>(c));
  a.cgrad = (float)(1.0 / sqrt((double)g.B * g.T * g.nbw * g.nba * g.P * g.O * (double)g.qp));  // lsq.py:323,330
  a.nchunks = W.nchunks_bwd;
  a.nwb = cdiv((long long)g.T * g.FBT * 16 * g.Opad, 64);
  a.nga = has_alpha ? cdiv((long long)g.T * g.nbw * g.nba * g.Opad, 64) : 0;
  a.napart = nparts;
  a.accum = (q->flags & CIMQ_LSQ_ACCUMULATE_GRADS) ? 1 : 0;
  hipLaunchKernelGGL(module_bwd_tail_kernel, dim3(a.nwb + a.nga), dim3(1024), 0, s, g, la, a);
  CIMQ_TRY(check_hip("module_bwd_tail"));
  hipLaunchKernelGGL(module_bwd_finish_kernel, dim3(1), dim3(1024), 0, s, la, a);
  return check_hip("module_bwd_finish");
}

int cimq_alpha_init(const cimq_conv_desc* d, const float* x, const float* w_q, const float* sa,
                    const float* sw, const int8_t* binary_mask, const float* signed_act,
                    float* alpha_init, void* ctx, void* ws, void* stream) {
  Geo g;
  CIMQ_TRY(make_geo(d, &g));
  if (!x || !w_q || !sa || !sw || !binary_mask || !signed_act || !alpha_init || !ctx || !ws)
    return fail(CIMQ_EINVAL, "null pointer argument");
  if (!(g.mode == ADC_SIGN || g.mode == ADC_TERNARY))
    return fail(CIMQ_EINVAL, "alpha_cim exists only for adc_bits 1 / 1.5");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint8_t* c = reinterpret_cast<uint8_t*>(ctx);
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  // the init path slices activations unsigned (lsq.py:51); the fused-LSQ codes are never
  // negative there, so the signed and unsigned slicings coincide
  CIMQ_TRY(prep_all(g, x, w_q, sa, sw, nullptr, binary_mask, signed_act, c, s, false, false));
  {
    Params pp = params_of(g, c);
    if (hipMemsetAsync(pp.flags, 0, 16, s) != hipSuccess) return fail(CIMQ_EHIP, "memset flags");
  }
  if (g.NBP == 4) CIMQ_TRY(dispatch_init<4>(g, c, sw, sa, signed_act, w, s));
  else CIMQ_TRY(dispatch_init<8>(g, c, sw, sa, signed_act, w, s));
  return launch_reduce_galpha(g, c, w, 0.f, 1, sw, sa, alpha_init, s);
}

int cimq_profile_start(int kernel_id, int max_launches) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.ev) return fail(CIMQ_EINVAL, "profiler already running");
  if (kernel_id < KID_FWD || kernel_id > KID_LAST || max_launches <= 0)
    return fail(CIMQ_EINVAL, "bad profiler arguments");
  p.ev = new hipEvent_t[2 * (size_t)max_launches];
  for (int i = 0; i < 2 * max_launches; ++i) {
    if (hipEventCreate(&p.ev[i]) != hipSuccess) {
      for (int k = 0; k < i; ++k) (void)hipEventDestroy(p.ev[k]);
      delete[] p.ev;
      p.ev = nullptr;
      return fail(CIMQ_EHIP, "hipEventCreate");
    }
  }
  p.kid = kernel_id;
  p.cap = max_launches;
  p.n = 0;
  p.bytes = p.flops = 0;
  return CIMQ_OK;
}

int cimq_profile_stop(double* total_ms, int* launches, double* algo_bytes, double* algo_flops) {
  Profiler& p = prof();
  std::lock_guard<std::mutex> lk(p.mu);
  if (!p.ev) return fail(CIMQ_EINVAL, "profiler not running");
  double tot = 0;
  int rc = CIMQ_OK;
  for (int i = 0; i < p.n; ++i) {
    float ms = 0;
    if (hipEventSynchronize(p.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, p.ev[2 * i], p.ev[2 * i + 1]) != hipSuccess) {
      rc = fail(CIMQ_EHIP, "hipEventElapsedTime");
      break;
    }
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = p.n;
  if (algo_bytes) *algo_bytes = p.bytes;
  if (algo_flops) *algo_flops = p.flops;
  for (int i = 0; i < 2 * p.cap; ++i) (void)hipEventDestroy(p.ev[i]);
  delete[] p.ev;
  p.ev = nullptr;
  p.kid = KID_NONE;
  p.cap = p.n = 0;
  return rc;
}

}  // extern "C"

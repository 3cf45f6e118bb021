// glibc_math.h — bit-exact device restatement of the host libm the reference ran on.
//
// The reference turns transcendental results into integer nanoseconds and prices
// (int(round(scale * -log(1-u))), int(round(r_T)) ...), so a correctly rounded or an
// ocml `log` is NOT enough for bit-exact parity (SURVEY.md §7 hard part 2: ~0.1 % of
// glibc results differ from the correctly rounded value).  These are the glibc 2.35
// x86-64 ifunc targets the reference resolves on an FMA+AVX2 host — __log_fma,
// __exp_fma and __pow_fma — restated instruction by instruction from their
// disassembly: every fused multiply-add the compiler formed there is an explicit
// __builtin_fma here, every other operation is a plain IEEE op (this header must be
// compiled with -ffp-contract=off).  Tables: glibc_math_tables.h (generated).
//
// Verified bit-exact against the host libm by tests/test_glibc_math.py (host build of
// this very header) and on the GPU by tests/test_gpu_parity.py.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GM_FN __host__ __device__ __forceinline__ static
#define GM_BIG __host__ __device__ __forceinline__ static
#define GM_TABLE_QUAL static __device__ __constant__ const
#else
#define GM_FN static inline
#define GM_BIG static inline
#define GM_TABLE_QUAL static const
#endif

#include "glibc_math_tables.h"

GM_FN uint64_t gm_asu64(double x) { return __builtin_bit_cast(uint64_t, x); }
GM_FN double gm_asf64(uint64_t x) { return __builtin_bit_cast(double, x); }

// ---------------------------------------------------------------- log (__log_fma)
GM_BIG double gm_log(double x) {
  uint64_t ix = gm_asu64(x);
  uint32_t top = (uint32_t)(ix >> 48);
  const uint64_t LO = 0x3fee000000000000ull, HI = 0x3ff1090000000000ull;
  if (ix - LO < HI - LO) {
    if (ix == 0x3ff0000000000000ull) return 0.0;
    double r = x - 1.0;
    double r2 = r * r;
    double r3 = r * r2;
    double p1 = __builtin_fma(r, GM_LOG_B2, GM_LOG_B1);
    double p2 = __builtin_fma(r, GM_LOG_B5, GM_LOG_B4);
    double p3 = __builtin_fma(r, GM_LOG_B8, GM_LOG_B7);
    p1 = __builtin_fma(r2, GM_LOG_B3, p1);
    p2 = __builtin_fma(r2, GM_LOG_B6, p2);
    double q = __builtin_fma(r2, GM_LOG_B9, p3);
    q = __builtin_fma(r3, GM_LOG_B10, q);
    q = __builtin_fma(q, r3, p2);
    q = __builtin_fma(q, r3, p1);
    double w = __builtin_fma(r, 0x1p27, r);       // r*2^27 + r   (fused "r + w")
    double rhi = __builtin_fma(-0x1p27, r, w);    // - w          (fused)
    double rhi2 = rhi * rhi;
    double rlo = r - rhi;
    double hi = __builtin_fma(rhi2, GM_LOG_B0, r);
    double lo = __builtin_fma(rhi2, GM_LOG_B0, r - hi);
    double t = GM_LOG_B0 * rlo;
    lo = __builtin_fma(t, r + rhi, lo);
    double y = __builtin_fma(q, r3, lo);
    return hi + y;
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if (ix * 2 == 0) return -__builtin_inf();
    if (ix == 0x7ff0000000000000ull) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return __builtin_nan("");
    ix = gm_asu64(x * 0x1p52);
    ix -= 52ull << 52;
  }
  uint64_t tmp = ix - 0x3fe6000000000000ull;
  int i = (int)((tmp >> 45) & 127);
  int k = (int)((int64_t)tmp >> 52);
  uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
  double invc = gm_log_tab[2 * i], logc = gm_log_tab[2 * i + 1];
  double z = gm_asf64(iz);
  double kd = (double)k;
  double r = __builtin_fma(z, invc, -1.0);
  double w = __builtin_fma(kd, GM_LOG_LN2HI, logc);
  double hi = w + r;
  double lo = __builtin_fma(kd, GM_LOG_LN2LO, (w - hi) + r);
  double r2 = r * r;
  double p1 = __builtin_fma(r, GM_LOG_A2, GM_LOG_A1);
  double p2 = __builtin_fma(r, GM_LOG_A4, GM_LOG_A3);
  double r3 = r * r2;
  double t = __builtin_fma(r2, GM_LOG_A0, lo);
  p2 = __builtin_fma(p2, r2, p1);
  double y = __builtin_fma(r3, p2, t);
  return y + hi;
}

// ---------------------------------------------------------------- exp (__exp_fma)
GM_FN double gm_exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {
    sbits -= 1009ull << 52;
    double scale = gm_asf64(sbits);
    return __builtin_fma(scale, tmp, scale) * 0x1p1009;
  }
  sbits += 1022ull << 52;
  double scale = gm_asf64(sbits);
  double y1 = tmp * scale;
  double y = scale + y1;
  if (1.0 > y) {
    double hi = y + 1.0;
    double lo = (scale - y) + y1;
    double t = ((1.0 - hi) + y) + lo;
    t = t + hi;
    y = t - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return y * 0x1p-1022;
}

GM_BIG double gm_exp(double x) {
  uint64_t ix = gm_asu64(x);
  uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ffu;
  if (abstop - 0x3c9u > 0x3eu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return x + 1.0;
    if (abstop >= 0x409u) {
      if (ix == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ffu) return x + 1.0;
      return (ix >> 63) ? 0.0 : __builtin_inf();
    }
    abstop = 0;
  }
  double kd = __builtin_fma(x, GM_EXP_INVLN2N, GM_EXP_SHIFT);
  uint64_t ki = gm_asu64(kd);
  kd = kd - GM_EXP_SHIFT;
  double r = __builtin_fma(kd, GM_EXP_NEGLN2HIN, x);
  r = __builtin_fma(kd, GM_EXP_NEGLN2LON, r);
  uint32_t idx = 2 * (uint32_t)(ki & 127);
  uint64_t top = ki << 45;
  double tail = gm_asf64(gm_exp_tab[idx]);
  uint64_t sbits = gm_exp_tab[idx + 1] + top;
  double r2 = r * r;
  double p = __builtin_fma(r, GM_EXP_C3, GM_EXP_C2);
  double t = r + tail;
  double q = __builtin_fma(r, GM_EXP_C5, GM_EXP_C4);
  p = __builtin_fma(p, r2, t);
  double r4 = r2 * r2;
  double tmp = __builtin_fma(r4, q, p);
  if (abstop == 0) return gm_exp_special(tmp, sbits, ki);
  double scale = gm_asf64(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// ---------------------------------------------------------------- pow (__pow_fma)
GM_FN int gm_checkint(uint64_t iy) {
  int e = (int)(iy >> 52 & 0x7ff);
  if (e < 0x3ff) return 0;
  if (e > 0x3ff + 52) return 2;
  if (iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
  if (iy & (1ull << (0x3ff + 52 - e))) return 1;
  return 2;
}
GM_FN int gm_zeroinfnan(uint64_t i) { return 2 * i - 1 >= 2 * 0x7ff0000000000000ull - 1; }

GM_FN double gm_pow_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {
    sbits -= 1009ull << 52;
    double scale = gm_asf64(sbits);
    return __builtin_fma(scale, tmp, scale) * 0x1p1009;
  }
  sbits += 1022ull << 52;
  double scale = gm_asf64(sbits);
  double y1 = tmp * scale;
  double y = scale + y1;
  if (1.0 > __builtin_fabs(y)) {
    double one = y < 0.0 ? -1.0 : 1.0;
    double lo = (scale - y) + y1;
    double hi = y + one;
    double t = ((one - hi) + y) + lo;
    t = t + hi;
    y = t - one;
    if (y == 0.0) y = gm_asf64(sbits & 0x8000000000000000ull);
  }
  return y * 0x1p-1022;
}

GM_BIG double gm_pow(double x, double y) {
  uint32_t sign_bias = 0;
  uint64_t ix = gm_asu64(x), iy = gm_asu64(y);
  uint32_t topx = (uint32_t)(ix >> 52), topy = (uint32_t)(iy >> 52);
  if (topx - 0x001u >= 0x7ffu - 0x001u || (topy & 0x7ffu) - 0x3beu >= 0x43eu - 0x3beu) {
    if (gm_zeroinfnan(iy)) {
      if (2 * iy == 0) return 1.0;
      if (ix == 0x3ff0000000000000ull) return 1.0;
      if (2 * ix > 2 * 0x7ff0000000000000ull || 2 * iy > 2 * 0x7ff0000000000000ull) return x + y;
      if (2 * ix == 2 * 0x3ff0000000000000ull) return 1.0;
      if ((2 * ix < 2 * 0x3ff0000000000000ull) == !(iy >> 63)) return 0.0;
      return y * y;
    }
    if (gm_zeroinfnan(ix)) {
      double x2 = x * x;
      if ((ix >> 63) && gm_checkint(iy) == 1) x2 = -x2;
      return (iy >> 63) ? 1 / x2 : x2;
    }
    if (ix >> 63) {
      int yint = gm_checkint(iy);
      if (yint == 0) return __builtin_nan("");
      if (yint == 1) sign_bias = 0x800u << 7;
      ix &= 0x7fffffffffffffffull;
      topx &= 0x7ffu;
    }
    if ((topy & 0x7ffu) - 0x3beu >= 0x43eu - 0x3beu) {
      if (ix == 0x3ff0000000000000ull) return 1.0;
      if ((topy & 0x7ffu) < 0x3beu) return ix > 0x3ff0000000000000ull ? 1.0 + y : 1.0 - y;
      return ((ix > 0x3ff0000000000000ull) == (topy < 0x800u)) ? __builtin_inf() : 0.0;
    }
    if (topx == 0) {
      ix = gm_asu64(x * 0x1p52);
      ix &= 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  // log_inline
  uint64_t tmp = ix - 0x3fe6955500000000ull;
  int i = (int)((tmp >> 45) & 127);
  int k = (int)((int64_t)tmp >> 52);
  uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
  double z = gm_asf64(iz);
  double kd = (double)k;
  double invc = gm_pow_tab[4 * i], logc = gm_pow_tab[4 * i + 2], logctail = gm_pow_tab[4 * i + 3];
  double t1 = __builtin_fma(kd, GM_POW_LN2HI, logc);
  double r = __builtin_fma(z, invc, -1.0);
  double ar = r * GM_POW_A0;
  double lo1 = __builtin_fma(kd, GM_POW_LN2LO, logctail);
  double q1 = __builtin_fma(r, GM_POW_A2, GM_POW_A1);
  double q2 = __builtin_fma(r, GM_POW_A4, GM_POW_A3);
  double t2 = r + t1;
  double ar2 = r * ar;
  double lo2a = t1 - t2;
  double ar3 = r * ar2;
  double lo3 = __builtin_fma(ar, r, -ar2);
  double lo2 = lo2a + r;
  double q3 = __builtin_fma(r, GM_POW_A6, GM_POW_A5);
  double hi = t2 + ar2;
  double lo4 = (t2 - hi) + ar2;
  q3 = __builtin_fma(q3, ar2, q2);
  double qq = __builtin_fma(ar2, q3, q1);
  double lo = lo1 + lo2;
  lo = lo + lo3;
  lo = lo + lo4;
  lo = __builtin_fma(ar3, qq, lo);
  double ly = hi + lo;
  double ltail = (hi - ly) + lo;
  // y * log(x) in double-double
  double ehi = y * ly;
  double elo = __builtin_fma(y, ltail, __builtin_fma(ly, y, -ehi));
  // exp_inline(ehi, elo, sign_bias)
  uint64_t ie = gm_asu64(ehi);
  uint32_t abstop = (uint32_t)(ie >> 52) & 0x7ffu;
  if (abstop - 0x3c9u > 0x3eu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) {
      double one = ehi + 1.0;
      return sign_bias ? -one : one;
    }
    if (abstop >= 0x409u) {
      if (ie >> 63) return sign_bias ? -0.0 : 0.0;
      return sign_bias ? -__builtin_inf() : __builtin_inf();
    }
    abstop = 0;
  }
  double ekd = __builtin_fma(ehi, GM_EXP_INVLN2N, GM_EXP_SHIFT);
  uint64_t ki = gm_asu64(ekd);
  ekd = ekd - GM_EXP_SHIFT;
  double er = __builtin_fma(ekd, GM_EXP_NEGLN2HIN, ehi);
  er = __builtin_fma(ekd, GM_EXP_NEGLN2LON, er);
  er = elo + er;
  uint32_t idx = 2 * (uint32_t)(ki & 127);
  uint64_t top = (ki + sign_bias) << 45;
  double tail = gm_asf64(gm_exp_tab[idx]);
  uint64_t sbits = gm_exp_tab[idx + 1] + top;
  double p = __builtin_fma(er, GM_EXP_C3, GM_EXP_C2);
  double t = er + tail;
  double r2 = er * er;
  double q = __builtin_fma(er, GM_EXP_C5, GM_EXP_C4);
  p = __builtin_fma(p, r2, t);
  double r4 = r2 * r2;
  double etmp = __builtin_fma(r4, q, p);
  if (abstop == 0) return gm_pow_special(etmp, sbits, ki);
  double scale = gm_asf64(sbits);
  return __builtin_fma(scale, etmp, scale);
}

// Bit-exact restatements of the glibc 2.35 (x86-64, FMA ifunc variants)
// single-precision elementary functions the reference's compiled physics
// calls (amdflang lowers EXP/LOG/x**y/2.0**y/TANH/ATAN on default reals to
// expf/logf/powf/exp2f/tanhf/atanf).  Same algorithm, same constants, same
// operation order, FMA exactly where the FMA build has it.  The code is
// __host__ __device__: tests/test_glibc_math.py compiles it for the host and
// compares against the host libm over all 2^32 inputs (univariate) and
// stratified samples (powf).
//
// Published algorithms restated:
//   expf/exp2f/logf/powf: ARM optimized-routines (Szabolcs Nagy), the
//     implementations glibc adopted in 2.28 (sysdeps/ieee754/flt-32/e_expf.c,
//     e_exp2f.c, e_logf.c, e_powf.c); table-driven, double internal arithmetic.
//   tanhf/atanf: fdlibm (Sun) float ports (s_tanhf.c + s_expm1f.c, s_atanf.c).
//
// Upstream notices (the algorithms and their constants / table values come
// from these sources; the code here is our own restatement):
//   ARM optimized-routines expf/exp2f/logf/powf: Copyright (c) 2017-2018, Arm
//     Limited; MIT License (SPDX-License-Identifier: MIT), as distributed in
//     glibc 2.35 under the LGPL-2.1-or-later with that notice retained.
//   fdlibm tanhf/expm1f/atanf/log10f/acosf/tanf float ports: Copyright (C)
//     1993 by Sun Microsystems, Inc.  "Developed at SunPro, a Sun Microsystems,
//     Inc. business.  Permission to use, copy, modify, and distribute this
//     software is freely granted, provided that this notice is preserved."
//     (float conversions by Ian Lance Taylor, Cygnus Support).
//   glibc 2.35 (GNU C Library): LGPL-2.1-or-later.
//
// Tables are parameters (struct GmTables) so the kernel can stage them in LDS.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD static inline
#endif

namespace gm {

GM_HD uint32_t asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
GM_HD float asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
GM_HD uint64_t asuint64(double f) { return __builtin_bit_cast(uint64_t, f); }
GM_HD double asdouble(uint64_t u) { return __builtin_bit_cast(double, u); }
GM_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

struct GmTables {
  uint64_t exp2f_tab[32];  // asuint64(2^(i/32)) - (i << 47)
  double logf_tab[32];     // {invc, logc} x 16 (logf_data.c)
  double powf_tab[32];     // {invc, log2(c)} x 16 (powf_log2_data.c)
};

// 2^(i/32), correctly rounded, minus i<<47 (exp2f_data.c construction)
#define GM_EXP2F_TAB                                                                  \
  {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full,               \
   0x3fef9301d0125b51ull, 0x3fef72b83c7d517bull, 0x3fef54873168b9aaull,               \
   0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, 0x3fef06fe0a31b715ull,               \
   0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,               \
   0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull,               \
   0x3feea47eb03a5585ull, 0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull,               \
   0x3feea11473eb0187ull, 0x3feea589994cce13ull, 0x3feeace5422aa0dbull,               \
   0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,               \
   0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull,               \
   0x3fef3720dcef9069ull, 0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full,               \
   0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

// logf_data.c: invc ~ 1/c for c near the centre of subinterval i of
// [0x1.6p-1, 0x1.6p0) (chosen values, not derivable), logc = round(log(c))
#define GM_LOGF_TAB                                                                     \
  {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2, 0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2, \
   0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2, 0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3, \
   0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3, 0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3, \
   0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4, 0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4, \
   0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5, 0x1.0000000000000p+0, 0x0.0p+0,             \
   0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5, 0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4,  \
   0x1.b2036576afce6p-1, 0x1.526e57720db08p-3, 0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3,  \
   0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2, 0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}

// powf_log2_data.c: same invc as logf_data.c, logc = round(log2(c))
#define GM_POWF_TAB                                                                     \
  {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2, 0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2, \
   0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2, 0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2, \
   0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2, 0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3, \
   0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3, 0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4, \
   0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5, 0x1.0000000000000p+0, 0x0.0p+0,             \
   0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4, 0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3,  \
   0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3, 0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2,  \
   0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2, 0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}

// ---- expf ------------------------------------------------------------------
GM_HD uint32_t top12(float x) { return asuint(x) >> 20; }

// GM_BRANCHLESS: the special-case exits of expf/logf as selects after the main
// path (same results for every input, tests/test_glibc_math.py), so an inlined
// call is one basic block and consecutive independent calls can interleave
#ifndef NMP_GM_BRANCHLESS
#define NMP_GM_BRANCHLESS 0
#endif
GM_HD float expf(float x, const GmTables& T) {
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32;
  const double C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32;
  const double C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double xd = (double)x;
#if !NMP_GM_BRANCHLESS
  const uint32_t abstop = top12(x) & 0x7ff;
  if (abstop >= top12(88.0f)) {
    if (asuint(x) == asuint(-__builtin_inff())) return 0.0f;
    if (abstop >= top12(__builtin_inff())) return x + x;
    if (x > 0x1.62e42ep6f) return __builtin_inff();  // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;             // underflow
  }
#endif
  const double z = InvLn2N * xd;
  double kd = z + SHIFT;
  const uint64_t ki = asuint64(kd);
  kd -= SHIFT;
  const double r = fma_(InvLn2N, xd, -kd);  // the FMA build contracts z - kd
  uint64_t t = T.exp2f_tab[ki % 32];
  t += ki << (52 - 5);
  const double s = asdouble(t);
  const double zz = fma_(C0, r, C1);
  const double r2 = r * r;
  double y = fma_(C2, r, 1.0);
  y = fma_(zz, r2, y);
  y = y * s;
#if NMP_GM_BRANCHLESS
  // |x| < 88 never meets the overflow / underflow bounds; -inf underflows to 0
  // and +inf overflows to inf as x + x would give; NaN -> x + x
  float res = (float)y;
  res = x > 0x1.62e42ep6f ? __builtin_inff() : res;
  res = x < -0x1.9fe368p6f ? 0.0f : res;
  return x != x ? x + x : res;
#else
  return (float)y;
#endif
}

// ---- exp2f -----------------------------------------------------------------
GM_HD float exp2f(float x, const GmTables& T) {
  const double SHIFT_SCALED = 0x1.8p+52 / 32;
  const double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
  const double xd = (double)x;
  const uint32_t abstop = top12(x) & 0x7ff;
  if (abstop >= top12(128.0f)) {
    if (asuint(x) == asuint(-__builtin_inff())) return 0.0f;
    if (abstop >= top12(__builtin_inff())) return x + x;
    if (x > 0.0f) return __builtin_inff();
    if (x <= -150.0f) return 0.0f;
  }
  double kd = xd + SHIFT_SCALED;
  const uint64_t ki = asuint64(kd);
  kd -= SHIFT_SCALED;
  const double r = xd - kd;
  uint64_t t = T.exp2f_tab[ki % 32];
  t += ki << (52 - 5);
  const double s = asdouble(t);
  const double z = fma_(C0, r, C1);
  const double r2 = r * r;
  double y = fma_(C2, r, 1.0);
  y = fma_(z, r2, y);
  y = y * s;
  return (float)y;
}

// ---- logf ------------------------------------------------------------------
GM_HD float logf(float x, const GmTables& T) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  const uint32_t OFF = 0x3f330000;
  uint32_t ix = asuint(x);
#if NMP_GM_BRANCHLESS
  const uint32_t ix0 = ix;
  const bool outside = ix - 0x00800000u >= 0x7f800000u - 0x00800000u;
  ix = outside ? asuint(x * 0x1p23f) - (23u << 23) : ix;  // subnormal: normalize
#else
  if (ix == 0x3f800000) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -__builtin_inff();
    if (ix == 0x7f800000) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
    ix = asuint(x * 0x1p23f);  // subnormal: normalize
    ix -= 23u << 23;
  }
#endif
  const uint32_t tmp = ix - OFF;
  const int i = (tmp >> (23 - 4)) % 16;
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0x1ffu << 23);
  const double invc = T.logf_tab[2 * i], logc = T.logf_tab[2 * i + 1];
  const double z = (double)asfloat(iz);
  const double r = fma_(z, invc, -1.0);
  const double y0 = fma_((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = fma_(A1, r, A2);
  y = fma_(A0, r2, y);
  y = fma_(y, r2, y0 + r);
#if NMP_GM_BRANCHLESS
  // x = 1 gives +0 through the main path as the early return does; the
  // outside-range inputs: +-0 -> -inf, +inf -> x, negative or NaN -> NaN,
  // positive subnormal -> the normalized main path
  const float res = (float)y;
  const float nan_or = ((ix0 & 0x80000000u) || ix0 * 2 >= 0xff000000u) ? __builtin_nanf("") : res;
  const float sp = ix0 * 2 == 0 ? -__builtin_inff() : ix0 == 0x7f800000 ? x : nan_or;
  return outside ? sp : res;
#else
  return (float)y;
#endif
}

// ---- powf ------------------------------------------------------------------
GM_HD double powf_log2(uint32_t ix, const GmTables& T) {
  const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2;
  const double A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (tmp >> (23 - 4)) % 16;
  const uint32_t top = tmp & 0xff800000u;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double invc = T.powf_tab[2 * i], logc = T.powf_tab[2 * i + 1];
  const double z = (double)asfloat(iz);
  const double r = fma_(z, invc, -1.0);
  const double y0 = logc + (double)k;
  const double r2 = r * r;
  double y = fma_(A0, r, A1);
  const double p = fma_(A2, r, A3);
  const double r4 = r2 * r2;
  double q = fma_(A4, r, y0);
  q = fma_(p, r2, q);
  y = fma_(y, r4, q);
  return y;
}

GM_HD float powf_exp2(double xd, uint32_t sign_bias, const GmTables& T) {
  const double SHIFT_SCALED = 0x1.8p+52 / 32;
  const double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
  double kd = xd + SHIFT_SCALED;
  const uint64_t ki = asuint64(kd);
  kd -= SHIFT_SCALED;
  const double r = xd - kd;
  uint64_t t = T.exp2f_tab[ki % 32];
  const uint64_t ski = ki + sign_bias;
  t += ski << (52 - 5);
  const double s = asdouble(t);
  const double z = fma_(C0, r, C1);
  const double r2 = r * r;
  double y = fma_(C2, r, 1.0);
  y = fma_(z, r2, y);
  y = y * s;
  return (float)y;
}

GM_HD int powf_checkint(uint32_t iy) {
  const int e = iy >> 23 & 0xff;
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}

GM_HD bool powf_issnan(uint32_t ix) { return 2 * (ix ^ 0x00400000u) > 2u * 0x7fc00000u; }

GM_HD bool powf_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000u - 1; }

// powf after the log2 of |x|: y*log2(x), the overflow / underflow exits, exp2
GM_HD float powf_tail(float y, double logx, uint32_t sign_bias, const GmTables& T) {
  const double ylogx = (double)y * logx;
  if ((asuint64(ylogx) >> 47 & 0xffff) >= asuint64(126.0) >> 47) {
    if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -__builtin_inff() : __builtin_inff();
    if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
  }
  return powf_exp2(ylogx, sign_bias, T);
}

GM_HD float powf(float x, float y, const GmTables& T) {
  uint32_t sign_bias = 0;
  uint32_t ix = asuint(x), iy = asuint(y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || powf_zeroinfnan(iy)) {
    if (powf_zeroinfnan(iy)) {
      if (2 * iy == 0) return powf_issnan(ix) ? x + y : 1.0f;
      if (ix == 0x3f800000) return powf_issnan(iy) ? x + y : 1.0f;
      if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
      if (2 * ix == 2 * 0x3f800000u) return 1.0f;
      if ((2 * ix < 2 * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
      return y * y;
    }
    if (powf_zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000u) && powf_checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000u) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000u) {
      const int yint = powf_checkint(iy);
      if (yint == 0) return __builtin_nanf("");
      if (yint == 1) sign_bias = 1u << (5 + 11);
      ix &= 0x7fffffffu;
    }
    if (ix < 0x00800000u) {
      ix = asuint(x * 0x1p23f);
      ix &= 0x7fffffffu;
      ix -= 23u << 23;
    }
  }
  return powf_tail(y, powf_log2(ix, T), sign_bias, T);
}

// x**y1 and x**y2, each equal to powf's result bit for bit.  When neither
// call takes powf's special-case block (x positive and normal, y1 and y2
// nonzero and finite) the log2 of x is formed once: powf's log2 depends on x
// alone.  (Not glibc code: the sharing is this restatement's, the arithmetic
// is powf's.)
GM_HD void powf_pair(float x, float y1, float y2, const GmTables& T, float& r1, float& r2) {
  const uint32_t ix = asuint(x);
  if (ix - 0x00800000u < 0x7f800000u - 0x00800000u && !powf_zeroinfnan(asuint(y1)) &&
      !powf_zeroinfnan(asuint(y2))) {
    const double logx = powf_log2(ix, T);
    r1 = powf_tail(y1, logx, 0, T);
    r2 = powf_tail(y2, logx, 0, T);
  } else {
    r1 = powf(x, y1, T);
    r2 = powf(x, y2, T);
  }
}

// ---- expm1f / tanhf (fdlibm float; plain fp32 arithmetic, no FMA) ------------
GM_HD float setexp(float y, int32_t k) { return asfloat(asuint(y) + ((uint32_t)k << 23)); }

GM_HD float expm1f(float x) {
  const float huge = 1.0e+30f, tiny = 1.0e-30f, o_threshold = 8.8721679688e+01f;
  const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
  const float invln2 = 1.4426950216e+00f;
  const float Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f, Q3 = -7.9365076090e-05f;
  const float Q4 = 4.0082177293e-06f, Q5 = -2.0109921195e-07f;
  float hi, lo, c = 0.0f, t, e, hxs, hfx, r1, y;
  int32_t k;
  uint32_t hx = asuint(x);
  const uint32_t xsb = hx & 0x80000000u;
  hx &= 0x7fffffffu;
  if (hx >= 0x4195b844u) {
    if (hx >= 0x42b17218u) {
      if (hx > 0x7f800000u) return x + x;
      if (hx == 0x7f800000u) return (xsb == 0) ? x : -1.0f;
      if (x > o_threshold) return huge * huge;
    }
    if (xsb != 0) return tiny - 1.0f;
  }
  if (hx > 0x3eb17218u) {
    if (hx < 0x3F851592u) {
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      } else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    } else {
      k = (int32_t)(invln2 * x + ((xsb == 0) ? 0.5f : -0.5f));
      t = (float)k;
      hi = x - t * ln2_hi;
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  } else if (hx < 0x33000000u) {
    t = huge + x;
    return x - (t - (huge + x));
  } else {
    k = 0;
  }
  hfx = 0.5f * x;
  hxs = x * hfx;
  r1 = 1.0f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
  t = 3.0f - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0f - x * t));
  if (k == 0) return x - (x * e - hxs);
  e = (x * (e - c) - c);
  e -= hxs;
  if (k == -1) return 0.5f * (x - e) - 0.5f;
  if (k == 1) {
    if (x < -0.25f) return -2.0f * (e - (x + 0.5f));
    return 1.0f + 2.0f * (x - e);
  }
  if (k <= -2 || k > 56) {
    y = 1.0f - (e - x);
    y = setexp(y, k);
    return y - 1.0f;
  }
  if (k < 23) {
    t = asfloat(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
    y = t - (e - x);
    y = setexp(y, k);
  } else {
    t = asfloat((uint32_t)(0x7f - k) << 23);  // 2^-k
    y = x - (e + t);
    y += 1.0f;
    y = setexp(y, k);
  }
  return y;
}

GM_HD float tanhf(float x) {
  const float tiny = 1.0e-30f;
  float t, z;
  const uint32_t jx = asuint(x);
  const uint32_t ix = jx & 0x7fffffffu;
  if (ix >= 0x7f800000u) {
    if (!(jx & 0x80000000u)) return 1.0f / x + 1.0f;
    return 1.0f / x - 1.0f;
  }
  if (ix < 0x41b00000u) {
    if (ix == 0) return x;
    if (ix < 0x24000000u) return x * (1.0f + x);
    if (ix >= 0x3f800000u) {
      t = expm1f(2.0f * __builtin_fabsf(x));
      z = 1.0f - 2.0f / (t + 2.0f);
    } else {
      t = expm1f(-2.0f * __builtin_fabsf(x));
      z = -t / (t + 2.0f);
    }
  } else {
    z = 1.0f - tiny;
  }
  return (jx & 0x80000000u) ? -z : z;
}

// ---- atanf (fdlibm float) -------------------------------------------------------
GM_HD float atanf(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f;
  const float atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f;
  const float atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f;
  const float aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f;
  const float aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f;
  const float aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  float w, s1, s2, z, hi = 0.0f, lo = 0.0f;
  int id;
  const uint32_t hx = asuint(x);
  const uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x4c000000u) {
    if (ix > 0x7f800000u) return x + x;
    if (!(hx & 0x80000000u)) return atanhi3 + atanlo3;
    return -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000u) {
    if (ix < 0x31000000u) return x;
    id = -1;
  } else {
    x = __builtin_fabsf(x);
    if (ix < 0x3f980000u) {
      if (ix < 0x3f300000u) {
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      } else {
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    } else {
      if (ix < 0x401c0000u) {
        id = 2;
        x = (x - 1.5f) / (1.0f + 1.5f * x);
      } else {
        id = 3;
        x = -1.0f / x;
      }
    }
  }
  z = x * x;
  w = z * z;
  s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return (hx & 0x80000000u) ? -z : z;
}

// ---- log10f (fdlibm float, calls the ARM logf) ----------------------------------
GM_HD float log10f(float x, const GmTables& T) {
  const float two25 = 3.3554432000e+07f, ivln10 = 4.3429449201e-01f;
  const float log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
  int32_t hx = (int32_t)asuint(x);
  int32_t k = 0;
  if (hx < 0x00800000) {
    if ((hx & 0x7fffffff) == 0) return -two25 / __builtin_fabsf(x);
    if (hx < 0) return (x - x) / (x - x);
    k -= 25;
    x *= two25;
    hx = (int32_t)asuint(x);
  }
  if (hx >= 0x7f800000) return x + x;
  k += (hx >> 23) - 127;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
  const float y = (float)(k + i);
  x = asfloat((uint32_t)hx);
  const float z = y * log10_2lo + ivln10 * logf(x, T);
  return z + y * log10_2hi;
}

// ---- acosf (fdlibm float) ------------------------------------------------------
GM_HD float acosf(float x) {
  const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
  const float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f;
  const float pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
  const float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f;
  const float qS4 = 7.7038154006e-02f;
  float z, p, q, r, w, s, c, df;
  const int32_t hx = (int32_t)asuint(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix <= 0x23000000) return pio2_hi + pio2_lo;
    z = x * x;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {
    z = (1.0f + x) * 0.5f;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    s = __builtin_sqrtf(z);
    r = p / q;
    w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  z = (1.0f - x) * 0.5f;
  s = __builtin_sqrtf(z);
  df = asfloat(asuint(s) & 0xfffff000u);
  c = (z - df * df) / (s + df);
  p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  r = p / q;
  w = r * s + c;
  return 2.0f * (df + w);
}

// ---- cosf (ARM sincosf family, FMA build) for |x| < 120 ------------------------
// __sincosf_table[0|1] = {sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4}
struct SinCosTab { double c0, c1, s1, c2, s2, c3, s3, c4; };
GM_HD SinCosTab sincos_tab(int which) {
  const double c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5;
  const double c3 = -0x1.6c087e89a359dp-10, c4 = 0x1.99343027bf8c3p-16;
  const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
  if (which == 0) return {1.0, c1, s1, c2, s2, c3, s3, c4};
  return {-1.0, -c1, s1, -c2, s2, -c3, s3, -c4};
}
GM_HD float sinf_poly(double x, double x2, const SinCosTab& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = fma_(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = fma_(x3, p.s1, x);
    return (float)fma_(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = fma_(x2, p.c4, p.c3);
  const double c1 = fma_(x2, p.c1, p.c0);
  const double x6 = x4 * x2;
  const double c = fma_(x4, p.c2, c1);
  return (float)fma_(x6, c2, c);
}
GM_HD uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

GM_HD float cosf(float y) {
  const double hpi_inv = 0x1.45f306dc9c883p+23, hpi = 0x1.921fb54442d18p+0;
  const double pio4 = 0x1.921FB6p-1;
  double x = y;
  if (abstop12(y) < abstop12((float)pio4)) {
    const double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x2, sincos_tab(0), 1);
  }
  if (abstop12(y) < abstop12(120.0f)) {
    const double r = x * hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = fma_(-(double)n, hpi, x);
    const double sgn = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sinf_poly(x * sgn, x * x, sincos_tab((n & 2) ? 1 : 0), n ^ 1);
  }
  return (float)::cos((double)y);  // |y| >= 120: not reached by the physics
}

// ---- tanf (fdlibm float: s_tanf + k_tanf + e_rem_pio2f) for |x| < 3pi/4 ---------
GM_HD float kernel_tanf(float x, float y, int iy) {
  const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
  const float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f;
  const float T3 = 2.1869488060e-02f, T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f;
  const float T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f, T8 = 2.4646313977e-04f;
  const float T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f;
  const float T12 = 2.5907305826e-05f;
  float z, r, v, w, s;
  const int32_t hx = (int32_t)asuint(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix < 0x39000000) {  // |x| < 2^-13 (glibc; fdlibm had 2^-28)
    if ((int)x == 0) {
      if ((ix | (iy + 1)) == 0) return 1.0f / __builtin_fabsf(x);
      if (iy == 1) return x;
      return -1.0f / x;
    }
  }
  if (ix >= 0x3f2ca140) {
    if (hx < 0) {
      x = -x;
      y = -y;
    }
    z = pio4 - x;
    w = pio4lo - y;
    x = z + w;
    y = 0.0f;
    if (__builtin_fabsf(x) < 0x1p-13f)
      return (float)(1 - ((hx >> 30) & 2)) * (float)iy * (1.0f - 2.0f * (float)iy * x);
  }
  z = x * x;
  w = z * z;
  r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
  v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
  s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (ix >= 0x3f2ca140) {
    v = (float)iy;
    return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) return w;
  z = asfloat(asuint(w) & 0xfffff000u);
  v = r - (z - x);
  float a = -1.0f / w;
  float t = asfloat(asuint(a) & 0xfffff000u);
  s = 1.0f + t * z;
  return t + a * (s + t * v);
}

GM_HD float tanf(float x) {
  // glibc 2.35 s_tanf.c: sincosf-style reduction in double (plain mul/sub, no
  // FMA in this generic build), then __kernel_tanf on the float hi/lo split.
  const double hpi_inv = 0x1.45f306dc9c883p+23, hpi = 0x1.921fb54442d18p+0;
  const uint32_t ix = asuint(x) & 0x7fffffffu;
  if (ix <= 0x3f490fdau) return kernel_tanf(x, 0.0f, 1);
  if (ix >= 0x7f800000u) return x - x;
  if (abstop12(x) <= 0x42e) {  // |x| < 120
    double xd = (double)x;
    const int n = ((int32_t)(xd * hpi_inv) + 0x800000) >> 24;
    xd = xd - (double)n * hpi;
    const float y0 = (float)xd;
    const float y1 = (float)(xd - (double)y0);
    return kernel_tanf(y0, y1, 1 - ((2 * n) & 2));
  }
  return (float)::tan((double)x);  // |x| >= 120: not reached by the physics
}

}  // namespace gm

// SPDX-License-Identifier: LGPL-2.1-or-later
// Derived from the GNU C Library 2.35 float math (sysdeps/ieee754/flt-32: e_expf.c,
// e_logf.c, e_powf.c, s_sinf.c, s_cosf.c and their data tables, contributed by
// Arm Ltd., Copyright (c) 2017-2018 Arm Ltd.; e_acosf.c, e_asinf.c, s_atanf.c,
// e_atan2f.c from fdlibm, Copyright (C) 1993 by Sun Microsystems, Inc. -- "Developed
// at SunPro, a Sun Microsystems, Inc. business.  Permission to use, copy, modify,
// and distribute this software is freely granted, provided that this notice is
// preserved.").  Copyright (C) 1991-2022 Free Software Foundation, Inc.
// The GNU C Library is free software; you can redistribute it and/or modify it
// under the terms of the GNU Lesser General Public License as published by the
// Free Software Foundation; either version 2.1 of the License, or (at your
// option) any later version.  It is distributed WITHOUT ANY WARRANTY; see the
// GNU Lesser General Public License (<https://www.gnu.org/licenses/>) for details.
// Provenance of every third-party-derived file: THIRD_PARTY_NOTICES.md.
//
// The reference's float libm calls, rounded exactly as on its host.
//
// The reference calls expf, logf, powf, sinf, cosf and acosf (via <cmath>'s float
// overloads: Erf / ErfInv common.h:26-78, the Beckmann sampler and D()
// microfacet_distribution.h:34-107,155-172, random_cosine_direction pdf.h:10-18,
// sphere light sampling sphere.h:7-15, Perlin noise).  glibc >= 2.28 computes
// them with table-driven double-precision algorithms (from ARM's
// optimized-routines) that are accurate but not always correctly rounded: a
// correctly rounded device libm differs in the last bit a few times per
// thousand calls, and a Beckmann path can turn such a bit into a different
// scattering direction.  These are the same algorithms on the same tables
// (glibc_mathf_tables.inc, extracted from libm.so.6 by tools/gen_glibc_mathf.py)
// with the fused multiply-adds of glibc's x86-64 FMA variants (selected on any
// CPU with FMA, e.g. e_expf-fma.c), so the device returns the host's float bit
// for bit.  tools/check_glibc_mathf.cpp compares them with libm over every float
// input (expf, logf, sinf, cosf, acosf, asinf, atanf) and over sampled pairs (powf, atan2f):
// all bit-exact except expf at 2 of the 2^32 inputs (1 ulp, |x| > 32).  acosf
// asinf / atanf / atan2f are glibc's fdlibm float routines, restated.
//
// Special powf operands (zero / inf / nan / negative or subnormal x, results
// beyond 2^+-126) take the double-precision route; the reference never meets them.
#pragma once
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define GM_FN __device__ __forceinline__
#define GM_TAB __device__ __constant__ const
#define GM_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define GM_SQRTF(x) ::srr::dev::rsqrt_exact(x)  // correctly rounded (devmath.h)
#else
#include <cmath>
#define GM_FN static inline
#define GM_TAB static const
#define GM_FMA(a, b, c) std::fma((a), (b), (c))
#define GM_SQRTF(x) std::sqrt((float)(x))
#endif

namespace srr {
namespace gm {

#include "glibc_mathf_tables.inc"

// (__builtin_bit_cast, not std::memcpy: on the device HIP's memcpy is a 4-byte
// loop through scratch memory, which the register allocator kept in k_paths)
GM_FN uint32_t asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
GM_FN float asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
GM_FN uint64_t asuint64(double f) { return __builtin_bit_cast(uint64_t, f); }
GM_FN double asdouble(uint64_t u) { return __builtin_bit_cast(double, u); }
GM_FN uint32_t top12(float x) { return asuint(x) >> 20; }

// e_expf.c: exp(x) = 2^(k/32) * 2^(r/32), k = round(x * 32/ln2)
GM_FN float expf_(float x) {
  const uint32_t abstop = top12(x) & 0x7ff;
  if (abstop >= top12(88.0f)) {
    if (asuint(x) == asuint(-INFINITY)) return 0.0f;
    if (abstop >= top12(INFINITY)) return x + x;
    if (x > 0x1.62e42ep6f) return INFINITY;
    if (x < -0x1.9fe368p6f) return 0.0f;
  }
  const double xd = (double)x;
  const double z = kExpfInvLn2N * xd;
  double kd = z + kExp2fShift;
  const uint64_t ki = asuint64(kd);
  kd -= kExp2fShift;
  const double r = z - kd;
  uint64_t t = kExp2fTab[ki % 32];
  t += ki << (52 - 5);
  const double s = asdouble(t);
  const double zz = GM_FMA(kExp2fPolyScaled[0], r, kExp2fPolyScaled[1]);
  const double r2 = r * r;
  double y = GM_FMA(kExp2fPolyScaled[2], r, 1.0);
  y = GM_FMA(zz, r2, y);
  y = y * s;
  return (float)y;
}

// e_logf.c: log(x) = log1p(z/c - 1) + log(c) + k ln2
GM_FN float logf_(float x) {
  uint32_t ix = asuint(x);
  if (ix == 0x3f800000) return 0.0f;
  if (ix - 0x00800000 >= 0x7f800000 - 0x00800000) {
    if (ix * 2 == 0) return -INFINITY;
    if (ix == 0x7f800000) return x;
    if ((ix & 0x80000000) || ix * 2 >= 0xff000000) return (x - x) / (x - x);
    ix = asuint(x * 0x1p23f);  // subnormal: normalise
    ix -= 23 << 23;
  }
  const uint32_t tmp = ix - 0x3f330000;
  const int i = (tmp >> (23 - 4)) % 16;
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const double invc = kLogfTab[2 * i], logc = kLogfTab[2 * i + 1];
  const double z = (double)asfloat(iz);
  const double r = GM_FMA(z, invc, -1.0);
  const double y0 = GM_FMA((double)k, kLogfLn2, logc);
  const double r2 = r * r;
  double y = GM_FMA(kLogfPoly[1], r, kLogfPoly[2]);
  y = GM_FMA(kLogfPoly[0], r2, y);
  y = GM_FMA(y, r2, y0 + r);
  return (float)y;
}

// e_powf.c: exp2(y * log2(x)), both in double, x > 0 normal and y finite non-zero
GM_FN float powf_(float x, float y) {
  const uint32_t ix = asuint(x), iy = asuint(y);
  const bool y_zeroinfnan = 2 * iy - 1 >= 2u * 0x7f800000 - 1;
  if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || y_zeroinfnan)
    return (float)pow((double)x, (double)y);  // special operands, negative / subnormal x
  // log2_inline
  const uint32_t tmp = ix - 0x3f330000;
  const int i = (tmp >> (23 - 4)) % 16;
  const uint32_t top = tmp & 0xff800000u;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double invc = kPowfLog2Tab[2 * i], logc = kPowfLog2Tab[2 * i + 1];
  const double z = (double)asfloat(iz);
  const double r = GM_FMA(z, invc, -1.0);
  const double y0 = logc + (double)k;
  const double r2 = r * r;
  double yy = GM_FMA(kPowfLog2Poly[0], r, kPowfLog2Poly[1]);
  const double p = GM_FMA(kPowfLog2Poly[2], r, kPowfLog2Poly[3]);
  const double r4 = r2 * r2;
  double q = GM_FMA(kPowfLog2Poly[4], r, y0);
  q = GM_FMA(p, r2, q);
  const double logx = GM_FMA(yy, r4, q);
  const double ylogx = (double)y * logx;
  if ((asuint64(ylogx) >> 47 & 0xffff) >= asuint64(126.0) >> 47)
    return (float)pow((double)x, (double)y);  // |y log2 x| >= 126: over/underflow range
  // exp2_inline (sign_bias 0)
  double kd = ylogx + kExp2fShiftScaled;
  const uint64_t ki = asuint64(kd);
  kd -= kExp2fShiftScaled;
  const double rr = ylogx - kd;
  uint64_t t = kExp2fTab[ki % 32];
  t += ki << (52 - 5);
  const double s = asdouble(t);
  const double zz = GM_FMA(kExp2fPoly[0], rr, kExp2fPoly[1]);
  const double rr2 = rr * rr;
  double e = GM_FMA(kExp2fPoly[2], rr, 1.0);
  e = GM_FMA(zz, rr2, e);
  return (float)(e * s);
}

// sincosf.h: polynomial of quadrant n on the reduced argument.  glibc picks
// __sincosf_table[1] for quadrants with n & 2, which is table 0 with the cosine
// coefficients negated, so that case is the cosine polynomial negated (exact).
GM_FN float sinf_poly(double x, double x2, bool neg_cos, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = GM_FMA(x2, kSc_s3, kSc_s2);
    const double x7 = x3 * x2;
    const double s = GM_FMA(x3, kSc_s1, x);
    return (float)GM_FMA(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = GM_FMA(x2, kSc_c4, kSc_c3);
  const double c1 = GM_FMA(x2, kSc_c1, kSc_c0);
  const double x6 = x4 * x2;
  const double c = GM_FMA(x4, kSc_c2, c1);
  const float r = (float)GM_FMA(x6, c2, c);
  return neg_cos ? -r : r;
}

// sign of sine in quadrant q = 0..3: {1, -1, -1, 1}
GM_FN double quadrant_sign(int q) { return ((q + 1) & 2) ? -1.0 : 1.0; }

// reduce_fast: n = round(x * 2/pi) (from x * 2^24 * 2/pi), x - n pi/2
GM_FN double reduce_fast(double x, int& n) {
  const double r = x * kSc_hpi_inv;
  n = ((int32_t)r + 0x800000) >> 24;
  return GM_FMA(-(double)n, kSc_hpi, x);
}

// reduce_large: |y| >= 120, Payne-Hanek with 4/pi to 192 bits; x in
// [-pi/4, pi/4] scaled by 2^62 in an integer, quadrant n
GM_FN double reduce_large(uint32_t xi, int& n) {
  const uint32_t* arr = &kInvPio4[(xi >> 26) & 15];
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint32_t)(xi * arr[0]);
  const uint64_t res1 = (uint64_t)xi * arr[4];
  const uint64_t res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t nn = (res0 + (1ULL << 61)) >> 62;
  res0 -= nn << 62;
  n = (int)nn;
  return (double)(int64_t)res0 * 0x1.921fb54442d18p-62;
}

GM_FN float sinf_(float y) {
  const uint32_t a = top12(y) & 0x7ff;
  double x = y;
  if (a < (top12(0x1.921fb6p-1f) & 0x7ff)) {  // |y| < pi/4
    if (a < (top12(0x1p-12f) & 0x7ff)) return y;
    return sinf_poly(x, x * x, false, 0);
  }
  if (a < (top12(120.0f) & 0x7ff)) {
    int n;
    x = reduce_fast(x, n);
    return sinf_poly(x * quadrant_sign(n & 3), x * x, (n & 2) != 0, n);
  }
  if (a < (top12(INFINITY) & 0x7ff)) {
    const uint32_t xi = asuint(y);
    const int sign = xi >> 31;
    int n;
    x = reduce_large(xi, n);
    return sinf_poly(x * quadrant_sign((n + sign) & 3), x * x, ((n + sign) & 2) != 0, n);
  }
  return y - y;  // inf / nan
}

GM_FN float cosf_(float y) {
  const uint32_t a = top12(y) & 0x7ff;
  double x = y;
  if (a < (top12(0x1.921fb6p-1f) & 0x7ff)) {
    if (a < (top12(0x1p-12f) & 0x7ff)) return 1.0f;
    return sinf_poly(x, x * x, false, 1);
  }
  if (a < (top12(120.0f) & 0x7ff)) {
    int n;
    x = reduce_fast(x, n);
    return sinf_poly(x * quadrant_sign(n & 3), x * x, (n & 2) != 0, n ^ 1);
  }
  if (a < (top12(INFINITY) & 0x7ff)) {
    const uint32_t xi = asuint(y);
    const int sign = xi >> 31;
    int n;
    x = reduce_large(xi, n);
    return sinf_poly(x * quadrant_sign((n + sign) & 3), x * x, ((n + sign) & 2) != 0, n ^ 1);
  }
  return y - y;  // inf / nan
}

// sinf_(y) and cosf_(y) together, each bit for bit the function's own result: one
// range reduction and, where |y| < 120, both polynomials evaluated once and picked per
// quadrant without a branch (sinf_poly's parity test splits a wave into both paths)
GM_FN void sincosf_(float y, float& so, float& co) {
  const uint32_t a = top12(y) & 0x7ff;
  if (a < (top12(0x1.921fb6p-1f) & 0x7ff) || !(a < (top12(120.0f) & 0x7ff))) {
    so = sinf_(y);
    co = cosf_(y);
    return;
  }
  int n;
  const double x = reduce_fast((double)y, n);
  const double xs = x * quadrant_sign(n & 3), x2 = x * x;
  // sinf_poly's two branches on (xs, x2) with the same sign flag
  const double x3 = xs * x2;
  const double s1 = GM_FMA(x2, kSc_s3, kSc_s2);
  const double x7 = x3 * x2;
  const double sv = GM_FMA(x3, kSc_s1, xs);
  const float S = (float)GM_FMA(x7, s1, sv);
  const double x4 = x2 * x2;
  const double c2 = GM_FMA(x2, kSc_c4, kSc_c3);
  const double c1 = GM_FMA(x2, kSc_c1, kSc_c0);
  const double x6 = x4 * x2;
  const double cv = GM_FMA(x4, kSc_c2, c1);
  const float r = (float)GM_FMA(x6, c2, cv);
  const float C = (n & 2) ? -r : r;
  const bool even = (n & 1) == 0;
  so = even ? S : C;
  co = even ? C : S;
}

// e_acosf.c (fdlibm's float acos, which glibc 2.35 keeps): float arithmetic,
// rational approximation on z = x^2 or z = (1 -+ x)/2
GM_FN float acosf_(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
  const float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
              pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f;
  const float qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
  const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    const float z = x * x;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  }
  if (hx < 0) {  // x < -0.5
    const float z = (one + x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = GM_SQRTF(z);
    const float r = p / q;
    const float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  }
  const float z = (one - x) * 0.5f;  // x > 0.5
  const float s = GM_SQRTF(z);
  const float df = asfloat(asuint(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  const float r = p / q;
  const float w = r * s + c;
  return 2.0f * (df + w);
}

// s_atanf.c / e_atan2f.c / e_asinf.c: glibc's fdlibm float routines (float
// arithmetic), restated; used by get_sphere_uv (hitable.h:10-15)
GM_FN float atanf_(float x) {
  const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
  const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
  const float a0 = 3.3333334327e-01f, a1 = -2.0000000298e-01f, a2 = 1.4285714924e-01f, a3 = -1.1111110449e-01f,
              a4 = 9.0908870101e-02f, a5 = -7.6918758452e-02f, a6 = 6.6610731184e-02f, a7 = -5.8335702866e-02f,
              a8 = 4.9768779427e-02f, a9 = -3.6531571299e-02f, a10 = 1.6285819933e-02f;
  const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x31000000) return x;
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {
      if (ix < 0x3f300000) id = 0, x = (2.0f * x - 1.0f) / (2.0f + x);
      else id = 1, x = (x - 1.0f) / (x + 1.0f);
    } else {
      if (ix < 0x401c0000) id = 2, x = (x - 1.5f) / (1.0f + 1.5f * x);
      else id = 3, x = -1.0f / x;
    }
  }
  const float z = x * x, w = z * z;
  const float s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
  const float s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
  if (id < 0) return x - x * (s1 + s2);
  const float zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -zz : zz;
}

GM_FN float atan2f_(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
              pi_lo = -8.7422776573e-08f;
  const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff, hy = (int32_t)asuint(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf_(y);
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2 * sign(x) + sign(y)
  if (iy == 0) return m <= 1 ? y : (m == 2 ? pi + tiny : -pi - tiny);
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      const float q[4] = {pi_o_4 + tiny, -pi_o_4 - tiny, 3.0f * pi_o_4 + tiny, -3.0f * pi_o_4 - tiny};
      return q[m];
    }
    const float q[4] = {0.0f, -0.0f, pi + tiny, -pi - tiny};
    return q[m];
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = atanf_(fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

GM_FN float asinf_(float x) {
  const float one = 1.0f, huge = 1.000e+30f, pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
              pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-1f, p1 = 7.495297643e-2f,
              p2 = 4.547037598e-2f, p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix < 0x32000000) {
      if (huge + x > one) return x;
    } else {
      const float t = x * x;
      const float w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
      return x + x * w;
    }
  }
  float w = one - fabsf(x);
  float t = w * 0.5f;
  float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  const float s = GM_SQRTF(t);
  if (ix >= 0x3F79999A) {  // |x| > 0.975
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = asfloat(asuint(s) & 0xfffff000u);
    const float c = (t - w * w) / (s + w);
    const float r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    const float q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return hx > 0 ? t : -t;
}

}  // namespace gm
}  // namespace srr

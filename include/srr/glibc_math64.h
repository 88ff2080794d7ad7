// SPDX-License-Identifier: LGPL-2.1-or-later
// Derived from the GNU C Library 2.35 (sysdeps/ieee754/dbl-64: s_sin.c, s_sincos.c,
// e_asin.c, e_atan2.c, and their data tables) -- IBM Accurate Mathematical Library,
// written by International Business Machines Corp.;
// Copyright (C) 2001-2022 Free Software Foundation, Inc.
// The GNU C Library is free software; you can redistribute it and/or modify it
// under the terms of the GNU Lesser General Public License as published by the
// Free Software Foundation; either version 2.1 of the License, or (at your
// option) any later version.  It is distributed WITHOUT ANY WARRANTY; see the
// GNU Lesser General Public License (<https://www.gnu.org/licenses/>) for details.
// Provenance of every third-party-derived file: THIRD_PARTY_NOTICES.md.
//
// The reference's double-precision libm calls of the MERL lookup (brdf.h:106-151:
// cos, sin, acos, atan2), rounded exactly as on its host.
//
// brdf::std_coords_to_half_diff_coords turns the (in, out) angles into the
// half / difference angles with double cos / sin / acos / atan2.  When out == in
// (brdfmaterial's own call, material.h:231) the difference vector is (0, 0, 1)
// up to ~1e-17 residues, so phi_diff = atan2(residue, residue) -- and with it the
// table cell -- is decided by the last-ulp rounding of every one of those calls.
// glibc's dbl-64 routines are not correctly rounded (a correctly rounded device
// libm differs from them on ~0.1 % of inputs), so these are glibc
// 2.35's own algorithms, restated from the x86-64 FMA variants the ifunc selects
// on any CPU with FMA (__sin_fma / __cos_fma of s_sin.c, __ieee754_acos_fma of
// e_asin.c, __ieee754_atan2_fma of e_atan2.c), with each fused multiply-add
// where the compiler put one in those builds, and sincos() (s_sincos.c, built
// once without FMA: g++ merges a sin and a cos of one argument into it), on the
// same data tables
// (glibc_math64_tables.inc, extracted from libm-2.35.a by tools/gen_glibc_math64.py).
// tools/check_glibc_math64.cpp compares them with the host libm.
//
// Domain: sin / cos take |x| < 105414350 (the reference's angles are within
// [-2pi, 2pi]); beyond that glibc's __branred reduction is not restated and the
// functions return NaN.  acos / atan2 cover every input.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GM64_FN __device__ __forceinline__
#define GM64_TAB __device__ __constant__ const
#define GM64_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#include <cmath>
#define GM64_FN static inline
#define GM64_TAB static const
#define GM64_FMA(a, b, c) std::fma((a), (b), (c))
#endif

namespace srr {
namespace gm64 {

#include "glibc_math64_tables.inc"

GM64_FN uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
GM64_FN double dbl(uint64_t u) { return __builtin_bit_cast(double, u); }
GM64_FN int32_t hi_word(double x) { return (int32_t)(bits(x) >> 32); }
GM64_FN uint32_t lo_word(double x) { return (uint32_t)bits(x); }
GM64_FN double fabs_(double x) { return dbl(bits(x) & 0x7fffffffffffffffULL); }
GM64_FN double copysign_(double x, double y) {
  return dbl((bits(x) & 0x7fffffffffffffffULL) | (bits(y) & 0x8000000000000000ULL));
}
GM64_FN double tab(const uint64_t* t, int k) { return dbl(t[k]); }

#define GM64_K(name, b) constexpr double name = __builtin_bit_cast(double, (uint64_t)b##ULL)
// usncs.h (s_sin.c)
GM64_K(kHp0, 0x3ff921fb54442d18);   // pi/2 high
GM64_K(kHp1, 0x3c91a62633145c07);   // pi/2 low
GM64_K(kBig, 0x42c8000000000000);   // 1.5 * 2^45: rounds |x| to a multiple of 1/128
GM64_K(kS1, 0xbfc5555555555555);    // TAYLOR_SIN
GM64_K(kS2, 0x3f81111111110ece);
GM64_K(kS3, 0xbf2a01a019db08b8);
GM64_K(kS4, 0x3ec71de27b9a7ed9);
GM64_K(kS5, 0xbe5addffc2fcdf59);
GM64_K(kSn3, 0xbfc5555555555515);   // do_sin / do_cos
GM64_K(kSn5, 0x3f811110e829872f);
GM64_K(kCs2, 0x3fe0000000000000);
GM64_K(kCs4, 0xbfa5555555555535);
GM64_K(kCs6, 0x3f56c16bedd9e239);
GM64_K(kHpInv, 0x3fe45f306dc9c883); // reduce_sincos
GM64_K(kToInt, 0x4338000000000000);
GM64_K(kMp1, 0x3ff921fb58000000);
GM64_K(kMp2, 0xbe4dde973c000000);
GM64_K(kPp3, 0xbc8cb3b398000000);
GM64_K(kPp4, 0xbacd747f23e32ed7);
// e_asin.c (acos)
GM64_K(kF1, 0x3fc55555555554f9);
GM64_K(kF2, 0x3fb333333336127d);
GM64_K(kF3, 0x3fa6db6dae42c0e4);
GM64_K(kF4, 0x3f9f1c7e04f4ad99);
GM64_K(kF5, 0x3f96e442c822d419);
GM64_K(kF6, 0x3f9292d80f453c72);
GM64_K(kRt0, 0x3fefffffffecc1dd);
GM64_K(kRt1, 0x3fdfffffff757304);
GM64_K(kRt2, 0x3fd800496769c91a);
GM64_K(kRt3, 0x3fd4006318d1dab9);
GM64_K(kT27, 0x41a0000000000000);
GM64_K(kPi, 0x400921fb54442d18);
// e_atan2.c (atnat2.h)
GM64_K(kOpi1, 0x3ca1a62633145c07);  // pi low
GM64_K(kQpi, 0x3fe921fb54442d18);   // pi/4
GM64_K(kTqpi, 0x4002d97c7f3321d2);  // 3pi/4
GM64_K(kD3, 0xbfd5555555555555);
GM64_K(kD5, 0x3fc99999999997fd);
GM64_K(kD7, 0xbfc24924923f7603);
GM64_K(kD9, 0x3fbc71c6e5129a3b);
GM64_K(kD11, 0xbfb7458022b13c25);
GM64_K(kD13, 0x3fb375f08b31cbce);
GM64_K(kTwoM500, 0x20b0000000000000);
GM64_K(kTwo500, 0x5f30000000000000);
GM64_K(kTwo52, 0x4330000000000000);
#undef GM64_K

// ---------------------------------------------------------------- s_sin.c

// TAYLOR_SIN (xx = a*a): a + (((P(xx) * a - 0.5 da) * xx) + da)
GM64_FN double taylor_sin(double a, double da) {
  const double xx = a * a;
  double p = GM64_FMA(kS5, xx, kS4);
  p = GM64_FMA(p, xx, kS3);
  p = GM64_FMA(p, xx, kS2);
  p = GM64_FMA(p, xx, kS1);
  const double t = GM64_FMA(p, a, -(0.5 * da));
  return a + GM64_FMA(xx, t, da);
}

// do_sin: sin(x + dx) from the sin / cos table at the nearest k/128 and short
// series of the remainder
GM64_FN double do_sin(double x, double dx) {
  const double xold = x;
  if (fabs_(x) < 0.126) return taylor_sin(x, dx);
  if (x <= 0) dx = -dx;
  const double u = fabs_(x) + kBig;
  x = fabs_(x) - (u - kBig);
  const double xx = x * x;
  const double s = x + GM64_FMA(x * xx, GM64_FMA(kSn5, xx, kSn3), dx);
  const double c = GM64_FMA(x, dx, xx * GM64_FMA(GM64_FMA(kCs6, xx, kCs4), xx, kCs2));
  const int k = (int)(lo_word(u) << 2);
  const double sn = tab(kSinCosTab, k), ssn = tab(kSinCosTab, k + 1), cs = tab(kSinCosTab, k + 2),
               ccs = tab(kSinCosTab, k + 3);
  const double cor = GM64_FMA(s, cs, GM64_FMA(-c, sn, GM64_FMA(ccs, s, ssn)));
  return copysign_(sn + cor, xold);
}

// do_cos: cos(x + dx), same table
GM64_FN double do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  const double u = fabs_(x) + kBig;
  x = fabs_(x) - (u - kBig) + dx;
  const double xx = x * x;
  const double s = GM64_FMA(x * xx, GM64_FMA(kSn5, xx, kSn3), x);
  const double c = xx * GM64_FMA(GM64_FMA(kCs6, xx, kCs4), xx, kCs2);
  const int k = (int)(lo_word(u) << 2);
  const double sn = tab(kSinCosTab, k), ssn = tab(kSinCosTab, k + 1), cs = tab(kSinCosTab, k + 2),
               ccs = tab(kSinCosTab, k + 3);
  const double cor = GM64_FMA(-s, sn, GM64_FMA(-c, cs, GM64_FMA(-s, ssn, ccs)));
  return cs + cor;
}

// reduce_sincos: x = n pi/2 + (a + da), |x| < 105414350, pi/2 to 136 bits
GM64_FN int reduce_sincos(double x, double& a, double& da) {
  const double t = GM64_FMA(x, kHpInv, kToInt);
  const double xn = t - kToInt;
  const double y = GM64_FMA(-xn, kMp2, GM64_FMA(-xn, kMp1, x));
  const int n = (int)(lo_word(t) & 3);
  const double t2 = GM64_FMA(-xn, kPp3, y);
  double db = GM64_FMA(-xn, kPp3, y - t2);
  const double b = GM64_FMA(-xn, kPp4, t2);
  db = db + GM64_FMA(-xn, kPp4, t2 - b);
  a = b;
  da = db;
  return n;
}

GM64_FN double do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}

GM64_FN double sin(double x) {
  const int32_t k = hi_word(x) & 0x7fffffff;
  if (k < 0x3e500000) return x;                       // |x| < 2^-26
  if (k < 0x3feb6000) return do_sin(x, 0.0);          // |x| < 0.855469
  if (k < 0x400368fd) {                                // |x| < 2.426265
    const double t = kHp0 - fabs_(x);
    return copysign_(do_cos(t, kHp1), x);
  }
  if (k < 0x419921fb) {                                // |x| < 105414350
    double a, da;
    const int n = reduce_sincos(x, a, da);
    return do_sincos(a, da, n);
  }
  if (k < 0x7ff00000) return dbl(0x7ff8000000000000ULL);  // __branred range: not restated
  return x / x;
}

GM64_FN double cos(double x) {
  const int32_t k = hi_word(x) & 0x7fffffff;
  if (k < 0x3e400000) return 1.0;                     // |x| < 2^-27
  if (k < 0x3feb6000) return do_cos(x, 0.0);
  if (k < 0x400368fd) {
    const double y = kHp0 - fabs_(x);
    const double a = y + kHp1;
    const double da = (y - a) + kHp1;
    return do_sin(a, da);
  }
  if (k < 0x419921fb) {
    double a, da;
    const int n = reduce_sincos(x, a, da);
    return do_sincos(a, da, n + 1);
  }
  if (k < 0x7ff00000) return dbl(0x7ff8000000000000ULL);
  return x / x;
}

// ---------------------------------------------------------------- s_sincos.c
// sincos() is not FMA-dispatched in glibc 2.35 (one generic build, no fused
// multiply-adds), and it reduces 0.855469 <= |x| < 2.426265 differently from
// sin(); g++ -O2 merges a sin and a cos of one argument into it, as the
// reference's std_coords_to_half_diff_coords does for its four input angles
// (brdf.h:111-123).  Same algorithms as above, evaluated in source order.

GM64_FN double taylor_sin_nofma(double a, double da) {
  const double xx = a * a;
  const double p = (((kS5 * xx + kS4) * xx + kS3) * xx + kS2) * xx + kS1;
  return a + ((p * a - 0.5 * da) * xx + da);
}

GM64_FN double do_sin_nofma(double x, double dx) {
  const double xold = x;
  if (fabs_(x) < 0.126) return taylor_sin_nofma(x, dx);
  if (x <= 0) dx = -dx;
  const double u = kBig + fabs_(x);
  x = fabs_(x) - (u - kBig);
  const double xx = x * x;
  const double s = x + (dx + x * xx * (kSn3 + xx * kSn5));
  const double c = x * dx + xx * (kCs2 + xx * (kCs4 + xx * kCs6));
  const int k = (int)(lo_word(u) << 2);
  const double sn = tab(kSinCosTab, k), ssn = tab(kSinCosTab, k + 1), cs = tab(kSinCosTab, k + 2),
               ccs = tab(kSinCosTab, k + 3);
  const double cor = (ssn + s * ccs - sn * c) + cs * s;
  return copysign_(sn + cor, xold);
}

GM64_FN double do_cos_nofma(double x, double dx) {
  if (x < 0) dx = -dx;
  const double u = kBig + fabs_(x);
  x = fabs_(x) - (u - kBig) + dx;
  const double xx = x * x;
  const double s = x + x * xx * (kSn3 + xx * kSn5);
  const double c = xx * (kCs2 + xx * (kCs4 + xx * kCs6));
  const int k = (int)(lo_word(u) << 2);
  const double sn = tab(kSinCosTab, k), ssn = tab(kSinCosTab, k + 1), cs = tab(kSinCosTab, k + 2),
               ccs = tab(kSinCosTab, k + 3);
  const double cor = (ccs - s * ssn - cs * c) - sn * s;
  return cs + cor;
}

GM64_FN int reduce_sincos_nofma(double x, double& a, double& da) {
  const double t = x * kHpInv + kToInt;
  const double xn = t - kToInt;
  const double y = (x - xn * kMp1) - xn * kMp2;
  const int n = (int)(lo_word(t) & 3);
  double t1 = xn * kPp3;
  const double t2 = y - t1;
  double db = (y - t2) - t1;
  t1 = xn * kPp4;
  const double b = t2 - t1;
  db += (t2 - b) - t1;
  a = b;
  da = db;
  return n;
}

GM64_FN double do_sincos_nofma(double a, double da, int n) {
  const double r = (n & 1) ? do_cos_nofma(a, da) : do_sin_nofma(a, da);
  return (n & 2) ? -r : r;
}

GM64_FN void sincos(double x, double& sinx, double& cosx) {
  const int32_t k = hi_word(x) & 0x7fffffff;
  if (k < 0x400368fd) {
    if (k < 0x3e400000) {  // |x| < 2^-27
      sinx = x;
      cosx = 1.0;
      return;
    }
    if (k < 0x3feb6000) {  // |x| < 0.855469
      sinx = do_sin_nofma(x, 0.0);
      cosx = do_cos_nofma(x, 0.0);
      return;
    }
    const double y = kHp0 - fabs_(x);  // |x| < 2.426265
    const double a = y + kHp1;
    const double da = (y - a) + kHp1;
    sinx = copysign_(do_cos_nofma(a, da), x);
    cosx = do_sin_nofma(a, da);
    return;
  }
  if (k < 0x419921fb) {
    double a, da;
    const int n = reduce_sincos_nofma(x, a, da);
    sinx = do_sincos_nofma(a, da, n);
    cosx = do_sincos_nofma(a, da, n + 1);
    return;
  }
  sinx = cosx = (k < 0x7ff00000) ? dbl(0x7ff8000000000000ULL) : x / x;
}

// ---------------------------------------------------------------- e_asin.c (acos)

// acos on [0.125, 0.96875): a polynomial of degree `deg` - 1 in xx = |x| - x_n
// around the interval's table point (asncs[n]): asin(|x|) = y_n + t, then
// acos = pi/2 -+ asin, pi/2 carried in two parts
GM64_FN double acos_table(double x, int32_t m, int n, int deg) {
  const double xx = (m > 0 ? x : -x) - tab(kAsnCs, n);
  double p = tab(kAsnCs, n + deg);
  for (int i = n + deg - 1; i >= n + 2; --i) p = GM64_FMA(p, xx, tab(kAsnCs, i));
  p = GM64_FMA(p, xx * xx, tab(kAsnCs, n + deg + 1));
  const double t = GM64_FMA(xx, tab(kAsnCs, n + 1), p);
  const double y = tab(kAsnCs, n + deg + 2);
  return m > 0 ? (kHp1 - t) + (kHp0 - y) : (t + kHp1) + (y + kHp0);
}

GM64_FN double acos(double x) {
  const int32_t m = hi_word(x);
  const int32_t k = m & 0x7fffffff;
  if (k < 0x3c880000) return kHp0;                    // |x| < 2^-55
  if (k < 0x3fc00000) {                                // |x| < 0.125
    const double x2 = x * x;
    double p = GM64_FMA(kF6, x2, kF5);
    p = GM64_FMA(p, x2, kF4);
    p = GM64_FMA(p, x2, kF3);
    p = GM64_FMA(p, x2, kF2);
    p = GM64_FMA(p, x2, kF1);
    const double r = kHp0 - x;
    const double cor = GM64_FMA(-p, x * x2, ((kHp0 - r) - x) + kHp1);
    return r + cor;
  }
  if (k < 0x3fd00000) return acos_table(x, m, 11 * ((k >> 15) & 0x1f), 6);         // [0.125, 0.25)
  if (k < 0x3fe00000) return acos_table(x, m, 11 * ((k >> 14) & 0x3f) + 352, 6);   // [0.25, 0.5)
  if (k < 0x3fe80000) return acos_table(x, m, 3 * ((k >> 11) & 0x1fc) + 1056, 7);  // [0.5, 0.75)
  if (k < 0x3fed8000) return acos_table(x, m, 13 * ((k >> 13) & 0x7f) + 992, 8);   // [0.75, 0.921875)
  if (k < 0x3fee8000) return acos_table(x, m, 14 * ((k >> 13) & 0x7f) + 884, 9);   // [0.921875, 0.953125)
  if (k < 0x3fef0000) return acos_table(x, m, 15 * ((k >> 13) & 0x7f) + 768, 10);  // [0.953125, 0.96875)
  if (k < 0x3ff00000) {                                // [0.96875, 1): acos = 2 asin(sqrt((1 - |x|)/2))
    const double z = 0.5 * (m > 0 ? 1.0 - x : x + 1.0);
    const uint64_t zb = bits(z);
    double t = tab(kInRoot, (int)((zb >> 46) & 0x7f)) * tab(kPowTwo, 511 - (int)((int64_t)zb >> 53));
    const double r = GM64_FMA(-(t * t), z, 1.0);
    t = GM64_FMA(GM64_FMA(GM64_FMA(kRt3, r, kRt2), r, kRt1), r, kRt0) * t;  // 1/sqrt(z), Newton-refined
    const double c = z * t;                                                  // sqrt(z)
    const double h = GM64_FMA(-(t * 0.5), c, 1.5);
    const double y = GM64_FMA(-kT27, c, GM64_FMA(c, kT27, c));               // sqrt(z) to 26 bits
    const double cc = GM64_FMA(-y, y, z) / GM64_FMA(h, c, y);               // and its remainder
    double p = GM64_FMA(kF6, z, kF5);
    p = GM64_FMA(p, z, kF4);
    p = GM64_FMA(p, z, kF3);
    p = GM64_FMA(p, z, kF2);
    p = GM64_FMA(p, z, kF1);
    p = p * z;
    const double q = p * (y + cc);
    if (m < 0) {
      const double res = ((kHp1 - cc) - q) + (kHp0 - y);
      return res + res;
    }
    const double res = (cc + q) + y;
    return res + res;
  }
  if (k == 0x3ff00000 && lo_word(x) == 0) return m > 0 ? 0.0 : kPi;
  if (k > 0x7ff00000 || (k == 0x7ff00000 && lo_word(x) != 0)) return x + x;
  const double d = x - x;  // |x| > 1 (or infinite): NaN
  return d / d;
}

// ---------------------------------------------------------------- e_atan2.c

GM64_FN double atan_poly(double v) {  // d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13))))
  double p = GM64_FMA(kD13, v, kD11);
  p = GM64_FMA(p, v, kD9);
  p = GM64_FMA(p, v, kD7);
  p = GM64_FMA(p, v, kD5);
  return GM64_FMA(p, v, kD3);
}

GM64_FN int atan_index(double u) {  // cij row: (TWO52 + 256 u) - TWO52 - 16
  return (int)(GM64_FMA(u, 256.0, kTwo52) - kTwo52) - 16;
}

GM64_FN double cij_poly(const uint64_t* c, double v) {  // c2 + v (c3 + v (c4 + v (c5 + v c6)))
  double p = GM64_FMA(dbl(c[6]), v, dbl(c[5]));
  p = GM64_FMA(p, v, dbl(c[4]));
  p = GM64_FMA(p, v, dbl(c[3]));
  return GM64_FMA(p, v, dbl(c[2]));
}

GM64_FN double atan2(double y, double x) {
  const int32_t ux = hi_word(x), uy = hi_word(y);
  const uint32_t dx = lo_word(x), dy = lo_word(y);
  const double mhp0 = -kHp0;
  if ((ux & 0x7ff00000) == 0x7ff00000 && ((ux & 0x000fffff) | dx) != 0) return x + y;  // x NaN
  if ((uy & 0x7ff00000) == 0x7ff00000 && ((uy & 0x000fffff) | dy) != 0) return y + y;  // y NaN
  if (uy == 0 && dy == 0) return (ux & 0x80000000) == 0 ? 0.0 : kPi;                   // y = +0
  if ((uint32_t)uy == 0x80000000u && dy == 0) return (ux & 0x80000000) == 0 ? -0.0 : -kPi;
  if (x == 0) return (uy & 0x80000000) == 0 ? kHp0 : mhp0;
  if (ux == 0x7ff00000 && dx == 0) {  // x = +inf
    if (uy == 0x7ff00000) { if (dy == 0) return kQpi; }
    else if ((uint32_t)uy == 0xfff00000u) { if (dy == 0) return -kQpi; }
    else return (uy & 0x80000000) == 0 ? 0.0 : -0.0;
  } else if ((uint32_t)ux == 0xfff00000u && dx == 0) {  // x = -inf
    if (uy == 0x7ff00000) { if (dy == 0) return kTqpi; }
    else if ((uint32_t)uy == 0xfff00000u) { if (dy == 0) return -kTqpi; }
    else return (uy & 0x80000000) == 0 ? kPi : -kPi;
  }
  if (uy == 0x7ff00000 && dy == 0) return kHp0;  // y = +-inf
  if ((uint32_t)uy == 0xfff00000u && dy == 0) return mhp0;

  double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int32_t de = (uy & 0x7ff00000) - (ux & 0x7ff00000);
  if (de >= 59768832) return y > 0 ? kHp0 : mhp0;  // ep = 57 * 16^5: x/y below an ulp of pi/2
  if (de <= -59768832) {                            // y/x negligible
    if (x > 0) return copysign_(ay / ax, y);
    return y > 0 ? kPi : -kPi;
  }
  if (ax < kTwoM500 || ay < kTwoM500) {
    ax *= kTwo500;
    ay *= kTwo500;
  }
  if (ax > kTwo500 || ay > kTwo500) {
    ax *= kTwoM500;
    ay *= kTwoM500;
  }
  // u + du = the smaller over the larger, to ~106 bits (EMULV)
  double u, du;
  const bool y_small = ay < ax;
  if (y_small) {
    u = ay / ax;
    const double v = ax * u, vv = GM64_FMA(ax, u, -v);
    du = ((ay - v) - vv) / ax;
  } else {
    u = ax / ay;
    const double v = ay * u, vv = GM64_FMA(ay, u, -v);
    du = ((ax - v) - vv) / ay;
  }
  double z;
  if (x > 0) {
    if (y_small) {  // (i) atan(ay/ax)
      if (u < 0.0625) {
        const double v = u * u;
        z = u + GM64_FMA(u * v, atan_poly(v), du);
      } else {
        const uint64_t* c = kCij + 7 * atan_index(u);
        const double t3 = u - dbl(c[0]);
        const double v = du + t3;  // EADD (t3, du)
        const double dv = fabs_(t3) > fabs_(du) ? (t3 - v) + du : (du - v) + t3;
        double p = GM64_FMA(dbl(c[6]), v, dbl(c[5]));
        p = GM64_FMA(p, v, dbl(c[4]));
        p = GM64_FMA(p, v, dbl(c[3]));
        const double zz = GM64_FMA(v, dbl(c[2]), GM64_FMA(dv, dbl(c[2]), (v * v) * p));
        z = zz + dbl(c[1]);
      }
    } else {  // (ii) pi/2 - atan(ax/ay)
      if (u < 0.0625) {
        const double v = u * u;
        const double zz = (u * v) * atan_poly(v);
        const double t2 = kHp0 - u;  // ESUB (hpi, u)
        const double cor = kHp0 > fabs_(u) ? (kHp0 - t2) - u : kHp0 - (u + t2);
        z = (((cor + kHp1) - du) - zz) + t2;
      } else {
        const uint64_t* c = kCij + 7 * atan_index(u);
        const double v = (u - dbl(c[0])) + du;
        const double zz = GM64_FMA(-cij_poly(c, v), v, kHp1);
        z = (kHp0 - dbl(c[1])) + zz;
      }
    }
  } else if (!(ay <= ax)) {  // (iii) pi/2 + atan(ax/ay)
    if (u < 0.0625) {
      const double v = u * u;
      const double zz = (v * u) * atan_poly(v);
      const double t2 = u + kHp0;  // EADD (hpi, u)
      const double cor = kHp0 > fabs_(u) ? (kHp0 - t2) + u : (u - t2) + kHp0;
      z = (((cor + kHp1) + du) + zz) + t2;
    } else {
      const uint64_t* c = kCij + 7 * atan_index(u);
      const double v = (u - dbl(c[0])) + du;
      const double zz = GM64_FMA(cij_poly(c, v), v, kHp1);
      z = (kHp0 + dbl(c[1])) + zz;
    }
  } else {  // (iv) pi - atan(ay/ax)
    if (u < 0.0625) {
      const double v = u * u;
      const double zz = (v * u) * atan_poly(v);
      const double t2 = kPi - u;  // ESUB (opi, u)
      const double cor = kPi > fabs_(u) ? (kPi - t2) - u : kPi - (t2 + u);
      z = (((cor + kOpi1) - du) - zz) + t2;
    } else {
      const uint64_t* c = kCij + 7 * atan_index(u);
      const double v = (u - dbl(c[0])) + du;
      const double zz = GM64_FMA(-cij_poly(c, v), v, kOpi1);
      z = (kPi - dbl(c[1])) + zz;
    }
  }
  return copysign_(z, y);
}

}  // namespace gm64
}  // namespace srr

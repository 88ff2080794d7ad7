// Device math that reproduces the reference's float/double promotions.
//
// The reference is compiled C++ on x86-64 (no FMA) linked to glibc's libm.  To
// track it on gfx950:
//  * kernels are compiled with -ffp-contract=off (no FMA contraction) and HIP's
//    default correctly rounded f32 division; f32 sqrt is made correctly rounded
//    here (rsqrt_exact);
//  * the reference's float libm calls run glibc's own algorithms and tables
//    (glibc_mathf.h: sinf, cosf, expf, logf, powf, acosf, asinf, atan2f --
//    bit-exact with the host's libm);
//  * double libm calls (sin/cos/log/pow of double) use the device double libm.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace srr {
namespace dev {

#define SRR_D __device__ __forceinline__

// Correctly rounded f32 sqrt.  v_sqrt_f32 (what __fsqrt_rn / sqrtf lower to on
// gfx950) is accurate to 1 ulp, not correctly rounded; the reference's sqrtf is.
// One step picks among s - 1ulp, s, s + 1ulp by the sign of the exact residual
// x - s'*s (fma), with the usual 2^32 pre-scaling of tiny inputs.
SRR_D float rsqrt_exact(float x) {
  const bool tiny = x < 0x1p-96f;
  const float sx = tiny ? x * 0x1p+32f : x;
  float s = __builtin_amdgcn_sqrtf(sx);
  if (sx > 0.0f && sx < INFINITY) {
    const float dn = __int_as_float(__float_as_int(s) - 1);
    const float up = __int_as_float(__float_as_int(s) + 1);
    const float vp = __builtin_fmaf(-dn, s, sx);
    const float vs = __builtin_fmaf(-up, s, sx);
    s = vp <= 0.0f ? dn : s;
    s = vs > 0.0f ? up : s;
  }
  return tiny ? s * 0x1p-16f : s;
}

}  // namespace dev
}  // namespace srr

#include "glibc_mathf.h"

namespace srr {
namespace dev {

#ifndef SRR_LIBM_DOUBLE  // (A/B builds only: -DSRR_LIBM_DOUBLE rounds double libm results instead)
SRR_D float rsin(float x) { return gm::sinf_(x); }
SRR_D float rcos(float x) { return gm::cosf_(x); }
SRR_D float rexp(float x) { return gm::expf_(x); }
SRR_D float rlog(float x) { return gm::logf_(x); }
SRR_D float rpow(float x, float y) { return gm::powf_(x, y); }
SRR_D float racos(float x) { return gm::acosf_(x); }
SRR_D float rasin(float x) { return gm::asinf_(x); }
SRR_D float ratan2(float y, float x) { return gm::atan2f_(y, x); }
#else
SRR_D float rsin(float x) { return (float)::sin((double)x); }
SRR_D float rcos(float x) { return (float)::cos((double)x); }
SRR_D float rexp(float x) { return (float)::exp((double)x); }
SRR_D float rlog(float x) { return (float)::log((double)x); }
SRR_D float rpow(float x, float y) { return (float)::pow((double)x, (double)y); }
SRR_D float racos(float x) { return (float)::acos((double)x); }
SRR_D float rasin(float x) { return (float)::asin((double)x); }
SRR_D float ratan2(float y, float x) { return (float)::atan2((double)y, (double)x); }
#endif
SRR_D float rdiv(float a, float b) { return __fdiv_rn(a, b); }

static constexpr double kPi = 3.14159265358979323846;  // mathf.h:10

// Comparisons of a float against a double literal that is not a float (the
// reference's `det < 0.0001`, `fabs(x) > 0.9`) as exact float comparisons:
// for float f and such a double d, f < d  <=>  f < up(d) and f > d <=> f >= up(d),
// where up(d) is the smallest float above d.
static constexpr float kUp1em4 = 0x1.a36e3p-14f;  // smallest float > 1e-4 (double)
static constexpr float kUp0p9 = 0x1.cccccep-1f;   // smallest float > 0.9 (double)

// Load of read-only scene data at a wave-uniform index through the constant
// address space, so the compiler can use scalar (SMEM) loads: the kernels
// write other buffers, which otherwise stops it from proving these never change.
template <class T>
SRR_D T cload(const T* p, int i) {
  T v;
  auto src = (const __attribute__((address_space(4))) uint32_t*)(p + i);
  uint32_t* dst = (uint32_t*)&v;
#pragma unroll
  for (int w = 0; w < (int)(sizeof(T) / 4); ++w) dst[w] = src[w];
  return v;
}

// Path-state streams are loaded and stored nontemporal so the scene (BVH nodes,
// triangles: ~1 MB) keeps its place in each XCD's L2.
template <class T>
SRR_D T ntl(const T* p) { return __builtin_nontemporal_load(p); }
template <class T>
struct NtId {
  typedef T type;
};
template <class T>
SRR_D void nts(T* p, typename NtId<T>::type v) { __builtin_nontemporal_store(v, p); }
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
SRR_D float4 ntl(const float4* p) {
  f32x4 v = __builtin_nontemporal_load((const f32x4*)p);
  return make_float4(v[0], v[1], v[2], v[3]);
}
SRR_D void nts(float4* p, float4 x) { __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w}, (f32x4*)p); }
SRR_D int4 ntl(const int4* p) {
  i32x4 v = __builtin_nontemporal_load((const i32x4*)p);
  return make_int4(v[0], v[1], v[2], v[3]);
}
SRR_D void nts(int4* p, int4 x) { __builtin_nontemporal_store(i32x4{x.x, x.y, x.z, x.w}, (i32x4*)p); }

// vec3.h: float x3 value type; every operator is the reference's per-component op
struct V3 {
  float x, y, z;
  SRR_D float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  SRR_D void set(int i, float v) {
    if (i == 0) x = v;
    else if (i == 1) y = v;
    else z = v;
  }
};
SRR_D V3 v3(float a, float b, float c) { return V3{a, b, c}; }
SRR_D V3 v3(float s) { return V3{s, s, s}; }
SRR_D V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
SRR_D V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
SRR_D V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
SRR_D V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
SRR_D V3 operator*(float t, V3 v) { return V3{t * v.x, t * v.y, t * v.z}; }
SRR_D V3 operator*(V3 v, float t) { return V3{t * v.x, t * v.y, t * v.z}; }
SRR_D V3 operator/(V3 v, float t) { return V3{rdiv(v.x, t), rdiv(v.y, t), rdiv(v.z, t)}; }
SRR_D float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
SRR_D V3 cross(V3 a, V3 b) { return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
SRR_D float length(V3 v) { return rsqrt_exact(v.x * v.x + v.y * v.y + v.z * v.z); }
SRR_D float squared_length(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
SRR_D V3 unit_vector(V3 v) { return v / length(v); }
SRR_D float ffmin(float a, float b) { return a < b ? a : b; }
SRR_D float ffmax(float a, float b) { return a > b ? a : b; }

struct Ray {  // ray.h
  V3 o, d;
  float tm;
  SRR_D V3 at(float t) const { return o + t * d; }
};

// mathf.h:14-19 (48-bit LCG) and rng.h:14-35 (PCG32), per path
struct Rng {
  uint64_t lcg;
  uint64_t pcg;
};
static constexpr uint64_t kPcgInc = 0xda3e39cb94b95bdbULL;
SRR_D double drand(Rng& r) {
  r.lcg = (0x5DEECE66DULL * r.lcg + 0xB16ULL) & 0xFFFFFFFFFFFFULL;
  return (double)(uint32_t)(r.lcg >> 16) / 4294967296.0;
}
SRR_D float pcg_uniform(Rng& r) {
  uint64_t old = r.pcg;
  r.pcg = old * 0x5851f42d4c957f2dULL + kPcgInc;
  uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  uint32_t rot = (uint32_t)(old >> 59u);
  uint32_t u = (xs >> rot) | (xs << ((~rot + 1u) & 31));
  return fminf(0.99999994f, float(u) * 2.3283064365386963e-10f);
}

}  // namespace dev
}  // namespace srr

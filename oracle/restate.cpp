// srr CPU oracle: a scalar restatement of the reference renderer's hot path
// (truemeat001/Simple-Raytracing-Render, Raytracing_n/), written from the
// reference's behaviour, function by function, with citations.  It keeps the
// reference's object-graph-and-recursion structure (virtual hit(), recursive
// color()) so it is an independent check of the product's flattened wavefront
// design, and it reproduces every float/double promotion of the reference so that
// on the same libm it is bit-identical to the reference itself.
//
// PARITY PINNED: tests/test_oracle_pins.py checks this restatement bit-for-bit
// against golden vectors made by the reference's own code (oracle/ref, committed
// under tests/golden/).
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load liboracle.so, and only as the checker / CPU baseline;
// the product path (simple-raytracing-render_amd/) never links or calls it.
//
// Differences from the reference, all SURVEY.md §8.0 build definitions:
//   * RNG state is per path (thread_local), reseeded from (x, y, s) (§8(c));
//   * beckmann_pdf's pdf value starts at 0 (Q11), teapot/4-arg triangles use
//     face normals (Q5), pixel index i = idx % nx (Q12).
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "scene_text.h"

namespace orc {

// ------------------------------------------------------------------ vec3.h
struct V {
  float e[3];
  V() : e{0, 0, 0} {}
  explicit V(float s) : e{s, s, s} {}
  V(float a, float b, float c) : e{a, b, c} {}
  float x() const { return e[0]; }
  float y() const { return e[1]; }
  float z() const { return e[2]; }
  float operator[](int i) const { return e[i]; }
  float& operator[](int i) { return e[i]; }
  V operator-() const { return V(-e[0], -e[1], -e[2]); }
  // vec3.h:38-41, evaluated left to right in float
  float length() const { return std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]); }
  float squared_length() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
  V& operator+=(const V& v) { e[0] += v.e[0]; e[1] += v.e[1]; e[2] += v.e[2]; return *this; }
  // vec3.h:160-167: k = 1.0 / t is a double division stored to float
  V& operator/=(float t) {
    float k = 1.0 / t;
    e[0] *= k; e[1] *= k; e[2] *= k;
    return *this;
  }
};
inline V operator+(const V& a, const V& b) { return V(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline V operator-(const V& a, const V& b) { return V(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline V operator*(const V& a, const V& b) { return V(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline V operator*(float t, const V& v) { return V(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline V operator*(const V& v, float t) { return V(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline V operator/(const V& v, float t) { return V(v.e[0] / t, v.e[1] / t, v.e[2] / t); }
inline float dot(const V& a, const V& b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline V cross(const V& a, const V& b) {
  return V(a.e[1] * b.e[2] - a.e[2] * b.e[1], a.e[2] * b.e[0] - a.e[0] * b.e[2], a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
inline V unit_vector(const V& v) { return v / v.length(); }  // vec3.h:169-172

struct Ray {  // ray.h:6-19
  V A, B;
  float tm = 0;
  Ray() {}
  Ray(const V& a, const V& b, float t = 0.0f) : A(a), B(b), tm(t) {}
  V at(float t) const { return A + t * B; }
};

static const double kPi = 3.14159265358979323846;  // mathf.h:10

// ------------------------------------------------------------ RNG (per path)
// mathf.h:14-19 (48-bit LCG, NOT glibc drand48) and rng.h:14-35 (PCG32 XSH-RR).
struct Rng {
  uint64_t lcg = 1;
  uint64_t pcg = 0x853c49e6748fea9bULL;
  uint64_t inc = 0xda3e39cb94b95bdbULL;
  double drand() {
    lcg = (0x5DEECE66DULL * lcg + 0xB16) & 0xFFFFFFFFFFFFULL;
    unsigned x = (unsigned)(lcg >> 16);
    return (double)x / (double)0x100000000LL;
  }
  uint32_t u32() {
    uint64_t old = pcg;
    pcg = old * 0x5851f42d4c957f2dULL + inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
  }
  float uniform() { return std::fmin(0.99999994f, float(u32() * 2.3283064365386963e-10f)); }
};
thread_local Rng R;
inline double drand48() { return R.drand(); }

// Traversal counters (SURVEY §8(d) N_node / N_tri / N_prim), per thread; only
// work done inside world->hit counts (light-pdf probes are excluded).
struct Counters { long long world = 0, node = 0, tri = 0, prim = 0, capped = 0; };
thread_local Counters C;
thread_local bool in_world = false;
#define COUNT(f) do { if (in_world) ++C.f; } while (0)

// ----------------------------------------------------------------- common.h
template <typename T, typename U, typename W>
inline T Clamp(T val, U low, W high) {
  if (val < low) return low;
  else if (val > high) return high;
  return val;
}
// common.h:26-46 -- Abramowitz & Stegun 7.1.26 with the reference's `+ exp`
// (SURVEY Q11 notes the bug; reproduced).
inline float Erf(float x) {
  float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f, a5 = 1.061405429f;
  float p = 0.3275911f;
  int sign = 1;
  if (x < 0) sign = -1;
  x = std::fabs(x);
  float t = 1 / (1 + p * x);
  float y = 1 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t + std::exp(-x * x);
  return sign * y;
}
// common.h:49-78 (Giles' single-precision erfinv)
inline float ErfInv(float x) {
  float w, p;
  x = Clamp(x, -.99999f, .99999f);
  w = -std::log((1 - x) * (1 + x));
  if (w < 5) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = 3.43273939e-07f + p * w;
    p = -3.5233877e-06f + p * w;
    p = -4.39150654e-06f + p * w;
    p = 0.00021858087f + p * w;
    p = -0.00125372503f + p * w;
    p = -0.00417768164f + p * w;
    p = 0.246640727f + p * w;
    p = 1.50140941f + p * w;
  } else {
    w = std::sqrt(w) - 3;
    p = -0.000200214257f;
    p = 0.000100950558f + p * w;
    p = 0.00134934322f + p * w;
    p = -0.00367342844f + p * w;
    p = 0.00573950773f + p * w;
    p = -0.0076224613f + p * w;
    p = 0.00943887047f + p * w;
    p = 1.00167406f + p * w;
    p = 2.83297682f + p * w;
  }
  return p * x;
}

// ------------------------------------------------------------- reflection.h
inline float CosTheta(const V& w) { return w.z(); }
inline float Cos2Theta(const V& w) { return w.z() * w.z(); }
inline float AbsCosTheta(const V& w) { return std::fabs(w.z()); }
inline float Sin2Theta(const V& w) { return std::fmax(0.0f, 1.0f - Cos2Theta(w)); }
inline float SinTheta(const V& w) { return std::sqrt(Sin2Theta(w)); }
inline float TanTheta(const V& w) { return SinTheta(w) / CosTheta(w); }
inline float Tan2Theta(const V& w) { return Sin2Theta(w) / Cos2Theta(w); }
inline float CosPhi(const V& w) {
  float s = SinTheta(w);
  return (s == 0) ? 1 : Clamp(w.x() / s, -1, 1);
}
inline float SinPhi(const V& w) {
  float s = SinTheta(w);
  return (s == 0) ? 0 : Clamp(w.y() / s, -1, 1);
}
inline float Cos2Phi(const V& w) { return CosPhi(w) * CosPhi(w); }
inline float Sin2Phi(const V& w) { return SinPhi(w) * SinPhi(w); }
inline V Reflect(const V& wo, const V& n) { return -wo + 2 * dot(wo, n) * n; }  // reflection.h:34-36
inline bool SameHemisphere(const V& a, const V& b) { return a.z() * b.z() > 0; }

// -------------------------------------------------------------------- onb.h
struct Onb {  // onb.h:6-30
  V ax[3];
  void build_from_w(const V& n) {
    ax[2] = unit_vector(n);
    V a = (std::fabs(ax[2].x()) > 0.9) ? V(0, 1, 0) : V(1, 0, 0);
    ax[1] = unit_vector(cross(ax[2], a));
    ax[0] = cross(ax[2], ax[1]);
  }
  V local(const V& a) const { return a.x() * ax[0] + a.y() * ax[1] + a.z() * ax[2]; }
};

// ------------------------------------------------- microfacet_distribution.h
// pbrt-v3 anisotropic Beckmann with visible-normal sampling (sampleVisibleArea
// is always true here: material.h:156).
struct Beckmann {
  float ax, ay;
  static float RoughnessToAlpha(float r) {  // :139-144
    r = std::fmax(r, 1e-3f);
    float x = std::log(r);
    return 1.62162f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
  }
  float D(const V& wh) const {  // :155-162
    float tan2 = Tan2Theta(wh);
    if (std::isinf(tan2)) return 0.;
    float cos4 = Cos2Theta(wh) * Cos2Theta(wh);
    return std::exp(-tan2 * (Cos2Phi(wh) / (ax * ax) + Sin2Phi(wh) / (ay * ay))) / (kPi * ax * ay * cos4);
  }
  float Lambda(const V& w) const {  // :164-173
    float absTan = std::fabs(TanTheta(w));
    if (std::isinf(absTan)) return 0;
    float alpha = std::sqrt(Cos2Phi(w) * ax * ax + Sin2Phi(w) * ay * ay);
    float a = 1 / (alpha * absTan);
    if (a > 1.6f) return 0;
    return (1 - 1.259f * a + 0.396f * a * a) / (3.535f * a + 2.181f * a * a);
  }
  float G1(const V& w) const { return 1 / (1 + Lambda(w)); }
  float G(const V& wo, const V& wi) const { return 1 / (1 + Lambda(wo) + Lambda(wi)); }
  float Pdf(const V& wo, const V& wh) const {  // :130-135
    return D(wh) * G1(wo) * std::fabs(dot(wo, wh)) / AbsCosTheta(wo);
  }
  static void Sample11(float cosThetaI, float u1, float u2, float* sx, float* sy) {  // :34-107
    if (cosThetaI > .9999) {
      float r = std::sqrt(-std::log(1.0f - u1));
      float sinPhi = std::sin(2 * kPi * u2);
      float cosPhi = std::cos(2 * kPi * u2);
      *sx = r * cosPhi;
      *sy = r * sinPhi;
      return;
    }
    float sinThetaI = std::sqrt(std::fmax(0.0f, 1.0f - cosThetaI * cosThetaI));
    float tanThetaI = sinThetaI / cosThetaI;
    float cotThetaI = 1 / tanThetaI;
    float a = -1, c = Erf(cosThetaI);
    float sample_x = std::fmax(u1, 1e-6f);
    float thetaI = std::acos(cosThetaI);
    float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
    float b = c - (1 + c) * std::pow(1 - sample_x, fit);
    static const float SQRT_PI_INV = 1.f / std::sqrt(kPi);
    float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * std::exp(-cotThetaI * cotThetaI));
    int it = 0;
    while (++it < 10) {
      if (!(b >= a && b <= c)) b = 0.5f * (a + c);
      float invErf = ErfInv(b);
      float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * (std::exp(-invErf * invErf))) - sample_x;
      float derivative = normalization * (1 - invErf * tanThetaI);
      if (std::fabs(value) < 1e-5f) break;
      if (value > 0) c = b;
      else a = b;
      b -= value / derivative;
    }
    *sx = ErfInv(b);
    *sy = ErfInv(2.0f * std::fmax(u2, 1e-6f) - 1.0f);
  }
  V SampleStretched(const V& wi, float u1, float u2) const {  // BeckmannSample :12-32
    V ws = unit_vector(V(ax * wi.x(), ay * wi.y(), wi.z()));
    float sx, sy;
    Sample11(CosTheta(ws), u1, u2, &sx, &sy);
    float tmp = CosPhi(ws) * sx - SinPhi(ws) * sy;
    sy = SinPhi(ws) * sx + CosPhi(ws) * sy;
    sx = tmp;
    sx = ax * sx;
    sy = ay * sy;
    return unit_vector(V(-sx, -sy, 1.f));
  }
  V Sample_wh(const V& wo, float u0, float u1) const {  // :175-211 (visible branch)
    bool flip = wo.z() < 0;
    V wh = SampleStretched(flip ? -wo : wo, u0, u1);
    if (flip) wh = -wh;
    return wh;
  }
};

// ---------------------------------------------------------------- textures
struct Texture {
  virtual ~Texture() {}
  virtual V value(float u, float v, const V& p) const = 0;
};
struct ConstTex : Texture {  // texture.h:25-33
  V c;
  explicit ConstTex(V c) : c(c) {}
  V value(float, float, const V&) const override { return c; }
};
struct ImageTex : Texture {  // texture.h:48-70 (nearest, 3 channels)
  std::vector<unsigned char> px;
  int nx, ny;
  V value(float u, float v, const V&) const override {
    int i = (u) * nx;
    int j = (1 - v) * ny - 0.001;
    if (i < 0) i = 0;
    if (j < 0) j = 0;
    if (i > nx - 1) i = nx - 1;
    if (j > ny - 1) j = ny - 1;
    float r = int(px[3 * i + 3 * nx * j]) / 255.0;
    float g = int(px[3 * i + 3 * nx * j + 1]) / 255.0;
    float b = int(px[3 * i + 3 * nx * j + 2]) / 255.0;
    return V(r, g, b);
  }
};
struct CheckerTex : Texture {  // texture.h:9-23
  const Texture *even, *odd;
  V value(float u, float v, const V& p) const override {
    float sines = std::sin(10 * p.x()) * std::sin(10 * p.y()) * std::sin(10 * p.z());
    return sines < 0 ? odd->value(u, v, p) : even->value(u, v, p);
  }
};
// perlin.h: tables from the reference's static initialisers (1,533 draws of the
// global LCG from seed 1; vec3 arguments are evaluated right to left by g++).
struct Perlin {
  V ranvec[256];
  int px[256], py[256], pz[256];
  Perlin() {
    Rng g;
    g.lcg = 1;
    for (int i = 0; i < 256; ++i) {
      float z = -1 + 2 * g.drand();
      float y = -1 + 2 * g.drand();
      float x = -1 + 2 * g.drand();
      ranvec[i] = unit_vector(V(x, y, z));
    }
    for (int* p : {px, py, pz}) {
      for (int i = 0; i < 256; ++i) p[i] = i;
      for (int i = 255; i > 0; i--) {
        int target = int(g.drand() * (i + 1));
        std::swap(p[i], p[target]);
      }
    }
  }
  float noise(const V& p) const {  // perlin.h:30-46
    float u = p.x() - std::floor(p.x()), v = p.y() - std::floor(p.y()), w = p.z() - std::floor(p.z());
    int i = std::floor(p.x()), j = std::floor(p.y()), k = std::floor(p.z());
    V c[2][2][2];
    for (int di = 0; di < 2; di++)
      for (int dj = 0; dj < 2; dj++)
        for (int dk = 0; dk < 2; dk++)
          c[di][dj][dk] = ranvec[px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255]];
    float uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    float accum = 0;
    for (int a = 0; a < 2; a++)
      for (int b = 0; b < 2; b++)
        for (int d = 0; d < 2; d++) {
          V wv(u - a, v - b, w - d);
          accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) * (d * ww + (1 - d) * (1 - ww)) *
                   dot(c[a][b][d], wv);
        }
    return accum;
  }
  float turb(const V& p, int depth = 7) const {
    float accum = 0;
    V t = p;
    float weight = 1.0;
    for (int i = 0; i < depth; i++) {
      accum += weight * noise(t);
      weight *= 0.5f;
      t = t * 2.0f;
    }
    return std::fabs(accum);
  }
};
const Perlin& perlin() {
  static Perlin P;
  return P;
}
struct NoiseTex : Texture {  // texture.h:35-46
  float scale;
  V value(float, float, const V& p) const override {
    return V(1, 1, 1) * 0.5 * (1 + std::sin(scale * p.z() + 5 * perlin().turb(scale * p)));
  }
};

// ------------------------------------------------------------------ hitable
struct Material;
struct Hit {  // hitable.h:17-25
  float t, u, v;
  V p, normal;
  const Material* mat;
};
struct AABB {  // aabb.h:10-52
  V mn, mx;
  bool hit(const Ray& r, float tmin, float tmax) const {
    COUNT(node);
    for (int a = 0; a < 3; a++) {
      float invD = 1.0f / r.B[a];
      float t0 = (mn[a] - r.A[a]) * invD;
      float t1 = (mx[a] - r.A[a]) * invD;
      if (invD < 0.0f) std::swap(t0, t1);
      tmin = t0 > tmin ? t0 : tmin;
      tmax = t1 < tmax ? t1 : tmax;
      if (tmax <= tmin) return false;
    }
    return true;
  }
};
inline float ffmin(float a, float b) { return a < b ? a : b; }
inline float ffmax(float a, float b) { return a > b ? a : b; }
inline AABB surrounding(const AABB& a, const AABB& b) {  // aabb.h:54-62
  return AABB{V(ffmin(a.mn.x(), b.mn.x()), ffmin(a.mn.y(), b.mn.y()), ffmin(a.mn.z(), b.mn.z())),
              V(ffmax(a.mx.x(), b.mx.x()), ffmax(a.mx.y(), b.mx.y()), ffmax(a.mx.z(), b.mx.z()))};
}

struct Hitable {  // hitable.h:27-33
  virtual ~Hitable() {}
  virtual bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool is_medium = false) const = 0;
  virtual bool bbox(float t0, float t1, AABB& b) const = 0;
  virtual float pdf_value(const V&, const V&) const { return 0.0; }
  virtual V random(const V&) const { return V(1, 0, 0); }
};

// hitable.h:10-15
inline void sphere_uv(const V& p, float& u, float& v) {
  float phi = std::atan2(p.z(), p.x());
  float theta = std::asin(p.y());
  u = 1 - (phi + kPi) / (2 * kPi);
  v = (theta + kPi / 2) / kPi;
}

struct Sphere : Hitable {  // sphere.h:17-86
  V center;
  float radius;
  const Material* mat;
  Sphere(V c, float r, const Material* m) : center(c), radius(r), mat(m) {}
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool) const override {
    COUNT(prim);
    V oc = r.A - center;
    float a = dot(r.B, r.B);
    float b = dot(oc, r.B);
    float c = dot(oc, oc) - radius * radius;
    float disc = b * b - a * c;
    if (disc > 0) {
      for (int k = 0; k < 2; ++k) {
        float temp = k == 0 ? (-b - std::sqrt(disc)) / a : (-b + std::sqrt(disc)) / a;
        if (temp < tmax && temp > tmin) {
          rec.t = temp;
          rec.p = r.at(rec.t);
          sphere_uv((rec.p - center) / radius, rec.u, rec.v);
          rec.normal = (rec.p - center) / radius;
          rec.mat = mat;
          return true;
        }
      }
    }
    return false;
  }
  bool bbox(float, float, AABB& b) const override {
    b = AABB{center - V(radius, radius, radius), center + V(radius, radius, radius)};
    return true;
  }
  float pdf_value(const V& o, const V& v) const override {  // sphere.h:69-78
    Hit rec;
    if (this->hit(Ray(o, v), 0.001, FLT_MAX, rec, false)) {
      float cos_theta_max = std::sqrt(1 - radius * radius / (center - o).squared_length());
      float solid_angle = 2 * kPi * (1 - cos_theta_max);
      return 1 / solid_angle;
    }
    return 0;
  }
  V random(const V& o) const override {  // sphere.h:7-15, 80-86
    V direction = center - o;
    float dist2 = direction.squared_length();
    Onb uvw;
    uvw.build_from_w(direction);
    float r1 = drand48();
    float r2 = drand48();
    float z = 1 + r2 * (std::sqrt(1 - radius * radius / dist2) - 1);
    float phi = 2 * kPi * r1;
    float x = std::cos(phi) * std::sqrt(1 - z * z);
    float y = std::sin(phi) * std::sqrt(1 - z * z);
    return uvw.local(V(x, y, z));
  }
};

struct MovingSphere : Hitable {  // moving_sphere.h:4-59
  V c0, c1;
  float t0, t1, radius;
  const Material* mat;
  V center(float time) const { return c0 + ((time - t0) / (t1 - t0)) * (c1 - c0); }
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool) const override {
    COUNT(prim);
    V oc = r.A - center(r.tm);
    float a = dot(r.B, r.B);
    float b = dot(oc, r.B);
    float c = dot(oc, oc) - radius * radius;
    float disc = b * b - a * c;
    if (disc > 0) {
      for (int k = 0; k < 2; ++k) {
        float temp = k == 0 ? (-b - std::sqrt(disc)) / a : (-b + std::sqrt(disc)) / a;
        if (temp < tmax && temp > tmin) {
          rec.t = temp;
          rec.p = r.at(rec.t);
          rec.normal = (rec.p - center(r.tm)) / radius;
          rec.mat = mat;
          return true;
        }
      }
    }
    return false;
  }
  bool bbox(float a, float b, AABB& box) const override {
    AABB b0{center(a) - V(radius, radius, radius), center(a) + V(radius, radius, radius)};
    AABB b1{center(b) - V(radius, radius, radius), center(b) + V(radius, radius, radius)};
    box = surrounding(b0, b1);
    return true;
  }
};

// aarect.h: axis-aligned rectangle in the plane axis `k_axis` = k.  The reference
// has three classes; axis a0/a1 are the in-plane coordinates (xy: x,y ; xz: x,z ;
// yz: y,z) and the normal is the unit vector of k_axis.
struct Rect : Hitable {
  int kax, a0, a1;
  float lo0, hi0, lo1, hi1, k;
  const Material* mat;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool) const override {  // aarect.h:96-147
    COUNT(prim);
    float t = (k - r.A[kax]) / r.B[kax];
    if (t < tmin || t > tmax) return false;
    float x = r.A[a0] + t * r.B[a0];
    float y = r.A[a1] + t * r.B[a1];
    if (x < lo0 || x > hi0 || y < lo1 || y > hi1) return false;
    rec.u = (x - lo0) / (hi0 - lo0);
    rec.v = (y - lo1) / (hi1 - lo1);
    rec.t = t;
    rec.mat = mat;
    rec.p = r.at(t);
    rec.normal = V(0, 0, 0);
    rec.normal[kax] = 1;
    return true;
  }
  bool bbox(float, float, AABB& b) const override {  // aarect.h:11-14,41-44,72-75
    V mn, mx;
    mn[a0] = lo0; mx[a0] = hi0;
    mn[a1] = lo1; mx[a1] = hi1;
    mn[kax] = k - 0.0001;
    mx[kax] = k + 0.0001;
    b = AABB{mn, mx};
    return true;
  }
  // Only xz_rect implements light sampling (aarect.h:45-60); xy/yz keep the
  // hitable defaults (their versions are commented out, aarect.h:15-29,76-91).
  float pdf_value(const V& o, const V& v) const override {
    if (kax != 1) return 0.0;
    Hit rec;
    if (this->hit(Ray(o, v), 0.001, FLT_MAX, rec, false)) {
      float area = (hi0 - lo0) * (hi1 - lo1);
      float distance_square = rec.t * rec.t * v.squared_length();
      float cosine = std::fabs(dot(v, rec.normal) / v.length());
      return distance_square / (cosine * area);
    }
    return 0;
  }
  V random(const V& o) const override {
    if (kax != 1) return V(1, 0, 0);
    // vec3(x0 + drand48()*(x1-x0), k, z0 + drand48()*(z1-z0)): g++ evaluates the
    // constructor arguments right to left, so the z draw comes first.
    float z = lo1 + drand48() * (hi1 - lo1);
    float x = lo0 + drand48() * (hi0 - lo0);
    return V(x, k, z) - o;
  }
};

struct List : Hitable {  // hitable_list.h:7-67
  std::vector<const Hitable*> l;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool med) const override {
    Hit tmp;
    bool any = false;
    double closest = tmax;
    for (const Hitable* h : l)
      if (h->hit(r, tmin, closest, tmp, med)) {
        any = true;
        closest = tmp.t;
        rec = tmp;
      }
    return any;
  }
  bool bbox(float t0, float t1, AABB& box) const override {  // Q10: merges list[0] only
    if (l.empty()) return false;
    AABB tb;
    if (!l[0]->bbox(t0, t1, tb)) return false;
    box = tb;
    for (size_t i = 0; i < l.size(); i++) {
      if (l[0]->bbox(t0, t1, tb)) box = surrounding(box, tb);
      else return false;
    }
    return true;
  }
  float pdf_value(const V& o, const V& v) const override {
    float weight = 1.0 / l.size();
    float sum = 0;
    for (const Hitable* h : l) sum += weight * h->pdf_value(o, v);
    return sum;
  }
  V random(const V& o) const override {
    int index = int(drand48() * l.size());
    return l[index]->random(o);
  }
};

struct Flip : Hitable {  // aarect.h:149-171
  const Hitable* p;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool med) const override {
    if (p->hit(r, tmin, tmax, rec, med)) {
      rec.normal = -rec.normal;
      return true;
    }
    return false;
  }
  bool bbox(float t0, float t1, AABB& b) const override { return p->bbox(t0, t1, b); }
  float pdf_value(const V& o, const V& v) const override { return p->pdf_value(o, v); }
  V random(const V& o) const override { return p->random(o); }
};

struct Translate : Hitable {  // hitable.h:35-61
  const Hitable* p;
  V off;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool med) const override {
    Ray moved(r.A - off, r.B, r.tm);
    if (p->hit(moved, tmin, tmax, rec, med)) {
      rec.p += off;
      return true;
    }
    return false;
  }
  bool bbox(float t0, float t1, AABB& b) const override {  // Q10: degenerate (Max+off, Max+off)
    if (p->bbox(t0, t1, b)) {
      b = AABB{b.mx + off, b.mx + off};
      return true;
    }
    return false;
  }
};

// rotate_y (hitable.h:65-132) and rotate_x (:135-203): rotation in the plane
// (ia, ib) = (x, z) for y and (y, z) for x; the ray goes in with -theta, the hit
// point and normal come out with +theta.
struct Rotate : Hitable {
  const Hitable* p;
  int ia, ib;
  bool about_y;
  float sin_t, cos_t;
  bool hasbox;
  AABB box;
  Rotate(const Hitable* ptr, float angle, bool y) : p(ptr), about_y(y) {
    ia = y ? 0 : 1;
    ib = 2;
    float radians = (kPi / 180.) * angle;
    sin_t = std::sin(radians);
    cos_t = std::cos(radians);
    hasbox = p->bbox(0, 1, box);
    V mn(FLT_MAX, FLT_MAX, FLT_MAX), mx(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          float x = i * box.mx.x() + (1 - i) * box.mn.x();
          float yy = j * box.mx.y() + (1 - j) * box.mn.y();
          float z = k * box.mx.z() + (1 - k) * box.mn.z();
          V tester;
          if (y) tester = V(cos_t * x + sin_t * z, yy, -sin_t * x + cos_t * z);
          else tester = V(x, cos_t * yy + sin_t * z, -sin_t * yy + cos_t * z);
          for (int c = 0; c < 3; c++) {
            if (tester[c] > mx[c]) mx[c] = tester[c];
            if (tester[c] < mn[c]) mn[c] = tester[c];
          }
        }
    box = AABB{mn, mx};
  }
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool med) const override {
    V o = r.A, d = r.B;
    o[ia] = cos_t * r.A[ia] - sin_t * r.A[ib];
    o[ib] = sin_t * r.A[ia] + cos_t * r.A[ib];
    d[ia] = cos_t * r.B[ia] - sin_t * r.B[ib];
    d[ib] = sin_t * r.B[ia] + cos_t * r.B[ib];
    if (p->hit(Ray(o, d, r.tm), tmin, tmax, rec, med)) {
      V pp = rec.p, nn = rec.normal;
      pp[ia] = cos_t * rec.p[ia] + sin_t * rec.p[ib];
      pp[ib] = -sin_t * rec.p[ia] + cos_t * rec.p[ib];
      nn[ia] = cos_t * rec.normal[ia] + sin_t * rec.normal[ib];
      nn[ib] = -sin_t * rec.normal[ia] + cos_t * rec.normal[ib];
      rec.p = pp;
      rec.normal = nn;
      return true;
    }
    return false;
  }
  bool bbox(float, float, AABB& b) const override {
    b = box;
    return hasbox;
  }
};

struct Triangle : Hitable {  // triangle.h:9-188
  V p0, p1, p2, normal, n0, n1, n2, uv0, uv1, uv2;
  const Material* mat;
  Triangle(V a, V b, V c, const Material* m) : p0(a), p1(b), p2(c), mat(m) {
    normal = unit_vector(cross(p1 - p0, p2 - p0));
  }
  bool hit(const Ray& r, float t0, float t1, Hit& rec, bool med) const override {  // :108-115
    bool h = hit_side(true, r, rec);
    if (!h && med) h = hit_side(false, r, rec);
    return h;
  }
  // :117-188 -- ignores t0/t1 and returns t as a DISTANCE
  bool hit_side(bool front, const Ray& r, Hit& rec) const {
    COUNT(tri);
    V e1 = p1 - p0, e2 = p2 - p0;
    if (!front) {
      e1 = p0 - p1;
      e2 = p2 - p1;
    }
    V dir = r.B / r.B.length();
    V P = cross(dir, e2);
    float det = dot(e1, P);
    V T;
    if (det > 0) T = r.A - p0;
    else {
      T = p0 - r.A;
      det = -det;
    }
    if (det < 0.0001) return false;
    float u = dot(T, P);
    if (u < 0.0f || u > det) return false;
    V Q = cross(T, e1);
    float v = dot(dir, Q);
    if (v < 0.0f || v + u > det) return false;
    float t = dot(e2, Q);
    float inv = 1.0f / det;
    t *= inv;
    u *= inv;
    v *= inv;
    if (t < 0.0001) return false;
    V uv = (1 - u - v) * uv0 + u * uv1 + v * uv2;
    rec.u = uv.x();
    rec.v = uv.y();
    rec.mat = mat;
    rec.normal = unit_vector((1 - u - v) * n0 + u * n1 + v * n2);  // FLAT_NORMAL == 1
    rec.p = (1 - u - v) * p0 + u * p1 + v * p2;
    rec.t = t;
    return true;
  }
  bool bbox(float, float, AABB& b) const override {  // :53-68
    b = AABB{V(ffmin(ffmin(p0.x(), p1.x()), p2.x()), ffmin(ffmin(p0.y(), p1.y()), p2.y()),
               ffmin(ffmin(p0.z(), p1.z()), p2.z())),
             V(ffmax(ffmax(p0.x(), p1.x()), p2.x()), ffmax(ffmax(p0.y(), p1.y()), p2.y()),
               ffmax(ffmax(p0.z(), p1.z()), p2.z()))};
    return true;
  }
  float pdf_value(const V& o, const V& v) const override {  // :70-87
    Hit rec;
    if (this->hit(Ray(o, v), 0.001, FLT_MAX, rec, false)) {
      V v01 = p1 - p0;
      V v01n = v01 / v01.length();
      V v02 = p2 - p0;
      V v02n = v02 / v02.length();
      float cos102 = dot(v01n, v02n);
      float sin102 = std::sqrt(1 - cos102 * cos102);
      float h = v02.length() * sin102;
      float area = 0.5 * v01.length() * h;
      float distance_square = rec.t * rec.t * v.squared_length();
      float cosine = std::fabs(dot(v, rec.normal)) / v.length();
      return distance_square / (cosine * area);
    }
    return 0;
  }
  V random(const V& o) const override {  // :89-94
    float u = drand48();
    float v = drand48() * (1 - u);
    V rp = p0 * (1 - u - v) + p1 * u + p2 * v;
    return rp - o;
  }
};

struct Bvh : Hitable {  // bvh.h:9-119
  const Hitable *left = nullptr, *right = nullptr;
  AABB box;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool med) const override {  // :64-93 (Q7)
    if (!box.hit(r, tmin, tmax)) return false;
    Hit lr, rr;
    bool hl = left->hit(r, tmin, tmax, lr, med);
    bool hr = right->hit(r, tmin, tmax, rr, med);
    if (hl && hr) {
      rec = (lr.t < rr.t) ? lr : rr;
      return true;
    }
    if (hl) { rec = lr; return true; }
    if (hr) { rec = rr; return true; }
    return false;
  }
  bool bbox(float, float, AABB& b) const override {
    b = box;
    return true;
  }
};

// bvh.h:21-55 comparators: -1 when a.min < b.min on the axis, else 1 (never 0);
// the boxes are taken at times (0, 0).  qsort here is the same glibc qsort the
// reference links.
template <int AX>
int box_compare(const void* a, const void* b) {
  AABB bl, br;
  (*(const Hitable* const*)a)->bbox(0, 0, bl);
  (*(const Hitable* const*)b)->bbox(0, 0, br);
  return (bl.mn[AX] - br.mn[AX] < 0.0) ? -1 : 1;
}

struct Store {  // owns every object of a scene
  std::vector<std::unique_ptr<Hitable>> h;
  std::vector<std::unique_ptr<Texture>> t;
  std::vector<std::unique_ptr<Material>> m;
  template <class T> T* add(T* p) { h.emplace_back(p); return p; }
};

const Hitable* build_bvh(Store& S, const Hitable** l, int n, float t0, float t1, Rng& lcg) {  // :96-119
  Bvh* node = S.add(new Bvh());
  int axis = int(3 * lcg.drand());
  if (axis == 0) qsort(l, n, sizeof(void*), box_compare<0>);
  else if (axis == 1) qsort(l, n, sizeof(void*), box_compare<1>);
  else qsort(l, n, sizeof(void*), box_compare<2>);
  if (n == 1) node->left = node->right = l[0];
  else if (n == 2) {
    node->left = l[0];
    node->right = l[1];
  } else {
    node->left = build_bvh(S, l, n / 2, t0, t1, lcg);
    node->right = build_bvh(S, l + n / 2, n - n / 2, t0, t1, lcg);
  }
  AABB bl, br;
  node->left->bbox(t0, t1, bl);
  node->right->bbox(t0, t1, br);
  node->box = surrounding(bl, br);
  return node;
}

// ------------------------------------------------------------------- pdf.h
struct Pdf {
  virtual ~Pdf() {}
  virtual float value(const V& wo, const V& wi) const = 0;
  virtual V generate(const V& wo) const = 0;
};

// pdf.h:10-18 -- note the `2 * sqrt(r2)`: non-unit, not cosine-distributed
inline V random_cosine_direction() {
  float r1 = drand48();
  float r2 = drand48();
  float phi = 2 * kPi * r1;
  float z = std::sqrt(1 - r2);
  float x = std::cos(phi) * 2 * std::sqrt(r2);
  float y = std::sin(phi) * 2 * std::sqrt(r2);
  return V(x, y, z);
}

struct CosinePdf : Pdf {  // pdf.h:30-59 (Q1: the sample is put opposite the viewer)
  Onb uvw;
  V n;
  explicit CosinePdf(const V& w) : n(w) { uvw.build_from_w(w); }
  float value(const V& wo, const V& wi) const override {
    float co = dot(unit_vector(wo), n);
    float ci = dot(unit_vector(wi), n);
    if (ci * co < 0) return std::fabs(ci) / kPi;
    return 0;
  }
  V generate(const V& wo) const override {
    V g = random_cosine_direction();
    if (dot(-wo, n) > 0) g.e[2] *= -1;
    return uvw.local(g);
  }
};

struct OrenNayarPdf : Pdf {  // pdf.h:61-116
  Onb uvw;
  V n;
  float A, B;
  OrenNayarPdf(const V& w, float a, float b) : n(w), A(a), B(b) { uvw.build_from_w(w); }
  V to_local(const V& d) const {
    return unit_vector(V(dot(unit_vector(d), uvw.ax[0]), dot(unit_vector(d), uvw.ax[1]), dot(unit_vector(d), uvw.ax[2])));
  }
  float value(const V& wwo, const V& wwi) const override {
    V wo = to_local(-wwo);
    V wi = to_local(wwi);
    float sinThetaI = SinTheta(wi), sinThetaO = SinTheta(wo);
    float maxCos = 0;
    if (sinThetaI > 1e-4 && sinThetaO > 1e-4) {
      float sinPhiI = SinPhi(wi), cosPhiI = CosPhi(wi);
      float sinPhiO = SinPhi(wo), cosPhiO = CosPhi(wo);
      float dCos = cosPhiI * cosPhiO + sinPhiI * sinPhiO;
      maxCos = ffmax(0.0f, dCos);
    }
    float sinAlpha, tanBeta;
    if (AbsCosTheta(wi) > AbsCosTheta(wo)) {
      sinAlpha = sinThetaO;
      tanBeta = sinThetaI / AbsCosTheta(wi);
    } else {
      sinAlpha = sinThetaI;
      tanBeta = sinThetaO / AbsCosTheta(wo);
    }
    float cosine = CosTheta(wi);
    if (cosine < 0) cosine = 0;
    return cosine * (A + B * maxCos * sinAlpha * tanBeta) / kPi;
  }
  V generate(const V& wo) const override {
    V g = random_cosine_direction();
    if (dot(-wo, n) > 0) g.e[2] *= -1;
    return uvw.local(g);
  }
};

struct BeckmannPdf : Pdf {  // pdf.h:119-156 (value = last generate()'s pdf, Q11; starts at 0)
  const Beckmann* dist;
  Onb uvw;
  mutable float pdf_value = 0;
  BeckmannPdf(const Beckmann* d, const V& n) : dist(d) { uvw.build_from_w(n); }
  float value(const V&, const V&) const override { return pdf_value; }
  V generate(const V& wo) const override {
    float u1 = R.uniform();
    float u2 = R.uniform();
    V wwo = unit_vector(V(dot(-wo, uvw.ax[0]), dot(-wo, uvw.ax[1]), dot(-wo, uvw.ax[2])));
    V wh = dist->Sample_wh(wwo, u1, u2);
    V wi = Reflect(unit_vector(wwo), wh);
    V wwi = unit_vector(wi.x() * uvw.ax[0] + wi.y() * uvw.ax[1] + wi.z() * uvw.ax[2]);
    // G is fed the WORLD-space incoming direction (pdf.h:145)
    pdf_value = dist->D(wh) * dist->G(wo, wi) / (4 * AbsCosTheta(wi) * AbsCosTheta(wwo));
    if (!SameHemisphere(wi, wwo)) pdf_value = 0;
    return wwi;
  }
};

struct HitablePdf : Pdf {  // pdf.h:159-171
  const Hitable* p;
  V o;
  float value(const V&, const V& wi) const override { return p->pdf_value(o, wi); }
  V generate(const V&) const override { return p->random(o); }
};

struct MixturePdf : Pdf {  // pdf.h:173-193 (ctor draws once, unused -- Q3)
  const Pdf* p[2];
  MixturePdf(const Pdf* a, const Pdf* b) {
    p[0] = a;
    p[1] = b;
    (void)drand48();
  }
  float value(const V& wo, const V& wi) const override { return 0.5 * p[0]->value(wo, wi) + 0.5 * p[1]->value(wo, wi); }
  V generate(const V& wo) const override {
    if (drand48() < 0.5) return p[0]->generate(wo);
    return p[1]->generate(wo);
  }
};

// -------------------------------------------------------------- material.h
struct Scatter {  // material.h:64-70
  Ray specular_ray;
  bool is_specular = false;
  V attenuation;
  std::unique_ptr<Pdf> pdf;
};

inline float rand01() { return drand48(); }  // material.h:37-41 (truncates to float)
inline V random_in_unit_sphere() {            // material.h:43-50; args drawn z, y, x
  V p;
  do {
    float z = rand01();
    float y = rand01();
    float x = rand01();
    p = 2.0f * V(x, y, z) - V(1, 1, 1);
  } while (dot(p, p) >= 1.0);
  return p;
}
inline float schlick(float cosine, float ref_idx) {  // material.h:14-19 (pow(float,int) is double)
  float r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1 - r0) * std::pow((double)(1 - cosine), 5);
}
inline bool refract(const V& v, const V& n, float ni_over_nt, V& refracted) {  // material.h:21-32
  V uv = unit_vector(v);
  float dt = dot(uv, n);
  float disc = 1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt);
  if (disc > 0) {
    refracted = ni_over_nt * (uv - n * dt) - n * std::sqrt(disc);
    return true;
  }
  return false;
}
inline V reflect(const V& v, const V& n) { return v - 2 * dot(v, n) * n; }  // material.h:34-36

struct Material {  // material.h:82-93
  virtual ~Material() {}
  virtual bool scatter(const Ray&, const Hit&, Scatter&) const = 0;
  virtual float scattering_pdf(const Ray&, const Hit&, const Ray&) const { return false; }
  virtual V emitted(const Ray&, const Hit&, float, float, const V&) const { return V(0, 0, 0); }
};

struct Lambertian : Material {  // material.h:95-114
  const Texture* albedo;
  float scattering_pdf(const Ray&, const Hit& rec, const Ray& sc) const override {
    float c = dot(rec.normal, unit_vector(sc.B));
    if (c < 0) c = 0;
    return c / kPi;
  }
  bool scatter(const Ray&, const Hit& h, Scatter& s) const override {
    s.is_specular = false;
    s.attenuation = albedo->value(h.u, h.v, h.p);
    s.pdf.reset(new CosinePdf(h.normal));
    return true;
  }
};

struct OrenNayar : Material {  // material.h:127-149
  const Texture* albedo;
  float A, B;
  OrenNayar(const Texture* a, float sigma) : albedo(a) {
    sigma = sigma / 180 * kPi;
    A = 1 - 0.5 * sigma * sigma / (sigma * sigma + 0.33);
    B = 0.45 * sigma * sigma / (sigma * sigma + 0.09);
  }
  float scattering_pdf(const Ray&, const Hit& rec, const Ray& sc) const override {
    float c = dot(rec.normal, unit_vector(sc.B));
    if (c < 0) c = 0;
    return c / kPi;
  }
  bool scatter(const Ray&, const Hit& h, Scatter& s) const override {
    s.is_specular = false;
    s.attenuation = albedo->value(h.u, h.v, h.p);
    s.pdf.reset(new OrenNayarPdf(h.normal, A, B));
    return true;
  }
};

struct BeckmannMat : Material {  // material.h:151-199
  const Texture* albedo;
  Beckmann dist;
  BeckmannMat(const Texture* a, float rx, float ry) : albedo(a) {
    dist.ax = Beckmann::RoughnessToAlpha(rx);
    dist.ay = Beckmann::RoughnessToAlpha(ry);
  }
  float scattering_pdf(const Ray& rin, const Hit& rec, const Ray& sc) const override {
    Onb uvw;
    uvw.build_from_w(rec.normal);
    V d = unit_vector(-rin.B);
    V wo = unit_vector(V(dot(d, uvw.ax[0]), dot(d, uvw.ax[1]), dot(d, uvw.ax[2])));
    V s = unit_vector(sc.B);
    V wi = unit_vector(V(dot(s, uvw.ax[0]), dot(s, uvw.ax[1]), dot(s, uvw.ax[2])));
    V wh = unit_vector(wi + wo);
    return dist.Pdf(wo, wh) / (4 * dot(wo, wh));
  }
  bool scatter(const Ray&, const Hit& h, Scatter& s) const override {
    s.is_specular = false;
    s.attenuation = albedo->value(h.u, h.v, h.p);
    s.pdf.reset(new BeckmannPdf(&dist, h.normal));
    return true;
  }
};

struct Metal : Material {  // material.h:243-261
  V albedo;
  float fuzz;
  bool scatter(const Ray& rin, const Hit& rec, Scatter& s) const override {
    V reflected = reflect(unit_vector(rin.B), rec.normal);
    s.specular_ray = Ray(rec.p, reflected + fuzz * random_in_unit_sphere());
    s.attenuation = albedo;
    s.is_specular = true;
    return true;
  }
};

struct Dielectric : Material {  // material.h:282-339 (Q21)
  float ref_idx;
  bool scatter(const Ray& rin, const Hit& rec, Scatter& s) const override {
    s.is_specular = true;
    s.attenuation = V(1.0, 1.0, 1.0);
    V outward;
    V reflected = reflect(rin.B, rec.normal);
    float ni_over_nt, reflect_prob, cosine;
    V refracted;
    if (dot(rin.B, rec.normal) > 0) {
      outward = -rec.normal;
      ni_over_nt = ref_idx;
      cosine = dot(rin.B, rec.normal) / rin.B.length();
    } else {
      outward = rec.normal;
      ni_over_nt = 1.0 / ref_idx;
      cosine = -dot(rin.B, rec.normal) / rin.B.length();
    }
    if (refract(rin.B, outward, ni_over_nt, refracted)) reflect_prob = schlick(cosine, ref_idx);
    else {
      s.specular_ray = Ray(rec.p, reflected);
      reflect_prob = 1.0;
    }
    if (rand01() < reflect_prob) s.specular_ray = Ray(rec.p, reflected);
    else s.specular_ray = Ray(rec.p, refracted);
    return true;
  }
};

struct DiffuseLight : Material {  // material.h:341-356 (Q16: one-sided)
  const Texture* emit;
  bool scatter(const Ray&, const Hit&, Scatter&) const override { return false; }
  V emitted(const Ray& rin, const Hit& rec, float u, float v, const V& p) const override {
    if (dot(rec.normal, rin.B) < 0.0) return emit->value(u, v, p);
    return V(0, 0, 0);
  }
};

struct Isotropic : Material {  // material.h:359-369
  const Texture* albedo;
  bool scatter(const Ray&, const Hit& rec, Scatter& s) const override {
    s.is_specular = true;
    s.specular_ray = Ray(rec.p, random_in_unit_sphere());
    s.attenuation = albedo->value(rec.u, rec.v, rec.p);
    return true;
  }
};

struct Medium : Hitable {  // constant_medium.h:4-50 (Q17)
  const Hitable* boundary;
  float density;
  const Material* phase;
  bool hit(const Ray& r, float tmin, float tmax, Hit& rec, bool) const override {
    (void)(drand48() < 0.00001);  // the debug-flag draw, then forced false
    Hit r1, r2;
    if (boundary->hit(r, -FLT_MAX, FLT_MAX, r1, true)) {
      if (boundary->hit(r, r1.t + 0.0001, FLT_MAX, r2, true)) {
        if (r1.t < tmin) r1.t = tmin;
        if (r2.t > tmax) r2.t = tmax;
        if (r1.t >= r2.t) return false;
        if (r1.t < 0) r1.t = 0;
        float inside = (r2.t - r1.t) * r.B.length();
        float hit_distance = -(1 / density) * std::log(drand48());
        if (hit_distance < inside) {
          rec.t = r1.t + hit_distance / r.B.length();
          rec.p = r.at(rec.t);
          rec.normal = V(1, 0, 0);
          rec.mat = phase;
          return true;
        }
      }
    }
    return false;
  }
  bool bbox(float t0, float t1, AABB& b) const override { return boundary->bbox(t0, t1, b); }
};

// ----------------------------------------------------------------- camera.h
struct Camera {  // camera.h:16-71 (9-argument ctor)
  V origin, llc, horizontal, vertical, u, v, w;
  float time0, time1, lens_radius;
  Camera(V lookfrom, V lookat, V vup, float vfov, float aspect, float aperture, float focus, float t0, float t1) {
    time0 = t0;
    time1 = t1;
    lens_radius = aperture / 2;
    float theta = vfov * kPi / 180;
    float half_height = std::tan(theta / 2);
    float half_width = aspect * half_height;
    origin = lookfrom;
    w = unit_vector(lookfrom - lookat);
    u = unit_vector(cross(vup, w));
    v = cross(w, u);
    llc = origin - half_width * focus * u - half_height * focus * v - focus * w;
    horizontal = 2 * half_width * focus * u;
    vertical = 2 * half_height * focus * v;
  }
  Ray get_ray(float s, float t) const {
    V p;
    do {  // random_in_unit_disk (camera.h:8-14), y drawn before x
      float y = drand48();
      float x = drand48();
      p = 2.0f * V(x, y, 0) - V(1, 1, 0);
    } while (dot(p, p) >= 1.0);
    V rd = lens_radius * p;
    V offset = u * rd.x() + v * rd.y();
    float time = time0 + drand48() * (time1 - time0);
    V dir = llc + s * horizontal + t * vertical - origin - offset;
    dir = unit_vector(dir);
    return Ray(origin + offset, dir, time);
  }
};

// -------------------------------------------------------------- integrator
struct Scene {
  Store store;
  std::map<long long, const Texture*> tex;
  std::map<long long, const Material*> mat;
  std::map<long long, const Hitable*> obj;
  std::map<long long, std::vector<const Hitable*>> grp;
  std::unique_ptr<Camera> cam;
  const Hitable* world = nullptr;
  const List* lights = nullptr;
};

constexpr int kMixtureGuard = 100000;  // attempts of one resampling loop (build definition)

// Raytracing_n.cpp:55-106 -- recursive; `depth` is shared down the recursion.
V color(const Scene& S, const Ray& r, int* depth, int max_depth) {
  Hit h;
  ++C.world;
  in_world = true;
  bool hit_any = S.world->hit(r, 0.001, std::numeric_limits<float>::max(), h);
  in_world = false;
  if (hit_any) {
    Scatter s;
    V emitted = h.mat->emitted(r, h, h.u, h.v, h.p);
    float pdf_val = 0;
    if (*depth < max_depth && h.mat->scatter(r, h, s)) {
      if (s.is_specular) {
        *depth += 1;
        return s.attenuation * color(S, s.specular_ray, depth, max_depth);
      }
      Ray scattered;
      pdf_val = 0;
      if (S.lights->l.size() > 0) {
        HitablePdf pl;
        pl.p = S.lights;
        pl.o = h.p;
        MixturePdf p(&pl, s.pdf.get());
        // Raytracing_n.cpp:79-83 loops without bound; a hit point in a light's own
        // plane never leaves it (every light sample runs parallel to the light, and
        // the BSDF half is 0, Q1).  Build definition, shared with the
        // product (kernels.hip kMixtureGuard): stop after kMixtureGuard attempts and
        // keep the last one (pdf_val 0).
        int attempts = 0;
        while (pdf_val == 0 && attempts < kMixtureGuard) {
          scattered = Ray(h.p, p.generate(r.B), r.tm);
          pdf_val = p.value(r.B, scattered.B);
          ++attempts;
        }
        if (pdf_val == 0) ++C.capped;
      } else {
        scattered = Ray(h.p, s.pdf->generate(r.B), r.tm);
        pdf_val = s.pdf->value(r.B, scattered.B);
      }
      *depth += 1;
      return emitted + s.attenuation * h.mat->scattering_pdf(r, h, scattered) * color(S, scattered, depth, max_depth) /
                           pdf_val;
    }
    return emitted;
  }
  return V(0.0f);
}

inline V de_nan(const V& c) {  // Raytracing_n.cpp:47-53
  V t = c;
  for (int k = 0; k < 3; ++k)
    if (!(t[k] == t[k])) t[k] = 0;
  return t;
}

// Joe-Kuo Sobol points, D = 2 (Raytracing_n.cpp:721-812): dimension 1 has all
// m = 1; dimension 2 is line "2 1 0 1" of new-joe-kuo-6.21201 (s=1, a=0, m1=1).
std::vector<double> sobol2(unsigned N) {
  unsigned L = (unsigned)std::ceil(std::log((double)N) / std::log(2.0));
  std::vector<unsigned> Cc(N);
  Cc[0] = 1;
  for (unsigned i = 1; i + 1 <= N; i++) {
    Cc[i] = 1;
    unsigned value = i;
    while (value & 1) { value >>= 1; Cc[i]++; }
  }
  std::vector<double> pts(2 * (size_t)N, 0.0);
  std::vector<unsigned> V1(L + 1), V2(L + 1);
  for (unsigned i = 1; i <= L; i++) V1[i] = 1u << (32 - i);
  const unsigned s = 1;
  for (unsigned i = 1; i <= (L < s ? L : s); i++) V2[i] = 1u << (32 - i);
  for (unsigned i = s + 1; i <= L; i++) V2[i] = V2[i - s] ^ (V2[i - s] >> s);
  unsigned X1 = 0, X2 = 0;
  for (unsigned i = 1; i + 1 <= N; i++) {
    X1 ^= V1[Cc[i - 1]];
    X2 ^= V2[Cc[i - 1]];
    pts[2 * i] = (double)X1 / std::pow(2.0, 32);
    pts[2 * i + 1] = (double)X2 / std::pow(2.0, 32);
  }
  return pts;
}

// ------------------------------------------------------------- scene text
std::vector<const Hitable*> make_teapot(Store& St, float scale, int divs, const Material* m);

V V3(const srr_text::Cmd& c, size_t k) { return V(c.f(k), c.f(k + 1), c.f(k + 2)); }

std::unique_ptr<Scene> build(const std::string& text) {
  auto cmds = srr_text::parse(text);
  std::unique_ptr<Scene> S(new Scene());
  Store& St = S->store;
  Rng lcg;
  lcg.lcg = srr_text::kPostPerlinSeed;
  auto M = [&](long long id) -> const Material* { return id < 0 ? nullptr : S->mat.at(id); };
  auto face = [](Triangle* t) { t->n0 = t->n1 = t->n2 = t->normal; };
  for (const auto& c : cmds) {
    const std::string& k = c.at(0);
    if (k == "srr_scene") continue;
    if (k == "lcg") { lcg.lcg = c.u(1); continue; }
    if (k == "tex") {
      const std::string& t = c.at(2);
      Texture* x = nullptr;
      if (t == "const") x = new ConstTex(V3(c, 3));
      else if (t == "image_gen") {
        auto* im = new ImageTex();
        im->nx = (int)c.i(3);
        im->ny = (int)c.i(4);
        im->px = srr_text::gen_image(im->nx, im->ny, (unsigned)c.u(5), (int)c.i(6));
        x = im;
      } else if (t == "image_raw") {
        auto* im = new ImageTex();
        im->nx = (int)c.i(3);
        im->ny = (int)c.i(4);
        im->px = srr_text::read_raw_image(c.at(5), im->nx, im->ny);
        x = im;
      } else if (t == "checker") {
        auto* ck = new CheckerTex();
        ck->even = S->tex.at(c.i(3));
        ck->odd = S->tex.at(c.i(4));
        x = ck;
      } else if (t == "noise") {
        auto* nt = new NoiseTex();
        nt->scale = c.f(3);
        x = nt;
      } else throw std::runtime_error("tex kind " + t);
      St.t.emplace_back(x);
      S->tex[c.i(1)] = x;
      continue;
    }
    if (k == "mat") {
      const std::string& t = c.at(2);
      Material* m = nullptr;
      if (t == "lambertian") { auto* q = new Lambertian(); q->albedo = S->tex.at(c.i(3)); m = q; }
      else if (t == "orennayar") m = new OrenNayar(S->tex.at(c.i(3)), c.f(4));
      else if (t == "beckmann") m = new BeckmannMat(S->tex.at(c.i(3)), c.f(4), c.f(5));
      else if (t == "metal") {
        auto* q = new Metal();
        q->albedo = V3(c, 3);
        float f = c.f(6);
        q->fuzz = (f < 1) ? f : 1;
        m = q;
      } else if (t == "dielectric") { auto* q = new Dielectric(); q->ref_idx = c.f(3); m = q; }
      else if (t == "diffuse_light") { auto* q = new DiffuseLight(); q->emit = S->tex.at(c.i(3)); m = q; }
      else if (t == "isotropic") { auto* q = new Isotropic(); q->albedo = S->tex.at(c.i(3)); m = q; }
      else throw std::runtime_error("mat kind " + t);
      St.m.emplace_back(m);
      S->mat[c.i(1)] = m;
      continue;
    }
    if (k == "grp") {
      S->grp[c.i(1)] = make_teapot(St, c.f(3), (int)c.i(4), M(c.i(5)));
      continue;
    }
    if (k == "obj") {
      long long id = c.i(1);
      const std::string& t = c.at(2);
      const Hitable* h = nullptr;
      auto rect = [&](int kax, int a0, int a1) {
        Rect* r = St.add(new Rect());
        r->kax = kax; r->a0 = a0; r->a1 = a1;
        r->lo0 = c.f(3); r->hi0 = c.f(4); r->lo1 = c.f(5); r->hi1 = c.f(6); r->k = c.f(7);
        r->mat = M(c.i(8));
        return r;
      };
      if (t == "sphere") h = St.add(new Sphere(V3(c, 3), c.f(6), M(c.i(7))));
      else if (t == "moving_sphere") {
        auto* ms = St.add(new MovingSphere());
        ms->c0 = V3(c, 3); ms->c1 = V3(c, 6); ms->t0 = c.f(9); ms->t1 = c.f(10); ms->radius = c.f(11);
        ms->mat = M(c.i(12));
        h = ms;
      } else if (t == "xy_rect") h = rect(2, 0, 1);
      else if (t == "xz_rect") h = rect(1, 0, 2);
      else if (t == "yz_rect") h = rect(0, 1, 2);
      else if (t == "box") {  // box.h:18-29: six rects in a hitable_list
        V p0 = V3(c, 3), p1 = V3(c, 6);
        const Material* m = M(c.i(9));
        auto mk = [&](int kax, int a0, int a1, float lo0, float hi0, float lo1, float hi1, float kk, bool flip) {
          Rect* r = St.add(new Rect());
          r->kax = kax; r->a0 = a0; r->a1 = a1;
          r->lo0 = lo0; r->hi0 = hi0; r->lo1 = lo1; r->hi1 = hi1; r->k = kk; r->mat = m;
          if (!flip) return (const Hitable*)r;
          Flip* f = St.add(new Flip());
          f->p = r;
          return (const Hitable*)f;
        };
        List* l = St.add(new List());
        l->l = {mk(2, 0, 1, p0.x(), p1.x(), p0.y(), p1.y(), p1.z(), false),
                mk(2, 0, 1, p0.x(), p1.x(), p0.y(), p1.y(), p0.z(), true),
                mk(1, 0, 2, p0.x(), p1.x(), p0.z(), p1.z(), p1.y(), false),
                mk(1, 0, 2, p0.x(), p1.x(), p0.z(), p1.z(), p0.y(), true),
                mk(0, 1, 2, p0.y(), p1.y(), p0.z(), p1.z(), p1.x(), false),
                mk(0, 1, 2, p0.y(), p1.y(), p0.z(), p1.z(), p0.x(), true)};
        struct Box : Hitable {  // box.h:5-34: own bbox (pmin, pmax), hit via the list
          const Hitable* l; AABB b;
          bool hit(const Ray& r, float a, float bb, Hit& rec, bool m) const override { return l->hit(r, a, bb, rec, m); }
          bool bbox(float, float, AABB& o) const override { o = b; return true; }
        };
        Box* bx = St.add(new Box());
        bx->l = l;
        bx->b = AABB{p0, p1};
        h = bx;
      } else if (t == "triangle" || t == "triangle_uv" || t == "triangle_uvn") {
        Triangle* tr = St.add(new Triangle(V3(c, 3), V3(c, 6), V3(c, 9), M(c.i(12))));
        if (t != "triangle") { tr->uv0 = V3(c, 13); tr->uv1 = V3(c, 16); tr->uv2 = V3(c, 19); }
        if (t == "triangle_uvn") { tr->n0 = V3(c, 22); tr->n1 = V3(c, 25); tr->n2 = V3(c, 28); }
        else face(tr);
        h = tr;
      } else if (t == "flip") { auto* f = St.add(new Flip()); f->p = S->obj.at(c.i(3)); h = f; }
      else if (t == "translate") {
        auto* tr = St.add(new Translate());
        tr->p = S->obj.at(c.i(3));
        tr->off = V3(c, 4);
        h = tr;
      } else if (t == "rotate_y") h = St.add(new Rotate(S->obj.at(c.i(3)), c.f(4), true));
      else if (t == "rotate_x") h = St.add(new Rotate(S->obj.at(c.i(3)), c.f(4), false));
      else if (t == "constant_medium") {
        auto* md = St.add(new Medium());
        md->boundary = S->obj.at(c.i(3));
        md->density = c.f(4);
        auto* iso = new Isotropic();
        iso->albedo = S->tex.at(c.i(5));
        St.m.emplace_back(iso);
        md->phase = iso;
        h = md;
      } else if (t == "list" || t == "list_group") {
        List* l = St.add(new List());
        if (t == "list")
          for (long long q = 0; q < c.i(3); ++q) l->l.push_back(S->obj.at(c.i(4 + q)));
        else l->l = S->grp.at(c.i(3));
        h = l;
      } else if (t == "bvh" || t == "bvh_group") {
        std::vector<const Hitable*> v;
        if (t == "bvh")
          for (long long q = 0; q < c.i(5); ++q) v.push_back(S->obj.at(c.i(6 + q)));
        else v = S->grp.at(c.i(5));
        h = build_bvh(St, v.data(), (int)v.size(), c.f(3), c.f(4), lcg);
      } else throw std::runtime_error("obj kind " + t);
      S->obj[id] = h;
      continue;
    }
    if (k == "camera") {
      S->cam.reset(new Camera(V3(c, 1), V3(c, 4), V3(c, 7), c.f(10), c.f(11), c.f(12), c.f(13), c.f(14), c.f(15)));
      continue;
    }
    if (k == "world") { S->world = S->obj.at(c.i(1)); continue; }
    if (k == "lights") {
      S->lights = dynamic_cast<const List*>(S->obj.at(c.i(1)));
      if (!S->lights) throw std::runtime_error("lights must be a hitable_list (Raytracing_n.cpp:75)");
      continue;
    }
    throw std::runtime_error("unknown command " + k);
  }
  if (!S->world || !S->lights || !S->cam) throw std::runtime_error("scene needs world, lights and camera");
  return S;
}

}  // namespace orc

// The Utah teapot data shared with the product tessellator (a data table, not logic).
#include "../include/srr/teapot_data.inc"

namespace orc {
// teapot.h:19-37 (Bezier evaluation) and :76-166 (tessellation), divs chosen.
static V bezier(const V* p, const float& t) {
  float b0 = (1 - t) * (1 - t) * (1 - t);
  float b1 = 3 * t * (1 - t) * (1 - t);
  float b2 = 3 * t * t * (1 - t);
  float b3 = t * t * t;
  return p[0] * b0 + p[1] * b1 + p[2] * b2 + p[3] * b3;
}
std::vector<const Hitable*> make_teapot(Store& St, float scale, int divs, const Material* m) {
  std::vector<V> P((divs + 1) * (divs + 1));
  std::vector<const Hitable*> tris;
  V cp[16];
  for (int np = 0; np < kSrrTeapotPatchCount; ++np) {
    for (int i = 0; i < 16; ++i)
      for (int c = 0; c < 3; ++c) cp[i][c] = kSrrTeapotVertex[kSrrTeapotPatch[np * 16 + i] * 3 + c] * scale;
    for (int j = 0, k = 0; j <= divs; ++j) {
      float v = (float)j / (float)divs;
      for (int i = 0; i <= divs; ++i, ++k) {
        float u = (float)i / (float)divs;
        V uc[4];
        for (int q = 0; q < 4; ++q) uc[q] = bezier(cp + 4 * q, u);
        P[k] = bezier(uc, v);
      }
    }
    for (int j = 0; j < divs; ++j)
      for (int i = 0; i < divs; ++i) {
        int q[4] = {(divs + 1) * j + i, (divs + 1) * j + i + 1, (divs + 1) * (j + 1) + i + 1, (divs + 1) * (j + 1) + i};
        for (int t = 0; t < 2; ++t) {
          Triangle* tr = St.add(new Triangle(P[q[0]], P[q[t + 1]], P[q[t + 2]], m));
          tr->n0 = tr->n1 = tr->n2 = tr->normal;
          tris.push_back(tr);
        }
      }
  }
  return tris;
}

thread_local std::string g_err;
}  // namespace orc

// =================================================================== C API
extern "C" {

const char* oracle_last_error() { return orc::g_err.c_str(); }

// Renders the pixels listed in `pixels` (PPM order index, row 0 = top) -- all
// pixels when pixels == NULL -- with per-path reseeding.  Outputs (any may be
// NULL): paths[n_pix*ns*3] raw color() per path (before de_nan), rays[n_pix*ns]
// world rays per path, img[n_pix*3] = mean of de_nan'd samples (before sqrt),
// img8[n_pix*3] tone-mapped (Raytracing_n.cpp:848-867).  stats[5] = world rays,
// box tests, triangle tests, analytic primitive tests, resampling loops stopped
// by the attempt cap (kMixtureGuard).
int oracle_render(const char* scene_text, int nx, int ny, int ns, int max_depth, const int* pixels, int n_pixels,
                  float* paths, unsigned char* rays, float* img, unsigned char* img8, long long* stats,
                  int n_threads) {
  try {
    std::unique_ptr<orc::Scene> S = orc::build(scene_text);
    std::vector<double> sp = orc::sobol2((unsigned)ns);
    int npix = pixels ? n_pixels : nx * ny;
    if (n_threads < 1) n_threads = 1;
    std::atomic<int> next(0);
    std::vector<orc::Counters> cnt(n_threads);
    auto work = [&](int tid) {
      orc::C = orc::Counters();
      for (;;) {
        int q = next.fetch_add(1);
        if (q >= npix) break;
        int pix = pixels ? pixels[q] : q;
        int i = pix % nx, j = ny - 1 - pix / nx;
        orc::V col(0, 0, 0);
        for (int s = 0; s < ns; ++s) {
          unsigned long long sd = srr_text::path_seed((unsigned)i, (unsigned)j, (unsigned)s);
          orc::R.lcg = sd;
          orc::R.pcg = 0x853c49e6748fea9bULL ^ (sd << 16);
          orc::R.inc = 0xda3e39cb94b95bdbULL;
          float u = float(sp[2 * s] + i) / float(nx);
          float v = float(sp[2 * s + 1] + j) / float(ny);
          orc::Ray r = S->cam->get_ray(u, v);
          int depth = 0;
          long long before = orc::C.world;
          orc::V c = orc::color(*S, r, &depth, max_depth);
          size_t p = (size_t)q * ns + s;
          if (paths) { paths[p * 3] = c[0]; paths[p * 3 + 1] = c[1]; paths[p * 3 + 2] = c[2]; }
          if (rays) rays[p] = (unsigned char)(orc::C.world - before);
          col += orc::de_nan(c);
        }
        col /= float(ns);
        if (img) { img[q * 3] = col[0]; img[q * 3 + 1] = col[1]; img[q * 3 + 2] = col[2]; }
        if (img8)
          for (int c = 0; c < 3; ++c) {
            int v = int(255.99 * std::sqrt(col[c]));
            img8[q * 3 + c] = (unsigned char)(v > 255 ? 255 : (v < 0 ? 0 : v));
          }
      }
      cnt[tid] = orc::C;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    if (stats) {
      stats[0] = stats[1] = stats[2] = stats[3] = stats[4] = 0;
      for (auto& c : cnt) {
        stats[0] += c.world; stats[1] += c.node; stats[2] += c.tri; stats[3] += c.prim; stats[4] += c.capped;
      }
    }
    return 0;
  } catch (const std::exception& e) {
    orc::g_err = e.what();
    return -1;
  }
}

int oracle_sobol(int n, double* out) {
  std::vector<double> p = orc::sobol2((unsigned)n);
  std::memcpy(out, p.data(), p.size() * sizeof(double));
  return 0;
}

int oracle_teapot(float scale, int divs, float* out) {  // p0 p1 p2 normal per triangle
  orc::Store st;
  auto tris = orc::make_teapot(st, scale, divs, nullptr);
  size_t k = 0;
  for (auto* h : tris) {
    const orc::Triangle* t = (const orc::Triangle*)h;
    for (const orc::V* v : {&t->p0, &t->p1, &t->p2, &t->normal})
      for (int c = 0; c < 3; ++c) out[k++] = (*v)[c];
  }
  return (int)tris.size();
}

}  // extern "C"

#include "restate_kat.inc"

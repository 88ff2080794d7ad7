// Host scene store, reference-compatible BVH builder, teapot tessellator, scene
// text parser and flattener.  Host arithmetic follows the reference's float /
// double promotions exactly (x86-64 baseline, no FMA), so the derived values
// the device reads (boxes, camera frame, rotation sin/cos, material constants)
// are bit-identical to the reference's.
#include "scene.h"

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iterator>
#include <map>
#include <sstream>

namespace srr {

static const double kPi = 3.14159265358979323846;  // mathf.h:10
static const uint64_t kPostPerlinSeed = 24561125610955ULL;

#include "../../include/srr/teapot_data.inc"

Scene::Scene() : lcg(kPostPerlinSeed) {}

double Scene::drand48() {  // mathf.h:14-19
  lcg = (0x5DEECE66DULL * lcg + 0xB16ULL) & 0xFFFFFFFFFFFFULL;
  unsigned x = (unsigned)(lcg >> 16);
  return (double)x / 4294967296.0;
}

// ----------------------------------------------------------------- small math
static inline float ffmin(float a, float b) { return a < b ? a : b; }  // aabb.h:7-8
static inline float ffmax(float a, float b) { return a > b ? a : b; }
static inline void cross3(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
static inline float len3(const float* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static inline void unit3(const float* v, float* o) {  // vec3.h:169-172
  float l = len3(v);
  o[0] = v[0] / l;
  o[1] = v[1] / l;
  o[2] = v[2] / l;
}
static inline Box3 surrounding(const Box3& a, const Box3& b) {  // aabb.h:54-62
  Box3 r;
  for (int k = 0; k < 3; ++k) {
    r.mn[k] = ffmin(a.mn[k], b.mn[k]);
    r.mx[k] = ffmax(a.mx[k], b.mx[k]);
  }
  return r;
}

// --------------------------------------------------------------- constructors
int Scene::add_tex(HTex t) {
  tex.push_back(std::move(t));
  return (int)tex.size() - 1;
}
int Scene::add_mat(HMat m) {
  mat.push_back(m);
  return (int)mat.size() - 1;
}
int Scene::add_obj(HObj o) {
  obj.push_back(std::move(o));
  return (int)obj.size() - 1;
}

// Derived constants exactly as the reference's constructors compute them.
int Scene::material(MatKind k, int t, const float* prm) {
  HMat m;
  m.kind = k;
  m.tex = t;
  switch (k) {
    case MAT_METAL:  // material.h:245: fuzz = f < 1 ? f : 1
      m.p[0] = prm[0]; m.p[1] = prm[1]; m.p[2] = prm[2];
      m.p[3] = (prm[3] < 1) ? prm[3] : 1;
      break;
    case MAT_DIELECTRIC:
      m.p[0] = prm[0];
      break;
    case MAT_ORENNAYAR: {  // material.h:129-133
      float sigma = prm[0];
      sigma = sigma / 180 * kPi;
      m.p[0] = 1 - 0.5 * sigma * sigma / (sigma * sigma + 0.33);
      m.p[1] = 0.45 * sigma * sigma / (sigma * sigma + 0.09);
      break;
    }
    case MAT_BECKMANN:  // material.h:153-157 via RoughnessToAlpha (microfacet_distribution.h:139-144)
      for (int q = 0; q < 2; ++q) {
        float r = std::fmax(prm[q], 1e-3f);
        float x = std::log(r);
        m.p[q] = 1.62162f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
      }
      break;
    default:
      break;
  }
  return add_mat(m);
}

int Scene::sphere(const float c[3], float r, int m) {
  HObj o;
  o.kind = H_SPHERE;
  o.mat = m;
  std::memcpy(o.f, c, 12);
  o.f[3] = r;
  return add_obj(o);
}

int Scene::moving_sphere(const float c0[3], const float c1[3], float t0, float t1, float r, int m) {
  HObj o;
  o.kind = H_MSPHERE;
  o.mat = m;
  std::memcpy(o.f, c0, 12);
  std::memcpy(o.f + 3, c1, 12);
  o.f[6] = t0;
  o.f[7] = t1;
  o.f[8] = r;
  return add_obj(o);
}

int Scene::rect(HKind k, float a0, float a1, float b0, float b1, float kk, int m) {
  HObj o;
  o.kind = k;
  o.mat = m;
  o.f[0] = a0; o.f[1] = a1; o.f[2] = b0; o.f[3] = b1; o.f[4] = kk;
  return add_obj(o);
}

int Scene::box(const float p0[3], const float p1[3], int m) {  // box.h:18-29
  int f[6];
  f[0] = rect(H_XY, p0[0], p1[0], p0[1], p1[1], p1[2], m);
  f[1] = wrap(H_FLIP, rect(H_XY, p0[0], p1[0], p0[1], p1[1], p0[2], m), nullptr);
  f[2] = rect(H_XZ, p0[0], p1[0], p0[2], p1[2], p1[1], m);
  f[3] = wrap(H_FLIP, rect(H_XZ, p0[0], p1[0], p0[2], p1[2], p0[1], m), nullptr);
  f[4] = rect(H_YZ, p0[1], p1[1], p0[2], p1[2], p1[0], m);
  f[5] = wrap(H_FLIP, rect(H_YZ, p0[1], p1[1], p0[2], p1[2], p0[0], m), nullptr);
  HObj o;
  o.kind = H_BOX;
  o.mat = m;
  std::memcpy(o.f, p0, 12);
  std::memcpy(o.f + 3, p1, 12);
  o.kids.assign(f, f + 6);
  return add_obj(o);
}

int Scene::triangle(const float p[9], int m, const float* uv9, const float* n9) {  // triangle.h:13-50
  HTri t;
  std::memcpy(t.p, p, 36);
  float e1[3] = {p[3] - p[0], p[4] - p[1], p[5] - p[2]};
  float e2[3] = {p[6] - p[0], p[7] - p[1], p[8] - p[2]};
  float c[3], nn[3];
  cross3(e1, e2, c);
  unit3(c, nn);
  if (n9) std::memcpy(t.n, n9, 36);
  else for (int k = 0; k < 3; ++k) std::memcpy(t.n + 3 * k, nn, 12);  // SURVEY Q5 build definition
  if (uv9) std::memcpy(t.uv, uv9, 36);
  else std::memset(t.uv, 0, 36);
  t.mat = m;
  tris.push_back(t);
  HObj o;
  o.kind = H_TRI;
  o.mat = m;
  o.tri = (int)tris.size() - 1;
  return add_obj(o);
}

int Scene::wrap(HKind k, int child, const float* f) {
  HObj o;
  o.kind = k;
  o.child = child;
  if (f) std::memcpy(o.f, f, 12);
  return add_obj(o);
}

int Scene::rotate(HKind k, int child, float angle) {  // hitable.h:81-107, 151-178
  HObj o;
  o.kind = k;
  o.child = child;
  float radians = (kPi / 180.) * angle;
  float s = std::sin(radians), c = std::cos(radians);
  o.f[0] = s;
  o.f[1] = c;
  Box3 b{};
  o.has_box = bbox(child, 0, 1, b);
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++)
      for (int kk = 0; kk < 2; kk++) {
        float x = i * b.mx[0] + (1 - i) * b.mn[0];
        float y = j * b.mx[1] + (1 - j) * b.mn[1];
        float z = kk * b.mx[2] + (1 - kk) * b.mn[2];
        float t[3];
        if (k == H_ROTY) {
          t[0] = c * x + s * z; t[1] = y; t[2] = -s * x + c * z;
        } else {
          t[0] = x; t[1] = c * y + s * z; t[2] = -s * y + c * z;
        }
        for (int q = 0; q < 3; q++) {
          if (t[q] > mx[q]) mx[q] = t[q];
          if (t[q] < mn[q]) mn[q] = t[q];
        }
      }
  std::memcpy(o.box.mn, mn, 12);
  std::memcpy(o.box.mx, mx, 12);
  return add_obj(o);
}

int Scene::medium(int boundary, float density, int t) {
  HObj o;
  o.kind = H_MEDIUM;
  o.child = boundary;
  o.f[0] = density;
  o.tex = t;
  return add_obj(o);
}

int Scene::list(const int* kids, int n) {
  HObj o;
  o.kind = H_LIST;
  o.kids.assign(kids, kids + n);
  return add_obj(o);
}

// glibc 2.35 qsort on an array of pointers is msort_with_tmp (stdlib/msort.c):
// top-down, n1 = n/2, and the merge takes the LEFT element when cmp <= 0.  With
// the reference's comparators (bvh.h:21-55, never 0) that fixes the order of
// equal keys, which fixes the BVH topology.
template <class T, class Cmp>
static void msort_rec(T* b, size_t n, T* tmp, Cmp cmp) {
  if (n <= 1) return;
  size_t n1 = n / 2, n2 = n - n1;
  T* b1 = b;
  T* b2 = b + n1;
  msort_rec(b1, n1, tmp, cmp);
  msort_rec(b2, n2, tmp, cmp);
  T* t = tmp;
  while (n1 > 0 && n2 > 0) {
    if (cmp(*b1, *b2) <= 0) { *t++ = *b1++; --n1; }
    else { *t++ = *b2++; --n2; }
  }
  if (n1 > 0) std::memcpy(t, b1, n1 * sizeof(T));
  std::memcpy(b, tmp, (n - n2) * sizeof(T));
}

int Scene::bvh(const int* kids, int n, float t0, float t1) {  // bvh.h:96-119
  HBvh B;
  B.input.assign(kids, kids + n);
  // the sort permutes POSITIONS into kids[]: the comparator reads its keys from
  // dense arrays (the same comparisons, so the same order, as sorting the
  // handles; a std::map lookup per comparison made a 640,000-triangle teapot's
  // build take 41 s)
  std::vector<int> l(n), tmp(n);
  for (int i = 0; i < n; ++i) l[i] = i;
  // box minima at times (0, 0) for the comparator, boxes at (t0, t1) for the nodes
  std::vector<float> key[3];
  for (auto& k : key) k.resize(n);
  std::vector<Box3> boxT(n);
  for (int i = 0; i < n; ++i) {
    Box3 b{};
    bbox(kids[i], 0, 0, b);
    for (int a = 0; a < 3; ++a) key[a][i] = b.mn[a];
    bbox(kids[i], t0, t1, b);
    boxT[i] = b;
  }
  std::function<int(int*, int)> build = [&](int* a, int m) -> int {
    int axis = int(3 * drand48());
    const float* kx = key[axis].data();
    auto cmp = [kx](int x, int y) { return (kx[x] - kx[y] < 0.0) ? -1 : 1; };
    msort_rec(a, (size_t)m, tmp.data(), cmp);
    int me = (int)B.nodes.size();
    B.nodes.push_back(HBvh::Node{});
    int L, R;
    Box3 bl, br;
    if (m <= 2) {
      auto leaf = [&](int pos) {
        B.leaves.push_back(kids[pos]);
        return ~((int)B.leaves.size() - 1);
      };
      L = leaf(a[0]);
      R = (m == 1) ? L : leaf(a[1]);
      bl = boxT[a[0]];
      br = boxT[a[m - 1]];
    } else {
      L = build(a, m / 2);
      R = build(a + m / 2, m - m / 2);
      bl = B.nodes[L].box;
      br = B.nodes[R].box;
    }
    B.nodes[me].left = L;
    B.nodes[me].right = R;
    B.nodes[me].box = surrounding(bl, br);
    return me;
  };
  if (n < 1) return -22;
  build(l.data(), n);
  B.box = B.nodes[0].box;
  bvhs.push_back(std::move(B));
  HObj o;
  o.kind = H_BVH;
  o.bvh = (int)bvhs.size() - 1;
  return add_obj(o);
}

void teapot_triangles(float scale, int divs, std::vector<float>& out) {  // teapot.h:19-37, 76-166
  auto bez = [](const float* p, const float& t, float* o) {
    float b0 = (1 - t) * (1 - t) * (1 - t);
    float b1 = 3 * t * (1 - t) * (1 - t);
    float b2 = 3 * t * t * (1 - t);
    float b3 = t * t * t;
    for (int c = 0; c < 3; ++c) o[c] = p[c] * b0 + p[3 + c] * b1 + p[6 + c] * b2 + p[9 + c] * b3;
  };
  std::vector<float> P((size_t)(divs + 1) * (divs + 1) * 3);
  out.clear();
  out.reserve((size_t)kSrrTeapotPatchCount * divs * divs * 2 * 9);
  float cp[48];
  for (int np = 0; np < kSrrTeapotPatchCount; ++np) {
    for (int i = 0; i < 16; ++i)
      for (int c = 0; c < 3; ++c) cp[i * 3 + c] = kSrrTeapotVertex[kSrrTeapotPatch[np * 16 + i] * 3 + c] * scale;
    for (int j = 0, k = 0; j <= divs; ++j) {
      float v = (float)j / (float)divs;
      for (int i = 0; i <= divs; ++i, ++k) {
        float u = (float)i / (float)divs;
        float uc[12];
        for (int q = 0; q < 4; ++q) bez(cp + 12 * q, u, uc + 3 * q);
        bez(uc, v, &P[(size_t)k * 3]);
      }
    }
    for (int j = 0; j < divs; ++j)
      for (int i = 0; i < divs; ++i) {
        int q[4] = {(divs + 1) * j + i, (divs + 1) * j + i + 1, (divs + 1) * (j + 1) + i + 1, (divs + 1) * (j + 1) + i};
        for (int t = 0; t < 2; ++t)
          for (int c : {q[0], q[t + 1], q[t + 2]})
            for (int d = 0; d < 3; ++d) out.push_back(P[(size_t)c * 3 + d]);
      }
  }
}

int Scene::teapot(float scale, int divs, int m, int* first) {
  std::vector<float> p;
  teapot_triangles(scale, divs, p);
  int n = (int)(p.size() / 9);
  int f = -1;
  for (int i = 0; i < n; ++i) {
    int h = triangle(&p[(size_t)i * 9], m, nullptr, nullptr);
    if (i == 0) f = h;
  }
  if (first) *first = f;
  return n;
}

void Scene::camera(const float lf[3], const float la[3], const float vup[3], float vfov, float aspect,
                   float aperture, float focus, float t0, float t1) {  // camera.h:33-48
  HCamera& C = cam;
  C.time0 = t0;
  C.time1 = t1;
  C.lens_radius = aperture / 2;
  float theta = vfov * kPi / 180;
  float half_height = std::tan(theta / 2);
  float half_width = aspect * half_height;
  std::memcpy(C.origin, lf, 12);
  float d[3] = {lf[0] - la[0], lf[1] - la[1], lf[2] - la[2]};
  float w[3], uu[3], vv[3], c[3];
  unit3(d, w);
  cross3(vup, w, c);
  unit3(c, uu);
  cross3(w, uu, vv);
  for (int k = 0; k < 3; ++k) {
    // origin - hw*focus*u - hh*focus*v - focus*w, evaluated left to right
    float a = half_width * focus * uu[k];
    float b = half_height * focus * vv[k];
    float e = focus * w[k];
    C.llc[k] = C.origin[k] - a - b - e;
    C.horizontal[k] = 2 * half_width * focus * uu[k];
    C.vertical[k] = 2 * half_height * focus * vv[k];
    C.u[k] = uu[k];
    C.v[k] = vv[k];
  }
  has_camera = true;
}

// ------------------------------------------------------------ bounding boxes
bool Scene::bbox(int h, float t0, float t1, Box3& b) const {
  const HObj& o = obj[h];
  switch (o.kind) {
    case H_SPHERE:  // sphere.h:31-34
      for (int k = 0; k < 3; ++k) { b.mn[k] = o.f[k] - o.f[3]; b.mx[k] = o.f[k] + o.f[3]; }
      return true;
    case H_MSPHERE: {  // moving_sphere.h:19-21, 53-59
      auto center = [&](float tm, float* c) {
        float s = (tm - o.f[6]) / (o.f[7] - o.f[6]);
        for (int k = 0; k < 3; ++k) c[k] = o.f[k] + s * (o.f[3 + k] - o.f[k]);
      };
      float c0[3], c1[3];
      center(t0, c0);
      center(t1, c1);
      Box3 a, bb;
      for (int k = 0; k < 3; ++k) {
        a.mn[k] = c0[k] - o.f[8]; a.mx[k] = c0[k] + o.f[8];
        bb.mn[k] = c1[k] - o.f[8]; bb.mx[k] = c1[k] + o.f[8];
      }
      b = surrounding(a, bb);
      return true;
    }
    case H_XY: case H_XZ: case H_YZ: {  // aarect.h:11-14, 41-44, 72-75
      int kax = o.kind == H_XY ? 2 : (o.kind == H_XZ ? 1 : 0);
      int a0 = o.kind == H_YZ ? 1 : 0;
      int a1 = o.kind == H_XY ? 1 : 2;
      b.mn[a0] = o.f[0]; b.mx[a0] = o.f[1];
      b.mn[a1] = o.f[2]; b.mx[a1] = o.f[3];
      b.mn[kax] = o.f[4] - 0.0001;
      b.mx[kax] = o.f[4] + 0.0001;
      return true;
    }
    case H_BOX:  // box.h:10-13
      for (int k = 0; k < 3; ++k) { b.mn[k] = o.f[k]; b.mx[k] = o.f[3 + k]; }
      return true;
    case H_TRI: {  // triangle.h:53-68
      const float* p = tris[o.tri].p;
      for (int k = 0; k < 3; ++k) {
        b.mn[k] = ffmin(ffmin(p[k], p[3 + k]), p[6 + k]);
        b.mx[k] = ffmax(ffmax(p[k], p[3 + k]), p[6 + k]);
      }
      return true;
    }
    case H_FLIP:
      return bbox(o.child, t0, t1, b);
    case H_TRANSLATE:  // hitable.h:54-61 (degenerate (Max+off, Max+off))
      if (bbox(o.child, t0, t1, b)) {
        for (int k = 0; k < 3; ++k) b.mn[k] = b.mx[k] = b.mx[k] + o.f[k];
        return true;
      }
      return false;
    case H_ROTY: case H_ROTX:
      b = o.box;
      return o.has_box;
    case H_MEDIUM:
      return bbox(o.child, t0, t1, b);
    case H_LIST: {  // hitable_list.h:35-52 (merges list[0] only)
      if (o.kids.empty()) return false;
      Box3 tb;
      if (!bbox(o.kids[0], t0, t1, tb)) return false;
      b = tb;
      for (size_t i = 0; i < o.kids.size(); ++i) {
        if (bbox(o.kids[0], t0, t1, tb)) b = surrounding(b, tb);
        else return false;
      }
      return true;
    }
    case H_BVH:
      b = bvhs[o.bvh].box;
      return true;
  }
  return false;
}

// ---------------------------------------------------------------- utilities
uint64_t path_seed(uint32_t x, uint32_t y, uint32_t s, uint64_t base) {
  uint64_t h = 0xcbf29ce484222325ULL ^ base;
  const uint32_t w[3] = {x, y, s};
  for (int k = 0; k < 3; ++k)
    for (int b = 0; b < 4; ++b) {
      h ^= (w[k] >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ULL;
    }
  return h & 0xFFFFFFFFFFFFULL;
}

void sobol2(unsigned N, double* pts) {  // Raytracing_n.cpp:721-812, D = 2
  unsigned L = (unsigned)std::ceil(std::log((double)N) / std::log(2.0));
  std::vector<unsigned> C(N ? N : 1);
  C[0] = 1;
  for (unsigned i = 1; i + 1 <= N; i++) {
    C[i] = 1;
    unsigned v = i;
    while (v & 1) { v >>= 1; C[i]++; }
  }
  // dimension 1: all m_i = 1; dimension 2: joe-kuo line "2 1 0 1" (s=1, a=0, m1=1)
  std::vector<unsigned> V1(L + 1), V2(L + 1);
  for (unsigned i = 1; i <= L; i++) V1[i] = 1u << (32 - i);
  if (L >= 1) V2[1] = 1u << 31;
  for (unsigned i = 2; i <= L; i++) V2[i] = V2[i - 1] ^ (V2[i - 1] >> 1);
  if (N) { pts[0] = 0; pts[1] = 0; }
  unsigned X1 = 0, X2 = 0;
  for (unsigned i = 1; i + 1 <= N; i++) {
    X1 ^= V1[C[i - 1]];
    X2 ^= V2[C[i - 1]];
    pts[2 * i] = (double)X1 / std::pow(2.0, 32);
    pts[2 * i + 1] = (double)X2 / std::pow(2.0, 32);
  }
}

static inline uint32_t hash32(uint32_t a) {
  a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
  return a;
}

std::vector<uint8_t> gen_image(int w, int h, uint32_t seed, int kind) {
  std::vector<uint8_t> px((size_t)w * h * 3);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      uint32_t n = hash32(seed * 0x9E3779B9u ^ hash32((uint32_t)(y * w + x)));
      int r, g, b;
      if (kind == 0) {
        int t = (y * 255) / (h > 1 ? h - 1 : 1);
        r = 90 + (t * 120) / 255 + (int)(n & 15);
        g = 140 + (t * 90) / 255 + (int)((n >> 4) & 15);
        b = 235 - (t * 60) / 255 + (int)((n >> 8) & 15);
      } else if (kind == 1) {
        int band = ((x * 7 + (int)((n >> 3) & 7)) / 13) & 15;
        r = 110 + band * 6 + (int)(n & 7);
        g = 70 + band * 4 + (int)((n >> 5) & 7);
        b = 40 + band * 2 + (int)((n >> 9) & 7);
      } else {
        int c = ((x >> 3) ^ (y >> 3)) & 1;
        r = g = b = c ? 230 : 25;
      }
      uint8_t* p = &px[((size_t)y * w + x) * 3];
      p[0] = (uint8_t)(r > 255 ? 255 : r);
      p[1] = (uint8_t)(g > 255 ? 255 : g);
      p[2] = (uint8_t)(b > 255 ? 255 : b);
    }
  return px;
}

// Perlin tables (perlin.h:67-97): the reference builds them in static
// initialisers from the global LCG at seed 1; vec3 arguments evaluate right to
// left under g++, so each ranvec draws z, y, x.
static void perlin_tables(std::vector<float>& ranvec, std::vector<int32_t>& perm) {
  uint64_t s = 1;
  auto dr = [&]() {
    s = (0x5DEECE66DULL * s + 0xB16ULL) & 0xFFFFFFFFFFFFULL;
    return (double)(unsigned)(s >> 16) / 4294967296.0;
  };
  ranvec.resize(256 * 3);
  for (int i = 0; i < 256; ++i) {
    float z = -1 + 2 * dr();
    float y = -1 + 2 * dr();
    float x = -1 + 2 * dr();
    float v[3] = {x, y, z}, u[3];
    unit3(v, u);
    std::memcpy(&ranvec[i * 3], u, 12);
  }
  perm.resize(3 * 256);
  for (int t = 0; t < 3; ++t) {
    int32_t* p = &perm[t * 256];
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int i = 255; i > 0; i--) {
      int target = int(dr() * (i + 1));
      std::swap(p[i], p[target]);
    }
  }
}

// ----------------------------------------------------------------- flattening
namespace {
struct Flattener {
  const Scene& S;
  Flat& F;
  std::string& err;
  std::map<int, int> mesh_of_bvh;
  std::vector<DObj> world, bound, inner;  // inner: object-BVH children
  std::map<int, int> rect_row, sphere_row;

  int chain_push(const std::vector<DXform>& ch) {
    int b = (int)F.xforms.size();
    F.xforms.insert(F.xforms.end(), ch.begin(), ch.end());
    return b;
  }
  int add_rect(int h) {
    auto it = rect_row.find(h);
    if (it != rect_row.end()) return it->second;
    const HObj& o = S.obj[h];
    DRect r{};
    r.kax = o.kind == H_XY ? 2 : (o.kind == H_XZ ? 1 : 0);
    r.a0 = o.kind == H_YZ ? 1 : 0;
    r.a1 = o.kind == H_XY ? 1 : 2;
    r.lo0 = o.f[0]; r.hi0 = o.f[1]; r.lo1 = o.f[2]; r.hi1 = o.f[3]; r.k = o.f[4];
    r.mat = o.mat;
    F.rects.push_back(r);
    return rect_row[h] = (int)F.rects.size() - 1;
  }
  int add_sphere(int h) {
    auto it = sphere_row.find(h);
    if (it != sphere_row.end()) return it->second;
    const HObj& o = S.obj[h];
    DSphere s{};
    if (o.kind == H_SPHERE) {
      for (int k = 0; k < 3; ++k) s.c0[k] = s.c1[k] = o.f[k];
      s.t0 = 0; s.t1 = 1; s.r = o.f[3];
    } else {
      for (int k = 0; k < 3; ++k) { s.c0[k] = o.f[k]; s.c1[k] = o.f[3 + k]; }
      s.t0 = o.f[6]; s.t1 = o.f[7]; s.r = o.f[8];
    }
    s.mat = o.mat;
    F.spheres.push_back(s);
    return sphere_row[h] = (int)F.spheres.size() - 1;
  }
  int add_stri(int h) {
    const HTri& t = S.tris[S.obj[h].tri];
    DStandaloneTri d{};
    std::memcpy(d.p, t.p, 36);
    std::memcpy(d.sh.n, t.n, 36);
    for (int k = 0; k < 3; ++k) { d.sh.uv[2 * k] = t.uv[3 * k]; d.sh.uv[2 * k + 1] = t.uv[3 * k + 1]; }
    d.sh.mat = t.mat;
    F.stris.push_back(d);
    return (int)F.stris.size() - 1;
  }
  // 4-wide BVH for near-first traversal with closest-hit pruning (kernels.hip
  // mesh_hit4).  The reference's result over a mesh depends only on which of its
  // LEAF boxes (1-2 triangles each, bvh.h:104-110) the ray's slab test passes:
  // every ancestor box contains its leaves, so an ancestor passes whenever a leaf
  // does.  Any hierarchy over the reference's exact leaf boxes therefore reaches
  // the same leaves.  By default the hierarchy is rebuilt with a binned SAH over
  // the leaf units (the reference splits at the median of a random axis, which
  // leaves loose, overlapping boxes); SRR_BVH4=ref collapses the reference
  // topology instead.  Leaf slots hold the reference's leaf box unchanged; inner
  // boxes are exact unions of their children.
  struct TNode {
    Box3 box;
    int left = -1, right = -1;
    int code = -1;  // leaf unit: (first triangle << 1) | (count - 1)
  };
  static float box_area(const Box3& b) {
    float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return dx * dy + dy * dz + dz * dx;
  }
  static Box3 box_union(const Box3& a, const Box3& b) {
    Box3 r;
    for (int k = 0; k < 3; ++k) {
      r.mn[k] = std::min(a.mn[k], b.mn[k]);
      r.mx[k] = std::max(a.mx[k], b.mx[k]);
    }
    return r;
  }
  static std::vector<TNode> tree_from_reference(const HBvh& B, int tri_off) {
    std::vector<TNode> T(B.nodes.size());
    for (size_t i = 0; i < B.nodes.size(); ++i) {
      const HBvh::Node& n = B.nodes[i];
      T[i].box = n.box;
      if (n.left < 0) {
        int first = ~n.left, last = ~n.right;
        T[i].code = ((first + tri_off) << 1) | (last != first ? 1 : 0);
      } else {
        T[i].left = n.left;
        T[i].right = n.right;
      }
    }
    return T;
  }
  static std::vector<TNode> tree_sah(const HBvh& B, int tri_off) {
    std::vector<TNode> units;
    for (const HBvh::Node& n : B.nodes)
      if (n.left < 0) {
        TNode u;
        u.box = n.box;
        int first = ~n.left, last = ~n.right;
        u.code = ((first + tri_off) << 1) | (last != first ? 1 : 0);
        units.push_back(u);
      }
    std::vector<TNode> T;
    T.reserve(2 * units.size());
    auto centroid = [](const TNode& u, int a) { return 0.5f * (u.box.mn[a] + u.box.mx[a]); };
    std::function<int(int, int)> build = [&](int lo, int hi) -> int {
      const int me = (int)T.size();
      T.push_back(TNode{});
      if (hi - lo == 1) {
        T[me] = units[lo];
        return me;
      }
      Box3 box = units[lo].box, cb;
      for (int a = 0; a < 3; ++a) cb.mn[a] = cb.mx[a] = centroid(units[lo], a);
      for (int i = lo; i < hi; ++i) {
        box = box_union(box, units[i].box);
        for (int a = 0; a < 3; ++a) {
          cb.mn[a] = std::min(cb.mn[a], centroid(units[i], a));
          cb.mx[a] = std::max(cb.mx[a], centroid(units[i], a));
        }
      }
      // SAH bins (SRR_SAH_BINS; 0 = full sweep).  Measured on C2 / 640k teapot / C4:
      // 16 bins 7,815 / 990 / -- Msamples/s, 64 bins 7,948 / 1,038 / 3,786, full sweep
      // 7,928 / 1,031 / 3,767
      static const int kBins = [] {
        const char* e = getenv("SRR_SAH_BINS");
        const int b = e ? atoi(e) : 64;
        return b == 0 || (b >= 2 && b <= 256) ? b : 64;
      }();
      if (kBins == 0) {  // full-sweep SAH: every split of the centroid order on each axis
        int best_axis = -1, best_k = -1;
        float best_cost = INFINITY;
        std::vector<float> rarea(hi - lo + 1);
        for (int a = 0; a < 3; ++a) {
          std::sort(units.begin() + lo, units.begin() + hi,
                    [&](const TNode& x, const TNode& y) { return centroid(x, a) < centroid(y, a); });
          Box3 acc = units[hi - 1].box;
          for (int i = hi - 1; i > lo; --i) {
            acc = box_union(acc, units[i].box);
            rarea[i - lo] = box_area(acc);
          }
          acc = units[lo].box;
          for (int i = lo + 1; i < hi; ++i) {  // left = [lo, i), right = [i, hi)
            const float cost = box_area(acc) * (i - lo) + rarea[i - lo] * (hi - i);
            if (cost < best_cost) { best_cost = cost; best_axis = a; best_k = i; }
            acc = box_union(acc, units[i].box);
          }
        }
        if (best_axis != 2)
          std::sort(units.begin() + lo, units.begin() + hi,
                    [&](const TNode& x, const TNode& y) { return centroid(x, best_axis) < centroid(y, best_axis); });
        const int l = build(lo, best_k);
        const int r = build(best_k, hi);
        T[me].box = box;
        T[me].left = l;
        T[me].right = r;
        return me;
      }
      int best_axis = -1, best_bin = -1;
      float best_cost = INFINITY;
      for (int a = 0; a < 3; ++a) {
        const float ext = cb.mx[a] - cb.mn[a];
        if (!(ext > 0.f)) continue;
        Box3 bb[256];
        int bn[256] = {};
        for (int i = lo; i < hi; ++i) {
          int b = std::min(kBins - 1, (int)(kBins * (centroid(units[i], a) - cb.mn[a]) / ext));
          bb[b] = bn[b] ? box_union(bb[b], units[i].box) : units[i].box;
          ++bn[b];
        }
        // the right sides of every split by one sweep from the top bin (box unions
        // are exact min / max, so the same boxes as unioning each side anew)
        Box3 rb[256];
        int rn[256];
        {
          Box3 R{};
          int nr = 0;
          for (int b = kBins - 1; b >= 1; --b) {
            if (bn[b]) { R = nr ? box_union(R, bb[b]) : bb[b]; nr += bn[b]; }
            rb[b] = R;
            rn[b] = nr;
          }
        }
        Box3 L{};
        int nl = 0;
        for (int s = 0; s < kBins - 1; ++s) {  // split after bin s
          if (bn[s]) { L = nl ? box_union(L, bb[s]) : bb[s]; nl += bn[s]; }
          const int nr = rn[s + 1];
          if (!nl || !nr) continue;
          float cost = box_area(L) * nl + box_area(rb[s + 1]) * nr;
          if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = s; }
        }
      }
      int mid;
      if (best_axis >= 0) {
        const int a = best_axis;
        const float ext = cb.mx[a] - cb.mn[a];
        auto it = std::partition(units.begin() + lo, units.begin() + hi, [&](const TNode& u) {
          return std::min(kBins - 1, (int)(kBins * (centroid(u, a) - cb.mn[a]) / ext)) <= best_bin;
        });
        mid = (int)(it - units.begin());
      } else {
        mid = (lo + hi) / 2;  // coincident centroids
      }
      if (mid <= lo || mid >= hi) mid = (lo + hi) / 2;
      const int l = build(lo, mid);
      const int r = build(mid, hi);
      T[me].box = box;
      T[me].left = l;
      T[me].right = r;
      return me;
    };
    build(0, (int)units.size());
    return T;
  }
  // SAH cost weights of the 4-wide walk (mesh_hit4): one node step tests 4 child
  // boxes; a leaf unit's 1-2 triangle tests cost kSahTri each.  Relative to the
  // root's area, as probabilities of a random ray reaching a box.
  static constexpr double kSahNode4 = 1.0, kSahNode2 = 0.5, kSahTri = 1.2;

  static int leaf_tris(const TNode& n) { return (n.code & 1) + 1; }

  // Treelet restructuring (Karras & Aila 2013) of the binary hierarchy over the
  // fixed leaf units: every treelet of up to 7 nodes' subtrees (its "leaves" may be
  // inner nodes) is rebuilt with the topology of least SAH cost, found by dynamic
  // programming over the subsets of those subtrees; a few bottom-up passes.  Leaf
  // units are never split or merged (they are the reference's leaves, whose slab
  // tests decide which triangles the reference tests), so any topology is exact.
  static void restructure(std::vector<TNode>& T, int root, int passes) {
    const int N = (int)T.size();
    std::vector<double> cost(N), area(N);
    std::vector<int> parent(N, -1);
    std::function<void(int)> eval = [&](int n) {
      area[n] = box_area(T[n].box);
      if (T[n].code >= 0) {
        cost[n] = kSahTri * leaf_tris(T[n]) * area[n];
        return;
      }
      parent[T[n].left] = n;
      parent[T[n].right] = n;
      eval(T[n].left);
      eval(T[n].right);
      cost[n] = kSahNode2 * area[n] + cost[T[n].left] + cost[T[n].right];
    };
    constexpr int K = 7;
    // per-treelet DP tables, reused (fixed size: 2^K subsets)
    Box3 sbox[1 << K];
    double sa[1 << K], copt[1 << K];
    int split[1 << K];
    for (int pass = 0; pass < passes; ++pass) {
      eval(root);
      const double cost_before = cost[root];
      // post-order list of inner nodes
      std::vector<int> order;
      std::function<void(int)> post = [&](int n) {
        if (T[n].code >= 0) return;
        post(T[n].left);
        post(T[n].right);
        order.push_back(n);
      };
      post(root);
      for (int tr : order) {
        // grow the treelet: repeatedly open the largest-area treelet leaf that is inner
        std::vector<int> leaves{T[tr].left, T[tr].right}, inner{tr};
        while ((int)leaves.size() < K) {
          int best = -1;
          double ba = -1;
          for (int k = 0; k < (int)leaves.size(); ++k)
            if (T[leaves[k]].code < 0 && area[leaves[k]] > ba) { ba = area[leaves[k]]; best = k; }
          if (best < 0) break;
          const int n = leaves[best];
          inner.push_back(n);
          leaves[best] = T[n].left;
          leaves.push_back(T[n].right);
        }
        const int nl = (int)leaves.size();
        if (nl < 3) continue;
        const int full = (1 << nl) - 1;
        for (int sset = 0; sset <= full; ++sset) split[sset] = 0;
        for (int sset = 1; sset <= full; ++sset) {
          bool first = true;
          for (int k = 0; k < nl; ++k)
            if (sset >> k & 1) {
              sbox[sset] = first ? T[leaves[k]].box : box_union(sbox[sset], T[leaves[k]].box);
              first = false;
            }
          sa[sset] = box_area(sbox[sset]);
        }
        for (int k = 0; k < nl; ++k) copt[1 << k] = cost[leaves[k]];
        for (int sset = 1; sset <= full; ++sset) {
          if ((sset & (sset - 1)) == 0) continue;
          double best = INFINITY;
          int bsplit = 0;
          // every split into two non-empty halves (each unordered pair once)
          for (int p = (sset - 1) & sset; p > 0; p = (p - 1) & sset) {
            const int q = sset ^ p;
            if (p < q) continue;
            const double c = copt[p] + copt[q];
            if (c < best) { best = c; bsplit = p; }
          }
          copt[sset] = kSahNode2 * sa[sset] + best;
          split[sset] = bsplit;
        }
        if (copt[full] + 1e-9 * copt[full] >= cost[tr]) continue;  // no better topology
        // rebuild the treelet with the optimal topology, reusing its inner nodes
        int next_inner = 1;  // inner[0] = tr stays the treelet root
        std::function<int(int, int)> emit = [&](int sset, int node) -> int {
          if ((sset & (sset - 1)) == 0) {
            for (int k = 0; k < nl; ++k)
              if (sset == (1 << k)) return leaves[k];
          }
          const int me = node >= 0 ? node : inner[next_inner++];
          const int p = split[sset];
          const int l = emit(p, -1), r = emit(sset ^ p, -1);
          T[me].left = l;
          T[me].right = r;
          T[me].code = -1;
          T[me].box = sbox[sset];
          cost[me] = kSahNode2 * sa[sset] + cost[l] + cost[r];
          area[me] = sa[sset];
          return me;
        };
        emit(full, tr);
      }
      // a pass that gained under 0.1 % of the SAH cost ends the restructuring
      eval(root);
      if (getenv("SRR_BVH_STATS"))
        fprintf(stderr, "srr treelets: pass %d SAH %.6g -> %.6g\n", pass, cost_before, cost[root]);
      if (!(cost[root] < cost_before * 0.999)) break;
    }
  }

  // SAH cost of the 4-wide hierarchy the collapse below makes of T (relative to
  // the root area): node steps plus triangle tests, kSahNode4 / kSahTri weights
  struct Collapse {
    const std::vector<TNode>& T;
    std::vector<std::array<double, 5>> f;  // f[n][k]: least cost of n's subtree as k slots
    std::vector<std::array<int, 5>> pick;  // the left child's share of the k slots
    explicit Collapse(const std::vector<TNode>& t) : T(t), f(t.size()), pick(t.size()) {
      for (auto& a : f) a.fill(-1.0);
    }
    // one slot holding n: a leaf unit (its triangle tests) or a 4-wide node
    double slot(int n) {
      const TNode& t = T[n];
      if (t.code >= 0) return kSahTri * leaf_tris(t) * box_area(t.box);
      double best = INFINITY;
      for (int k = 2; k <= 4; ++k) best = std::min(best, open(n, k));
      return kSahNode4 * box_area(t.box) + best;
    }
    // n opened into exactly k slots (k >= 2) split between its children
    double open(int n, int k) {
      if (f[n][k] >= 0) return f[n][k];
      const TNode& t = T[n];
      double best = INFINITY;
      int bi = 0;
      for (int i = 1; i < k; ++i) {
        const double c = slots(t.left, i) + slots(t.right, k - i);
        if (c < best) { best = c; bi = i; }
      }
      pick[n][k] = bi;
      return f[n][k] = best;
    }
    double slots(int n, int k) {  // n's subtree as exactly k slots
      if (k == 1) return slot(n);
      if (T[n].code >= 0) return INFINITY;
      return open(n, k);
    }
    // the k slots chosen for n's subtree
    void cut(int n, int k, std::vector<int>& out) {
      if (k == 1) { out.push_back(n); return; }
      open(n, k);
      const int i = pick[n][k];
      cut(T[n].left, i, out);
      cut(T[n].right, k - i, out);
    }
    // the children of n as a 4-wide node: the best k in 2..4
    std::vector<int> children(int n) {
      int bk = 2;
      double best = INFINITY;
      for (int k = 2; k <= 4; ++k)
        if (open(n, k) < best) { best = open(n, k); bk = k; }
      std::vector<int> out;
      cut(n, bk, out);
      return out;
    }
  };

  void build_node4(const HBvh& B, DMesh& m) {
    static const bool ref_topology = [] {
      const char* e = getenv("SRR_BVH4");
      return e && !strcmp(e, "ref");
    }();
    // SRR_BVH_OPT: 0 = binned SAH + greedy collapse (round 3), 1 = + treelet
    // restructuring + SAH-optimal collapse (default)
    static const int opt = [] {
      const char* e = getenv("SRR_BVH_OPT");
      return e ? atoi(e) : 1;
    }();
    std::vector<TNode> T = ref_topology ? tree_from_reference(B, m.tri_off) : tree_sah(B, m.tri_off);
    const int root = 0;
    if (!ref_topology && opt >= 1 && T.size() > 2) restructure(T, root, 3);
    Collapse col(T);
    m.node4_off = (int)(F.node4.size() / 32);
    double sah4 = 0;  // SAH cost of the 4-wide hierarchy built (SRR_BVH_STATS)
    std::function<int(int)> build = [&](int top) -> int {
      std::vector<int> kids{top};
      if (!ref_topology && opt >= 1 && T[top].code < 0) {
        kids = col.children(top);
      } else {
        while (kids.size() < 4) {  // open the largest inner node until 4 children
          int best = -1;
          float ba = -1.f;
          for (size_t k = 0; k < kids.size(); ++k)
            if (T[kids[k]].code < 0 && box_area(T[kids[k]].box) > ba) { ba = box_area(T[kids[k]].box); best = (int)k; }
          if (best < 0) break;
          const TNode n = T[kids[best]];
          kids[best] = n.left;
          kids.insert(kids.begin() + best + 1, n.right);
        }
      }
      sah4 += kSahNode4 * box_area(T[top].box);
      for (int k : kids)
        if (T[k].code >= 0) sah4 += kSahTri * leaf_tris(T[k]) * box_area(T[k].box);
      const int me = (int)(F.node4.size() / 32);
      F.node4.resize(F.node4.size() + 32);
      int32_t child[4] = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};  // empty: never descended
      float lo[3][4], hi[3][4];
      for (int c = 0; c < 4; ++c) {
        for (int a = 0; a < 3; ++a) { lo[a][c] = INFINITY; hi[a][c] = -INFINITY; }  // empty slot
        if (c >= (int)kids.size()) continue;
        const TNode& n = T[kids[c]];
        for (int a = 0; a < 3; ++a) { lo[a][c] = n.box.mn[a]; hi[a][c] = n.box.mx[a]; }
        child[c] = n.code >= 0 ? ~n.code : build(kids[c]);
      }
      float* d = &F.node4[32 * (size_t)me];
      for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 4; ++c) { d[4 * a + c] = lo[a][c]; d[12 + 4 * a + c] = hi[a][c]; }
      std::memcpy(d + 24, child, 16);
      return me;
    };
    build(root);
    m.n_node4 = (int)(F.node4.size() / 32) - m.node4_off;
    if (getenv("SRR_BVH_STATS"))
      fprintf(stderr, "srr bvh4: %d leaf units, %d nodes, SAH cost %.4f (x root area)\n", (int)(T.size() + 1) / 2,
              m.n_node4, sah4 / std::max(1e-30, (double)box_area(T[root].box)));
    // breadth-first layout: the top levels come first, so the path kernel can
    // keep a prefix of the array in LDS (SceneView::node4_lds)
    std::vector<int> order{m.node4_off}, newidx(F.node4.size() / 32, -1);
    for (size_t i = 0; i < order.size(); ++i) {
      newidx[order[i]] = m.node4_off + (int)i;
      int32_t ch[4];
      std::memcpy(ch, &F.node4[32 * (size_t)order[i] + 24], 16);
      for (int c = 0; c < 4; ++c)
        if (ch[c] >= 0) order.push_back(ch[c]);
    }
    std::vector<float> bfs(32 * order.size());
    for (size_t i = 0; i < order.size(); ++i) {
      std::memcpy(&bfs[32 * i], &F.node4[32 * (size_t)order[i]], 32 * sizeof(float));
      int32_t ch[4];
      std::memcpy(ch, &bfs[32 * i + 24], 16);
      for (int c = 0; c < 4; ++c)
        if (ch[c] >= 0) ch[c] = newidx[ch[c]];
      std::memcpy(&bfs[32 * i + 24], ch, 16);
    }
    std::copy(bfs.begin(), bfs.end(), F.node4.begin() + 32 * (size_t)m.node4_off);
  }

  int add_mesh(int h) {  // a bvh_node whose leaves are all bare triangles
    auto it = mesh_of_bvh.find(h);
    if (it != mesh_of_bvh.end()) return it->second;
    const HBvh& B = S.bvhs[S.obj[h].bvh];
    for (int l : B.leaves)
      if (S.obj[l].kind != H_TRI) return -1;
    DMesh m{};
    m.node_off = (int)(F.nodes.size() / 8);
    m.tri_off = (int)(F.tri_shade.size());
    m.n_nodes = (int)B.nodes.size();
    m.n_tris = (int)B.leaves.size();
    // Threaded (stackless) layout: HBvh nodes are already in preorder with the
    // left child at i + 1; skip[i] = i + size(subtree i) is where a traversal
    // goes when it is done with, or prunes, node i.  Leaves record their 1-2
    // triangles (consecutive in DFS leaf order) as (first << 1) | (count - 1).
    std::vector<int> size(B.nodes.size(), 1);
    for (int i = (int)B.nodes.size() - 1; i >= 0; --i)
      if (B.nodes[i].left >= 0) size[i] = 1 + size[B.nodes[i].left] + size[B.nodes[i].right];
    for (size_t i = 0; i < B.nodes.size(); ++i) {
      const HBvh::Node& n = B.nodes[i];
      int32_t skip = m.node_off + (int32_t)i + size[i];
      int32_t leaf = -1;
      if (n.left < 0) {
        int first = ~n.left, last = ~n.right;
        leaf = ((first + m.tri_off) << 1) | (last != first ? 1 : 0);
      }
      float sf, lf;
      std::memcpy(&sf, &skip, 4);
      std::memcpy(&lf, &leaf, 4);
      F.nodes.insert(F.nodes.end(), {n.box.mn[0], n.box.mn[1], n.box.mn[2], sf, n.box.mx[0], n.box.mx[1], n.box.mx[2], lf});
    }
    build_node4(B, m);
    const size_t tri_first = F.tri_pos.size() / 16;
    for (int l : B.leaves) {
      const HTri& t = S.tris[S.obj[l].tri];
      for (int k = 0; k < 3; ++k) F.tri_pos.insert(F.tri_pos.end(), {t.p[3 * k], t.p[3 * k + 1], t.p[3 * k + 2], 0.f});
      F.tri_pos.insert(F.tri_pos.end(), {0.f, 0.f, 0.f, 0.f});  // pad to one 64-B line
      TriShade sh{};
      std::memcpy(sh.n, t.n, 36);
      for (int k = 0; k < 3; ++k) { sh.uv[2 * k] = t.uv[3 * k]; sh.uv[2 * k + 1] = t.uv[3 * k + 1]; }
      sh.mat = t.mat;
      F.tri_shade.push_back(sh);
    }
    build_node4q(m, tri_first);
    F.meshes.push_back(m);
    return mesh_of_bvh[h] = (int)F.meshes.size() - 1;
  }

  // Quantised bound on one axis: the smallest q with fl(o + q*s) <= v (lower) or
  // the largest-needed q with fl(o + q*s) >= v (upper), in the device's float
  // arithmetic (no contraction); false when 8 bits do not reach.
  static bool quant(float o, float sc, float v, bool upper, uint32_t& q) {
    if (!(v == v)) return false;
    double g = ((double)v - (double)o) / (double)sc;
    long long k = upper ? (long long)std::ceil(g) : (long long)std::floor(g);
    k = std::max(0LL, std::min(255LL, k));
    auto at = [&](long long x) {
      volatile float d = (float)x * sc;  // (volatile: one float rounding per step, as on the device)
      volatile float r = o + d;
      return (float)r;
    };
    if (upper) {
      while (k < 255 && at(k) < v) ++k;
      if (at(k) < v) return false;
    } else {
      while (k > 0 && at(k) > v) --k;
      if (at(k) > v) return false;
    }
    q = (uint32_t)k;
    return true;
  }

  // The 64-B compressed copy of this mesh's 4-wide nodes (device_scene.h
  // kNode4qWords).  A leaf child's exact box must be what the device recomputes
  // from its 1-2 triangles (ffmin / ffmax of the vertices, triangle.h:53-68,
  // bvh.h's surrounding_box): checked here; a mismatch (NaN vertices) turns the
  // compressed nodes off for the scene.
  void build_node4q(const DMesh& m, size_t tri_first) {
    F.node4q.resize(F.node4.size() / 2, 0.f);
    auto ffmin = [](float a, float b) { return a < b ? a : b; };
    auto ffmax = [](float a, float b) { return a > b ? a : b; };
    for (int ni = m.node4_off; ni < m.node4_off + m.n_node4; ++ni) {
      const float* d = &F.node4[32 * (size_t)ni];
      int32_t ch[4];
      std::memcpy(ch, d + 24, 16);
      float o[3], sc[3];
      uint32_t q[6] = {0, 0, 0, 0, 0, 0};
      for (int a = 0; a < 3; ++a) {
        float lo = INFINITY, hi = -INFINITY;
        for (int c = 0; c < 4; ++c)
          if (ch[c] != INT32_MIN) {
            lo = std::min(lo, d[4 * a + c]);
            hi = std::max(hi, d[12 + 4 * a + c]);
          }
        if (!(lo <= hi)) { lo = hi = 0.f; }  // all-empty node (not built) or NaN: handled below
        o[a] = lo;
        // scale: a power of two with 255 steps covering the extent, at least an
        // ulp-sized step of the coordinates
        const float ext = hi - lo;
        int e = -126;
        if (ext > 0) e = std::max(e, (int)std::ceil(std::log2((double)ext / 250.0)));
        const float mag = std::max(std::fabs(lo), std::fabs(hi));
        if (mag > 0) e = std::max(e, std::ilogb(mag) - 23);
        for (;; ++e) {
          sc[a] = std::ldexp(1.0f, e);
          bool ok = true;
          uint32_t qlo = 0, qhi = 0;
          for (int c = 0; c < 4 && ok; ++c) {
            uint32_t bl = 255, bh = 0;  // empty slot: lo > hi
            if (ch[c] != INT32_MIN)
              ok = quant(o[a], sc[a], d[4 * a + c], false, bl) && quant(o[a], sc[a], d[12 + 4 * a + c], true, bh);
            qlo |= bl << (8 * c);
            qhi |= bh << (8 * c);
          }
          if (ok) {
            q[a] = qlo;
            q[3 + a] = qhi;
            break;
          }
          if (e > 127) {
            F.node4q_ok = false;
            break;
          }
        }
      }
      // leaf children: the exact box the device recomputes must be the stored one
      for (int c = 0; c < 4; ++c) {
        if (ch[c] >= 0 || ch[c] == INT32_MIN) continue;
        const int leaf = ~ch[c], first = leaf >> 1, count = (leaf & 1) + 1;
        float mn[3], mx[3];
        for (int t = 0; t < count; ++t) {
          const float* p = &F.tri_pos[16 * (tri_first + (size_t)(first - m.tri_off + t))];
          for (int a = 0; a < 3; ++a) {
            const float tmn = ffmin(ffmin(p[a], p[4 + a]), p[8 + a]);
            const float tmx = ffmax(ffmax(p[a], p[4 + a]), p[8 + a]);
            mn[a] = t ? ffmin(mn[a], tmn) : tmn;
            mx[a] = t ? ffmax(mx[a], tmx) : tmx;
          }
        }
        for (int a = 0; a < 3; ++a)
          if (std::memcmp(&mn[a], &d[4 * a + c], 4) || std::memcmp(&mx[a], &d[12 + 4 * a + c], 4)) F.node4q_ok = false;
      }
      float* w = &F.node4q[kNode4qWords * (size_t)ni];
      for (int a = 0; a < 3; ++a) { w[a] = o[a]; w[3 + a] = sc[a]; }
      std::memcpy(w + 6, q, 24);
      std::memcpy(w + 12, ch, 16);
    }
  }

  // bvh_node over other hitables: the same threaded BVH2 records as add_mesh,
  // leaves naming children (DFS order); each child flattened to DObjs relative to
  // the node (its own instance chain only).  Children must be analytic
  // primitives, boxes, lists or instances of those: a mesh or medium nested in
  // an object BVH is refused.
  std::map<int, int> obvh_of_bvh;
  int add_obvh(int h) {
    auto it = obvh_of_bvh.find(h);
    if (it != obvh_of_bvh.end()) return it->second;
    const HBvh& B = S.bvhs[S.obj[h].bvh];
    DObvh o{};
    o.node_off = (int)(F.nodes.size() / 8);
    o.n_nodes = (int)B.nodes.size();
    o.child_off = (int)F.obvh_children.size();
    o.n_children = (int)B.leaves.size();
    for (int l : B.leaves) {
      std::vector<DObj> tmp;
      if (!walk(l, {}, tmp, false)) return -1;
      for (const DObj& d : tmp)
        if (d.kind != OBJ_SPHERE && d.kind != OBJ_MSPHERE && d.kind != OBJ_RECT && d.kind != OBJ_TRI) {
          err = "bvh_node over hitables that contain a bvh_node or constant_medium is not supported on the device";
          return -1;
        }
      F.obvh_children.push_back(DObvhChild{(int)inner.size(), (int)tmp.size()});  // rebased in flatten()
      inner.insert(inner.end(), tmp.begin(), tmp.end());
    }
    std::vector<int> size(B.nodes.size(), 1);
    for (int i = (int)B.nodes.size() - 1; i >= 0; --i)
      if (B.nodes[i].left >= 0) size[i] = 1 + size[B.nodes[i].left] + size[B.nodes[i].right];
    for (size_t i = 0; i < B.nodes.size(); ++i) {
      const HBvh::Node& n = B.nodes[i];
      int32_t skip = o.node_off + (int32_t)i + size[i];
      int32_t leaf = -1;
      if (n.left < 0) {
        int first = ~n.left, last = ~n.right;
        leaf = ((first + o.child_off) << 1) | (last != first ? 1 : 0);
      }
      float sf, lf;
      std::memcpy(&sf, &skip, 4);
      std::memcpy(&lf, &leaf, 4);
      F.nodes.insert(F.nodes.end(), {n.box.mn[0], n.box.mn[1], n.box.mn[2], sf, n.box.mx[0], n.box.mx[1], n.box.mx[2], lf});
    }
    F.obvhs.push_back(o);
    return obvh_of_bvh[h] = (int)F.obvhs.size() - 1;
  }

  // Appends the objects `h` contributes to `out`, under transform chain `ch`.
  bool walk(int h, std::vector<DXform> ch, std::vector<DObj>& out, bool in_medium) {
    const HObj& o = S.obj[h];
    auto emit = [&](int kind, int idx) {
      // flip_normals only negates the normal, which commutes with the rotations
      // and is untouched by translations: the chain keeps the moving transforms
      // and the flips become one parity bit (kXfFlipBit), applied last on the way out
      std::vector<DXform> moving;
      int flips = 0;
      for (const DXform& x : ch) {
        if (x.kind == XF_FLIP) ++flips;
        else moving.push_back(x);
      }
      DObj d;
      d.kind = kind;
      d.xf_begin = chain_push(moving);
      d.xf_count = (int)moving.size() | ((flips & 1) ? kXfFlipBit : 0);
      d.idx = idx;
      out.push_back(d);
    };
    switch (o.kind) {
      case H_LIST:
      case H_BOX:
        // hitable_list::hit passes closest_so_far along in order, so a nested list
        // (and box, box.h:31-33) behaves exactly like its children inlined in place.
        for (int k : o.kids)
          if (!walk(k, ch, out, in_medium)) return false;
        return true;
      case H_FLIP: ch.push_back(DXform{XF_FLIP, 0, 0, 0}); return walk(o.child, ch, out, in_medium);
      case H_TRANSLATE: ch.push_back(DXform{XF_TRANSLATE, o.f[0], o.f[1], o.f[2]}); return walk(o.child, ch, out, in_medium);
      case H_ROTY: ch.push_back(DXform{XF_ROTY, o.f[0], o.f[1], 0}); return walk(o.child, ch, out, in_medium);
      case H_ROTX: ch.push_back(DXform{XF_ROTX, o.f[0], o.f[1], 0}); return walk(o.child, ch, out, in_medium);
      case H_SPHERE:
      case H_MSPHERE: emit(o.kind == H_SPHERE ? OBJ_SPHERE : OBJ_MSPHERE, add_sphere(h)); return true;
      case H_XY: case H_XZ: case H_YZ: emit(OBJ_RECT, add_rect(h)); return true;
      case H_TRI: emit(OBJ_TRI, add_stri(h)); return true;
      case H_BVH: {
        int m = add_mesh(h);
        if (m >= 0) {
          emit(OBJ_MESH, m);
          return true;
        }
        int ob = add_obvh(h);
        if (ob < 0) return false;
        emit(OBJ_OBVH, ob);
        return true;
      }
      case H_MEDIUM: {
        if (in_medium) {
          err = "constant_medium nested inside a constant_medium boundary is not supported";
          return false;
        }
        DMedium md{};
        md.bnd_begin = (int)bound.size();
        std::vector<DObj> tmp;
        if (!walk(o.child, {}, tmp, true)) return false;
        bound.insert(bound.end(), tmp.begin(), tmp.end());
        md.bnd_count = (int)tmp.size();
        md.density = o.f[0];
        // constant_medium owns an isotropic phase material (constant_medium.h:6-9)
        DMat iso{};
        iso.kind = MAT_ISOTROPIC;
        iso.tex = o.tex;
        F.mats.push_back(iso);
        md.phase_mat = (int)F.mats.size() - 1;
        F.media.push_back(md);
        emit(OBJ_MEDIUM, (int)F.media.size() - 1);
        return true;
      }
    }
    err = "unknown hitable";
    return false;
  }

  DLight light(int h) {  // hitable_list.h:54-67 targets; flip forwards (aarect.h:163-169)
    const HObj* o = &S.obj[h];
    while (o->kind == H_FLIP) o = &S.obj[o->child];
    int hh = (int)(o - S.obj.data());
    if (o->kind == H_XZ) return DLight{LIGHT_XZRECT, add_rect(hh)};
    if (o->kind == H_SPHERE) return DLight{LIGHT_SPHERE, add_sphere(hh)};
    if (o->kind == H_TRI) return DLight{LIGHT_TRI, add_stri(hh)};
    return DLight{LIGHT_NONE, 0};  // hitable defaults: pdf 0, random (1,0,0) (hitable.h:31-32)
  }
};
}  // namespace

// Keeps only the materials the flattened objects reference and the textures
// (and image bytes) those materials reach, in their construction order.  The
// reference's builders construct materials they never place (cornell_box makes
// 20, uses 4); dropping them changes no lookup, shrinks the LDS-staged world
// tables, lets the diffuse-only kernel variant run when only diffuse materials
// are placed, and makes two builds of one scene flatten to identical tables
// whatever unused materials either constructed (srr_scene_digest).
static void compact_materials(Flat& F) {
  const int nm = (int)F.mats.size(), nt = (int)F.texs.size();
  std::vector<int> mmap(nm, -1), tmap(nt, -1);
  auto use_mat = [&](int m) {
    if (m >= 0 && m < nm) mmap[m] = 0;
  };
  for (const DSphere& x : F.spheres) use_mat(x.mat);
  for (const DRect& x : F.rects) use_mat(x.mat);
  for (const DStandaloneTri& x : F.stris) use_mat(x.sh.mat);
  for (const TriShade& x : F.tri_shade) use_mat(x.mat);
  for (const DMedium& x : F.media) use_mat(x.phase_mat);
  std::vector<int> stack;
  for (int m = 0; m < nm; ++m)
    if (mmap[m] == 0 && F.mats[m].tex >= 0) stack.push_back(F.mats[m].tex);
  while (!stack.empty()) {  // textures reached, through checker children
    const int t = stack.back();
    stack.pop_back();
    if (t < 0 || t >= nt || tmap[t] == 0) continue;
    tmap[t] = 0;
    if (F.texs[t].kind == TEX_CHECKER) {
      stack.push_back(F.texs[t].even);
      stack.push_back(F.texs[t].odd);
    }
  }
  std::vector<DTex> texs;
  std::vector<uint8_t> images;
  for (int t = 0; t < nt; ++t) {
    if (tmap[t] < 0) continue;
    tmap[t] = (int)texs.size();
    DTex d = F.texs[t];
    if (d.kind == TEX_IMAGE) {
      const size_t bytes = 3 * (size_t)d.nx * d.ny;
      const int64_t off = (int64_t)images.size();
      images.insert(images.end(), F.images.begin() + d.off, F.images.begin() + d.off + bytes);
      d.off = off;
    }
    texs.push_back(d);
  }
  for (DTex& d : texs)
    if (d.kind == TEX_CHECKER) {
      d.even = tmap[d.even];
      d.odd = tmap[d.odd];
    }
  std::vector<DMat> mats;
  for (int m = 0; m < nm; ++m) {
    if (mmap[m] < 0) continue;
    mmap[m] = (int)mats.size();
    DMat d = F.mats[m];
    if (d.tex >= 0) d.tex = tmap[d.tex];
    mats.push_back(d);
  }
  auto remap = [&](int32_t& m) {
    if (m >= 0 && m < nm) m = mmap[m];
  };
  for (DSphere& x : F.spheres) remap(x.mat);
  for (DRect& x : F.rects) remap(x.mat);
  for (DStandaloneTri& x : F.stris) remap(x.sh.mat);
  for (TriShade& x : F.tri_shade) remap(x.mat);
  for (DMedium& x : F.media) remap(x.phase_mat);
  F.mats = std::move(mats);
  F.texs = std::move(texs);
  F.images = std::move(images);
}

// Sphere runs (device_scene.h DSGroup): every run of >= kSGroupMinRun consecutive
// world objects that are plain spheres / moving spheres without an instance
// wrapper becomes one OBJ_SGROUP object over a BVH of their boxes; the spheres'
// DObjs go to `grouped` (their position in the run is the item's `pos`).
// SRR_SGROUP=0 keeps the plain list (A/B, parity).
static std::vector<DObj> group_sphere_runs(const Scene& S, Flat& F, const std::vector<DObj>& in,
                                           std::vector<DObj>& grouped) {
  static const bool on = [] {
    const char* e = getenv("SRR_SGROUP");
    return !e || atoi(e) != 0;
  }();
  // ray times: camera rays carry [time0, time1] (camera.h:57) and keep it through
  // diffuse bounces; specular rays are built with time 0 (ray.h:10)
  const double tlo = std::min(0.0, (double)std::min(S.cam.time0, S.cam.time1));
  const double thi = std::max(0.0, (double)std::max(S.cam.time0, S.cam.time1));
  auto plain = [&](const DObj& d) {
    if ((d.kind != OBJ_SPHERE && d.kind != OBJ_MSPHERE) || d.xf_count != 0) return false;
    const DSphere& sp = F.spheres[d.idx];
    bool ok = std::isfinite(sp.r);
    for (int k = 0; k < 3; ++k) ok = ok && std::isfinite(sp.c0[k]) && std::isfinite(sp.c1[k]);
    if (d.kind == OBJ_MSPHERE) ok = ok && std::isfinite(sp.t0) && std::isfinite(sp.t1) && sp.t1 != sp.t0;
    return ok;
  };
  std::vector<DObj> out;
  for (size_t i = 0; i < in.size();) {
    size_t j = i;
    while (j < in.size() && plain(in[j])) ++j;
    if (!on || j - i < (size_t)kSGroupMinRun) {
      out.insert(out.end(), in.begin() + i, in.begin() + (j > i ? j : i + 1));
      i = j > i ? j : i + 1;
      continue;
    }
    // items and their boxes (the center's whole path over the ray times, widened by
    // a relative 1e-5 for the float center arithmetic; sgroup_hit adds the per-ray pad)
    struct It { DSGItem it; double mn[3], mx[3], c[3]; };
    std::vector<It> items;
    for (size_t k = i; k < j; ++k) {
      const DSphere& sp = F.spheres[in[k].idx];
      It e{};
      e.it.s = sp;
      e.it.pos = (int)(k - i);
      e.it.moving = in[k].kind == OBJ_MSPHERE ? 1 : 0;
      e.it.obj = (int)grouped.size();  // rebased onto the objs table in flatten()
      grouped.push_back(in[k]);
      const double r = std::fabs((double)sp.r);
      for (int a = 0; a < 3; ++a) {
        double c0 = sp.c0[a], c1 = c0;
        if (e.it.moving) {  // center(t) = c0 + ((t - t0) / (t1 - t0)) (c1 - c0), linear in t
          const double s0 = (tlo - sp.t0) / ((double)sp.t1 - sp.t0), s1 = (thi - sp.t0) / ((double)sp.t1 - sp.t0);
          c1 = c0 + s1 * ((double)sp.c1[a] - sp.c0[a]);
          c0 = c0 + s0 * ((double)sp.c1[a] - sp.c0[a]);
        }
        const double lo = std::min(c0, c1) - r, hi = std::max(c0, c1) + r;
        const double w = 1e-5 * (std::max(std::fabs(lo), std::fabs(hi)) + r) + 1e-30;
        e.mn[a] = lo - w;
        e.mx[a] = hi + w;
        e.c[a] = 0.5 * (e.mn[a] + e.mx[a]);
      }
      items.push_back(e);
    }
    DSGroup g{};
    g.node_off = (int)(F.nodes.size() / 8);
    g.item_off = (int)F.sg_items.size();
    g.n_items = (int)items.size();
    // top-down median split on the widest centroid axis, leaves of 1-2 spheres, in
    // preorder with skip links (the threaded format of `nodes`)
    std::vector<float> nodes;
    std::function<void(int, int)> build = [&](int lo, int hi) {
      double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
      double cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int k = lo; k < hi; ++k)
        for (int a = 0; a < 3; ++a) {
          mn[a] = std::min(mn[a], items[k].mn[a]);
          mx[a] = std::max(mx[a], items[k].mx[a]);
          cmn[a] = std::min(cmn[a], items[k].c[a]);
          cmx[a] = std::max(cmx[a], items[k].c[a]);
        }
      const size_t me = nodes.size() / 8;
      nodes.resize(nodes.size() + 8);
      // float box rounded outward
      for (int a = 0; a < 3; ++a) {
        float fl = (float)mn[a], fh = (float)mx[a];
        if ((double)fl > mn[a]) fl = std::nextafter(fl, -INFINITY);
        if ((double)fh < mx[a]) fh = std::nextafter(fh, INFINITY);
        nodes[8 * me + a] = fl;
        nodes[8 * me + 4 + a] = fh;
      }
      int32_t leaf = -1;
      if (hi - lo <= 2) {
        leaf = ((int)F.sg_items.size() << 1) | (hi - lo - 1);
        for (int k = lo; k < hi; ++k) F.sg_items.push_back(items[k].it);
      } else {
        int ax = 0;
        for (int a = 1; a < 3; ++a)
          if (cmx[a] - cmn[a] > cmx[ax] - cmn[ax]) ax = a;
        const int mid = (lo + hi) / 2;
        std::nth_element(items.begin() + lo, items.begin() + mid, items.begin() + hi,
                         [ax](const It& x, const It& y) { return x.c[ax] < y.c[ax]; });
        build(lo, mid);
        build(mid, hi);
      }
      const int32_t skip = g.node_off + (int32_t)(nodes.size() / 8);
      std::memcpy(&nodes[8 * me + 3], &skip, 4);
      std::memcpy(&nodes[8 * me + 7], &leaf, 4);
    };
    build(0, (int)items.size());
    g.n_nodes = (int)(nodes.size() / 8);
    F.nodes.insert(F.nodes.end(), nodes.begin(), nodes.end());
    F.sgroups.push_back(g);
    DObj d{};
    d.kind = OBJ_SGROUP;
    d.idx = (int)F.sgroups.size() - 1;
    out.push_back(d);
    i = j;
  }
  return out;
}

int flatten(const Scene& S, Flat& F, std::string& err) {
  F = Flat();
  if (S.world < 0 || S.lights < 0 || !S.has_camera) {
    err = "scene needs world, lights and a camera";
    return -22;
  }
  if (S.obj[S.lights].kind != H_LIST) {
    err = "lights must be a hitable_list (Raytracing_n.cpp:75 casts it)";
    return -22;
  }
  // materials first: object rows reference them by handle
  for (const HMat& m : S.mat) {
    DMat d{};
    d.kind = m.kind;
    d.tex = m.tex;
    std::memcpy(d.p, m.p, 16);
    F.mats.push_back(d);
  }
  for (const HTex& t : S.tex) {
    DTex d{};
    d.kind = t.kind;
    std::memcpy(d.c, t.c, 12);
    d.nx = t.nx;
    d.ny = t.ny;
    d.even = t.even;
    d.odd = t.odd;
    if (t.kind == TEX_IMAGE) {
      d.off = (int64_t)F.images.size();
      F.images.insert(F.images.end(), t.px.begin(), t.px.end());
    }
    F.texs.push_back(d);
  }
  Flattener fl{S, F, err};
  if (!fl.walk(S.world, {}, fl.world, false)) return -95;
  std::vector<DObj> grouped_objs;  // the spheres moved into sphere groups, kept after every other DObj
  const std::vector<DObj> world = group_sphere_runs(S, F, fl.world, grouped_objs);
  F.n_world = (int)world.size();
  F.objs = world;
  for (DObj d : fl.bound) F.objs.push_back(d);
  for (DMedium& m : F.media) m.bnd_begin += F.n_world;
  const int inner_base = (int)F.objs.size();
  for (DObj d : fl.inner) F.objs.push_back(d);
  for (DObvhChild& c : F.obvh_children) c.obj_begin += inner_base;
  const int grouped_base = (int)F.objs.size();
  for (DObj d : grouped_objs) F.objs.push_back(d);
  for (DSGItem& it : F.sg_items) it.obj += grouped_base;
  for (int k : S.obj[S.lights].kids) {
    if (S.obj[k].kind == H_LIST) {
      err = "nested hitable_list inside the light list is not supported";
      return -95;
    }
    F.lights.push_back(fl.light(k));
  }
  compact_materials(F);
  perlin_tables(F.perlin_ranvec, F.perlin_perm);
  const HCamera& c = S.cam;
  std::memcpy(F.cam.origin, c.origin, 12);
  std::memcpy(F.cam.llc, c.llc, 12);
  std::memcpy(F.cam.horizontal, c.horizontal, 12);
  std::memcpy(F.cam.vertical, c.vertical, 12);
  std::memcpy(F.cam.u, c.u, 12);
  std::memcpy(F.cam.v, c.v, 12);
  F.cam.time0 = c.time0;
  F.cam.time1 = c.time1;
  F.cam.lens_radius = c.lens_radius;
  return 0;
}

// --------------------------------------------------------------- text parser
namespace {
struct Tok {
  std::vector<std::string> t;
  int line;
  float f(size_t i) const { return std::strtof(t.at(i).c_str(), nullptr); }
  long long i(size_t k) const { return std::strtoll(t.at(k).c_str(), nullptr, 10); }
  unsigned long long u(size_t k) const { return std::strtoull(t.at(k).c_str(), nullptr, 10); }
  void v3(size_t k, float* o) const { o[0] = f(k); o[1] = f(k + 1); o[2] = f(k + 2); }
};
}  // namespace

int scene_from_text(const std::string& text, Scene& S, std::string& err) {
  std::istringstream is(text);
  std::string line;
  int ln = 0;
  bool header = false;
  std::map<long long, int> T, M, O;
  std::map<long long, std::pair<int, int>> G;  // group: first handle, count
  auto need = [&](std::map<long long, int>& mp, long long id, const char* what) -> int {
    if (id == -1 && std::string(what) == "mat") return -1;
    auto it = mp.find(id);
    if (it == mp.end()) throw std::runtime_error(std::string("undefined ") + what + " " + std::to_string(id));
    return it->second;
  };
  try {
    while (std::getline(is, line)) {
      ++ln;
      size_t h = line.find('#');
      if (h != std::string::npos) line.resize(h);
      Tok c;
      c.line = ln;
      std::istringstream ls(line);
      std::string w;
      while (ls >> w) c.t.push_back(w);
      if (c.t.empty()) continue;
      const std::string& k = c.t[0];
      if (!header) {
        if (k != "srr_scene" || c.i(1) != 1) throw std::runtime_error("not an srr_scene v1 description");
        header = true;
        continue;
      }
      float a[3], b[3], cc[3];
      if (k == "lcg") S.lcg = c.u(1) & 0xFFFFFFFFFFFFULL;
      else if (k == "tex") {
        const std::string& t = c.t.at(2);
        HTex x;
        if (t == "const") { x.kind = TEX_CONST; c.v3(3, x.c); }
        else if (t == "image_gen") {
          x.kind = TEX_IMAGE;
          x.nx = (int)c.i(3);
          x.ny = (int)c.i(4);
          x.px = gen_image(x.nx, x.ny, (uint32_t)c.u(5), (int)c.i(6));
        } else if (t == "image_raw") {  // decoded RGB8 file, w*h*3 bytes, row 0 = top
          x.kind = TEX_IMAGE;
          x.nx = (int)c.i(3);
          x.ny = (int)c.i(4);
          std::ifstream f(c.t.at(5), std::ios::binary);
          if (!f) throw std::runtime_error("image_raw: cannot open " + c.t.at(5));
          x.px.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
          if (x.nx <= 0 || x.ny <= 0 || x.px.size() != (size_t)x.nx * x.ny * 3)
            throw std::runtime_error("image_raw " + c.t.at(5) + ": size does not match " + c.t.at(3) + "x" + c.t.at(4));
        } else if (t == "checker") {
          x.kind = TEX_CHECKER;
          x.even = need(T, c.i(3), "tex");
          x.odd = need(T, c.i(4), "tex");
        } else if (t == "noise") { x.kind = TEX_NOISE; x.c[0] = c.f(3); }
        else throw std::runtime_error("tex kind " + t);
        T[c.i(1)] = S.add_tex(std::move(x));
      } else if (k == "mat") {
        const std::string& t = c.t.at(2);
        float prm[4] = {0, 0, 0, 0};
        int hm;
        if (t == "metal") { c.v3(3, prm); prm[3] = c.f(6); hm = S.material(MAT_METAL, -1, prm); }
        else if (t == "dielectric") { prm[0] = c.f(3); hm = S.material(MAT_DIELECTRIC, -1, prm); }
        else {
          int tx = need(T, c.i(3), "tex");
          if (t == "lambertian") hm = S.material(MAT_LAMBERTIAN, tx, prm);
          else if (t == "orennayar") { prm[0] = c.f(4); hm = S.material(MAT_ORENNAYAR, tx, prm); }
          else if (t == "beckmann") { prm[0] = c.f(4); prm[1] = c.f(5); hm = S.material(MAT_BECKMANN, tx, prm); }
          else if (t == "diffuse_light") hm = S.material(MAT_DIFFUSE_LIGHT, tx, prm);
          else if (t == "isotropic") hm = S.material(MAT_ISOTROPIC, tx, prm);
          else throw std::runtime_error("mat kind " + t);
        }
        M[c.i(1)] = hm;
      } else if (k == "grp") {
        if (c.t.at(2) != "teapot") throw std::runtime_error("grp kind");
        int first = -1;
        int n = S.teapot(c.f(3), (int)c.i(4), need(M, c.i(5), "mat"), &first);
        G[c.i(1)] = {first, n};
      } else if (k == "obj") {
        const std::string& t = c.t.at(2);
        int hnd = -1;
        if (t == "sphere") { c.v3(3, a); hnd = S.sphere(a, c.f(6), need(M, c.i(7), "mat")); }
        else if (t == "moving_sphere") {
          c.v3(3, a); c.v3(6, b);
          hnd = S.moving_sphere(a, b, c.f(9), c.f(10), c.f(11), need(M, c.i(12), "mat"));
        } else if (t == "xy_rect" || t == "xz_rect" || t == "yz_rect") {
          HKind kk = t == "xy_rect" ? H_XY : (t == "xz_rect" ? H_XZ : H_YZ);
          hnd = S.rect(kk, c.f(3), c.f(4), c.f(5), c.f(6), c.f(7), need(M, c.i(8), "mat"));
        } else if (t == "box") { c.v3(3, a); c.v3(6, b); hnd = S.box(a, b, need(M, c.i(9), "mat")); }
        else if (t == "triangle" || t == "triangle_uv" || t == "triangle_uvn") {
          float p[9], uv[9], n[9];
          for (int q = 0; q < 9; ++q) p[q] = c.f(3 + q);
          if (t != "triangle") for (int q = 0; q < 9; ++q) uv[q] = c.f(13 + q);
          if (t == "triangle_uvn") for (int q = 0; q < 9; ++q) n[q] = c.f(22 + q);
          hnd = S.triangle(p, need(M, c.i(12), "mat"), t != "triangle" ? uv : nullptr,
                           t == "triangle_uvn" ? n : nullptr);
        } else if (t == "flip") hnd = S.wrap(H_FLIP, need(O, c.i(3), "obj"), nullptr);
        else if (t == "translate") { c.v3(4, a); hnd = S.wrap(H_TRANSLATE, need(O, c.i(3), "obj"), a); }
        else if (t == "rotate_y") hnd = S.rotate(H_ROTY, need(O, c.i(3), "obj"), c.f(4));
        else if (t == "rotate_x") hnd = S.rotate(H_ROTX, need(O, c.i(3), "obj"), c.f(4));
        else if (t == "constant_medium") hnd = S.medium(need(O, c.i(3), "obj"), c.f(4), need(T, c.i(5), "tex"));
        else if (t == "list" || t == "bvh") {
          size_t base = t == "bvh" ? 5 : 3;
          long long n = c.i(base);
          std::vector<int> kids;
          for (long long q = 0; q < n; ++q) kids.push_back(need(O, c.i(base + 1 + q), "obj"));
          hnd = t == "bvh" ? S.bvh(kids.data(), (int)n, c.f(3), c.f(4)) : S.list(kids.data(), (int)n);
        } else if (t == "bvh_group" || t == "list_group") {
          auto it = G.find(c.i(t == "bvh_group" ? 5 : 3));
          if (it == G.end()) throw std::runtime_error("undefined grp");
          std::vector<int> kids(it->second.second);
          for (int q = 0; q < it->second.second; ++q) kids[q] = it->second.first + q;
          hnd = t == "bvh_group" ? S.bvh(kids.data(), (int)kids.size(), c.f(3), c.f(4))
                                 : S.list(kids.data(), (int)kids.size());
        } else throw std::runtime_error("obj kind " + t);
        if (hnd < 0) throw std::runtime_error("constructor failed");
        O[c.i(1)] = hnd;
        S.text_ids.emplace_back(c.i(1), hnd);
      } else if (k == "camera") {
        c.v3(1, a); c.v3(4, b); c.v3(7, cc);
        S.camera(a, b, cc, c.f(10), c.f(11), c.f(12), c.f(13), c.f(14), c.f(15));
      } else if (k == "world") S.world = need(O, c.i(1), "obj");
      else if (k == "lights") S.lights = need(O, c.i(1), "obj");
      else throw std::runtime_error("unknown command " + k);
    }
  } catch (const std::exception& e) {
    err = "scene line " + std::to_string(ln) + ": " + e.what();
    return -22;
  }
  if (!header) {
    err = "empty scene description";
    return -22;
  }
  return 0;
}

}  // namespace srr

/* srr reference-compatible C++ scene API.
 *
 * Header-only C++ over the C-ABI (include/srr_capi.h): the class names and
 * constructor signatures the reference's scene builders call
 * (Raytracing_n.cpp:108-711), so a builder written for the reference compiles
 * against srr unchanged apart from its includes:
 *
 *     #include "srr/ref_api.h"
 *     using namespace srr::ref;
 *     srr::ref::scene_scope scope(scene);          // where the constructors record
 *     material* white = new lambertian(new constant_texture(vec3(0.73f, 0.73f, 0.73f)));
 *     hitable** list = new hitable*[8];
 *     list[0] = new flip_normals(new yz_rect(0, 555, 0, 555, 555, green));
 *     ...
 *     *world = new hitable_list(list, i);
 *
 * Every constructor records one object in the current scene (scene_scope) through
 * the C-ABI and keeps its integer handle; the objects themselves are small
 * proxies (the reference leaks its graph; so may a caller here -- the scene owns
 * the real data).  Errors throw srr::ref::error (the reference never reports any).
 *
 * Build definitions: the 7-argument camera's shutter times,
 * uninitialised in the reference (camera.h:19-31), are 0; teapot and 4-argument
 * triangles carry face normals (Q5); drand48() draws from the scene's LCG, which
 * starts at the reference's post-Perlin state (Q14). */
#pragma once

#include <stdlib.h>  // glibc's drand48 declared before the reference's name is mapped below

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../srr_capi.h"
#include "merl.h"

/* The reference defines its own global drand48() (mathf.h:14-19), which clashes
 * with glibc's; as in the reference's Linux build (oracle/ref/shim.h), the name is
 * mapped to the scene-build LCG below. */
#define drand48 srr_ref_drand48

namespace srr {
namespace ref {

struct error : std::runtime_error {
  int code;
  error(int c, const char* msg) : std::runtime_error(std::string("srr: ") + (msg ? msg : "")), code(c) {}
};

inline srr_scene*& current_scene() {
  thread_local srr_scene* s = nullptr;
  return s;
}

/* Makes `s` the scene the constructors below record into, for this thread. */
struct scene_scope {
  srr_scene* prev;
  explicit scene_scope(srr_scene* s) : prev(current_scene()) { current_scene() = s; }
  ~scene_scope() { current_scene() = prev; }
  scene_scope(const scene_scope&) = delete;
  scene_scope& operator=(const scene_scope&) = delete;
};

inline srr_scene* cur() {
  srr_scene* s = current_scene();
  if (!s) throw error(SRR_EINVAL, "no scene_scope active");
  return s;
}
inline int check(int h) {
  if (h < 0) throw error(h, srr_last_error());
  return h;
}

/* mathf.h:14-19 drand48() on the scene-build LCG (bvh_node's random axis uses it) */
inline double srr_ref_drand48() { return srr_scene_drand48(cur()); }

/* stb_image's stbi_load (stb_image.h v2.19) as the builders call it, through srr's
 * stb-exact decoder (srr_image_load); free with stbi_image_free. */
inline unsigned char* stbi_load(const char* path, int* x, int* y, int* comp, int req_comp) {
  unsigned char* p = nullptr;
  return srr_image_load(path, req_comp, x, y, comp, &p) < 0 ? nullptr : p;
}
inline void stbi_image_free(void* p) { srr_image_free((unsigned char*)p); }

/* vec3.h: the value type the builders pass around (float x3) */
class vec3 {
 public:
  float e[3];
  vec3() : e{0, 0, 0} {}
  vec3(float e0) : e{e0, e0, e0} {}
  vec3(float e0, float e1, float e2) : e{e0, e1, e2} {}
  vec3(const float* p) : e{p[0], p[1], p[2]} {}
  float x() const { return e[0]; }
  float y() const { return e[1]; }
  float z() const { return e[2]; }
  float r() const { return e[0]; }
  float g() const { return e[1]; }
  float b() const { return e[2]; }
  float operator[](int i) const { return e[i]; }
  float& operator[](int i) { return e[i]; }
  vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
  float squared_length() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }  // vec3.h
  float length() const { return std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]); }
};
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline vec3 operator*(const vec3& a, const vec3& b) { return vec3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline vec3 operator*(float t, const vec3& v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3& v, float t) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator/(const vec3& v, float t) { return vec3(v.e[0] / t, v.e[1] / t, v.e[2] / t); }

/* ------------------------------------------------------------------ textures */
class texture {  // texture.h:4-7
 public:
  int handle = -1;
  virtual ~texture() = default;
};
class constant_texture : public texture {  // texture.h:25-33
 public:
  constant_texture(vec3 c) { handle = check(srr_constant_texture(cur(), c.x(), c.y(), c.z())); }
};
class image_texture : public texture {  // texture.h:48-70 (bytes copied; the reference borrows them)
 public:
  image_texture(unsigned char* pixels, int A, int B) { handle = check(srr_image_texture(cur(), pixels, A, B)); }
};
class checker_texture : public texture {  // texture.h:9-23
 public:
  checker_texture(texture* t0, texture* t1) { handle = check(srr_checker_texture(cur(), t0->handle, t1->handle)); }
};
class noise_texture : public texture {  // texture.h:35-46
 public:
  noise_texture(float sc) { handle = check(srr_noise_texture(cur(), sc)); }
};
/* srr extension (not a reference class): an image_texture over a synthetic RGB8
 * image (srr_image_texture_gen; kind 0 sky, 1 wood, 2 checker) -- the BASELINE
 * stand-in scenes' textures, generated in code instead of read from contents/. */
class generated_texture : public texture {
 public:
  generated_texture(int nx, int ny, unsigned seed, int kind) {
    handle = check(srr_image_texture_gen(cur(), nx, ny, seed, kind));
  }
};

/* ----------------------------------------------------------------- materials */
class material {  // material.h:82-93
 public:
  int handle = -1;
  virtual ~material() = default;
};
inline int mat_handle(const material* m) {  // null material*: -1
  if (m && m->handle == -2) throw error(SRR_ENOTSUP, "brdfmaterial cannot be rendered (it sets no pdf, SURVEY Q23)");
  return m ? m->handle : -1;
}
class lambertian : public material {  // material.h:95-114
 public:
  lambertian(texture* a) { handle = check(srr_lambertian(cur(), a->handle)); }
};
class orennayar : public material {  // material.h:127-149
 public:
  orennayar(texture* a, float sigma) { handle = check(srr_orennayar(cur(), a->handle, sigma)); }
};
class beckmann : public material {  // material.h:151-199
 public:
  beckmann(texture* a, float roughx, float roughy) { handle = check(srr_beckmann(cur(), a->handle, roughx, roughy)); }
};
class metal : public material {  // material.h:243-261
 public:
  metal(const vec3& a, float f) { handle = check(srr_metal(cur(), a.x(), a.y(), a.z(), f)); }
};
class dielectric : public material {  // material.h:282-339
 public:
  dielectric(float ri) { handle = check(srr_dielectric(cur(), ri)); }
};
class diffuse_light : public material {  // material.h:341-356
 public:
  diffuse_light(texture* a) { handle = check(srr_diffuse_light(cur(), a->handle)); }
};
class isotropic : public material {  // material.h:359-369
 public:
  isotropic(texture* a) { handle = check(srr_isotropic(cur(), a->handle)); }
};

/* brdf.h's MERL reader (brdf::read_brdf, :156-185; messages as the reference
 * prints them) and lookup (brdf::lookup_brdf_val, :190-214), on the host.  The
 * GPU lookup is srr_merl_lookup. */
class brdf {
 public:
  bool read_brdf(const char* filename, double*& table) {
    FILE* f = std::fopen(filename, "rb");
    std::printf(f ? "the file was opened\n" : "the file was not opened\n");
    if (!f) return false;
    int dims[3] = {0, 0, 0};
    const bool hdr = std::fread(dims, sizeof(int), 3, f) == 3;
    const long long n = (long long)dims[0] * dims[1] * dims[2];
    if (!hdr || n != merl::kCells) {
      std::fprintf(stderr, "Dimensions don't match\n");
      std::fclose(f);
      return false;
    }
    table = (double*)std::malloc(sizeof(double) * 3 * n);
    const size_t got = std::fread(table, sizeof(double), 3 * n, f);
    std::fclose(f);
    return got == (size_t)(3 * n);
  }
  void lookup_brdf_val(double* table, double theta_in, double fi_in, double theta_out, double fi_out, double& red,
                       double& green, double& blue) {
    merl::rgb_of(table, merl::cell_of(theta_in, fi_in, theta_out, fi_out), red, green, blue);
    if (red < 0.0 || green < 0.0 || blue < 0.0) std::fprintf(stderr, "Below horizon.\n");
  }
};

/* material.h:201-241.  The reference reads the table but its scatter() never
 * sets a pdf, so a hitable carrying one cannot be rendered there:
 * constructing one works (cornell_box and soldier_scene do, unused); putting it
 * on a primitive throws. */
constexpr int kUnrenderableMaterial = -2;
class brdfmaterial : public material {
 public:
  brdfmaterial(const char* brdf_filename, const vec3& a) : albedo(a) {
    brdf_reader = new brdf();
    brdf_reader->read_brdf(brdf_filename, brdf_data);
    handle = kUnrenderableMaterial;
  }
  brdf* brdf_reader;
  double* brdf_data = nullptr;
  vec3 albedo;
};

/* ------------------------------------------------------------------ hitables */
class hitable {  // hitable.h:27-33
 public:
  int handle = -1;
  virtual ~hitable() = default;
};
class sphere : public hitable {  // sphere.h:21
 public:
  sphere(vec3 cen, float r, material* m) { handle = check(srr_sphere(cur(), cen.e, r, mat_handle(m))); }
};
class moving_sphere : public hitable {  // moving_sphere.h:8
 public:
  moving_sphere(vec3 cen0, vec3 cen1, float t0, float t1, float r, material* m) {
    handle = check(srr_moving_sphere(cur(), cen0.e, cen1.e, t0, t1, r, mat_handle(m)));
  }
};
class xy_rect : public hitable {  // aarect.h:8
 public:
  xy_rect(float x0, float x1, float y0, float y1, float k, material* mat) {
    handle = check(srr_xy_rect(cur(), x0, x1, y0, y1, k, mat_handle(mat)));
  }
};
class xz_rect : public hitable {  // aarect.h:38
 public:
  xz_rect(float x0, float x1, float z0, float z1, float k, material* mat) {
    handle = check(srr_xz_rect(cur(), x0, x1, z0, z1, k, mat_handle(mat)));
  }
};
class yz_rect : public hitable {  // aarect.h:69
 public:
  yz_rect(float y0, float y1, float z0, float z1, float k, material* mat) {
    handle = check(srr_yz_rect(cur(), y0, y1, z0, z1, k, mat_handle(mat)));
  }
};
class box : public hitable {  // box.h:18-29
 public:
  box(const vec3& p0, const vec3& p1, material* ptr) { handle = check(srr_box(cur(), p0.e, p1.e, mat_handle(ptr))); }
};
class flip_normals : public hitable {  // aarect.h:149-171
 public:
  flip_normals(hitable* p) { handle = check(srr_flip_normals(cur(), p->handle)); }
};
class translate : public hitable {  // hitable.h:35-61
 public:
  translate(hitable* p, const vec3& displacement) { handle = check(srr_translate(cur(), p->handle, displacement.e)); }
};
class rotate_y : public hitable {  // hitable.h:65-132
 public:
  rotate_y(hitable* p, float angle) { handle = check(srr_rotate_y(cur(), p->handle, angle)); }
};
class rotate_x : public hitable {  // hitable.h:135-203
 public:
  rotate_x(hitable* p, float angle) { handle = check(srr_rotate_x(cur(), p->handle, angle)); }
};
class triangle : public hitable {  // triangle.h:13-50
 public:
  explicit triangle(int h) { handle = h; }  // a triangle the scene already holds (teapot)
  triangle(vec3 p0, vec3 p1, vec3 p2, material* mat) { make(p0, p1, p2, mat, nullptr, nullptr); }
  triangle(vec3 p0, vec3 p1, vec3 p2, material* mat, vec3 uv0, vec3 uv1, vec3 uv2) {
    const float uv[9] = {uv0.x(), uv0.y(), uv0.z(), uv1.x(), uv1.y(), uv1.z(), uv2.x(), uv2.y(), uv2.z()};
    make(p0, p1, p2, mat, uv, nullptr);
  }
  triangle(vec3 p0, vec3 p1, vec3 p2, material* mat, vec3 uv0, vec3 uv1, vec3 uv2, vec3 n0, vec3 n1, vec3 n2) {
    const float uv[9] = {uv0.x(), uv0.y(), uv0.z(), uv1.x(), uv1.y(), uv1.z(), uv2.x(), uv2.y(), uv2.z()};
    const float n[9] = {n0.x(), n0.y(), n0.z(), n1.x(), n1.y(), n1.z(), n2.x(), n2.y(), n2.z()};
    make(p0, p1, p2, mat, uv, n);
  }

 private:
  void make(const vec3& p0, const vec3& p1, const vec3& p2, material* mat, const float* uv, const float* n) {
    const float p[9] = {p0.x(), p0.y(), p0.z(), p1.x(), p1.y(), p1.z(), p2.x(), p2.y(), p2.z()};
    handle = check(srr_triangle(cur(), p, mat_handle(mat), uv, n));
  }
};
class constant_medium : public hitable {  // constant_medium.h:6
 public:
  constant_medium(hitable* b, float d, texture* a) { handle = check(srr_constant_medium(cur(), b->handle, d, a->handle)); }
};
inline std::vector<int> handles_of(hitable** l, int n) {
  std::vector<int> h((size_t)(n > 0 ? n : 0));
  for (int i = 0; i < n; ++i) h[(size_t)i] = l[i]->handle;
  return h;
}
class hitable_list : public hitable {  // hitable_list.h:11
 public:
  hitable_list(hitable** l, int n) {
    std::vector<int> h = handles_of(l, n);
    handle = check(srr_hitable_list(cur(), h.data(), n));
  }
};
class bvh_node : public hitable {  // bvh.h:96-119 (consumes the scene LCG like the reference)
 public:
  bvh_node(hitable** l, int n, float time0, float time1) {
    std::vector<int> h = handles_of(l, n);
    handle = check(srr_bvh_node(cur(), h.data(), n, time0, time1));
  }
};
/* teapot.h:13-166.  The reference hard-codes divs = 100 (640,000 triangles);
 * `divs` is exposed because BASELINE's "~6k tris" is divs = 10. */
class teapot {
 public:
  teapot(float scale, material* mat, int divs = 100) : scale_(scale), mat_(mat), divs_(divs) {}
  hitable** createPloyTeapot() {
    int first = 0;
    count_ = check(srr_teapot(cur(), scale_, divs_, mat_handle(mat_), &first));
    hitable** list = new hitable*[(size_t)count_];
    for (int k = 0; k < count_; ++k) list[k] = new triangle(first + k);
    return list;
  }
  int getTriangleCount() const { return count_; }

 private:
  float scale_;
  material* mat_;
  int divs_;
  int count_ = 0;
};

/* model.h:13-102 (assimp replaced by srr's PLY / binary-FBX loader, srr_model):
 * the file is read in the constructor; genhitablemodel() and gettrianglecount()
 * cover mesh 0 only, as the reference's do (model.h:90, :101). */
class model {
 public:
  model(const std::string& filename, bool flipUVs, bool flipWindingOrder, material* mat, vec3 scale) {
    count_ = check(srr_model(cur(), filename.c_str(), flipUVs, flipWindingOrder, mat_handle(mat), scale.e, &first_));
  }
  hitable** genhitablemodel() {
    hitable** list = new hitable*[(size_t)count_];
    for (int k = 0; k < count_; ++k) list[k] = new triangle(first_ + k);
    return list;
  }
  int gettrianglecount() const { return count_; }

 private:
  int first_ = 0, count_ = 0;
};

/* camera.h:19-48 */
class camera {
 public:
  camera(vec3 lookfrom, vec3 lookat, vec3 vup, float vfov, float aspect, float aperture, float focus_dist)
      : camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, 0.f, 0.f) {}
  camera(vec3 lookfrom, vec3 lookat, vec3 vup, float vfov, float aspect, float aperture, float focus_dist, float t0,
         float t1) {
    check(srr_camera(cur(), lookfrom.e, lookat.e, vup.e, vfov, aspect, aperture, focus_dist, t0, t1));
  }
};

/* The builder's outputs: world (renderthread's `world`) and hlist (light shapes). */
inline void capture(hitable* world, hitable* hlist) {
  check(srr_scene_set_world(cur(), world->handle));
  if (hlist) check(srr_scene_set_lights(cur(), hlist->handle));
}

}  // namespace ref
}  // namespace srr

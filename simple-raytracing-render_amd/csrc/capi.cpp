// C-ABI (include/srr_capi.h) and the host render driver: scene upload, the
// wavefront bounce loop on one HIP stream, batch bookkeeping and timing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/srr_capi.h"
#include "imageio.h"
#include "meshio.h"
#include "../../include/srr/merl.h"
#include "multi.h"
#include "renderer.h"

using namespace srr;

struct srr_scene {
  Scene s;
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail(SRR_EIO, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
int upload(T** dst, const std::vector<T>& v) {
  size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  HIPCHK(hipMalloc((void**)dst, bytes));
  if (!v.empty()) HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}
}  // namespace

extern "C" {

const char* srr_last_error(void) { return g_err.c_str(); }
const char* srr_version(void) { return "srr 0.1 (gfx950 wavefront path tracer)"; }

// ------------------------------------------------------------------ scene
srr_scene* srr_scene_create(void) { return new srr_scene(); }
void srr_scene_destroy(srr_scene* s) { delete s; }

int srr_scene_from_text(const char* text, srr_scene** out) {
  if (!text || !out) return fail(SRR_EINVAL, "null argument");
  std::unique_ptr<srr_scene> s(new srr_scene());
  std::string err;
  int rc = scene_from_text(text, s->s, err);
  if (rc < 0) return fail(rc, err);
  *out = s.release();
  return 0;
}

int srr_scene_text_handle(const srr_scene* s, int id) {
  if (!s) return fail(SRR_EINVAL, "null scene");
  for (auto& kv : s->s.text_ids)
    if (kv.first == id) return kv.second;
  return fail(SRR_EINVAL, "no such text object id");
}

// FNV-1a 64 over the flattened device tables (scene.h Flat): two scenes with the
// same digest upload byte-identical objects, transforms, primitives, BVHs (both
// layouts), triangles, media, materials, textures and image bytes, lights and camera.
// parts (optional, SRR_DIGEST_PARTS entries): one digest per table, in that order.
int srr_scene_digest(const srr_scene* s, uint64_t* out, uint64_t* parts) {
  if (!s || !out) return fail(SRR_EINVAL, "null argument");
  Flat f;
  std::string err;
  const int rc = flatten(s->s, f, err);
  if (rc < 0) return fail(rc, err);
  uint64_t h = 0xcbf29ce484222325ULL;
  int part = 0;
  auto mix = [](uint64_t& x, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) x = (x ^ b[i]) * 0x100000001b3ULL;
  };
  auto blob = [&](const void* p, size_t n) {
    mix(h, &n, sizeof n);
    mix(h, p, n);
    if (const char* dd = getenv("SRR_DIGEST_DUMP")) {  // diagnostics: each table to <prefix>.<part>
      FILE* df = fopen((std::string(dd) + "." + std::to_string(part)).c_str(), "wb");
      if (df) { fwrite(p, 1, n, df); fclose(df); }
    }
    if (parts) {
      uint64_t x = 0xcbf29ce484222325ULL;
      mix(x, p, n);
      parts[part] = x;
    }
    ++part;
  };
  auto vec = [&blob](const auto& v) { blob(v.data(), v.size() * sizeof(v[0])); };
  vec(f.objs);
  blob(&f.n_world, sizeof f.n_world);
  vec(f.xforms);
  vec(f.spheres);
  vec(f.rects);
  vec(f.stris);
  vec(f.meshes);
  vec(f.nodes);
  vec(f.node4);
  vec(f.tri_pos);
  vec(f.tri_shade);
  vec(f.media);
  {  // object BVHs, with the sphere groups and their items (device_scene.h DSGroup) in the same part
    std::vector<uint8_t> b;
    auto put = [&b](const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); };
    put(f.obvhs.data(), f.obvhs.size() * sizeof(DObvh));
    put(f.sgroups.data(), f.sgroups.size() * sizeof(DSGroup));
    put(f.sg_items.data(), f.sg_items.size() * sizeof(DSGItem));
    vec(b);
  }
  vec(f.obvh_children);
  vec(f.mats);
  vec(f.texs);
  vec(f.images);
  vec(f.perlin_ranvec);
  vec(f.perlin_perm);
  vec(f.lights);
  blob(&f.cam, sizeof f.cam);
  *out = h;
  return 0;
}

int srr_scene_set_lcg(srr_scene* s, uint64_t state) {
  if (!s) return fail(SRR_EINVAL, "null scene");
  s->s.lcg = state & 0xFFFFFFFFFFFFULL;
  return 0;
}
uint64_t srr_scene_get_lcg(const srr_scene* s) { return s ? s->s.lcg : 0; }
double srr_scene_drand48(srr_scene* s) { return s ? s->s.drand48() : 0.0; }

#define SCN(s) \
  if (!(s)) return fail(SRR_EINVAL, "null scene");
#define TEXOK(s, t) \
  if (!(s)->s.valid_tex(t)) return fail(SRR_EINVAL, "bad texture handle " + std::to_string(t));
#define MATOK(s, m) \
  if (!(s)->s.valid_mat(m)) return fail(SRR_EINVAL, "bad material handle " + std::to_string(m));
#define OBJOK(s, o) \
  if (!(s)->s.valid_obj(o)) return fail(SRR_EINVAL, "bad hitable handle " + std::to_string(o));

int srr_constant_texture(srr_scene* s, float r, float g, float b) {
  SCN(s);
  HTex t;
  t.kind = TEX_CONST;
  t.c[0] = r; t.c[1] = g; t.c[2] = b;
  return s->s.add_tex(std::move(t));
}
int srr_image_texture(srr_scene* s, const unsigned char* rgb, int nx, int ny) {
  SCN(s);
  if (!rgb || nx <= 0 || ny <= 0) return fail(SRR_EINVAL, "bad image");
  HTex t;
  t.kind = TEX_IMAGE;
  t.nx = nx;
  t.ny = ny;
  t.px.assign(rgb, rgb + (size_t)nx * ny * 3);
  return s->s.add_tex(std::move(t));
}
int srr_image_texture_file(srr_scene* s, const char* path) {
  SCN(s);
  if (!path) return fail(SRR_EINVAL, "null path");
  srr::Image im;
  std::string err;
  if (srr::load_image(path, 0, im, err) < 0) return fail(SRR_EIO, err);
  // image_texture reads 3 bytes per texel from the buffer stbi_load returned,
  // whatever its channel count (texture.h:58-70): keep exactly the
  // bytes it can address.  Fewer than 3 channels would read past that buffer.
  if (im.n < 3) return fail(SRR_EINVAL, std::string(path) + ": image_texture needs 3 or 4 channels");
  HTex t;
  t.kind = TEX_IMAGE;
  t.nx = im.w;
  t.ny = im.h;
  t.px.assign(im.px.begin(), im.px.begin() + (size_t)im.w * im.h * 3);
  return s->s.add_tex(std::move(t));
}
int srr_image_texture_gen(srr_scene* s, int nx, int ny, uint32_t seed, int kind) {
  SCN(s);
  if (nx <= 0 || ny <= 0 || kind < 0 || kind > 2) return fail(SRR_EINVAL, "bad image_gen");
  HTex t;
  t.kind = TEX_IMAGE;
  t.nx = nx;
  t.ny = ny;
  t.px = gen_image(nx, ny, seed, kind);
  return s->s.add_tex(std::move(t));
}
int srr_checker_texture(srr_scene* s, int even, int odd) {
  SCN(s);
  TEXOK(s, even);
  TEXOK(s, odd);
  HTex t;
  t.kind = TEX_CHECKER;
  t.even = even;
  t.odd = odd;
  return s->s.add_tex(std::move(t));
}
int srr_noise_texture(srr_scene* s, float scale) {
  SCN(s);
  HTex t;
  t.kind = TEX_NOISE;
  t.c[0] = scale;
  return s->s.add_tex(std::move(t));
}

static int mat_with_tex(srr_scene* s, MatKind k, int tex, float a = 0, float b = 0) {
  SCN(s);
  TEXOK(s, tex);
  float p[4] = {a, b, 0, 0};
  return s->s.material(k, tex, p);
}
int srr_lambertian(srr_scene* s, int t) { return mat_with_tex(s, MAT_LAMBERTIAN, t); }
int srr_orennayar(srr_scene* s, int t, float sigma) { return mat_with_tex(s, MAT_ORENNAYAR, t, sigma); }
int srr_beckmann(srr_scene* s, int t, float rx, float ry) { return mat_with_tex(s, MAT_BECKMANN, t, rx, ry); }
int srr_diffuse_light(srr_scene* s, int t) { return mat_with_tex(s, MAT_DIFFUSE_LIGHT, t); }
int srr_isotropic(srr_scene* s, int t) { return mat_with_tex(s, MAT_ISOTROPIC, t); }
int srr_metal(srr_scene* s, float r, float g, float b, float fuzz) {
  SCN(s);
  float p[4] = {r, g, b, fuzz};
  return s->s.material(MAT_METAL, -1, p);
}
int srr_dielectric(srr_scene* s, float ri) {
  SCN(s);
  float p[4] = {ri, 0, 0, 0};
  return s->s.material(MAT_DIELECTRIC, -1, p);
}

int srr_sphere(srr_scene* s, const float c[3], float r, int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.sphere(c, r, m);
}
int srr_moving_sphere(srr_scene* s, const float c0[3], const float c1[3], float t0, float t1, float r, int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.moving_sphere(c0, c1, t0, t1, r, m);
}
int srr_xy_rect(srr_scene* s, float x0, float x1, float y0, float y1, float k, int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.rect(H_XY, x0, x1, y0, y1, k, m);
}
int srr_xz_rect(srr_scene* s, float x0, float x1, float z0, float z1, float k, int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.rect(H_XZ, x0, x1, z0, z1, k, m);
}
int srr_yz_rect(srr_scene* s, float y0, float y1, float z0, float z1, float k, int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.rect(H_YZ, y0, y1, z0, z1, k, m);
}
int srr_box(srr_scene* s, const float p0[3], const float p1[3], int m) {
  SCN(s);
  MATOK(s, m);
  return s->s.box(p0, p1, m);
}
int srr_triangle(srr_scene* s, const float p[9], int m, const float* uv9, const float* n9) {
  SCN(s);
  MATOK(s, m);
  if (!p) return fail(SRR_EINVAL, "null vertices");
  return s->s.triangle(p, m, uv9, n9);
}
int srr_flip_normals(srr_scene* s, int c) {
  SCN(s);
  OBJOK(s, c);
  return s->s.wrap(H_FLIP, c, nullptr);
}
int srr_translate(srr_scene* s, int c, const float off[3]) {
  SCN(s);
  OBJOK(s, c);
  return s->s.wrap(H_TRANSLATE, c, off);
}
int srr_rotate_y(srr_scene* s, int c, float a) {
  SCN(s);
  OBJOK(s, c);
  return s->s.rotate(H_ROTY, c, a);
}
int srr_rotate_x(srr_scene* s, int c, float a) {
  SCN(s);
  OBJOK(s, c);
  return s->s.rotate(H_ROTX, c, a);
}
int srr_constant_medium(srr_scene* s, int b, float density, int tex) {
  SCN(s);
  OBJOK(s, b);
  TEXOK(s, tex);
  return s->s.medium(b, density, tex);
}
int srr_hitable_list(srr_scene* s, const int* kids, int n) {
  SCN(s);
  if (n < 0 || (n > 0 && !kids)) return fail(SRR_EINVAL, "bad list");
  for (int i = 0; i < n; ++i) OBJOK(s, kids[i]);
  return s->s.list(kids, n);
}
int srr_bvh_node(srr_scene* s, const int* kids, int n, float t0, float t1) {
  SCN(s);
  if (n < 1 || !kids) return fail(SRR_EINVAL, "bvh_node needs n >= 1 children");
  for (int i = 0; i < n; ++i) OBJOK(s, kids[i]);
  return s->s.bvh(kids, n, t0, t1);
}
int srr_teapot(srr_scene* s, float scale, int divs, int m, int* first) {
  SCN(s);
  MATOK(s, m);
  if (divs < 1 || divs > 400) return fail(SRR_EINVAL, "teapot divs out of range");
  return s->s.teapot(scale, divs, m, first);
}
int srr_camera(srr_scene* s, const float lf[3], const float la[3], const float vup[3], float vfov, float aspect,
               float aperture, float focus, float t0, float t1) {
  SCN(s);
  s->s.camera(lf, la, vup, vfov, aspect, aperture, focus, t0, t1);
  return 0;
}
int srr_scene_set_world(srr_scene* s, int o) {
  SCN(s);
  OBJOK(s, o);
  s->s.world = o;
  return 0;
}
int srr_scene_set_lights(srr_scene* s, int o) {
  SCN(s);
  OBJOK(s, o);
  if (s->s.obj[o].kind != H_LIST) return fail(SRR_EINVAL, "lights must be a hitable_list (Raytracing_n.cpp:75)");
  s->s.lights = o;
  return 0;
}

// --------------------------------------------------------------- renderer
int srr_renderer_create(const srr_scene* sc, int device, srr_renderer** out) {
  if (!sc || !out) return fail(SRR_EINVAL, "null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(SRR_ENODEV, "no HIP device (the srr renderer has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(SRR_ENODEV, "device index out of range");
  std::string err;
  int rc = renderer_create(sc->s, device, out, err);
  if (rc < 0) return fail(rc, err);
  return 0;
}

void srr_renderer_destroy(srr_renderer* r) { delete r; }

int srr_renderer_create_multi(const srr_scene* sc, int n, const int* ids, srr_renderer** out) {
  if (!sc || !out || !ids) return fail(SRR_EINVAL, "null argument");
  std::string err;
  int rc = multi_create(sc->s, n, ids, out, err);
  if (rc < 0) return fail(rc, err);
  return 0;
}

int srr_renderer_devices(const srr_renderer* r, int* ids, int cap) {
  if (!r) return fail(SRR_EINVAL, "null renderer");
  if (r->multi) return multi_devices(r->multi, ids, cap);
  if (ids && cap > 0) ids[0] = r->device;
  return 1;
}

const char* srr_renderer_transport(const srr_renderer* r) {
  return !r ? "" : r->multi ? multi_transport(r->multi) : "none";
}

int64_t srr_multi_plan(const srr_params* p, int n, int32_t* index, int64_t* off) {
  std::string err;
  const int64_t rc = multi_plan(p, n, nullptr, index, off, err);
  if (rc < 0) return fail((int)rc, err);
  return rc;
}

int64_t srr_shard_pixels(const srr_params* p, int32_t* out) {
  if (!p || p->nx <= 0 || p->ny <= 0 || p->shard_count < 1 || p->shard_index < 0 ||
      p->shard_index >= p->shard_count)
    return fail(SRR_EINVAL, "bad params");
  // shard tiles round-robin, each tile row rotated by one: tile
  // t = tr * tiles_x + tc (tr = row / tile, tc = col / tile) belongs to shard
  // (t + tr) % shard_count.  Without the rotation a frame tiles_x tiles wide splits
  // into whole tile columns whenever shard_count divides tiles_x (C2 at 8 GPUs:
  // rank k renders columns k and k + 8, 4.7 % above the mean in world rays; with it
  // 1.4 %).  Pixels in PPM order within the shard, emitted row by row as runs of a
  // tile's columns.
  const int tile = p->shard_count == 1 ? p->nx : (p->tile > 0 ? p->tile : 32);
  const int tiles_x = (p->nx + tile - 1) / tile;
  int64_t n = 0;
  for (int row = 0; row < p->ny; ++row) {
    const int tr = row / tile, t0 = tr * tiles_x + tr;
    for (int tc = 0; tc < tiles_x; ++tc) {
      if ((t0 + tc) % p->shard_count != p->shard_index) continue;
      const int c1 = std::min(p->nx, (tc + 1) * tile);
      for (int col = tc * tile; col < c1; ++col) {
        if (out) out[n] = row * p->nx + col;
        ++n;
      }
    }
  }
  return n;
}

int srr_render_device(srr_renderer* r, const srr_params* p, float* d_mean, srr_stats* stats) {
  if (!r || !p || !d_mean) return fail(SRR_EINVAL, "null argument");
  if (p->spp < 1 || p->max_depth < 0 || p->max_depth > 64) return fail(SRR_EINVAL, "spp >= 1, 0 <= max_depth <= 64");
  if (p->sample_begin < 0 || p->sample_begin > INT32_MAX - p->spp)
    return fail(SRR_EINVAL, "sample_begin must be >= 0 and sample_begin + spp must fit in int32");
  if (r->multi) {
    std::string err;
    const int rc = multi_render_device(r, p, d_mean, stats, err);
    return rc < 0 ? fail(rc, err) : 0;
  }
  // the shard's pixel list is built and uploaded once per shard (srr_renderer::pix_key)
  const int key[5] = {p->nx, p->ny, p->shard_index, p->shard_count, p->tile};
  const bool held = std::equal(key, key + 5, r->pix_key);
  int64_t npix = held ? r->pix_n : srr_shard_pixels(p, nullptr);
  if (npix < 0) return (int)npix;
  std::vector<int32_t> pix;
  if (!held) {
    pix.resize(npix);
    srr_shard_pixels(p, pix.data());
  }
  // a new list overwrites the held one before anything can fail: forget its key
  // until the render succeeds (a failed call must not leave the old shard "held")
  if (!held) r->pix_key[0] = -1;
  std::string err;
  int rc = render_device(r, p, held ? nullptr : pix.data(), npix, d_mean, stats, err);
  if (rc < 0) return fail(rc, err);
  if (!held) {
    std::copy(key, key + 5, r->pix_key);
    r->pix_n = npix;
  }
  return 0;
}

int srr_render_device_async(srr_renderer* r, const srr_params* p, float* d_mean, int64_t* ticket) {
  if (!r || !p || !d_mean || !ticket) return fail(SRR_EINVAL, "null argument");
  if (p->spp < 1 || p->max_depth < 0 || p->max_depth > 64) return fail(SRR_EINVAL, "spp >= 1, 0 <= max_depth <= 64");
  if (p->sample_begin < 0 || p->sample_begin > INT32_MAX - p->spp)
    return fail(SRR_EINVAL, "sample_begin must be >= 0 and sample_begin + spp must fit in int32");
  if (r->multi) {
    std::string err;
    const int rc = multi_render_device_async(r, p, d_mean, ticket, err);
    return rc < 0 ? fail(rc, err) : 0;
  }
  const int key[5] = {p->nx, p->ny, p->shard_index, p->shard_count, p->tile};
  const bool held = std::equal(key, key + 5, r->pix_key);
  int64_t npix = held ? r->pix_n : srr_shard_pixels(p, nullptr);
  if (npix < 0) return (int)npix;
  std::vector<int32_t> pix;
  if (!held) {
    pix.resize(npix);
    srr_shard_pixels(p, pix.data());
  }
  // a new list overwrites the held one before anything can fail: forget its key
  // until the render succeeds (a failed call must not leave the old shard "held")
  if (!held) r->pix_key[0] = -1;
  std::string err;
  int rc = render_device_async(r, p, held ? nullptr : pix.data(), npix, d_mean, ticket, err);
  if (rc < 0) return fail(rc, err);
  if (!held) {
    std::copy(key, key + 5, r->pix_key);
    r->pix_n = npix;
  }
  return 0;
}

int srr_render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats) {
  if (!r) return fail(SRR_EINVAL, "null renderer");
  std::string err;
  int rc = r->multi ? multi_render_wait(r, ticket, stats, err) : render_wait(r, ticket, stats, err);
  if (rc < 0) return fail(rc, err);
  return 0;
}

int srr_render(srr_renderer* r, const srr_params* p, float* mean, unsigned char* rgb8, srr_stats* stats) {
  if (!r || !p) return fail(SRR_EINVAL, "null argument");
  if (r->multi && p->shard_count > 1)
    return fail(SRR_EINVAL, "a multi-device renderer shards the frame itself: shard_count must be 0 or 1");
  int64_t npix = r->multi ? (p->nx > 0 && p->ny > 0 ? (int64_t)p->nx * p->ny : -1) : srr_shard_pixels(p, nullptr);
  if (npix < 0 && r->multi) return fail(SRR_EINVAL, "bad params");
  if (npix < 0) return (int)npix;
  float* d = nullptr;
  HIPCHK(hipSetDevice(r->device));
  HIPCHK(hipMalloc((void**)&d, 3 * npix * sizeof(float)));
  int rc = srr_render_device(r, p, d, stats);
  std::vector<float> h(3 * npix);
  if (rc == 0) {
    hipError_t e = hipMemcpy(h.data(), d, h.size() * sizeof(float), hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(SRR_EIO, hipGetErrorString(e));
  }
  hipFree(d);
  if (rc < 0) return rc;
  if (mean) std::memcpy(mean, h.data(), h.size() * sizeof(float));
  if (rgb8) srr_tonemap(h.data(), npix, rgb8);
  return 0;
}

int srr_accum_get(srr_renderer* r, float* sums, int64_t* npix, int64_t* samples) {
  if (!r) return fail(SRR_EINVAL, "null renderer");
  if (r && r->multi) return fail(SRR_EINVAL, "progressive sums and kept paths are per device: use a one-device renderer");
  if (npix) *npix = r->acc_npix;
  if (samples) *samples = r->acc_samples;
  if (sums && r->acc_npix) {
    HIPCHK(hipSetDevice(r->device));
    HIPCHK(hipMemcpy(sums, r->acc, 3 * r->acc_npix * sizeof(float), hipMemcpyDeviceToHost));
  }
  return 0;
}

int srr_accum_set(srr_renderer* r, const float* sums, int64_t npix, int64_t samples) {
  if (!r || !sums || npix <= 0 || samples < 0) return fail(SRR_EINVAL, "bad accumulator state");
  if (r && r->multi) return fail(SRR_EINVAL, "progressive sums and kept paths are per device: use a one-device renderer");
  HIPCHK(hipSetDevice(r->device));
  drain_async(r);  // frames in flight read the pixel list this may reallocate
  if ((size_t)npix > r->pix_cap) {
    r->pix_key[0] = -1;  // the held pixel list goes with the buffer
    (void)hipFree(r->pixels);
    (void)hipFree(r->acc);
    r->pixels = nullptr;
    r->acc = nullptr;
    r->pix_cap = 0;
    HIPCHK(hipMalloc((void**)&r->pixels, npix * sizeof(int32_t)));
    HIPCHK(hipMalloc((void**)&r->acc, 3 * npix * sizeof(float)));
    r->pix_cap = npix;
  }
  HIPCHK(hipMemcpy(r->acc, sums, 3 * npix * sizeof(float), hipMemcpyHostToDevice));
  r->acc_npix = npix;
  r->acc_samples = samples;
  std::fill(r->acc_key, r->acc_key + 5, -1);  // any frame / shard of npix pixels may continue them
  return 0;
}

int srr_copy_paths(srr_renderer* r, float* radiance, unsigned char* rays) {
  if (r && r->multi) return fail(SRR_EINVAL, "progressive sums and kept paths are per device: use a one-device renderer");
  if (!r || !r->raw_all) return fail(SRR_EINVAL, "render with SRR_FLAG_KEEP_PATHS first");
  HIPCHK(hipSetDevice(r->device));
  if (radiance) HIPCHK(hipMemcpy(radiance, r->raw_all, r->kept_paths * 3 * sizeof(float), hipMemcpyDeviceToHost));
  if (rays) HIPCHK(hipMemcpy(rays, r->rays_all, r->kept_paths, hipMemcpyDeviceToHost));
  return 0;
}

int srr_tonemap(const float* mean, int64_t n, unsigned char* rgb8) {  // Raytracing_n.cpp:850-862
  if (!mean || !rgb8) return fail(SRR_EINVAL, "null argument");
  for (int64_t i = 0; i < 3 * n; ++i) {
    float c = std::sqrt(mean[i]);
    int q = int(255.99 * c);
    q = q > 255 ? 255 : q;
    q = q < 0 ? 0 : q;
    rgb8[i] = (unsigned char)q;
  }
  return 0;
}

int srr_mesh_file_triangles(const char* path, int flip_uvs, int flip_winding, const float scale[3], float* pos9,
                            float* uv9, float* nrm9, int* flags_out) {
  if (!path || !scale) return fail(SRR_EINVAL, "null argument");
  srr::MeshData m;
  std::string err;
  if (srr::load_mesh_file(path, m, err) < 0) return fail(SRR_EIO, err);
  srr::apply_model_semantics(m, flip_uvs != 0, flip_winding != 0, scale);
  for (size_t t = 0; t < m.tris.size(); ++t)
    for (int j = 0; j < 3; ++j) {
      const srr::MeshData::Corner& c = m.tris[t][j];
      if (pos9) std::memcpy(pos9 + 9 * t + 3 * j, c.p, 12);
      if (uv9) std::memcpy(uv9 + 9 * t + 3 * j, c.uv, 12);
      if (nrm9) std::memcpy(nrm9 + 9 * t + 3 * j, c.n, 12);
    }
  if (flags_out) *flags_out = (m.has_normals ? 1 : 0) | (m.has_uvs ? 2 : 0);
  if (m.tris.size() > (size_t)INT32_MAX / 2) return fail(SRR_EINVAL, "mesh too large");
  return (int)m.tris.size();
}

int srr_model(srr_scene* s, const char* path, int flip_uvs, int flip_winding, int mat, const float scale[3],
              int* first_handle) {
  if (!s || !path || !scale) return fail(SRR_EINVAL, "null argument");
  srr::MeshData m;
  std::string err;
  if (srr::load_mesh_file(path, m, err) < 0) return fail(SRR_EIO, err);
  srr::apply_model_semantics(m, flip_uvs != 0, flip_winding != 0, scale);
  if (m.tris.empty()) return fail(SRR_EINVAL, std::string(path) + ": mesh 0 has no triangles");
  int first = -1;
  for (const auto& t : m.tris) {
    float p[9], uv[9], n[9];
    for (int j = 0; j < 3; ++j) {
      std::memcpy(p + 3 * j, t[j].p, 12);
      std::memcpy(uv + 3 * j, t[j].uv, 12);
      std::memcpy(n + 3 * j, t[j].n, 12);
    }
    int h = srr_triangle(s, p, mat, uv, m.has_normals ? n : nullptr);
    if (h < 0) return h;
    if (first < 0) first = h;
  }
  if (first_handle) *first_handle = first;
  return (int)m.tris.size();
}

int srr_write_ppm(const char* path, int nx, int ny, const unsigned char* rgb8) {
  FILE* f = fopen(path, "w");
  if (!f) return fail(SRR_EIO, std::string("cannot open ") + path);
  fprintf(f, "P3\n%d %d\n255\n", nx, ny);
  for (int i = 0; i < nx * ny; ++i) fprintf(f, "%d %d %d\n", rgb8[3 * i], rgb8[3 * i + 1], rgb8[3 * i + 2]);
  fclose(f);
  return 0;
}

int srr_write_png(const char* path, int nx, int ny, const unsigned char* rgb8) {
  if (!path || !rgb8) return fail(SRR_EINVAL, "null argument");
  std::vector<uint8_t> png;
  std::string err;
  int rc = srr::encode_png(rgb8, nx, ny, 3, png, err);
  if (rc < 0) return fail(rc, err);
  FILE* f = fopen(path, "wb");
  if (!f) return fail(SRR_EIO, std::string("cannot open ") + path);
  size_t w = fwrite(png.data(), 1, png.size(), f);
  fclose(f);
  return w == png.size() ? 0 : fail(SRR_EIO, std::string("short write to ") + path);
}

int srr_image_load(const char* path, int req_comp, int* x, int* y, int* comp, unsigned char** out) {
  if (!path || !x || !y || !out) return fail(SRR_EINVAL, "null argument");
  *out = nullptr;
  srr::Image im;
  std::string err;
  int rc = srr::load_image(path, req_comp, im, err);
  if (rc < 0) return fail(rc == -2 ? SRR_EIO : SRR_EINVAL, err);
  *x = im.w;
  *y = im.h;
  if (comp) *comp = im.file_n;
  *out = (unsigned char*)malloc(im.px.size());
  if (!*out) return fail(SRR_ENOMEM, "out of memory");
  std::memcpy(*out, im.px.data(), im.px.size());
  return im.n;
}

void srr_image_free(unsigned char* pixels) { free(pixels); }

int srr_device_kat(const char* name, int n, int width, float* records) {
  if (!name || !records || n <= 0 || width <= 0) return fail(SRR_EINVAL, "bad KAT arguments");
  static const char* kNames[] = {"erf",   "beckmann11", "beckmann_dist", "beckmann_pdf", "cosine_pdf",
                                 "orennayar_pdf", "dielectric", "metal", "triangle", "aabb", "sqrt",
                                 "camera", "lights", "light_list"};
  static const int kWidth[] = {3, 5, 16, 21, 21, 21, 14, 14, 26, 15, 2, 23, 15, 15};
  int kind = -1;
  for (int k = 0; k < 14; ++k)
    if (!strcmp(name, kNames[k])) kind = k;
  if (kind < 0) return fail(SRR_EINVAL, std::string("no device KAT named ") + name);
  if (width != kWidth[kind]) return fail(SRR_EINVAL, std::string("KAT ") + name + ": unexpected record width");
  // host-side parameters the scene builder would compute (material ctors, face normals)
  std::vector<float> aux(4 * (size_t)n, 0.f);
  std::vector<DStandaloneTri> tris(kind == 8 ? n : 1);
  Scene hs;
  for (int q = 0; q < n; ++q) {
    const float* r = records + (size_t)q * width;
    if (kind == 2 || kind == 3) {
      const float prm[4] = {r[0], r[1], 0, 0};
      const HMat& m = hs.mat[hs.material(MAT_BECKMANN, -1, prm)];
      aux[4 * q] = m.p[0];
      aux[4 * q + 1] = m.p[1];
    } else if (kind == 4 || kind == 5) {
      const float prm[4] = {r[0], 0, 0, 0};
      const HMat& m = hs.mat[hs.material(MAT_ORENNAYAR, -1, prm)];
      aux[4 * q] = m.p[0];
      aux[4 * q + 1] = m.p[1];
    } else if (kind == 8) {  // triangle(p0, p1, p2, mat, uv0, uv1, uv2) with face normals (kat.inc)
      const float uv9[9] = {0.1f, 0.2f, 0, 0.7f, 0.1f, 0, 0.3f, 0.9f, 0};
      const int h = hs.triangle(r, -1, uv9, nullptr);
      const HTri& t = hs.tris[hs.obj[h].tri];
      DStandaloneTri& d = tris[q];
      std::memcpy(d.p, t.p, 36);
      std::memcpy(d.sh.n, t.n, 36);
      for (int k = 0; k < 3; ++k) d.sh.uv[2 * k] = t.uv[3 * k], d.sh.uv[2 * k + 1] = t.uv[3 * k + 1];
      d.sh.mat = -1;
    }
  }
  // camera KAT: camera(lookfrom, lookat, (0,1,0), vfov, aspect, aperture, focus, 0, 1) per record, built
  // by the host scene code exactly as a scene's camera (camera.h:33-48)
  std::vector<DCamera> cams(kind == 11 ? n : 1);
  if (kind == 11) {
    for (int q = 0; q < n; ++q) {
      const float* r = records + (size_t)q * width;
      const float vup[3] = {0, 1, 0};
      Scene cs;
      cs.camera(r, r + 3, vup, r[6], r[7], r[8], r[9], 0.0f, 1.0f);
      const HCamera& c = cs.cam;
      DCamera& d = cams[q];
      std::memcpy(d.origin, c.origin, 12);
      std::memcpy(d.llc, c.llc, 12);
      std::memcpy(d.horizontal, c.horizontal, 12);
      std::memcpy(d.vertical, c.vertical, 12);
      std::memcpy(d.u, c.u, 12);
      std::memcpy(d.v, c.v, 12);
      d.time0 = c.time0;
      d.time1 = c.time1;
      d.lens_radius = c.lens_radius;
    }
  }
  // light KATs: the light list {flip(xz_rect(213,343,227,332,554)), sphere((278,700,280),50),
  // triangle((150,500,150),(400,520,180),(260,540,420))} of oracle/ref/kat.inc, flattened like a scene's
  Flat lf;
  if (kind == 12 || kind == 13) {
    Scene ls;
    const int rect = ls.wrap(H_FLIP, ls.rect(H_XZ, 213, 343, 227, 332, 554, -1), nullptr);
    const float c[3] = {278, 700, 280};
    const int sph = ls.sphere(c, 50, -1);
    const float p9[9] = {150, 500, 150, 400, 520, 180, 260, 540, 420};
    const int tri = ls.triangle(p9, -1, nullptr, nullptr);
    const int kids[3] = {rect, sph, tri};
    ls.world = ls.lights = ls.list(kids, 3);
    const float lf3[3] = {0, 0, -1}, la3[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    ls.camera(lf3, la3, up, 40, 1, 0, 1, 0, 1);
    ls.has_camera = true;
    std::string e;
    if (flatten(ls, lf, e) < 0 || lf.lights.size() != 3) return fail(SRR_EINVAL, "light KAT scene: " + e);
  }
  float* d_rec = nullptr;
  float* d_aux = nullptr;
  DStandaloneTri* d_tris = nullptr;
  DCamera* d_cams = nullptr;
  DRect* d_rects = nullptr;
  DSphere* d_sph = nullptr;
  DStandaloneTri* d_stris = nullptr;
  DLight* d_lights = nullptr;
  const size_t rb = (size_t)n * width * sizeof(float);
  int rc = 0;
  if (hipMalloc((void**)&d_rec, rb) != hipSuccess || hipMalloc((void**)&d_aux, aux.size() * 4) != hipSuccess ||
      hipMalloc((void**)&d_tris, tris.size() * sizeof(DStandaloneTri)) != hipSuccess)
    rc = fail(SRR_ENOMEM, "device allocation failed");
  if (!rc && (hipMemcpy(d_rec, records, rb, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_aux, aux.data(), aux.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_tris, tris.data(), tris.size() * sizeof(DStandaloneTri), hipMemcpyHostToDevice) != hipSuccess))
    rc = fail(SRR_EIO, "copy to device failed");
  auto upload = [&rc](auto*& dst, const auto& v) {
    if (rc || v.empty()) return;
    const size_t b = v.size() * sizeof(v[0]);
    if (hipMalloc((void**)&dst, b) != hipSuccess) rc = fail(SRR_ENOMEM, "device allocation failed");
    else if (hipMemcpy(dst, v.data(), b, hipMemcpyHostToDevice) != hipSuccess) rc = fail(SRR_EIO, "copy to device failed");
  };
  upload(d_cams, cams);
  upload(d_rects, lf.rects);
  upload(d_sph, lf.spheres);
  upload(d_stris, lf.stris);
  upload(d_lights, lf.lights);
  const KatTables kt{d_cams, d_rects, d_sph, d_stris, d_lights, (int)lf.lights.size()};
  if (!rc && launch_kat(kind, n, width, d_rec, d_aux, d_tris, kt) < 0) rc = fail(SRR_EIO, "KAT kernel launch failed");
  if (!rc && (hipDeviceSynchronize() != hipSuccess || hipMemcpy(records, d_rec, rb, hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail(SRR_EIO, "KAT kernel failed");
  for (void* p : {(void*)d_rec, (void*)d_aux, (void*)d_tris, (void*)d_cams, (void*)d_rects, (void*)d_sph,
                  (void*)d_stris, (void*)d_lights})
    (void)hipFree(p);
  return rc;
}

// ---- MERL tables (brdf.h)
struct srr_merl {
  int device = 0;
  double* table = nullptr;  // device: 3 * merl::kCells doubles
};

int srr_merl_create(const double* table, int64_t n_doubles, int device, srr_merl** out) {
  if (!table || !out) return fail(SRR_EINVAL, "null argument");
  if (n_doubles != 3 * (int64_t)merl::kCells) return fail(SRR_EINVAL, "MERL table: dimensions don't match");
  HIPCHK(hipSetDevice(device));
  auto m = std::make_unique<srr_merl>();
  m->device = device;
  HIPCHK(hipMalloc((void**)&m->table, (size_t)n_doubles * sizeof(double)));
  if (hipMemcpy(m->table, table, (size_t)n_doubles * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(m->table);
    return fail(SRR_EIO, "MERL table upload failed");
  }
  *out = m.release();
  return 0;
}

int srr_merl_load(const char* path, int device, srr_merl** out) {  // brdf::read_brdf (brdf.h:156-185)
  if (!path || !out) return fail(SRR_EINVAL, "null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(SRR_EIO, std::string("cannot open MERL table ") + path);
  int32_t dims[3] = {0, 0, 0};
  const bool hdr = fread(dims, sizeof(int32_t), 3, f) == 3;
  const int64_t n = (int64_t)dims[0] * dims[1] * dims[2];
  if (!hdr || n != merl::kCells) {
    fclose(f);
    return fail(SRR_EINVAL, "MERL table: dimensions don't match");
  }
  std::vector<double> t(3 * (size_t)n);
  const size_t got = fread(t.data(), sizeof(double), t.size(), f);
  fclose(f);
  if (got != t.size()) return fail(SRR_EINVAL, "MERL table: truncated file");
  return srr_merl_create(t.data(), (int64_t)t.size(), device, out);
}

void srr_merl_destroy(srr_merl* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  (void)hipFree(m->table);
  delete m;
}

int srr_merl_lookup(srr_merl* m, int64_t n, const double* angles, double* rgb, int32_t* cell) {
  if (!m || n < 0 || (n > 0 && (!angles || !rgb))) return fail(SRR_EINVAL, "bad MERL lookup arguments");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(m->device));
  double *d_ang = nullptr, *d_rgb = nullptr;
  int32_t* d_cell = nullptr;
  int rc = 0;
  if (hipMalloc((void**)&d_ang, 4 * (size_t)n * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&d_rgb, 3 * (size_t)n * sizeof(double)) != hipSuccess ||
      (cell && hipMalloc((void**)&d_cell, (size_t)n * sizeof(int32_t)) != hipSuccess))
    rc = fail(SRR_ENOMEM, "device allocation failed");
  if (!rc && hipMemcpy(d_ang, angles, 4 * (size_t)n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(SRR_EIO, "copy to device failed");
  if (!rc && launch_merl_lookup(m->table, n, d_ang, d_rgb, d_cell) < 0) rc = fail(SRR_EIO, "MERL kernel launch failed");
  if (!rc && (hipDeviceSynchronize() != hipSuccess ||
              hipMemcpy(rgb, d_rgb, 3 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
              (cell && hipMemcpy(cell, d_cell, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)))
    rc = fail(SRR_EIO, "MERL kernel failed");
  (void)hipFree(d_ang);
  (void)hipFree(d_rgb);
  (void)hipFree(d_cell);
  return rc;
}

int srr_teapot_vertices(float scale, int divs, float* out) {
  if (divs < 1 || divs > 400) return fail(SRR_EINVAL, "teapot divs out of range");
  std::vector<float> p;
  teapot_triangles(scale, divs, p);
  if (out) std::memcpy(out, p.data(), p.size() * sizeof(float));
  return (int)(p.size() / 9);
}

int64_t srr_bvh_topology(const srr_scene* s, int o, char* buf, int64_t cap) {
  if (!s || !s->s.valid_obj(o) || s->s.obj[o].kind != H_BVH) return fail(SRR_EINVAL, "not a bvh_node handle");
  const HBvh& B = s->s.bvhs[s->s.obj[o].bvh];
  std::map<int, int> pos;
  for (size_t q = 0; q < B.input.size(); ++q) pos[B.input[q]] = (int)q;
  std::string txt;
  char line[256];
  snprintf(line, sizeof line, "box %g %g %g %g %g %g\n", B.box.mn[0], B.box.mn[1], B.box.mn[2], B.box.mx[0],
           B.box.mx[1], B.box.mx[2]);
  txt += line;
  std::vector<int> stack{0};
  while (!stack.empty()) {
    int n = stack.back();
    stack.pop_back();
    const HBvh::Node& nd = B.nodes[n];
    if (nd.left < 0) {
      snprintf(line, sizeof line, "L %d %d\n", pos[B.leaves[~nd.left]], pos[B.leaves[~nd.right]]);
      txt += line;
    } else {
      txt += "N\n";
      stack.push_back(nd.right);
      stack.push_back(nd.left);
    }
  }
  if (buf && cap > 0) {
    int64_t m = std::min<int64_t>(cap - 1, (int64_t)txt.size());
    std::memcpy(buf, txt.data(), m);
    buf[m] = 0;
  }
  return (int64_t)txt.size() + 1;
}

int srr_sobol_points(int n, double* out) {
  if (n < 1 || !out) return fail(SRR_EINVAL, "bad args");
  sobol2((unsigned)n, out);
  return 0;
}

}  // extern "C"

// Reference harness: compiles the REFERENCE translation unit itself
// (/root/reference/Raytracing_n/Raytracing_n.cpp, transcoded UTF-16 -> UTF-8 by
// oracle/ref/Makefile into a scratch dir that never enters git or the GPU-box
// snapshot) and drives the reference's own classes and functions to produce
// golden vectors under tests/golden/.  TEST INFRASTRUCTURE ONLY: nothing under
// oracle/ is linked into, or called by, the product path.
//
// Deterministic mode: single thread, and the reference's global
// RNGs -- `seed` (mathf.h:12) and `s_rng` (pdf.h:20) -- are re-seeded per path
// from (x, y, s) with srr_text::path_seed, so every path is order independent.
//
// Commands:
//   render <scene.txt> <nx> <ny> <ns> <maxdepth> <out_prefix>
//   sums   <scene.txt> <nx> <ny> <ns> <maxdepth> <pix0> <pix1> <out_prefix>
//                                                 per-pixel digest (full frames)
//   bvh    <scene.txt> <obj_id> <out.txt>          reference BVH topology
//   teapot <scale> <divs> <out.f32>                tessellated vertices
//   sobol  <N> <out.f64>
//   kat    <name> <n> <seed> <out.bin>             per-function known answers
//   image  <file> <req_comp> <out.raw>             stbi_load (stb_image v2.19)
//   builder <name> <nx> <ny> <ns> <maxdepth> <out_prefix>   a reference scene builder
#define private public
#define main ref_main
#include "Raytracing_n.cpp"
#undef main
#undef private

#include "../scene_text.h"

#include <unistd.h>

using srr_text::Cmd;

namespace {

// ---------------------------------------------------------------- scene build
struct RefScene {
  std::map<long long, texture*> tex;
  std::map<long long, material*> mat;
  std::map<long long, hitable*> obj;
  std::map<long long, std::vector<hitable*>> grp;
  camera* cam = nullptr;
  hitable* world = nullptr;
  hitable* lights = nullptr;
  std::vector<std::vector<unsigned char>*> images;
};

material* M(RefScene& S, long long id) {
  if (id < 0) return nullptr;
  return S.mat.at(id);
}

vec3 V3(const Cmd& c, size_t k) { return vec3(c.f(k), c.f(k + 1), c.f(k + 2)); }

// Triangles made with the 4- and 7-argument constructors leave n0..n2
// unset (triangle.h:13-34), while FLAT_NORMAL (triangle.h:7,178-183) shades with
// them: SURVEY Q5's build definition gives them the face normal.
void face_normals(triangle* t) { t->n0 = t->n1 = t->n2 = t->normal; }

// Teapot with a chosen subdivision: the same per-patch grid and quad split as
// teapot::createPloyTeapot (teapot.h:76-166, which hard-codes divs=100), built
// with the reference's own evalBezierPatch and the 10-argument triangle ctor.
std::vector<hitable*> make_teapot(float scale, int divs, material* m) {
  teapot tp(scale, m);
  std::vector<vec3> P((divs + 1) * (divs + 1));
  std::vector<hitable*> tris;
  vec3 cp[16];
  for (int np = 0; np < kTeapotNumPatches; ++np) {
    for (int i = 0; i < 16; ++i)
      for (int c = 0; c < 3; ++c) cp[i][c] = teapotVertices[teapotPatches[np][i] - 1][c] * scale;
    for (int j = 0, k = 0; j <= divs; ++j) {
      float v = (float)j / (float)divs;
      for (int i = 0; i <= divs; ++i, ++k) {
        float u = (float)i / (float)divs;
        P[k] = tp.evalBezierPatch(cp, u, v);
      }
    }
    for (int j = 0; j < divs; ++j)
      for (int i = 0; i < divs; ++i) {
        int q[4] = {(divs + 1) * j + i, (divs + 1) * j + i + 1, (divs + 1) * (j + 1) + i + 1,
                    (divs + 1) * (j + 1) + i};
        for (int t = 0; t < 2; ++t) {
          triangle* tri = new triangle(P[q[0]], P[q[t + 1]], P[q[t + 2]], m);
          face_normals(tri);
          tris.push_back(tri);
        }
      }
  }
  return tris;
}

RefScene build(const std::vector<Cmd>& cmds) {
  RefScene S;
  seed = srr_text::kPostPerlinSeed;
  for (const Cmd& c : cmds) {
    const std::string& k = c.at(0);
    if (k == "srr_scene") continue;
    if (k == "lcg") { seed = c.u(1); continue; }
    if (k == "tex") {
      long long id = c.i(1);
      const std::string& t = c.at(2);
      if (t == "const") S.tex[id] = new constant_texture(V3(c, 3));
      else if (t == "image_gen") {
        int w = (int)c.i(3), h = (int)c.i(4);
        auto* px = new std::vector<unsigned char>(srr_text::gen_image(w, h, (unsigned)c.u(5), (int)c.i(6)));
        S.images.push_back(px);
        S.tex[id] = new image_texture(px->data(), w, h);
      } else if (t == "image_raw") {
        int w = (int)c.i(3), h = (int)c.i(4);
        auto* px = new std::vector<unsigned char>(srr_text::read_raw_image(c.at(5), w, h));
        S.images.push_back(px);
        S.tex[id] = new image_texture(px->data(), w, h);
      } else if (t == "checker") S.tex[id] = new checker_texture(S.tex.at(c.i(3)), S.tex.at(c.i(4)));
      else if (t == "noise") S.tex[id] = new noise_texture(c.f(3));
      else throw std::runtime_error("tex kind " + t);
      continue;
    }
    if (k == "mat") {
      long long id = c.i(1);
      const std::string& t = c.at(2);
      if (t == "lambertian") S.mat[id] = new lambertian(S.tex.at(c.i(3)));
      else if (t == "orennayar") S.mat[id] = new orennayar(S.tex.at(c.i(3)), c.f(4));
      else if (t == "beckmann") S.mat[id] = new beckmann(S.tex.at(c.i(3)), c.f(4), c.f(5));
      else if (t == "metal") S.mat[id] = new metal(V3(c, 3), c.f(6));
      else if (t == "dielectric") S.mat[id] = new dielectric(c.f(3));
      else if (t == "diffuse_light") S.mat[id] = new diffuse_light(S.tex.at(c.i(3)));
      else if (t == "isotropic") S.mat[id] = new isotropic(S.tex.at(c.i(3)));
      else throw std::runtime_error("mat kind " + t);
      continue;
    }
    if (k == "grp") {
      long long gid = c.i(1);
      if (c.at(2) != "teapot") throw std::runtime_error("grp kind");
      S.grp[gid] = make_teapot(c.f(3), (int)c.i(4), M(S, c.i(5)));
      continue;
    }
    if (k == "obj") {
      long long id = c.i(1);
      const std::string& t = c.at(2);
      hitable* h = nullptr;
      if (t == "sphere") h = new sphere(V3(c, 3), c.f(6), M(S, c.i(7)));
      else if (t == "moving_sphere")
        h = new moving_sphere(V3(c, 3), V3(c, 6), c.f(9), c.f(10), c.f(11), M(S, c.i(12)));
      else if (t == "xy_rect") h = new xy_rect(c.f(3), c.f(4), c.f(5), c.f(6), c.f(7), M(S, c.i(8)));
      else if (t == "xz_rect") h = new xz_rect(c.f(3), c.f(4), c.f(5), c.f(6), c.f(7), M(S, c.i(8)));
      else if (t == "yz_rect") h = new yz_rect(c.f(3), c.f(4), c.f(5), c.f(6), c.f(7), M(S, c.i(8)));
      else if (t == "box") h = new box(V3(c, 3), V3(c, 6), M(S, c.i(9)));
      else if (t == "triangle") {
        triangle* tr = new triangle(V3(c, 3), V3(c, 6), V3(c, 9), M(S, c.i(12)));
        face_normals(tr);
        h = tr;
      } else if (t == "triangle_uv") {
        triangle* tr = new triangle(V3(c, 3), V3(c, 6), V3(c, 9), M(S, c.i(12)), V3(c, 13), V3(c, 16), V3(c, 19));
        face_normals(tr);
        h = tr;
      } else if (t == "triangle_uvn")
        h = new triangle(V3(c, 3), V3(c, 6), V3(c, 9), M(S, c.i(12)), V3(c, 13), V3(c, 16), V3(c, 19),
                         V3(c, 22), V3(c, 25), V3(c, 28));
      else if (t == "flip") h = new flip_normals(S.obj.at(c.i(3)));
      else if (t == "translate") h = new translate(S.obj.at(c.i(3)), V3(c, 4));
      else if (t == "rotate_y") h = new rotate_y(S.obj.at(c.i(3)), c.f(4));
      else if (t == "rotate_x") h = new rotate_x(S.obj.at(c.i(3)), c.f(4));
      else if (t == "constant_medium") h = new constant_medium(S.obj.at(c.i(3)), c.f(4), S.tex.at(c.i(5)));
      else if (t == "list" || t == "bvh") {
        size_t base = (t == "bvh") ? 5 : 3;
        long long n = c.i(base);
        hitable** l = new hitable*[n];
        for (long long q = 0; q < n; ++q) l[q] = S.obj.at(c.i(base + 1 + q));
        h = (t == "bvh") ? (hitable*)new bvh_node(l, (int)n, c.f(3), c.f(4)) : (hitable*)new hitable_list(l, (int)n);
      } else if (t == "bvh_group" || t == "list_group") {
        std::vector<hitable*>& g = S.grp.at(c.i(t == "bvh_group" ? 5 : 3));
        hitable** l = new hitable*[g.size()];
        for (size_t q = 0; q < g.size(); ++q) l[q] = g[q];
        h = (t == "bvh_group") ? (hitable*)new bvh_node(l, (int)g.size(), c.f(3), c.f(4))
                               : (hitable*)new hitable_list(l, (int)g.size());
      } else throw std::runtime_error("obj kind " + t);
      S.obj[id] = h;
      continue;
    }
    if (k == "camera") {
      S.cam = new camera(V3(c, 1), V3(c, 4), V3(c, 7), c.f(10), c.f(11), c.f(12), c.f(13), c.f(14), c.f(15));
      continue;
    }
    if (k == "world") { S.world = S.obj.at(c.i(1)); continue; }
    if (k == "lights") { S.lights = S.obj.at(c.i(1)); continue; }
    throw std::runtime_error("unknown command " + k);
  }
  if (!S.world || !S.lights || !S.cam) throw std::runtime_error("scene needs world, lights and camera");
  return S;
}

// Counts world->hit calls made by color() (Raytracing_n.cpp:58): the metric's
// "sample" (SURVEY §8(d)).  Light-pdf probes go to light_shape and are not counted.
struct counting_world : public hitable {
  hitable* w;
  mutable long long n = 0;
  explicit counting_world(hitable* p) : w(p) {}
  bool hit(const ray& r, float a, float b, hit_record& rec, bool m = false) const override {
    ++n;
    return w->hit(r, a, b, rec, m);
  }
  bool bounding_box(float t0, float t1, aabb& box) const override { return w->bounding_box(t0, t1, box); }
};

void reseed_path(unsigned x, unsigned y, unsigned s) {
  seed = srr_text::path_seed(x, y, s);
  s_rng.state = PCG32_DEFAULT_STATE ^ (seed << 16);
  s_rng.inc = PCG32_DEFAULT_STREAM;
}

double** sobol(unsigned N) {
  // The reference reads its direction numbers from new-joe-kuo-6.21201; for
  // D = 2 only the header line and line 2 ("2 1 0 1") are consumed.
  // (per-process file: several harness processes may run at once)
  char path[64];
  snprintf(path, sizeof path, "/tmp/srr_ref_sobol_dirs.%d.txt", (int)getpid());
  FILE* f = fopen(path, "w");
  fprintf(f, "d       s       a       m_i\n2       1       0       1\n");
  fclose(f);
  double** sp = sobol_points(N, 2, path);
  remove(path);
  return sp;
}

void write(const std::string& path, const void* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  fwrite(p, 1, n, f);
  fclose(f);
}

int render_to(hitable* world, hitable* lights, camera* cam, const std::string& out) {
  counting_world cw(world);
  double** sp = sobol(ns);
  std::vector<float> paths((size_t)nx * ny * ns * 3);
  std::vector<unsigned char> rays((size_t)nx * ny * ns);
  std::vector<float> img((size_t)nx * ny * 3);
  std::vector<int> img8((size_t)nx * ny * 3);
  auto t0 = std::chrono::steady_clock::now();
  for (int pix = 0; pix < nx * ny; ++pix) {
    // PPM order (Raytracing_n.cpp:873-876) with SURVEY Q12's fix i = pix % nx.
    int i = pix % nx;
    int j = ny - 1 - pix / nx;
    vec3 col(0, 0, 0);
    for (int s = 0; s < ns; ++s) {
      reseed_path((unsigned)i, (unsigned)j, (unsigned)s);
      float u = float(sp[s][0] + i) / float(nx);
      float v = float(sp[s][1] + j) / float(ny);
      ray r = cam->get_ray(u, v);
      int depth = 0;
      long long before = cw.n;
      vec3 c = color(r, &cw, lights, &depth);
      size_t p = ((size_t)pix * ns + s);
      paths[p * 3 + 0] = c[0];
      paths[p * 3 + 1] = c[1];
      paths[p * 3 + 2] = c[2];
      rays[p] = (unsigned char)(cw.n - before);
      col += de_nan(c);
    }
    col /= float(ns);
    img[pix * 3 + 0] = col[0];
    img[pix * 3 + 1] = col[1];
    img[pix * 3 + 2] = col[2];
    col = vec3(sqrt(col[0]), sqrt(col[1]), sqrt(col[2]));
    for (int c = 0; c < 3; ++c) {
      int q = int(255.99 * col[c]);
      q = q > 255 ? 255 : q;
      q = q < 0 ? 0 : q;
      img8[pix * 3 + c] = q;
    }
  }
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  write(out + ".paths.f32", paths.data(), paths.size() * 4);
  write(out + ".rays.u8", rays.data(), rays.size());
  write(out + ".img.f32", img.data(), img.size() * 4);
  std::ofstream ppm(out + ".ppm");
  ppm << "P3\n" << nx << " " << ny << "\n255\n";
  for (int p = 0; p < nx * ny; ++p) ppm << img8[p * 3] << " " << img8[p * 3 + 1] << " " << img8[p * 3 + 2] << "\n";
  printf("{\"paths\": %lld, \"world_rays\": %lld, \"ms\": %.3f, \"msamples_per_s\": %.4f}\n",
         (long long)nx * ny * ns, cw.n, ms, cw.n / (ms * 1e3));
  return 0;
}

// Per-pixel digest of a render, for frames too large to keep per path (the full
// 512x512x1024 C2 frame is 268 M paths).  Per pixel, in PPM order:
//   rays  uint32  sum of the pixel's world->hit calls over its ns paths
//   hash  uint32  FNV-1a-32 (word-wise: h = (h ^ w) * 16777619) over the words (r, g, b, rays) of each path in
//                 sample order, every NaN canonicalised to 0x7fc00000 (x86 and
//                 gfx950 produce different NaN payloads)
//   mean  3 x f32 the pixel's mean radiance (Raytracing_n.cpp:841-848)
inline uint32_t fnv_word(uint32_t h, uint32_t w) { return (h ^ w) * 16777619u; }
inline uint32_t canon_bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (f != f) ? 0x7fc00000u : u;
}

// sums <scene.txt> <nx> <ny> <ns> <maxdepth> <pix0> <pix1> <out_prefix> [stride]
// (pixels pix0, pix0 + stride, ... below pix1; out_prefix "-" writes no files:
// bench.py's cpu_baseline times the reference this way, one process per core)
int cmd_sums(int argc, char** argv) {
  if (argc < 10) return 2;
  RefScene S = build(srr_text::parse(srr_text::read_file(argv[2])));
  nx = atoi(argv[3]);
  ny = atoi(argv[4]);
  ns = atoi(argv[5]);
  maxDepth = atoi(argv[6]);
  const int p0 = atoi(argv[7]), p1 = atoi(argv[8]);
  const std::string out = argv[9];
  const int stride = argc > 10 ? std::max(1, atoi(argv[10])) : 1;
  counting_world cw(S.world);
  double** sp = sobol(ns);
  std::vector<uint32_t> rays, hash;
  std::vector<float> mean;
  auto t0 = std::chrono::steady_clock::now();
  int npx = 0;
  for (int pix = p0; pix < p1; pix += stride, ++npx) {
    int i = pix % nx;
    int j = ny - 1 - pix / nx;
    vec3 col(0, 0, 0);
    uint32_t h = 2166136261u, rs = 0;
    for (int s = 0; s < ns; ++s) {
      reseed_path((unsigned)i, (unsigned)j, (unsigned)s);
      float u = float(sp[s][0] + i) / float(nx);
      float v = float(sp[s][1] + j) / float(ny);
      ray r = S.cam->get_ray(u, v);
      int depth = 0;
      long long before = cw.n;
      vec3 c = color(r, &cw, S.lights, &depth);
      uint32_t nr = (uint32_t)(cw.n - before);
      h = fnv_word(fnv_word(fnv_word(fnv_word(h, canon_bits(c[0])), canon_bits(c[1])), canon_bits(c[2])), nr);
      rs += nr;
      col += de_nan(c);
    }
    col /= float(ns);
    rays.push_back(rs);
    hash.push_back(h);
    for (int c = 0; c < 3; ++c) mean.push_back(col[c]);
  }
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (out != "-") {
    write(out + ".rays.u32", rays.data(), rays.size() * 4);
    write(out + ".hash.u32", hash.data(), hash.size() * 4);
    write(out + ".mean.f32", mean.data(), mean.size() * 4);
  }
  printf("{\"pixels\": %d, \"world_rays\": %lld, \"ms\": %.3f}\n", npx, cw.n, ms);
  return 0;
}

// paths <scene.txt> <nx> <ny> <ns> <maxdepth> <pixels, comma-separated PPM-order indices> <out_prefix>:
// every path of the listed pixels of the nx x ny frame (out.paths.f32 [n][ns][3]
// raw color(), out.rays.u8 [n][ns] world rays) -- goldens for chosen pixels of a
// frame too large to keep whole (tests/golden/make_tail.py)
int cmd_paths(int argc, char** argv) {
  if (argc < 9) return 2;
  RefScene S = build(srr_text::parse(srr_text::read_file(argv[2])));
  nx = atoi(argv[3]);
  ny = atoi(argv[4]);
  ns = atoi(argv[5]);
  maxDepth = atoi(argv[6]);
  std::vector<int> pixels;
  for (const char* q = argv[7]; *q;) {
    pixels.push_back(atoi(q));
    while (*q && *q != ',') ++q;
    if (*q == ',') ++q;
  }
  const std::string out = argv[8];
  counting_world cw(S.world);
  double** sp = sobol(ns);
  std::vector<float> paths(pixels.size() * ns * 3);
  std::vector<unsigned char> rays(pixels.size() * ns);
  for (size_t q = 0; q < pixels.size(); ++q) {
    const int pix = pixels[q];
    int i = pix % nx;
    int j = ny - 1 - pix / nx;
    for (int s = 0; s < ns; ++s) {
      reseed_path((unsigned)i, (unsigned)j, (unsigned)s);
      float u = float(sp[s][0] + i) / float(nx);
      float v = float(sp[s][1] + j) / float(ny);
      ray r = S.cam->get_ray(u, v);
      int depth = 0;
      long long before = cw.n;
      vec3 c = color(r, &cw, S.lights, &depth);
      const size_t k = q * ns + s;
      paths[3 * k] = c[0];
      paths[3 * k + 1] = c[1];
      paths[3 * k + 2] = c[2];
      rays[k] = (unsigned char)(cw.n - before);
    }
  }
  write(out + ".paths.f32", paths.data(), paths.size() * 4);
  write(out + ".rays.u8", rays.data(), rays.size());
  printf("{\"pixels\": %zu, \"world_rays\": %lld}\n", pixels.size(), cw.n);
  return 0;
}

int cmd_render(int argc, char** argv) {
  if (argc < 8) return 2;
  RefScene S = build(srr_text::parse(srr_text::read_file(argv[2])));
  nx = atoi(argv[3]);
  ny = atoi(argv[4]);
  ns = atoi(argv[5]);
  maxDepth = atoi(argv[6]);
  return render_to(S.world, S.lights, S.cam, argv[7]);
}

// builder <name> <nx> <ny> <ns> <maxdepth> <out_prefix>: one of the reference's
// OWN scene builders (Raytracing_n.cpp:108-711), called exactly as main() does
// (aspect = nx / ny, :895-919) from the state the scene LCG has at main() entry,
// then rendered like `render`.  The builders open their assets by relative
// Windows paths ("..\\contents\\..."): the caller runs this in a directory
// holding entries with those literal names (tests/golden/make_scenes.py).
int cmd_builder(int argc, char** argv) {
  if (argc < 8) return 2;
  std::string name = argv[2];
  nx = atoi(argv[3]);
  ny = atoi(argv[4]);
  ns = atoi(argv[5]);
  maxDepth = atoi(argv[6]);
  hitable* world = nullptr;
  hitable* hl = nullptr;
  camera* cam = nullptr;
  float aspect = float(nx) / float(ny);
  if (name == "random_scene") random_scene(&world, &cam, &hl, aspect);
  else if (name == "ball_scenes") ball_scenes(&world, &cam, &hl, aspect);
  else if (name == "ball_orennayar_scenes") ball_orennayar_scenes(&world, &cam, &hl, aspect);
  else if (name == "final") final(&world, &cam, &hl, aspect);
  else throw std::runtime_error("builder " + name + " not available (model.h scenes need assimp)");
  return render_to(world, hl, cam, argv[7]);
}

// Reference BVH topology in preorder: "N" = interior node, "L a b" = leaf over
// child indices a, b (a == b for the n == 1 leaf, bvh.h:104-105).
void dump_bvh(const hitable* h, const std::map<const hitable*, int>& idx, std::ostream& os) {
  const bvh_node* b = dynamic_cast<const bvh_node*>(h);
  auto li = idx.find(b->left), ri = idx.find(b->right);
  if (li != idx.end() && ri != idx.end()) {
    os << "L " << li->second << " " << ri->second << "\n";
    return;
  }
  os << "N\n";
  dump_bvh(b->left, idx, os);
  dump_bvh(b->right, idx, os);
}

int cmd_bvh(int argc, char** argv) {
  if (argc < 5) return 2;
  std::vector<Cmd> cmds = srr_text::parse(srr_text::read_file(argv[2]));
  long long want = atoll(argv[3]);
  // Child pointers of the wanted bvh in command order, captured before the
  // reference's qsort permutes its array.
  std::vector<long long> child_ids;
  long long grp = -1;
  for (const Cmd& c : cmds)
    if (c.at(0) == "obj" && c.i(1) == want) {
      if (c.at(2) == "bvh")
        for (long long q = 0; q < c.i(5); ++q) child_ids.push_back(c.i(6 + q));
      else if (c.at(2) == "bvh_group") grp = c.i(5);
    }
  RefScene S = build(cmds);
  std::map<const hitable*, int> idx;
  if (grp >= 0) {
    auto& g = S.grp.at(grp);
    for (size_t q = 0; q < g.size(); ++q) idx[g[q]] = (int)q;
  } else {
    for (size_t q = 0; q < child_ids.size(); ++q) idx[S.obj.at(child_ids[q])] = (int)q;
  }
  std::ofstream os(argv[4]);
  const bvh_node* root = dynamic_cast<const bvh_node*>(S.obj.at(want));
  aabb bx = root->box;
  os << "box " << bx._min[0] << " " << bx._min[1] << " " << bx._min[2] << " " << bx._max[0] << " " << bx._max[1]
     << " " << bx._max[2] << "\n";
  dump_bvh(root, idx, os);
  printf("seed_after=%llu\n", seed);
  return 0;
}

int cmd_teapot(int argc, char** argv) {
  if (argc < 5) return 2;
  std::vector<hitable*> tris = make_teapot((float)atof(argv[2]), atoi(argv[3]), nullptr);
  std::vector<float> v;
  for (hitable* h : tris) {
    triangle* t = (triangle*)h;
    for (const vec3* p : {&t->p0, &t->p1, &t->p2, &t->normal})
      for (int c = 0; c < 3; ++c) v.push_back((*p)[c]);
  }
  write(argv[4], v.data(), v.size() * 4);
  printf("tris=%zu\n", tris.size());
  return 0;
}

int cmd_sobol(int argc, char** argv) {
  if (argc < 4) return 2;
  unsigned N = (unsigned)atoi(argv[2]);
  double** sp = sobol(N);
  std::vector<double> v;
  for (unsigned i = 0; i < N; ++i) {
    v.push_back(sp[i][0]);
    v.push_back(sp[i][1]);
  }
  write(argv[3], v.data(), v.size() * 8);
  return 0;
}

// Utah teapot control data (teapotdata.h, Newell's public-domain set) as exact
// C99 hex-float / integer initialisers, for the product's tessellator.
int cmd_teapot_data(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[2], "w");
  fprintf(f, "// Generated by oracle/ref (ref_harness teapot_data) from the public-domain Utah\n"
             "// teapot (Newell) as used by the reference renderer; exact float bit patterns.\n");
  fprintf(f, "static const int kSrrTeapotPatchCount = %d;\nstatic const int kSrrTeapotVertexCount = %d;\n",
          kTeapotNumPatches, kTeapotNumVertices);
  fprintf(f, "static const float kSrrTeapotVertex[%d] = {\n", kTeapotNumVertices * 3);
  for (int i = 0; i < kTeapotNumVertices; ++i)
    fprintf(f, "  %a, %a, %a,\n", teapotVertices[i][0], teapotVertices[i][1], teapotVertices[i][2]);
  fprintf(f, "};\n// 16 control-point indices per patch, 0-based\nstatic const short kSrrTeapotPatch[%d] = {\n",
          kTeapotNumPatches * 16);
  for (int p = 0; p < kTeapotNumPatches; ++p) {
    fprintf(f, " ");
    for (int i = 0; i < 16; ++i) fprintf(f, " %d,", teapotPatches[p][i] - 1);
    fprintf(f, "\n");
  }
  fprintf(f, "};\n");
  fclose(f);
  return 0;
}

// image <file> <req_comp> <out.raw>: the reference's own stbi_load (stb_image
// v2.19 compiled inside Raytracing_n.cpp), decoded bytes to out.raw; prints
// "x y comp".
int cmd_image(int argc, char** argv) {
  if (argc < 5) return 2;
  int x = 0, y = 0, n = 0, req = atoi(argv[3]);
  unsigned char* px = stbi_load(argv[2], &x, &y, &n, req);
  if (!px) {
    fprintf(stderr, "stbi_load failed: %s\n", stbi_failure_reason());
    return 1;
  }
  write(argv[4], px, (size_t)x * y * (req ? req : n));
  stbi_image_free(px);
  printf("%d %d %d\n", x, y, n);
  return 0;
}

int cmd_kat(int argc, char** argv);

}  // namespace

#include "kat.inc"

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: ref_harness render|bvh|teapot|sobol|kat ...\n");
    return 2;
  }
  try {
    std::string c = argv[1];
    if (c == "render") return cmd_render(argc, argv);
    if (c == "sums") return cmd_sums(argc, argv);
    if (c == "paths") return cmd_paths(argc, argv);
    if (c == "bvh") return cmd_bvh(argc, argv);
    if (c == "teapot") return cmd_teapot(argc, argv);
    if (c == "sobol") return cmd_sobol(argc, argv);
    if (c == "kat") return cmd_kat(argc, argv);
    if (c == "image") return cmd_image(argc, argv);
    if (c == "builder") return cmd_builder(argc, argv);
    if (c == "teapot_data") return cmd_teapot_data(argc, argv);
  } catch (const std::exception& e) {
    fprintf(stderr, "ref_harness: %s\n", e.what());
    return 1;
  }
  fprintf(stderr, "unknown command\n");
  return 2;
}

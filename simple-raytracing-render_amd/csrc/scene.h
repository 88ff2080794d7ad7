// Host scene store behind the C-ABI: one record per reference constructor call,
// built eagerly where the reference is eager (bvh_node, rotate_*, orennayar,
// beckmann, camera compute their derived values in the constructor), then
// flattened into the device tables of device_scene.h.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "device_scene.h"

namespace srr {

enum HKind : int32_t {
  H_SPHERE, H_MSPHERE, H_XY, H_XZ, H_YZ, H_BOX, H_TRI, H_FLIP, H_TRANSLATE, H_ROTY, H_ROTX, H_MEDIUM, H_LIST, H_BVH
};

struct Box3 {
  float mn[3], mx[3];
};

struct HTex {
  TexKind kind;
  float c[3] = {0, 0, 0};
  int nx = 0, ny = 0;
  std::vector<uint8_t> px;
  int even = -1, odd = -1;
};

struct HMat {
  MatKind kind;
  int tex = -1;
  float p[4] = {0, 0, 0, 0};
};

struct HTri {
  float p[9];
  float n[9];
  float uv[9];
  int mat;
};

struct HBvh {  // reference-topology BVH2 (bvh.h:96-119)
  struct Node {
    Box3 box;
    int left, right;  // >= 0: node index; < 0: ~(position in leaf_objs)
  };
  std::vector<Node> nodes;  // nodes[0] = root
  std::vector<int> leaves;  // object handles in DFS leaf order
  std::vector<int> input;   // children as given to bvh_node (before its sort)
  Box3 box;
};

struct HObj {
  HKind kind;
  int mat = -1;
  float f[11] = {0};  // sphere: c r | msphere: c0 c1 t0 t1 r | rect: lo0 hi0 lo1 hi1 k |
                      // box: p0 p1 | translate: off | rotate: sin cos
  int child = -1;     // wrappers; medium boundary
  int tex = -1;       // medium phase texture
  int tri = -1;       // H_TRI row
  int bvh = -1;       // H_BVH row
  std::vector<int> kids;  // H_LIST; H_BOX's six faces
  bool has_box = false;   // rotate_*: bounding box of the child at construction
  Box3 box{};
};

struct HCamera {
  float origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
  float time0, time1, lens_radius;
};

class Scene {
 public:
  Scene();
  uint64_t lcg;  // scene-build LCG (mathf.h:12), post-Perlin by default
  double drand48();

  std::vector<HTex> tex;
  std::vector<HMat> mat;
  std::vector<HObj> obj;
  std::vector<HTri> tris;
  std::vector<HBvh> bvhs;
  bool has_camera = false;
  HCamera cam{};
  int world = -1, lights = -1;
  std::vector<std::pair<long long, int>> text_ids;  // text `obj` id -> handle

  // constructors (C-ABI srr_*), each returns a handle or a negative code
  int add_tex(HTex t);
  int add_mat(HMat m);
  int add_obj(HObj o);
  int material(MatKind k, int tex, const float* prm);  // material.h constructors
  int sphere(const float c[3], float r, int m);
  int moving_sphere(const float c0[3], const float c1[3], float t0, float t1, float r, int m);
  int rect(HKind k, float a0, float a1, float b0, float b1, float kk, int m);
  int box(const float p0[3], const float p1[3], int m);
  int triangle(const float p[9], int m, const float* uv9, const float* n9);
  int wrap(HKind k, int child, const float* f);
  int rotate(HKind k, int child, float angle);
  int medium(int boundary, float density, int tex);
  int list(const int* kids, int n);
  int bvh(const int* kids, int n, float t0, float t1);
  int teapot(float scale, int divs, int m, int* first);
  void camera(const float lf[3], const float la[3], const float vup[3], float vfov, float aspect, float aperture,
              float focus, float t0, float t1);

  // hitable::bounding_box of every kind (the reference's float ops)
  bool bbox(int h, float t0, float t1, Box3& b) const;
  bool valid_obj(int h) const { return h >= 0 && h < (int)obj.size(); }
  bool valid_mat(int m) const { return m == -1 || (m >= 0 && m < (int)mat.size()); }
  bool valid_tex(int t) const { return t >= 0 && t < (int)tex.size(); }
};

// Parse srr scene description v1.
int scene_from_text(const std::string& text, Scene& s, std::string& err);

// Flattened tables (device_scene.h) ready for upload.
struct Flat {
  std::vector<DObj> objs;
  int n_world = 0;
  std::vector<DXform> xforms;
  std::vector<DSphere> spheres;
  std::vector<DRect> rects;
  std::vector<DStandaloneTri> stris;
  std::vector<DMesh> meshes;
  std::vector<float> nodes;             // 2 float4 per node (lo, hi)
  std::vector<float> node4;             // 8 float4 per 4-wide node
  // the same 4-wide nodes compressed to 64 B (device_scene.h kNode4qWords):
  // child boxes quantised to 8 bits per bound against the node's own box,
  // rounded outward; leaf boxes are recomputed exactly from the triangles
  std::vector<float> node4q;
  bool node4q_ok = true;                // every mesh's leaf boxes recompute exactly
  std::vector<float> tri_pos;           // float4 x4 per triangle (p0, p1, p2, pad)
  std::vector<TriShade> tri_shade;
  std::vector<DMedium> media;
  std::vector<DObvh> obvhs;
  std::vector<DObvhChild> obvh_children;
  std::vector<DSGroup> sgroups;         // runs of plain spheres behind a BVH (device_scene.h)
  std::vector<DSGItem> sg_items;
  std::vector<DMat> mats;
  std::vector<DTex> texs;
  std::vector<uint8_t> images;
  std::vector<float> perlin_ranvec;  // 256 x 3
  std::vector<int32_t> perlin_perm;  // 3 x 256
  std::vector<DLight> lights;
  DCamera cam{};
};

int flatten(const Scene& s, Flat& f, std::string& err);

// Utah teapot vertices (teapot.h:19-37,76-166) with a chosen subdivision.
void teapot_triangles(float scale, int divs, std::vector<float>& p9);

// Per-path seeding: FNV-1a-64 over (x, y, s) bytes, low 48 bits.
uint64_t path_seed(uint32_t x, uint32_t y, uint32_t s, uint64_t base);

// Joe-Kuo Sobol (Raytracing_n.cpp:721-812), D = 2.
void sobol2(unsigned n, double* out);

// Synthetic RGB8 image (same bytes as every other consumer).
std::vector<uint8_t> gen_image(int w, int h, uint32_t seed, int kind);

}  // namespace srr

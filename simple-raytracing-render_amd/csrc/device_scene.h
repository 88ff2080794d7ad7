// Flattened device scene: plain-old-data tables the host flattener
// (scene.cpp) fills and the HIP kernels (kernels.hip) read.  Layout in HBM:
//
//   world objects  DObj[n_world]            the reference's top-level
//                                           hitable_list, nested lists / boxes
//                                           inlined in order, instance wrappers
//                                           distributed onto each child as a
//                                           transform chain (xforms[])
//   mesh BVH       float4 nodes[2N]         reference-topology BVH2 (bvh.h:96-119) in
//                                           preorder, threaded for stackless traversal,
//                                           one 32-B record per node (half a cache line):
//                                           lo = (min.xyz, skip), hi = (max.xyz, leaf)
//                                           skip = next node once this subtree is done;
//                                           leaf = (first_tri << 1) | (count - 1), or -1
//   mesh BVH4      float4 node4[8*N4]       the same BVH collapsed to 4-wide nodes: each
//                                           node holds up to 4 reference nodes' boxes
//                                           (SoA: lo.x[4], lo.y[4], lo.z[4], hi.x[4],
//                                           hi.y[4], hi.z[4]) and child refs (int4):
//                                           >= 0 node4 index, < 0 ~leaf code, INT32_MIN
//                                           empty slot; 128 B
//   triangles      float4 tri_pos[4*T]      p0, p1, p2, pad (one 64-B line) in BVH leaf (DFS) order
//                  TriShade tri_shade[T]    n0..n2, uv0..uv2, material
//   materials/textures/images/lights/camera   small tables
//
// All indices are 32-bit; a scene is far below 2^31 of anything.
#pragma once
#include <cstdint>

namespace srr {

enum ObjKind : int32_t {
  OBJ_SPHERE = 0,
  OBJ_MSPHERE = 1,
  OBJ_RECT = 2,
  OBJ_TRI = 3,
  OBJ_MESH = 4,
  OBJ_MEDIUM = 5,
  OBJ_OBVH = 6,  // bvh_node over analytic hitables (spheres, boxes, rects, ...)
  OBJ_SGROUP = 7,  // a run of consecutive plain spheres of a hitable_list behind a BVH (DSGroup)
};

enum XformKind : int32_t { XF_FLIP = 0, XF_TRANSLATE = 1, XF_ROTY = 2, XF_ROTX = 3 };

struct DXform {  // one instance wrapper (hitable.h:35-203, aarect.h:149-171)
  int32_t kind;
  float a, b, c;  // translate: offset; rotate: sin, cos
};

// DObj::xf_count: moving transforms (translate / rotate) in the low bits, and
// kXfFlipBit when an odd number of flip_normals wrap the object
constexpr int32_t kXfFlipBit = 1 << 30;
constexpr int32_t kXfCountMask = 0xFFFF;

struct DObj {
  int32_t kind;
  int32_t xf_begin, xf_count;  // chain, outermost first (xf_count: see kXfFlipBit)
  int32_t idx;                 // row in the kind's table
};

struct DSphere {  // sphere.h / moving_sphere.h (static: c1 = c0, t0 = 0, t1 = 1)
  float c0[3], c1[3];
  float t0, t1, r;
  int32_t mat;
};

struct DRect {  // aarect.h: plane axis kax at k, in-plane axes a0, a1
  int32_t kax, a0, a1, mat;
  float lo0, hi0, lo1, hi1, k;
  float pad[3];
};

struct TriShade {  // triangle.h fields used after a hit
  float n[9];      // n0, n1, n2
  float uv[6];     // uv0.xy, uv1.xy, uv2.xy (uv.z is never read: triangle.h:172-175)
  int32_t mat;
};

// Compressed 4-wide node (Flat::node4q), 16 words = 64 B, same index and child
// references as the 128-B node: origin xyz, scale xyz (powers of two), then per
// bound one word of 4 bytes (child c in byte c): lo.x lo.y lo.z hi.x hi.y hi.z,
// then the 4 child references.  Child c's box on axis a is
//   [o_a + q_lo * s_a, o_a + q_hi * s_a]   (float mul, then float add)
// which contains the child's exact box (the builder checks the rounding).
constexpr int kNode4qWords = 16;

struct DMesh {
  int32_t node_off;  // into node arrays (root = node_off)
  int32_t tri_off;   // into tri arrays
  int32_t n_nodes, n_tris;
  int32_t node4_off; // root of the 4-wide view in node4[]
  int32_t n_node4;
};

// bvh_node whose leaves are not bare triangles (e.g. final's 400 boxes and 1,000
// spheres, Raytracing_n.cpp:483-496, :515-519): the reference-topology BVH2 in the
// same threaded node format as a mesh, whose leaves name children instead of
// triangles; each child is a run of DObjs hit with hitable_list semantics (a box
// is its 6 rects, box.h:31-33), with its transform chain relative to the node.
struct DObvh {
  int32_t node_off, n_nodes;
  int32_t child_off, n_children;
};

struct DObvhChild {
  int32_t obj_begin, obj_count;  // into the DObj table
};

// A run of >= kSGroupMinRun consecutive spheres / moving spheres of a
// hitable_list (random_scene's ~480, ball_scenes' 121), with no instance wrapper,
// replaced in the list by one object: a BVH over their boxes (threaded preorder
// records in the mesh BVH2 format of `nodes`, whose leaves name 1-2 items) gives
// the same answer as testing them in order.  In hitable_list::hit
// (hitable_list.h:21-33) sphere j reports its first root above t_min --
// v_j = temp1 if temp1 > t_min, else temp2 if temp2 > t_min (sphere.h:36-66, temp1
// <= temp2) -- and replaces the record iff v_j < closest_so_far: the run yields
// the smallest v_j below the closest-so-far it was entered with, ties to the
// EARLIEST sphere, whatever order the candidates are met in (kernels.hip
// sgroup_hit).  Boxes and pruning are conservative (the float roots of a
// near-tangent ray can lie ~1e-3 x distance off the sphere).
constexpr int kSGroupMinRun = 8;

struct DSGroup {
  int32_t node_off, n_nodes;  // threaded BVH2 records in `nodes` (leaf code: (first item << 1) | (count - 1))
  int32_t item_off, n_items;  // into sg_items, in BVH leaf order
};

struct DSGItem {   // one sphere of a run
  DSphere s;
  int32_t pos;     // its place in the run (ties go to the smaller)
  int32_t moving;  // moving_sphere (center at the ray's time)
  int32_t obj;     // its DObj (kept after the world list, for the hit record)
  int32_t pad;
};

struct DMedium {  // constant_medium.h:4-50
  int32_t bnd_begin, bnd_count;  // boundary objects (list semantics), in DObj
  float density;
  int32_t phase_mat;
};

enum MatKind : int32_t {
  MAT_LAMBERTIAN = 0,
  MAT_ORENNAYAR = 1,
  MAT_BECKMANN = 2,
  MAT_METAL = 3,
  MAT_DIELECTRIC = 4,
  MAT_DIFFUSE_LIGHT = 5,
  MAT_ISOTROPIC = 6,
  MAT_COUNT = 7,
};

struct DMat {
  int32_t kind;
  int32_t tex;       // albedo / emit texture (-1: none)
  float p[4];        // orennayar: A, B | beckmann: alphax, alphay | metal: rgb, fuzz | dielectric: ri
};

enum TexKind : int32_t { TEX_CONST = 0, TEX_IMAGE = 1, TEX_CHECKER = 2, TEX_NOISE = 3 };

struct DTex {
  int32_t kind;
  int32_t nx, ny;    // image
  int32_t even, odd; // checker
  int64_t off;       // image byte offset
  float c[3];        // const colour; noise: c[0] = scale
};

enum LightKind : int32_t { LIGHT_NONE = 0, LIGHT_XZRECT = 1, LIGHT_SPHERE = 2, LIGHT_TRI = 3 };

struct DLight {  // hitable_pdf targets (hitable_list.h:54-67)
  int32_t kind;
  int32_t idx;   // rect / sphere / standalone-triangle row
};

struct DCamera {  // camera.h:61-67
  float origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
  float time0, time1, lens_radius;
};

struct DStandaloneTri {  // triangle outside any BVH
  float p[9];
  TriShade sh;
};

}  // namespace srr

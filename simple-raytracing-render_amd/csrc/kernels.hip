// srr HIP kernels for gfx950 (MI355X): a wavefront path tracer.
//
// One bounce of every live path is one pass over three kernels:
//   srr_trace  closest hit against the flattened world (the reference's
//              hitable_list / bvh_node / aabb / triangle / sphere / rect /
//              constant_medium hit functions) -> SoA hit records     [HOT]
//   srr_shade  material::scatter + pdf sampling + light pdf (the body of
//              color(), Raytracing_n.cpp:55-106) -> next ray, or the folded
//              path radiance; survivors are compacted into the next active
//              list with one wave-aggregated atomic per wave
//   (srr_raygen / srr_accumulate / srr_finish around the bounce loop)
// Semantics follow the reference exactly; see DESIGN.md.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "device_scene.h"
#include "devmath.h"
#include "kernels.h"
#include "../../include/srr/merl.h"

namespace srr {
namespace dev {

// ===================================================================== hits
// sphere.h:36-66 and moving_sphere.h:24-51 (static spheres have c1 = c0)
SRR_D V3 sphere_center(const DSphere& s, float tm, bool moving) {
  V3 c0 = v3(s.c0[0], s.c0[1], s.c0[2]);
  if (!moving) return c0;
  V3 c1 = v3(s.c1[0], s.c1[1], s.c1[2]);
  return c0 + ((tm - s.t0) / (s.t1 - s.t0)) * (c1 - c0);
}

SRR_D bool sphere_hit(const DSphere& s, bool moving, const Ray& r, float tmin, float tmax, float& t) {
  V3 oc = r.o - sphere_center(s, r.tm, moving);
  float a = dot(r.d, r.d);
  float b = dot(oc, r.d);
  float c = dot(oc, oc) - s.r * s.r;
  float disc = b * b - a * c;
  if (disc > 0) {
    float sq = rsqrt_exact(disc);
    float temp = (-b - sq) / a;
    if (temp < tmax && temp > tmin) { t = temp; return true; }
    temp = (-b + sq) / a;
    if (temp < tmax && temp > tmin) { t = temp; return true; }
  }
  return false;
}

// rect_hit with the plane axis a compile-time constant (xy: 2, xz: 1, yz: 0), for the
// world list's hit test (t only), dispatched on the rect's (uniform) axis
template <int KAX>
SRR_D bool rect_hit_t(const DRect& q, const Ray& r, float tmin, float tmax, float& t) {
  constexpr int A0 = KAX == 0 ? 1 : 0, A1 = KAX == 2 ? 1 : 2;
  const float tt = (q.k - r.o[KAX]) / r.d[KAX];
  if (tt < tmin || tt > tmax) return false;
  const float x = r.o[A0] + tt * r.d[A0];
  const float y = r.o[A1] + tt * r.d[A1];
  if (x < q.lo0 || x > q.hi0 || y < q.lo1 || y > q.hi1) return false;
  t = tt;
  return true;
}

#ifndef SRR_RECTAX
#define SRR_RECTAX 1  // rect tests specialised on the plane axis (A/B: -DSRR_RECTAX=0)
#endif
// aarect.h:96-147
SRR_D bool rect_hit(const DRect& q, const Ray& r, float tmin, float tmax, float& t, float& u, float& v) {
#ifdef SRR_EXP_FASTRECT  // timing probe only (not the reference's quotient)
  float tt = (q.k - r.o[q.kax]) * __builtin_amdgcn_rcpf(r.d[q.kax]);
#else
  float tt = (q.k - r.o[q.kax]) / r.d[q.kax];
#endif
  if (tt < tmin || tt > tmax) return false;
  float x = r.o[q.a0] + tt * r.d[q.a0];
  float y = r.o[q.a1] + tt * r.d[q.a1];
  if (x < q.lo0 || x > q.hi0 || y < q.lo1 || y > q.hi1) return false;
  u = (x - q.lo0) / (q.hi0 - q.lo0);
  v = (y - q.lo1) / (q.hi1 - q.lo1);
  t = tt;
  return true;
}

// triangle.h:117-188: two-sided Moller-Trumbore variant on the NORMALISED
// direction; ignores t_min/t_max and returns a distance.
SRR_D bool tri_hit(V3 p0, V3 p1, V3 p2, bool front, V3 o, V3 dir, float& t, float& u, float& v) {
  V3 e1, e2;
  if (front) { e1 = p1 - p0; e2 = p2 - p0; }
  else { e1 = p0 - p1; e2 = p2 - p1; }
  V3 P = cross(dir, e2);
  float det = dot(e1, P);
  V3 T;
  if (det > 0) T = o - p0;
  else { T = p0 - o; det = -det; }
  if (det < kUp1em4) return false;  // det < 0.0001 (double)
  float uu = dot(T, P);
  if (uu < 0.0f || uu > det) return false;
  V3 Q = cross(T, e1);
  float vv = dot(dir, Q);
  if (vv < 0.0f || vv + uu > det) return false;
  float tt = dot(e2, Q);
  float inv = 1.0f / det;
  tt *= inv;
  uu *= inv;
  vv *= inv;
  if (tt < kUp1em4) return false;  // t < 0.0001 (double)
  t = tt; u = uu; v = vv;
  return true;
}

// tri_hit's front test from p0 and the edges e1 = p1 - p0, e2 = p2 - p0 (the same
// arithmetic after those two differences)
SRR_D bool tri_hit_e(V3 p0, V3 e1, V3 e2, V3 o, V3 dir, float& t) {
  V3 P = cross(dir, e2);
  float det = dot(e1, P);
  V3 T;
  if (det > 0) T = o - p0;
  else { T = p0 - o; det = -det; }
  if (det < kUp1em4) return false;
  float uu = dot(T, P);
  if (uu < 0.0f || uu > det) return false;
  V3 Q = cross(T, e1);
  float vv = dot(dir, Q);
  if (vv < 0.0f || vv + uu > det) return false;
  float tt = dot(e2, Q);
  float inv = 1.0f / det;
  tt *= inv;
  if (tt < kUp1em4) return false;
  t = tt;
  return true;
}

// Triangles are padded to 64 B (kTriStride float4) so a test touches one cache line.
constexpr int kTriStride = 4;

// aabb.h:33-49 with the per-axis reciprocal hoisted (same value each test).
// Branchless: the reference returns false at the first axis with tmax <= tmin;
// tmin only grows and tmax only shrinks over the axes (NaN slabs leave both
// unchanged), so testing once after all three axes gives the same answer.
SRR_D bool slab(float4 lo, float4 hi, V3 o, V3 inv, float tmin, float tmax) {
#define SRR_AX(A)                                     \
  {                                                   \
    float t0 = (lo.A - o.A) * inv.A;                  \
    float t1 = (hi.A - o.A) * inv.A;                  \
    bool sw = inv.A < 0.0f;                           \
    float n_ = sw ? t1 : t0, f_ = sw ? t0 : t1;       \
    tmin = n_ > tmin ? n_ : tmin;                     \
    tmax = f_ < tmax ? f_ : tmax;                     \
  }
  SRR_AX(x) SRR_AX(y) SRR_AX(z)
#undef SRR_AX
  return !(tmax <= tmin);
}

struct MeshHit {
  float t;
  int tri;
};

// bvh.h:83-86 reduces the two subtrees' hits with `left.t < right.t ? left :
// right`.  Over leaves in DFS order that is a left fold in which a later
// triangle replaces the current one unless current.t < later.t: the smallest t
// with ties to the later triangle, and -- for a NaN ray, whose every triangle
// test yields t = NaN -- the last triangle.  `wins` applies that fold for a
// candidate met in any order (ti is the DFS position).
SRR_D bool wins(float t, int ti, float best_t, int best_i) {
  return ti > best_i ? !(best_t < t) : (t < best_t);
}

// bvh.h:64-93 over the reference-topology BVH: a node is tested against the
// incoming [tmin, tmax] (never shrunk: the reference tests both children with
// the same t_max), and among the tested triangles that hit, the smallest t wins,
// ties to the later DFS leaf (left.t < right.t ? left : right).  The reference
// visits nodes left-first and never reorders, so a threaded preorder layout
// (device_scene.h) reproduces its visit set exactly with no stack: box hit ->
// next node (the left child); box miss or leaf done -> the skip link.
template <bool PREFETCH>
SRR_D bool mesh_hit(const SceneView& S, const DMesh& m, const Ray& r, float tmin, float tmax, bool is_medium,
                    MeshHit& out, unsigned long long* ctr) {
  V3 inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  V3 dir = r.d / length(r.d);
  int node = m.node_off;
  const int end = m.node_off + m.n_nodes;
  bool found = false;
  float best_t = 0;
  int best_i = -1;
  uint32_t nbox = 0, ntri = 0;
  float4 lo = S.nodes[2 * (node)], hi = S.nodes[2 * (node) + 1];
  for (;;) {
    ++nbox;
    const int skip = __float_as_int(lo.w);
    const int leaf = __float_as_int(hi.w);
    // both possible successors are known before the box test: fetch them now so
    // their latency overlaps this node's work (one-node lookahead)
    float4 lo_c, hi_c, lo_s, hi_s;
    if (PREFETCH) {
      if (leaf < 0) { lo_c = S.nodes[2 * (node + 1)]; hi_c = S.nodes[2 * (node + 1) + 1]; }
      if (skip < end) { lo_s = S.nodes[2 * (skip)]; hi_s = S.nodes[2 * (skip) + 1]; }
    }
    bool hit = slab(lo, hi, r.o, inv, tmin, tmax);
    if (hit && leaf >= 0) {
      int first = leaf >> 1, count = (leaf & 1) + 1;
      ntri += 2;  // the reference tests a one-triangle leaf twice (bvh.h:104-105)
      for (int ti = first; ti < first + count; ++ti) {
        const float4* tp = S.tri_pos + kTriStride * (size_t)ti;
        float4 a = tp[0], b = tp[1], c = tp[2];
        V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(c.x, c.y, c.z);
        float t, u, v;
        bool h = tri_hit(p0, p1, p2, true, r.o, dir, t, u, v);
        if (!h && is_medium) { ++ntri; h = tri_hit(p0, p1, p2, false, r.o, dir, t, u, v); }
        if (h && (!found || wins(t, ti, best_t, best_i))) {
          found = true;
          best_t = t;
          best_i = ti;
        }
      }
    }
    const bool down = hit && leaf < 0;
    const int next = down ? node + 1 : skip;
    if (next >= end) break;
    if (PREFETCH) {
      lo = down ? lo_c : lo_s;
      hi = down ? hi_c : hi_s;
    } else {
      lo = S.nodes[2 * (next)];
      hi = S.nodes[2 * (next) + 1];
    }
    node = next;
  }
  if (ctr) { atomicAdd(ctr, (unsigned long long)nbox); atomicAdd(ctr + 1, (unsigned long long)ntri); }
  out.t = best_t;
  out.tri = best_i;
  return found;
}

// Traversal modes of the trace kernel (SRR_TRAVERSAL): the reference BVH2
// threaded and stackless, or its 4-wide view (device_scene.h) near-first with an
// LDS stack, optionally pruning subtrees by the closest hit found so far.
enum Traversal : int { TR_BVH2 = 0, TR_BVH4 = 1, TR_BVH4_PRUNE = 2, TR_BVH4_TIMED = 3 };
// TR | TR_WL: the world tables (objects, transforms, primitives, meshes, media)
// were staged in LDS by the kernel, so they are read with plain (ds_read) loads
constexpr int TR_WL = 16;
constexpr int tr_mode(int tr) { return tr & 15; }
template <int TR, class T>
SRR_D T wload(const T* p, int i) {
  if constexpr ((TR & TR_WL) != 0) return p[i];
  else return cload(p, i);
}
// World-list tables are read at wave-uniform addresses (every active lane is at
// the same object), but the compiler cannot know the loaded words are uniform:
// uni() moves them to scalar registers, so the dispatch on object / transform
// kinds becomes scalar branches instead of exec-mask regions (SRR_UNIFORM)
#ifndef SRR_UNIFORM
#define SRR_UNIFORM 1
#endif
template <class T>
SRR_D T uni(T v) {
  static_assert(sizeof(T) % 4 == 0, "uni: whole words");
  int* w = (int*)&v;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) w[i] = __builtin_amdgcn_readfirstlane(w[i]);
  return v;
}
template <bool U, class T>
SRR_D T maybe_uni(T v) {
  if constexpr (U) return uni(v);
  else return v;
}
constexpr int kTraceBlock = 256;
constexpr int kStack = kPathsLdsStack;  // LDS stack entries per ray; deeper -> global extension, then the exact BVH2 re-walk
constexpr int kWorldLdsBytes = kPathsWorldLdsBytes;  // world tables staged in LDS up to this size
constexpr unsigned long long kTimingCap = 1 << 16;  // SRR_TIMING wave records

// LDS pointers in the LDS address space: generic pointers to the stacks let the
// backend merge LDS and global-extension stack addresses into one flat pointer,
// whose null check it can emit as an illegal compare on gfx950
template <class T>
using lds_ptr = __attribute__((address_space(3))) T*;
template <class T>
SRR_D lds_ptr<T> to_lds(T* p) { return (lds_ptr<T>)(uint32_t)(uintptr_t)p; }

struct TraceCtx {
  unsigned long long* ctr;  // optional counters: boxes tested, triangle tests, stack overflows
  lds_ptr<int> st_node;    // this thread's LDS stack (stride kTraceBlock)
  lds_ptr<float> st_t;     // entry distance of each stacked node
  const __attribute__((address_space(3))) f32x4* lds_nodes = nullptr;  // LDS copy of node4[0, lds_count) (k_paths)
  int lds_count = 0;
  int st_cap = kStack;                   // stack entries used (<= kStack; SRR_STACK_CAP tests the re-walk)
  unsigned long long* ovf = nullptr;     // optional: += 1 per traversal that overflowed into the re-walk
  // optional global extension of the stack (k_paths): entries kStack.. of lane
  // `slot` at gst[(sp - st_cap) * gst_stride + slot] = (node, entry t bits), up to
  // gst_cap of them; only a traversal deeper than that re-walks the BVH2
  int2* gst = nullptr;
  int gst_cap = 0;
  int gst_stride = 0;
  int slot = 0;
  // Suspendable mesh walks (k_paths, TR_SUSP): a lane whose walk has
  // taken a node step in this call leaves it once at most walk_thr lanes of its
  // wave are still walking (<= 0: never), its walk state saved in the save area that
  // follows the stack's global extension (walk_save(): [3][gst_stride] float4 at
  // `slot`); `resume` (in) continues the walk saved there, `susp` (out) says the
  // lane suspended.  All three are per-lane VGPR ints (vreg()): the path kernel's
  // scalar registers are full, and every scalar value live across the walk loop
  // spills to VGPR lanes (v_writelane / v_readlane in the loop)
  int walk_thr = -1;
  mutable int resume = 0;
  mutable int susp = 0;
  mutable int obj_k = -1;  // (SUSP) the world-list object under test (set by world_hit; wave-uniform)
  // SRR_TIMING diagnostics (wave-uniform): cycles inside mesh traversals, steps
  mutable uint64_t mesh_cycles = 0;
  mutable int mesh_steps = 0;       // node steps of the wave's longest walk
  mutable int mesh_lane_steps = 0;  // node steps summed over the wave's lanes
  mutable int mesh_walkers = 0;     // lanes that took a node step
  mutable uint64_t leaf_cycles = 0;  // cycles in mesh_hit4's leaf-triangle queue (longest walk's lane)
  mutable int leaf_passes = 0;       // passes of that queue (the same lane's)
  mutable uint64_t step_parts[3] = {0, 0, 0};  // node fetch, slab + queue set-up, order + push + pop
#ifdef SRR_SLOW_RAYS
  mutable int last_steps = 0;  // diagnostics build: node steps | 1 << 30 on overflow, of this lane's last walk
#endif
};

// Pruning margin: a subtree is skipped only when its box's UNCLIPPED entry
// (the slab intersection of the whole line, not clipped to tmin) lies beyond
// best_t * kPruneSlack along the ray.  The reference tests every leaf box the
// ray segment [tmin, tmax] crosses and keeps the smallest triangle t (a
// distance) with ties to the later leaf -- and triangle::hit ignores tmin
// (SURVEY Q4), so a leaf box that passes the [tmin, tmax] test can hold a hit
// at a parameter below tmin, anywhere from the box's own entry on.  A box whose
// unclipped entry is beyond the bound therefore holds no hit nearer than
// best_t, unless the triangle's float t were more than 6 % short of its box
// entry -- far beyond the few-ulp error of both computations.  (Pruning on the
// tmin-clipped entry, as round 1 did, lost the nearer self-hits of rays leaving
// the mesh's own surface: 1,115 world rays of the 512x512x1024 C2 frame.)
constexpr float kPruneSlack = 1.0625f;

// a value the compiler must keep in a VGPR (see TraceCtx::walk_thr)
SRR_D int vreg(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// the suspended-walk save area: [3][gst_stride] float4 right after the stack's
// global extension (renderer.cpp allocates both at once), lane `slot`, word w
SRR_D float4* walk_save(const TraceCtx& cx, int w) {
  return (float4*)(cx.gst + (size_t)cx.gst_cap * cx.gst_stride) + ((size_t)w * cx.gst_stride + cx.slot);
}

// A NaN t bound (tmax): the world list's closest-so-far goes NaN when an
// earlier object reports a hit at t = NaN -- e.g. a ray lying in an xz_rect
// light's plane, (k - o.y) / d.y = 0 / 0, which passes every comparison of
// aarect.h:115-121.  aabb::hit then rejects no box (tmax stays NaN, and
// `tmax <= tmin` is false, aabb.h:33-49), so the reference walks the whole BVH
// and folds every triangle: the result is the fold over all triangles of the
// mesh, which `wins` reproduces in any order.  Walking the tree here cost up
// to 17 ms for one such ray (~2,000 node steps with the global stack, then
// 6,400 triangle tests, every fetch dependent): it set the end of a tile shard
// (profiles/r03/slow_rays_s2.txt).  Instead the wave's active lanes scan the
// triangles together for each such ray and reduce by `wins`: the same
// (found, t, triangle) as the walk, bit for bit.
SRR_D void mesh_scan_nan(const SceneView& S, const DMesh& m, const Ray& r, bool is_medium, uint64_t nanm,
                         bool& found, float& best_t, int& best_i) {
  const uint64_t act = __ballot(true);
  const int nact = __popcll(act);
  const int me = __popcll(act & ((1ull << __lane_id()) - 1));
  const int t_end = m.tri_off + m.n_tris;
  while (nanm) {
    const int L = __ffsll((unsigned long long)nanm) - 1;
    nanm &= nanm - 1;
    const V3 o = v3(__shfl(r.o.x, L), __shfl(r.o.y, L), __shfl(r.o.z, L));
    const V3 d = v3(__shfl(r.d.x, L), __shfl(r.d.y, L), __shfl(r.d.z, L));
    const V3 dir = d / length(d);
    bool f = false;
    float bt = 0;
    int bi = -1;
    for (int ti = m.tri_off + me; ti < t_end; ti += nact) {
      const float4* tp = S.tri_pos + kTriStride * (size_t)ti;
      const float4 a = tp[0], b = tp[1], c = tp[2];
      const V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(c.x, c.y, c.z);
      float t, u, v;
      bool h = tri_hit(p0, p1, p2, true, o, dir, t, u, v);
      if (!h && is_medium) h = tri_hit(p0, p1, p2, false, o, dir, t, u, v);
      if (h && (!f || wins(t, ti, bt, bi))) {
        f = true;
        bt = t;
        bi = ti;
      }
    }
    // reduce over the active lanes in lane order (wins is a strict total order
    // on (t, index), so the order does not change the winner)
    bool rf = false;
    float rt = 0;
    int ri = -1;
    for (uint64_t a2 = act; a2; a2 &= a2 - 1) {
      const int j = __ffsll((unsigned long long)a2) - 1;
      const bool fj = __shfl((int)f, j) != 0;
      const float tj = __shfl(bt, j);
      const int ij = __shfl(bi, j);
      if (fj && (!rf || wins(tj, ij, rt, ri))) {
        rf = true;
        rt = tj;
        ri = ij;
      }
    }
    if ((int)__lane_id() == L) {
      found = rf;
      best_t = rt;
      best_i = ri;
    }
  }
}

// A slab's running entry / exit over the axes, from -inf / +inf (never NaN): the
// reference's `t0 > tmin ? t0 : tmin` keeps tmin for a NaN t0, as fmaxf does (and a
// +-0 difference compares equal everywhere the entry is used), so with SRR_FMINMAX the
// compare + select pairs become single v_max_f32 / v_min_f32
#ifndef SRR_FMINMAX
#define SRR_FMINMAX 1  // (A/B: -DSRR_FMINMAX=0)
#endif
#if SRR_FMINMAX
#define SRR_SMAX(n, acc) fmaxf((n), (acc))
#define SRR_SMIN(f, acc) fminf((f), (acc))
#else
#define SRR_SMAX(n, acc) ((n) > (acc) ? (n) : (acc))
#define SRR_SMIN(f, acc) ((f) < (acc) ? (f) : (acc))
#endif

// SRR_SLIM: in mesh_hit4's walk (whose lanes never carry a NaN bound: those took
// the fold over all triangles), a child's [max(entry, tmin), min(exit, tmax)] by
// fmaxf / fminf, and the child sort's swap test on the entries alone (a child not
// taken has entry +inf and node -1; a taken child's entry is finite or -inf)
#ifndef SRR_SLIM
#define SRR_SLIM 1  // (A/B: -DSRR_SLIM=0)
#endif
#if SRR_SLIM
#define SRR_CMAX(x, t) fmaxf((x), (t))
#define SRR_CMIN(x, t) fminf((x), (t))
#define SRR_CSWAP_IF(a, b) (kt[b] < kt[a])
#else
#define SRR_CMAX(x, t) ((x) > (t) ? (x) : (t))
#define SRR_CMIN(x, t) ((x) < (t) ? (x) : (t))
#define SRR_CSWAP_IF(a, b) (kn[b] >= 0 && (kn[a] < 0 || kt[b] < kt[a]))
#endif

// one axis of a slab test on the whole line (as SRR_CHILD's): entry / exit
SRR_D void slab_axis(float L, float H, float O, float I, float& lo, float& hi) {
  const float t0 = (L - O) * I, t1 = (H - O) * I;
  const bool sw = I < 0.0f;
  const float n = sw ? t1 : t0, f = sw ? t0 : t1;
  lo = SRR_SMAX(n, lo);
  hi = SRR_SMIN(f, hi);
}

// A compressed node's box bound (device_scene.h kNode4qWords): o + q * s with
// q = byte c of the word, one float multiply (exact) and one float add
SRR_D float q_bound(float o, float s, uint32_t w, int c) { return o + (float)((w >> (8 * c)) & 255u) * s; }

// 4-wide traversal of one mesh; same result as mesh_hit (the reference's
// leaf set, min t, ties to the later DFS triangle).
// Q: the 64-B compressed nodes (SceneView::node4q): inner children are tested
// against their outward-rounded boxes (a larger box only visits and prunes
// less), leaf children against the rounded box first and then against their
// exact box, recomputed from the leaf's 1-2 triangles (ffmin / ffmax of the
// vertices: the reference's triangle / bvh_node box, triangle.h:53-68) with the
// reference's slab arithmetic -- the same leaf set as the 128-B nodes.
#ifndef SRR_LEAFQ
#define SRR_LEAFQ 1
#endif
constexpr bool LEAFQ = SRR_LEAFQ != 0;  // mesh_hit4's leaf-triangle queue (A/B: -DSRR_LEAFQ=0)
#ifndef SRR_TRIPF
#define SRR_TRIPF 1
#endif
#ifndef SRR_TOPREG
#define SRR_TOPREG 1  // the stack's top entry kept in registers (A/B: -DSRR_TOPREG=0)
#endif
#ifndef SRR_EDGEREC
#define SRR_EDGEREC 1  // leaf pairs from packed p0 / e1 / e2 records (A/B: -DSRR_EDGEREC=0)
#endif
#ifndef SRR_LEAFPAIR
#define SRR_LEAFPAIR 1  // one leaf (both triangles) per pass of the leaf queue (A/B: -DSRR_LEAFPAIR=0)
#endif

// SUSP: the walk may stop part-way (TraceCtx::walk_thr) and continue in a later
// call with TraceCtx::resume; its state at the loop top -- next node, stack depth
// and top entry (the deeper entries stay in the lane's LDS stack and global
// extension, which nothing else touches), best hit, bound, flags -- is all it needs.
template <bool PRUNE, bool TIMING = false, bool Q = false, int STRIDE = kTraceBlock, bool SUSP = false>
SRR_D bool mesh_hit4(const SceneView& S, const DMesh& m, const Ray& r, float tmin, float tmax, bool is_medium,
                     MeshHit& out, const TraceCtx& cx) {
  static_assert(!SUSP || (SRR_TOPREG && !Q), "suspendable walks: the register top entry, 128-B nodes");
  if (const uint64_t nanm = __ballot(!(tmax == tmax))) {  // NaN bound: the fold over all triangles
    bool f = false;
    float bt = 0;
    int bi = -1;
    mesh_scan_nan(S, m, r, is_medium, nanm, f, bt, bi);
    if (!(tmax == tmax)) {
#ifdef SRR_SLOW_RAYS
      cx.last_steps |= 1 << 28;  // diagnostics build: this lane took the NaN-bound scan
#endif
      out.t = bt;
      out.tri = bi;
      return f;
    }
  }
  const V3 inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  const float len = length(r.d);
  const V3 dir = r.d / len;
  const float to_param = kPruneSlack / len;
  bool found = false;
  float best_t = 0;
  int best_i = -1;
  float bound = tmax;
  int node = m.node4_off;
  int sp = 0;
  bool overflow = false, deep = false;
  uint32_t nbox = 0, ntri = 0;
  const uint64_t tm_enter = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  // (step-part stamps; per lane: the longest walk's lane was in every step of the wave)
  uint64_t ts = TIMING ? __builtin_amdgcn_s_memtime() : 0, sp0 = 0, sp1 = 0, sp2 = 0, slf = 0;
  int spass = 0;
#if SRR_TOPREG
  int top_n = -1;
  float top_t = 0.f;
#endif
  if constexpr (SUSP) {
    if (cx.resume) {  // the walk this lane suspended in an earlier wave-iteration, if it is this object's
      const float4 b = *walk_save(cx, 1);
      const int fl = __float_as_int(b.w);
      if ((fl >> 2) == cx.obj_k) {
        const float4 a = *walk_save(cx, 0);
        node = __float_as_int(a.x);
        sp = __float_as_int(a.y);
        top_n = __float_as_int(a.z);
        top_t = a.w;
        best_t = b.x;
        best_i = __float_as_int(b.y);
        found = best_i >= 0;
        bound = b.z;
        overflow = (fl & 1) != 0;
        deep = (fl & 2) != 0;
        cx.resume = 0;
      }
    }
  }
  for (;;) {
    if (TIMING) {
      asm volatile("" ::"v"(node), "v"(sp));
      const uint64_t t = __builtin_amdgcn_s_memtime();
      sp2 += t - ts;
      ts = t;
    }
    float4 LX, LY, LZ, HX, HY, HZ;
    int4 CH;
    if constexpr (Q) {
      f32x4 A, B, C, D;
      if (node < cx.lds_count) {  // top levels: LDS copy (k_paths)
        const __attribute__((address_space(3))) f32x4* N = cx.lds_nodes + 4 * node;
        A = N[0], B = N[1], C = N[2], D = N[3];
      } else {
        const f32x4* N = (const f32x4*)(S.node4q + 4 * (size_t)node);
        A = N[0], B = N[1], C = N[2], D = N[3];
      }
      // A = (o.x, o.y, o.z, s.x), B = (s.y, s.z, lo.x, lo.y), C = (lo.z, hi.x, hi.y, hi.z), D = children
      const uint32_t qlx = __float_as_uint(B[2]), qly = __float_as_uint(B[3]), qlz = __float_as_uint(C[0]);
      const uint32_t qhx = __float_as_uint(C[1]), qhy = __float_as_uint(C[2]), qhz = __float_as_uint(C[3]);
#define SRR_QB(O, S_, W) make_float4(q_bound(O, S_, W, 0), q_bound(O, S_, W, 1), q_bound(O, S_, W, 2), q_bound(O, S_, W, 3))
      LX = SRR_QB(A[0], A[3], qlx), LY = SRR_QB(A[1], B[0], qly), LZ = SRR_QB(A[2], B[1], qlz);
      HX = SRR_QB(A[0], A[3], qhx), HY = SRR_QB(A[1], B[0], qhy), HZ = SRR_QB(A[2], B[1], qhz);
#undef SRR_QB
      CH = make_int4(__float_as_int(D[0]), __float_as_int(D[1]), __float_as_int(D[2]), __float_as_int(D[3]));
    } else if (node < cx.lds_count) {  // top levels: LDS copy (k_paths)
      const __attribute__((address_space(3))) f32x4* N = cx.lds_nodes + 8 * node;
      auto f4 = [](f32x4 v) { return make_float4(v[0], v[1], v[2], v[3]); };
      LX = f4(N[0]), LY = f4(N[1]), LZ = f4(N[2]), HX = f4(N[3]), HY = f4(N[4]), HZ = f4(N[5]);
      const f32x4 c4 = N[6];
      CH = make_int4(__float_as_int(c4[0]), __float_as_int(c4[1]), __float_as_int(c4[2]), __float_as_int(c4[3]));
    } else {
      const float4* N = S.node4 + 8 * (size_t)node;
      LX = N[0], LY = N[1], LZ = N[2], HX = N[3], HY = N[4], HZ = N[5];
      CH = *(const int4*)(N + 6);
    }
    nbox += 4;
    if (TIMING) {  // the node's words are in registers
      asm volatile("" ::"v"(LX.x), "v"(HZ.w), "v"(CH.x), "v"(CH.w));
      __builtin_amdgcn_s_waitcnt(0);
      const uint64_t t = __builtin_amdgcn_s_memtime();
      sp0 += t - ts;
      ts = t;
    }
    float near[4];
    bool hit[4];
#define SRR_CHILD(c, C)                                                                  \
  {                                                                                      \
    float lo_ = -INFINITY, hi_ = INFINITY;                                               \
    SRR_SLAB_AX(LX.C, HX.C, r.o.x, inv.x) SRR_SLAB_AX(LY.C, HY.C, r.o.y, inv.y)          \
    SRR_SLAB_AX(LZ.C, HZ.C, r.o.z, inv.z)                                                \
    near[c] = lo_;                                                                       \
    const float a_ = SRR_CMAX(lo_, tmin), b_ = SRR_CMIN(hi_, tmax);                      \
    hit[c] = !(b_ <= a_) && !(PRUNE && lo_ > bound);                                     \
  }
#define SRR_SLAB_AX(L, H, O, I)                      \
  {                                                  \
    float t0 = (L - O) * I, t1 = (H - O) * I;        \
    bool sw = I < 0.0f;                              \
    float n_ = sw ? t1 : t0, f_ = sw ? t0 : t1;      \
    lo_ = SRR_SMAX(n_, lo_);                         \
    hi_ = SRR_SMIN(f_, hi_);                         \
  }
    SRR_CHILD(0, x) SRR_CHILD(1, y) SRR_CHILD(2, z) SRR_CHILD(3, w)
#undef SRR_SLAB_AX
#undef SRR_CHILD
    const int ch[4] = {CH.x, CH.y, CH.z, CH.w};
    if constexpr (!Q && LEAFQ) {
      // The leaf children this step hit, as a queue of (leaf, triangle) work: one
      // pass of the loop tests one triangle of every lane that has one, whatever
      // child slot its leaves sit in (slot by slot, a wave ran the triangle test
      // once per slot with a leaf, each time for a few lanes).  The fold is
      // order-free (`wins`), and the bound may only shrink: the same result.
      int q0 = -1, q1 = -1, q2 = -1, q3 = -1;  // leaf codes ~child, in slot order
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        // (a NaN ray passes every slab test, as in the reference, so empty slots
        // are told apart by their INT_MIN child, not by their inverted box)
        if (!hit[c] || ch[c] >= 0 || ch[c] == INT32_MIN) continue;
        const int leaf = ~ch[c];
        ntri += 2;
        if (q0 < 0) q0 = leaf;
        else if (q1 < 0) q1 = leaf;
        else if (q2 < 0) q2 = leaf;
        else q3 = leaf;
      }
      int sub = 0;  // triangle of leaf q0 under test
      if (TIMING) asm volatile("" ::"v"(q0), "v"(q3), "v"(near[0]), "v"(near[3]));
      const uint64_t tl_enter = TIMING ? __builtin_amdgcn_s_memtime() : 0;
      if (TIMING) sp1 += tl_enter - ts;
      int npass = 0;
#if SRR_LEAFPAIR
      // one pass per leaf: both its triangles' vertices are loaded together (a
      // one-triangle leaf loads its triangle twice, from L1) and tested, so a pass
      // waits for one round trip per leaf, not one per triangle
      (void)sub;
      while (q0 >= 0) {
        if (TIMING) ++npass;
        const int t0 = q0 >> 1;
        const bool two = (q0 & 1) != 0;
#if SRR_EDGEREC
        if (!is_medium) {  // the packed edge record of t0: p0, e1, e2 of t0 and t0 + 1
          const float4* lp = S.tri_edge + 8 * (size_t)t0;
          const float4 w0 = lp[0], w1 = lp[1], w2 = lp[2], w3 = lp[3];
          const float2 w4 = *(const float2*)(lp + 4);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (j == 1 && !two) break;
            const V3 p0 = j ? v3(w2.y, w2.z, w2.w) : v3(w0.x, w0.y, w0.z);
            const V3 e1 = j ? v3(w3.x, w3.y, w3.z) : v3(w0.w, w1.x, w1.y);
            const V3 e2 = j ? v3(w3.w, w4.x, w4.y) : v3(w1.z, w1.w, w2.x);
            const int ti = t0 + j;
            float t;
            if (tri_hit_e(p0, e1, e2, r.o, dir, t) && (!found || wins(t, ti, best_t, best_i))) {
              found = true;
              best_t = t;
              best_i = ti;
            }
          }
          if (PRUNE && found && best_t * to_param < bound) bound = best_t * to_param;
          q0 = q1;
          q1 = q2;
          q2 = q3;
          q3 = -1;
          continue;
        }
#endif
        const float4* tp = S.tri_pos + kTriStride * (size_t)t0;
        const float4* tq = tp + (two ? kTriStride : 0);
        const float4 a0 = tp[0], b0 = tp[1], c0 = tp[2];
        const float4 a1 = tq[0], b1 = tq[1], c1 = tq[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j == 1 && !two) break;
          const float4 a = j ? a1 : a0, b = j ? b1 : b0, cc = j ? c1 : c0;
          const int ti = t0 + j;
          const V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(cc.x, cc.y, cc.z);
          float t, u, v;
          bool h = tri_hit(p0, p1, p2, true, r.o, dir, t, u, v);
          if (!h && is_medium) h = tri_hit(p0, p1, p2, false, r.o, dir, t, u, v);
          if (h && (!found || wins(t, ti, best_t, best_i))) {
            found = true;
            best_t = t;
            best_i = ti;
          }
        }
        // shrink only with ordered compares: a NaN bound (the reference passes
        // every box then) or a NaN best keeps the bound as it is
        if (PRUNE && found && best_t * to_param < bound) bound = best_t * to_param;
        q0 = q1;
        q1 = q2;
        q2 = q3;
        q3 = -1;
      }
#else
#if SRR_TRIPF
      // software pipelined: the next triangle's vertices are in flight while
      // this one is tested (one L2 / Infinity Cache latency per pass, not two)
      float4 na{}, nb{}, nc{};
      if (q0 >= 0) {
        const float4* tp = S.tri_pos + kTriStride * (size_t)(q0 >> 1);
        na = tp[0], nb = tp[1], nc = tp[2];
      }
#endif
      while (q0 >= 0) {
        if (TIMING) ++npass;
        const int ti = (q0 >> 1) + sub;
#if SRR_TRIPF
        const float4 a = na, b = nb, cc = nc;
        {
          const int nti = (sub == 0 && (q0 & 1)) ? ti + 1 : (q1 >= 0 ? (q1 >> 1) : -1);
          if (nti >= 0) {
            const float4* tp = S.tri_pos + kTriStride * (size_t)nti;
            na = tp[0], nb = tp[1], nc = tp[2];
          }
        }
#else
        const float4* tp = S.tri_pos + kTriStride * (size_t)ti;
        const float4 a = tp[0], b = tp[1], cc = tp[2];
#endif
        const V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(cc.x, cc.y, cc.z);
        float t, u, v;
        bool h = tri_hit(p0, p1, p2, true, r.o, dir, t, u, v);
        if (!h && is_medium) h = tri_hit(p0, p1, p2, false, r.o, dir, t, u, v);
        if (h && (!found || wins(t, ti, best_t, best_i))) {
          found = true;
          best_t = t;
          best_i = ti;
        }
        // shrink only with ordered compares: a NaN bound (the reference passes
        // every box then) or a NaN best keeps the bound as it is
        if (PRUNE && found && best_t * to_param < bound) bound = best_t * to_param;
        if (sub == 0 && (q0 & 1)) {
          sub = 1;
        } else {
          sub = 0;
          q0 = q1;
          q1 = q2;
          q2 = q3;
          q3 = -1;
        }
      }
#endif
      if (TIMING) {
        spass += npass;
        ts = __builtin_amdgcn_s_memtime();
        slf += ts - tl_enter;
      }
    } else
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      // (a NaN ray passes every slab test, as in the reference, so empty slots
      // are told apart by their INT_MIN child, not by their inverted box)
      if (!hit[c] || ch[c] >= 0 || ch[c] == INT32_MIN) continue;
      const int leaf = ~ch[c];
      const int first = leaf >> 1, count = (leaf & 1) + 1;
      if constexpr (Q) {  // the exact leaf box from the vertices (the tests below re-read them from L1)
        const float4* tp = S.tri_pos + kTriStride * (size_t)first;
        V3 mn, mx;
        for (int t = 0; t < count; ++t) {
          const float4 a = tp[kTriStride * t], b = tp[kTriStride * t + 1], cc = tp[kTriStride * t + 2];
          const V3 tmn = v3(ffmin(ffmin(a.x, b.x), cc.x), ffmin(ffmin(a.y, b.y), cc.y), ffmin(ffmin(a.z, b.z), cc.z));
          const V3 tmx = v3(ffmax(ffmax(a.x, b.x), cc.x), ffmax(ffmax(a.y, b.y), cc.y), ffmax(ffmax(a.z, b.z), cc.z));
          mn = t ? v3(ffmin(mn.x, tmn.x), ffmin(mn.y, tmn.y), ffmin(mn.z, tmn.z)) : tmn;
          mx = t ? v3(ffmax(mx.x, tmx.x), ffmax(mx.y, tmx.y), ffmax(mx.z, tmx.z)) : tmx;
        }
        float lo_ = -INFINITY, hi_ = INFINITY;
        slab_axis(mn.x, mx.x, r.o.x, inv.x, lo_, hi_);
        slab_axis(mn.y, mx.y, r.o.y, inv.y, lo_, hi_);
        slab_axis(mn.z, mx.z, r.o.z, inv.z, lo_, hi_);
        const float a_ = lo_ > tmin ? lo_ : tmin, b_ = hi_ < tmax ? hi_ : tmax;
        if ((b_ <= a_) || (PRUNE && lo_ > bound)) continue;  // the exact leaf box misses
      }
      ntri += 2;
      for (int ti = first; ti < first + count; ++ti) {
        const float4* tp = S.tri_pos + kTriStride * (size_t)ti;
        const float4 a = tp[0], b = tp[1], cc = tp[2];
        V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(cc.x, cc.y, cc.z);
        float t, u, v;
        bool h = tri_hit(p0, p1, p2, true, r.o, dir, t, u, v);
        if (!h && is_medium) h = tri_hit(p0, p1, p2, false, r.o, dir, t, u, v);
        if (h && (!found || wins(t, ti, best_t, best_i))) {
          found = true;
          best_t = t;
          best_i = ti;
        }
      }
      // shrink only with ordered compares: a NaN bound (the reference passes
      // every box then) or a NaN best keeps the bound as it is
      if (PRUNE && found && best_t * to_param < bound) bound = best_t * to_param;
    }
    // inner children that (still) overlap [tmin, bound], nearest first
    float kt[4];
    int kn[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bool take = hit[c] && ch[c] >= 0 && !(PRUNE && near[c] > bound);
      kt[c] = take ? near[c] : INFINITY;
      kn[c] = take ? ch[c] : -1;
    }
#define SRR_CSWAP(a, b)                                          \
  if (SRR_CSWAP_IF(a, b)) {                                      \
    float tt_ = kt[a]; kt[a] = kt[b]; kt[b] = tt_;               \
    int nn_ = kn[a]; kn[a] = kn[b]; kn[b] = nn_;                 \
  }
    SRR_CSWAP(0, 1) SRR_CSWAP(2, 3) SRR_CSWAP(0, 2) SRR_CSWAP(1, 3) SRR_CSWAP(1, 2)
#undef SRR_CSWAP
#if SRR_TOPREG
    // the stack's top entry is also kept in registers (top_n, top_t: entry sp - 1
    // whenever sp > 0), so a pop has its node at once and reads the entry below it
    // from LDS while the next step runs
    int nx = -1;  // the next node (the nearest child, or the nearest pending subtree), -1: done
    if (kn[0] >= 0) {
      nx = kn[0];
#pragma unroll
      for (int c = 3; c >= 1; --c) {
        if (kn[c] < 0) continue;
        if (sp < cx.st_cap) {
          cx.st_node[sp * STRIDE] = kn[c];
          cx.st_t[sp * STRIDE] = kt[c];
          ++sp;
          top_n = kn[c];
          top_t = kt[c];
        } else if (sp < cx.st_cap + cx.gst_cap) {
          cx.gst[(size_t)(sp - cx.st_cap) * cx.gst_stride + cx.slot] = make_int2(kn[c], __float_as_int(kt[c]));
          ++sp;
          deep = true;
          top_n = kn[c];
          top_t = kt[c];
        } else {
          overflow = true;
        }
      }
    } else {
      while (sp > 0) {
        --sp;
        const int cand = top_n;
        const float ct = top_t;
        if (sp > 0) {  // the new top
          if (sp - 1 < cx.st_cap) {
            top_n = cx.st_node[(sp - 1) * STRIDE];
            top_t = cx.st_t[(sp - 1) * STRIDE];
          } else {
            const int2 e = cx.gst[(size_t)(sp - 1 - cx.st_cap) * cx.gst_stride + cx.slot];
            top_n = e.x;
            top_t = __int_as_float(e.y);
          }
        }
        if (!(PRUNE && ct > bound)) { nx = cand; break; }
      }
    }
    if constexpr (SUSP) {
      // (SUSP) the walk also stops, to continue in a later wave-iteration, once at most
      // walk_thr of the wave's lanes have a next node (wave-uniform; every lane has taken
      // this step, so each progresses): one exit with the finished walks, node = next
      if (nx < 0 || (int)__popcll(__ballot(nx >= 0)) <= cx.walk_thr) {
        node = nx;
        break;
      }
      node = nx;
      continue;
    }
#else
    if (kn[0] >= 0) {
      node = kn[0];
#pragma unroll
      for (int c = 3; c >= 1; --c) {
        if (kn[c] < 0) continue;
        if (sp < cx.st_cap) {
          cx.st_node[sp * STRIDE] = kn[c];
          cx.st_t[sp * STRIDE] = kt[c];
          ++sp;
        } else if (sp < cx.st_cap + cx.gst_cap) {
          cx.gst[(size_t)(sp - cx.st_cap) * cx.gst_stride + cx.slot] = make_int2(kn[c], __float_as_int(kt[c]));
          ++sp;
          deep = true;
        } else {
          overflow = true;
        }
      }
      continue;
    }
    // pop the nearest pending subtree that may still hold a closer hit
    int nx = -1;
    while (sp > 0) {
      --sp;
      int cand;
      float ct;
      if (sp < cx.st_cap) {
        cand = cx.st_node[sp * STRIDE];
        ct = cx.st_t[sp * STRIDE];
      } else {
        const int2 e = cx.gst[(size_t)(sp - cx.st_cap) * cx.gst_stride + cx.slot];
        cand = e.x;
        ct = __int_as_float(e.y);
      }
      if (!(PRUNE && ct > bound)) { nx = cand; break; }
    }
#endif
    if (nx < 0) break;
    node = nx;
  }
  bool suspended = false;
  if constexpr (SUSP) {
    if (node >= 0) {  // stopped with a next node: the walk's state at the top of that step
      *walk_save(cx, 0) = make_float4(__int_as_float(node), __int_as_float(sp), __int_as_float(top_n), top_t);
      *walk_save(cx, 1) = make_float4(best_t, __int_as_float(best_i), bound,
                                      __int_as_float((overflow ? 1 : 0) | (deep ? 2 : 0) | (cx.obj_k << 2)));
      cx.susp = 1;
      suspended = true;
    }
  }
  if (cx.ctr && !TIMING) {
    atomicAdd(cx.ctr, (unsigned long long)nbox);
    atomicAdd(cx.ctr + 1, (unsigned long long)ntri);
    if (overflow) atomicAdd(cx.ctr + 2, 1ull);
    // diagnostics: histograms of node steps per ray and per wave (max over lanes)
    const int steps = (int)(nbox / 4);
    atomicAdd(cx.ctr + 3 + min(steps, 63), 1ull);
    int wmax = steps;
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o));
    if ((int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) atomicAdd(cx.ctr + 67 + min(wmax, 63), 1ull);
  }
  if (TIMING) {
    sp2 += __builtin_amdgcn_s_memtime() - ts;
    {  // the parts of the lane with the longest walk (it ran in every step of the wave's loop)
      int lm = (int)nbox;
      for (int o = 32; o > 0; o >>= 1) lm = max(lm, __shfl_xor(lm, o));
      const int src = __ffsll((unsigned long long)__ballot((int)nbox == lm)) - 1;
      cx.step_parts[0] += (uint64_t)__shfl((unsigned long long)sp0, src);
      cx.step_parts[1] += (uint64_t)__shfl((unsigned long long)sp1, src);
      cx.step_parts[2] += (uint64_t)__shfl((unsigned long long)sp2, src);
      cx.leaf_cycles += (uint64_t)__shfl((unsigned long long)slf, src);
      cx.leaf_passes += __shfl(spass, src);
    }
    int st = (int)(nbox / 4), sum = st, walk = st > 0;
    for (int o = 32; o > 0; o >>= 1) {
      st = max(st, __shfl_xor(st, o));
      sum += __shfl_xor(sum, o);
      walk += __shfl_xor(walk, o);
    }
    cx.mesh_steps += st;
    cx.mesh_lane_steps += sum;
    cx.mesh_walkers += walk;
    cx.mesh_cycles += __builtin_amdgcn_s_memtime() - tm_enter;
  }
  if (cx.ovf && cx.gst) {  // traversals that used the global stack (one atomic per wave; a suspended walk counts when it ends)
    const uint64_t dm = __ballot(deep && !suspended);
    if (dm && (int)__lane_id() == __ffsll((unsigned long long)dm) - 1) atomicAdd(cx.ovf + 1, (unsigned long long)__popcll(dm));
  }
#ifdef SRR_SLOW_RAYS
  cx.last_steps += (int)(nbox / 4) | (overflow ? 1 << 30 : 0) | (deep ? 1 << 29 : 0);
#endif
  if (SUSP && suspended) return false;  // (the caller sees cx.susp)
  if (overflow) {  // rare: exact re-walk
    if (cx.ovf) atomicAdd(cx.ovf, 1ull);
    return mesh_hit<false>(S, m, r, tmin, tmax, is_medium, out, cx.ctr);
  }
  out.t = best_t;
  out.tri = best_i;
  return found;
}

// ------------------------------------------------ quad-cooperative traversal
// In a path kernel wave most rays miss a mesh's root box (C2: 87 % of world rays
// never enter the teapot's), and the few that enter hold the whole wave for their
// 10-40 node steps.  mesh_hit4_quad gives each entering ray a hardware quad of
// lanes (up to 16 rays per round): lane c of the quad tests child c of the node
// (the reference's slab arithmetic; leaf children test their 1-2 triangles), the
// quad reduces the hits with `wins` (a strict total order on (t, index), so any
// reduction order gives the fold's winner) and orders its inner children nearest
// first through DPP exchanges, and the quad's lane 0 lends its LDS stack (and
// global extension).  Same visit rules, pruning and result as mesh_hit4; a quad
// whose stack overflows leaves its ray to the exact BVH2 re-walk.
constexpr int TR_QUAD = 32;
constexpr int TR_Q = 64;  // meshes traced over the compressed 64-B nodes (SceneView::node4q)
constexpr int TR_BIG = 128;  // the 1,024-lane path kernel: LDS stacks with stride 1,024
constexpr int tr_stride(int tr) { return (tr & TR_BIG) ? 1024 : kTraceBlock; }
constexpr int TR_SUSP = 256;  // the path kernel: mesh walks may suspend and resume (TraceCtx::walk_thr)

template <int CTRL>
SRR_D int quad_dpp(int x) { return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false); }
template <int CTRL>
SRR_D float quad_dpp(float x) { return __int_as_float(quad_dpp<CTRL>(__float_as_int(x))); }
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E;  // quad_perm [1,0,3,2], [2,3,0,1]
template <int K>
constexpr int kQuadBcast = K * 0x55;               // quad_perm [K,K,K,K]

// the quad's winning candidate among its four lanes' (f, t, i)
SRR_D void quad_best(bool& f, float& t, int& i) {
#define SRR_QSTEP(CTRL)                                                      \
  {                                                                          \
    const bool of = quad_dpp<CTRL>((int)f) != 0;                             \
    const float ot = quad_dpp<CTRL>(t);                                      \
    const int oi = quad_dpp<CTRL>(i);                                        \
    if (of && (!f || wins(ot, oi, t, i))) { f = true; t = ot; i = oi; }       \
  }
  SRR_QSTEP(kQuadXor1) SRR_QSTEP(kQuadXor2)
#undef SRR_QSTEP
}

template <bool PRUNE, int STRIDE = kTraceBlock>
SRR_D bool mesh_hit4_quad(const SceneView& S, const DMesh& m, const Ray& r, float tmin, float tmax, bool is_medium,
                          MeshHit& out, const TraceCtx& cx) {
  if (const uint64_t nanm = __ballot(!(tmax == tmax))) {  // NaN bound: the fold over all triangles (mesh_scan_nan)
    bool f = false;
    float bt = 0;
    int bi = -1;
    mesh_scan_nan(S, m, r, is_medium, nanm, f, bt, bi);
    if (!(tmax == tmax)) {
#ifdef SRR_SLOW_RAYS
      cx.last_steps |= 1 << 28;  // diagnostics build: this lane took the NaN-bound scan
#endif
      out.t = bt;
      out.tri = bi;
      return f;
    }
  }
  const V3 inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  // every lane tests the mesh's root box -- the reference's bvh_node root, whose
  // own box test comes first in bvh.h:64-66 -- itself
  const bool want = slab(S.nodes[2 * m.node_off], S.nodes[2 * m.node_off + 1], r.o, inv, tmin, tmax);
  if (__ballot(1) != ~0ull) {  // not a full wave (its last paths): per lane
    if (!want) return false;
    return mesh_hit4<PRUNE, false, false, STRIDE>(S, m, r, tmin, tmax, is_medium, out, cx);
  }
  const int lane = __lane_id(), q = lane >> 2, c = lane & 3;
  const float len = length(r.d);
  const V3 dir = r.d / len;
  const float to_param = kPruneSlack / len;
  // quad lane 0's stacks serve its quad (entry e of lane l - c is cx.st_*[e * STRIDE - c])
  const int gslot = cx.slot - c;
  bool found_me = false, redo_me = false;
  float t_me = 0;
  int i_me = -1;
  uint64_t W = __ballot(want);
  if (__popcll(W) > S.quad_max) {  // many rays enter: one per lane
    if (!want) return false;
    return mesh_hit4<PRUNE, false, false, STRIDE>(S, m, r, tmin, tmax, is_medium, out, cx);
  }
  while (W) {
    // this round: up to 16 wanting lanes, quad k serving the k-th
    int owner = 0, nb = 0;
    uint64_t Wr = 0;
    for (; nb < 16 && W; ++nb) {  // wave-uniform: the round's lanes in order
      const int l = __ffsll((unsigned long long)W) - 1;
      W &= W - 1;
      Wr |= 1ull << l;
      if (q == nb) owner = l;
    }
    bool run = q < nb;
    // the owner's ray
    const V3 o = v3(__shfl(r.o.x, owner), __shfl(r.o.y, owner), __shfl(r.o.z, owner));
    const V3 iv = v3(__shfl(inv.x, owner), __shfl(inv.y, owner), __shfl(inv.z, owner));
    const V3 dr = v3(__shfl(dir.x, owner), __shfl(dir.y, owner), __shfl(dir.z, owner));
    const float q_tmin = __shfl(tmin, owner), q_tmax = __shfl(tmax, owner), q_tp = __shfl(to_param, owner);
    const bool q_med = __shfl((int)is_medium, owner) != 0;
    int node = m.node4_off, sp = 0;
    float bound = q_tmax, best_t = 0;
    int best_i = -1;
    bool found = false, overflow = false, deep = false;
    while (__ballot(run)) {
      if (run) {
        // child c of the node
        float lx, ly, lz, hx, hy, hz;
        int ch;
        if (node < cx.lds_count) {
          const __attribute__((address_space(3))) float* N =
              (const __attribute__((address_space(3))) float*)(cx.lds_nodes + 8 * node);
          lx = N[c], ly = N[4 + c], lz = N[8 + c], hx = N[12 + c], hy = N[16 + c], hz = N[20 + c];
          ch = __float_as_int(N[24 + c]);
        } else {
          const float* N = (const float*)(S.node4 + 8 * (size_t)node);
          lx = N[c], ly = N[4 + c], lz = N[8 + c], hx = N[12 + c], hy = N[16 + c], hz = N[20 + c];
          ch = __float_as_int(N[24 + c]);
        }
        float lo_ = -INFINITY, hi_ = INFINITY;
#define SRR_QAX(L, H, O, I)                      \
  {                                              \
    float t0 = (L - O) * I, t1 = (H - O) * I;    \
    bool sw = I < 0.0f;                          \
    float n_ = sw ? t1 : t0, f_ = sw ? t0 : t1;  \
    lo_ = SRR_SMAX(n_, lo_);                     \
    hi_ = SRR_SMIN(f_, hi_);                     \
  }
        SRR_QAX(lx, hx, o.x, iv.x) SRR_QAX(ly, hy, o.y, iv.y) SRR_QAX(lz, hz, o.z, iv.z)
#undef SRR_QAX
        const float a_ = lo_ > q_tmin ? lo_ : q_tmin, b_ = hi_ < q_tmax ? hi_ : q_tmax;
        const bool hit = !(b_ <= a_) && !(PRUNE && lo_ > bound);
        // a leaf child: its triangles
        bool cf = false;
        float ct = 0;
        int ci = -1;
        if (hit && ch < 0 && ch != INT32_MIN) {
          const int leaf = ~ch;
          const int first = leaf >> 1, count = (leaf & 1) + 1;
          for (int ti = first; ti < first + count; ++ti) {
            const float4* tp = S.tri_pos + kTriStride * (size_t)ti;
            const float4 a = tp[0], b = tp[1], cc = tp[2];
            const V3 p0 = v3(a.x, a.y, a.z), p1 = v3(b.x, b.y, b.z), p2 = v3(cc.x, cc.y, cc.z);
            float t, u, v;
            bool h = tri_hit(p0, p1, p2, true, o, dr, t, u, v);
            if (!h && q_med) h = tri_hit(p0, p1, p2, false, o, dr, t, u, v);
            if (h && (!cf || wins(t, ti, ct, ci))) {
              cf = true;
              ct = t;
              ci = ti;
            }
          }
        }
        quad_best(cf, ct, ci);
        if (cf && (!found || wins(ct, ci, best_t, best_i))) {
          found = true;
          best_t = ct;
          best_i = ci;
        }
        if (PRUNE && found && best_t * q_tp < bound) bound = best_t * q_tp;
        // inner children that still overlap [tmin, bound], nearest first (ties: lower c)
        const bool take = hit && ch >= 0 && !(PRUNE && lo_ > bound);
        const float nk[4] = {quad_dpp<kQuadBcast<0>>(lo_), quad_dpp<kQuadBcast<1>>(lo_), quad_dpp<kQuadBcast<2>>(lo_),
                             quad_dpp<kQuadBcast<3>>(lo_)};
        const int tk = quad_dpp<kQuadBcast<0>>((int)take) | (quad_dpp<kQuadBcast<1>>((int)take) << 1) |
                       (quad_dpp<kQuadBcast<2>>((int)take) << 2) | (quad_dpp<kQuadBcast<3>>((int)take) << 3);
        const int ck[4] = {quad_dpp<kQuadBcast<0>>(ch), quad_dpp<kQuadBcast<1>>(ch), quad_dpp<kQuadBcast<2>>(ch),
                           quad_dpp<kQuadBcast<3>>(ch)};
        const int ntake = __popc(tk);
        if (ntake > 0) {
          int rank = 0, first_k = -1;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (!((tk >> k) & 1)) continue;
            if (k != c && (nk[k] < lo_ || (nk[k] == lo_ && k < c))) ++rank;
            if (first_k < 0) first_k = k;
            else if (nk[k] < nk[first_k]) first_k = k;
          }
          if (take && rank > 0) {  // pushed farthest first: rank 1 ends on top
            const int pos = sp + (ntake - 1 - rank);
            if (pos < cx.st_cap) {
              cx.st_node[pos * STRIDE - c] = ch;
              cx.st_t[pos * STRIDE - c] = lo_;
            } else if (pos < cx.st_cap + cx.gst_cap) {
              cx.gst[(size_t)(pos - cx.st_cap) * cx.gst_stride + gslot] = make_int2(ch, __float_as_int(lo_));
              deep = true;
            } else {
              overflow = true;
            }
          }
          sp = min(sp + ntake - 1, cx.st_cap + cx.gst_cap);
          node = ck[first_k];
        } else {
          int nx = -1;
          while (sp > 0) {
            --sp;
            int cand;
            float ctt;
            if (sp < cx.st_cap) {
              cand = cx.st_node[sp * STRIDE - c];
              ctt = cx.st_t[sp * STRIDE - c];
            } else {
              const int2 e = cx.gst[(size_t)(sp - cx.st_cap) * cx.gst_stride + gslot];
              cand = e.x;
              ctt = __int_as_float(e.y);
            }
            if (!(PRUNE && ctt > bound)) {
              nx = cand;
              break;
            }
          }
          if (nx < 0) run = false;
          else node = nx;
        }
      }
    }
    // the quad's overflow / deep flags, then the result back to its owner
    overflow = (quad_dpp<kQuadBcast<0>>((int)overflow) | quad_dpp<kQuadBcast<1>>((int)overflow) |
                quad_dpp<kQuadBcast<2>>((int)overflow) | quad_dpp<kQuadBcast<3>>((int)overflow)) != 0;
    deep = (quad_dpp<kQuadBcast<0>>((int)deep) | quad_dpp<kQuadBcast<1>>((int)deep) |
            quad_dpp<kQuadBcast<2>>((int)deep) | quad_dpp<kQuadBcast<3>>((int)deep)) != 0;
    const int my_q = __popcll(Wr & ((1ull << lane) - 1));  // owners: their quad
    const int from = 4 * my_q;
    const bool f_r = __shfl((int)found, from) != 0;
    const float t_r = __shfl(best_t, from);
    const int i_r = __shfl(best_i, from);
    const bool o_r = __shfl((int)overflow, from) != 0;
    const bool d_r = __shfl((int)deep, from) != 0;
    if ((Wr >> lane) & 1) {
      found_me = f_r;
      t_me = t_r;
      i_me = i_r;
      redo_me = o_r;
      if (cx.ovf && d_r) atomicAdd(cx.ovf + 1, 1ull);
    }
  }
  if (redo_me) {  // rare: exact re-walk
    if (cx.ovf) atomicAdd(cx.ovf, 1ull);
    return mesh_hit<false>(S, m, r, tmin, tmax, is_medium, out, cx.ctr);
  }
  out.t = t_me;
  out.tri = i_me;
  return found_me;
}

#ifndef SRR_XFAX
#define SRR_XFAX 1  // rotations, record rects and light corners specialised on their axis (A/B: -DSRR_XFAX=0)
#endif
template <int IA>  // rotate_y (IA 0) / rotate_x (IA 1), the ray going in: the arithmetic of chain_in's generic branch
SRR_D void rot_in(const DXform& x, Ray& r) {
  const float s = x.a, c = x.b;
  V3 o = r.o, d = r.d;
  o.set(IA, c * r.o[IA] - s * r.o.z);
  o.z = s * r.o[IA] + c * r.o.z;
  d.set(IA, c * r.d[IA] - s * r.d.z);
  d.z = s * r.d[IA] + c * r.d.z;
  r.o = o;
  r.d = d;
}
template <int IA>  // ...and the record coming out
SRR_D void rot_out(const DXform& x, V3& p, V3& n) {
  const float s = x.a, c = x.b;
  V3 pp = p, nn = n;
  pp.set(IA, c * p[IA] + s * p.z);
  pp.z = -s * p[IA] + c * p.z;
  nn.set(IA, c * n[IA] + s * n.z);
  nn.z = -s * n[IA] + c * n.z;
  p = pp;
  n = nn;
}

// Instance chain (outermost first): the ray going in (hitable.h:44-52, 109-116,
// 180-188; flip leaves the ray alone)
template <int TR = 0, bool U = false>
SRR_D Ray chain_in(const SceneView& S, const DObj& ob, Ray r) {
  const int n = ob.xf_count & kXfCountMask;
  for (int k = 0; k < n; ++k) {
    DXform x = maybe_uni<U>(wload<TR>(S.xforms, ob.xf_begin + k));
    if (x.kind == XF_TRANSLATE) r.o = r.o - v3(x.a, x.b, x.c);
#if SRR_XFAX  // the rotation's axis a compile-time constant in each branch (no run-time indexing)
    else if (x.kind == XF_ROTY) rot_in<0>(x, r);
    else if (x.kind == XF_ROTX) rot_in<1>(x, r);
#else
    else if (x.kind == XF_ROTY || x.kind == XF_ROTX) {
      int ia = x.kind == XF_ROTY ? 0 : 1;
      float s = x.a, c = x.b;
      V3 o = r.o, d = r.d;
      o.set(ia, c * r.o[ia] - s * r.o.z);
      o.z = s * r.o[ia] + c * r.o.z;
      d.set(ia, c * r.d[ia] - s * r.d.z);
      d.z = s * r.d[ia] + c * r.d.z;
      r.o = o;
      r.d = d;
    }
#endif
  }
  return r;
}

// ...and the hit record coming out, innermost first
SRR_D void chain_out(const SceneView& S, const DObj& ob, V3& p, V3& n) {
  for (int k = (ob.xf_count & kXfCountMask) - 1; k >= 0; --k) {
    DXform x = S.xforms[ob.xf_begin + k];
    if (x.kind == XF_TRANSLATE) p = p + v3(x.a, x.b, x.c);
#if SRR_XFAX
    else if (x.kind == XF_ROTY) rot_out<0>(x, p, n);
    else rot_out<1>(x, p, n);
#else
    else {
      int ia = x.kind == XF_ROTY ? 0 : 1;
      float s = x.a, c = x.b;
      V3 pp = p, nn = n;
      pp.set(ia, c * p[ia] + s * p.z);
      pp.z = -s * p[ia] + c * p.z;
      nn.set(ia, c * n[ia] + s * n.z);
      nn.z = -s * n[ia] + c * n.z;
      p = pp;
      n = nn;
    }
#endif
  }
  if (ob.xf_count & kXfFlipBit) n = -n;  // flip_normals (aarect.h:149-171), exact in any order
}

struct ObjHit {
  float t;
  int prim;  // triangle index for meshes
};

// hit of one analytic primitive (sphere, moving sphere, rect, standalone
// triangle) in its local frame
template <int TR, bool U = false>
SRR_D bool prim_hit(const SceneView& S, const DObj& ob, const Ray& lr, float tmin, float tmax, bool is_medium,
                    float& t) {
  switch (ob.kind) {
    case OBJ_SPHERE:
    case OBJ_MSPHERE:
      return sphere_hit(maybe_uni<U>(wload<TR>(S.spheres, ob.idx)), ob.kind == OBJ_MSPHERE, lr, tmin, tmax, t);
    case OBJ_RECT: {
#if SRR_RECTAX
      const DRect q = maybe_uni<U>(wload<TR>(S.rects, ob.idx));
      switch (q.kax) {
        case 0: return rect_hit_t<0>(q, lr, tmin, tmax, t);
        case 1: return rect_hit_t<1>(q, lr, tmin, tmax, t);
        default: return rect_hit_t<2>(q, lr, tmin, tmax, t);
      }
#else
      float u, v;
      return rect_hit(maybe_uni<U>(wload<TR>(S.rects, ob.idx)), lr, tmin, tmax, t, u, v);
#endif
    }
    case OBJ_TRI: {
      const DStandaloneTri T = maybe_uni<U>(wload<TR>(S.stris, ob.idx));
      V3 p0 = v3(T.p[0], T.p[1], T.p[2]), p1 = v3(T.p[3], T.p[4], T.p[5]), p2 = v3(T.p[6], T.p[7], T.p[8]);
      V3 dir = lr.d / length(lr.d);
      float u, v;
      bool hh = tri_hit(p0, p1, p2, true, lr.o, dir, t, u, v);
      if (!hh && is_medium) hh = tri_hit(p0, p1, p2, false, lr.o, dir, t, u, v);
      return hh;
    }
  }
  return false;
}

// bvh.h:64-93 over an object BVH (device_scene.h DObvh): the threaded walk of
// mesh_hit -- every node tested against the incoming [tmin, tmax], the
// reference's visit set, smallest t with ties to the later DFS child (`wins`) --
// where a leaf child is a run of primitives hit like a hitable_list (its own
// closest-so-far, from tmax).  Returns the winning primitive's DObj index.
template <int TR>
SRR_D bool obvh_hit(const SceneView& S, const DObvh& o, const Ray& r, float tmin, float tmax, bool is_medium,
                    float& out_t, int& out_obj) {
  const V3 inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  const int end = o.node_off + o.n_nodes;
  bool found = false;
  float best_t = 0;
  int best_i = -1;
  for (int node = o.node_off; node < end;) {
    const float4 lo = S.nodes[2 * node], hi = S.nodes[2 * node + 1];
    const int skip = __float_as_int(lo.w), leaf = __float_as_int(hi.w);
    const bool hit = slab(lo, hi, r.o, inv, tmin, tmax);
    if (hit && leaf >= 0) {
      const int first = leaf >> 1, count = (leaf & 1) + 1;
      for (int ci = first; ci < first + count; ++ci) {
        const DObvhChild c = S.obvh_children[ci];
        float closest = tmax, ct = 0;
        int cobj = -1;
        for (int k = c.obj_begin; k < c.obj_begin + c.obj_count; ++k) {
          const DObj pb = wload<TR>(S.objs, k);
          float t;
          if (prim_hit<TR>(S, pb, chain_in<TR>(S, pb, r), tmin, closest, is_medium, t)) {
            closest = t;
            ct = t;
            cobj = k;
          }
        }
        if (cobj >= 0 && (!found || wins(ct, ci, best_t, best_i))) {
          found = true;
          best_t = ct;
          best_i = ci;
          out_obj = cobj;
        }
      }
    }
    node = (hit && leaf < 0) ? node + 1 : skip;
  }
  out_t = best_t;
  return found;
}

// A run of spheres behind a BVH (device_scene.h DSGroup): the result of testing
// them in list order -- hitable_list.h:21-33 with sphere.h:36-66 -- found in any
// order.  Sphere j's value is its first root above tmin, v_j = temp1 if temp1 >
// tmin else temp2 if temp2 > tmin (computed exactly as sphere_hit does); the run
// returns the smallest v_j < tmax, ties to the earliest sphere (a later equal
// root fails sphere_hit's `temp < t_max`).  Boxes only prune, so they are padded
// per ray by 4e-3 of the L1 distance from the ray origin to the box: a
// near-tangent ray's float root can lie ~sqrt(10 eps) |oc| ~ 1.1e-3 |oc| off the
// sphere (the cancellation in b*b - a*c), and a subtree is skipped only when its
// padded entry lies beyond 1.0625 x the current bound.  NaN slab terms leave the
// interval as it is (never reject).  Returns the winner's item index.
template <int TR>
SRR_D bool sgroup_hit(const SceneView& S, const DSGroup& g, const Ray& r, float tmin, float tmax, float& out_t,
                      int& out_item) {
  const V3 inv = v3(__frcp_rn(r.d.x), __frcp_rn(r.d.y), __frcp_rn(r.d.z));  // (pruning only)
  bool found = false;
  float best = tmax;
  int best_pos = 0, best_item = -1;
  const int end = g.node_off + g.n_nodes;
  for (int node = g.node_off; node < end;) {
    const float4 lo = S.nodes[2 * node], hi = S.nodes[2 * node + 1];
    const int skip = __float_as_int(lo.w), leaf = __float_as_int(hi.w);
    const float pad = 4e-3f * (fabsf(r.o.x - 0.5f * (lo.x + hi.x)) + fabsf(r.o.y - 0.5f * (lo.y + hi.y)) +
                               fabsf(r.o.z - 0.5f * (lo.z + hi.z)) + (hi.x - lo.x) + (hi.y - lo.y) + (hi.z - lo.z));
    float tn = -INFINITY, tf = INFINITY;
#define SRR_AX(A)                                         \
  {                                                       \
    const float t0 = (lo.A - pad - r.o.A) * inv.A;        \
    const float t1 = (hi.A + pad - r.o.A) * inv.A;        \
    const bool sw = inv.A < 0.0f;                         \
    const float n_ = sw ? t1 : t0, f_ = sw ? t0 : t1;     \
    tn = SRR_SMAX(n_, tn);                                \
    tf = SRR_SMIN(f_, tf);                                \
  }
    SRR_AX(x) SRR_AX(y) SRR_AX(z)
#undef SRR_AX
    const bool hit = !(tf < tn) && !(tn > best * kPruneSlack);
    if (hit && leaf >= 0) {
      const int first = leaf >> 1, count = (leaf & 1) + 1;
      for (int i = first; i < first + count; ++i) {
        const DSGItem it = S.sg_items[i];
        const V3 oc = r.o - sphere_center(it.s, r.tm, it.moving != 0);  // sphere_hit's arithmetic
        const float a = dot(r.d, r.d);
        const float b = dot(oc, r.d);
        const float c = dot(oc, oc) - it.s.r * it.s.r;
        const float disc = b * b - a * c;
        if (!(disc > 0)) continue;
        const float sq = rsqrt_exact(disc);
        const float t1 = (-b - sq) / a;
        float v;
        if (t1 > tmin) v = t1;
        else {
          const float t2 = (-b + sq) / a;
          if (!(t2 > tmin)) continue;
          v = t2;
        }
        if (!(v < tmax)) continue;
        if (!found || v < best || (v == best && it.pos < best_pos)) {
          found = true;
          best = v;
          best_pos = it.pos;
          best_item = i;
        }
      }
    }
    node = (hit && leaf < 0) ? node + 1 : skip;
  }
  out_t = best;
  out_item = best_item;
  return found;
}

// hit of one non-medium flattened object (in its local frame)
template <int TR, bool U = false>
SRR_D bool basic_hit(const SceneView& S, const DObj& ob, const Ray& lr, float tmin, float tmax, bool is_medium,
                     ObjHit& h, const TraceCtx& cx) {
  switch (ob.kind) {
    case OBJ_MESH: {
#ifdef SRR_EXP_NOMESH  // timing experiment only (wrong image): meshes never hit
      return false;
#endif
      MeshHit mh;
      const DMesh m = maybe_uni<U>(wload<TR>(S.meshes, ob.idx));
      bool hit;
      if (tr_mode(TR) == TR_BVH2) hit = mesh_hit<false>(S, m, lr, tmin, tmax, is_medium, mh, cx.ctr);
      else if (TR & TR_QUAD)
        hit = mesh_hit4_quad<tr_mode(TR) != TR_BVH4, tr_stride(TR)>(S, m, lr, tmin, tmax, is_medium, mh, cx);
      else if (TR & TR_Q)
        hit = mesh_hit4<tr_mode(TR) != TR_BVH4, false, true, tr_stride(TR)>(S, m, lr, tmin, tmax, is_medium, mh, cx);
      else
        hit = mesh_hit4<tr_mode(TR) != TR_BVH4, tr_mode(TR) == TR_BVH4_TIMED, false, tr_stride(TR), (TR & TR_SUSP) != 0>(
            S, m, lr, tmin, tmax, is_medium, mh, cx);
      if (!hit) return false;
      h.t = mh.t;
      h.prim = mh.tri;
      return true;
    }
    case OBJ_OBVH:
      return obvh_hit<TR>(S, S.obvhs[ob.idx], lr, tmin, tmax, is_medium, h.t, h.prim);
    case OBJ_SGROUP:
      return sgroup_hit<TR>(S, S.sgroups[ob.idx], lr, tmin, tmax, h.t, h.prim);
    case OBJ_MEDIUM:
      return false;
    default:
      return prim_hit<TR, U>(S, ob, lr, tmin, tmax, is_medium, h.t);
  }
}

// hitable_list::hit (hitable_list.h:21-33) over objects [b, b+n) -- a medium's
// boundary, which sees is_medium = true
template <int TR>
SRR_D bool list_hit(const SceneView& S, int b, int n, const Ray& r, float tmin, float tmax, float& t,
                    const TraceCtx& cx) {
  bool any = false;
  float closest = tmax;
  for (int k = 0; k < n; ++k) {
    const DObj ob = maybe_uni<SRR_UNIFORM != 0>(wload<TR>(S.objs, b + k));
    const Ray lr = chain_in<TR, SRR_UNIFORM != 0>(S, ob, r);
    float th = 0;
    bool hit;
    if (ob.kind == OBJ_MESH) {
      // a mesh inside a boundary (rare: the shipped scenes bound their media with
      // spheres and boxes) takes the exact stackless BVH2 walk, so the medium path
      // does not inline two more copies of the LDS-stack BVH4 traversal into the
      // path kernel (that pushed the MEDIA variants to ~110 spilled VGPRs)
      MeshHit mh;
      hit = mesh_hit<false>(S, wload<TR>(S.meshes, ob.idx), lr, tmin, closest, true, mh, nullptr);
      th = mh.t;
    } else if (ob.kind == OBJ_OBVH) {
      int po;
      hit = obvh_hit<TR>(S, S.obvhs[ob.idx], lr, tmin, closest, true, th, po);
    } else if (ob.kind == OBJ_MEDIUM) {
      hit = false;
    } else {
      hit = prim_hit<TR, SRR_UNIFORM != 0>(S, ob, lr, tmin, closest, true, th);
    }
    if (hit) {
      any = true;
      closest = th;
      t = th;
    }
  }
  return any;
}

// constant_medium.h:19-50 (two draws, one even on a miss)
template <int TR>
SRR_D bool medium_hit(const SceneView& S, const DMedium& md, const Ray& r, float tmin, float tmax, Rng& rng,
                      float& t, const TraceCtx& cx) {
  (void)(drand(rng) < 0.00001);
  // the boundary's entry (from -FLT_MAX) and exit (from entry + 0.0001, a double
  // sum rounded to the float parameter): one inlined list walk, run twice
  float tb[2] = {0, 0};
  float lo = -FLT_MAX;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    float th;
    if (!list_hit<TR>(S, md.bnd_begin, md.bnd_count, r, lo, FLT_MAX, th, cx)) return false;
    tb[pass] = th;
    lo = (float)((double)th + 0.0001);
  }
  float t1 = tb[0], t2 = tb[1];
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return false;
  if (t1 < 0) t1 = 0;
  float len = length(r.d);
  float inside = (t2 - t1) * len;
  float hit_distance = -(1 / md.density) * ::log(drand(rng));
  if (hit_distance < inside) {
    t = t1 + hit_distance / len;
    return true;
  }
  return false;
}

// The world's hitable_list::hit over the flattened objects, in order; a later
// object that reports a hit always replaces the record.
struct WorldHit {
  int obj;  // -1: miss
  int prim;
  float t;
};

// objects [k0, k1) of the world list, continuing a closest-so-far `closest`
template <bool MEDIA, int TR>
SRR_D void world_objs(const SceneView& S, const Ray& r, Rng& rng, const TraceCtx& cx, int k0, int k1, WorldHit& w,
                      float& closest) {
  const float tmin = 0.001f;
  for (int k = k0; k < k1; ++k) {
    const DObj ob = maybe_uni<SRR_UNIFORM != 0>(wload<TR>(S.objs, k));
    Ray lr = chain_in<TR, SRR_UNIFORM != 0>(S, ob, r);
    ObjHit h;
    bool hit;
    if (MEDIA && ob.kind == OBJ_MEDIUM) {
      hit = medium_hit<TR>(S, maybe_uni<SRR_UNIFORM != 0>(wload<TR>(S.media, ob.idx)), lr, tmin, closest, rng, h.t, cx);
      h.prim = -1;
    } else {
      hit = basic_hit<TR, SRR_UNIFORM != 0>(S, ob, lr, tmin, closest, false, h, cx);
    }
    if (hit) {
      closest = h.t;
      w.obj = k;
      w.prim = h.prim;
      w.t = h.t;
    }
  }
}

// TR_SUSP: a lane's mesh walk may suspend (cx.susp) and its world hit is then
// redone in a later wave-iteration (cx.resume), the walk continuing from its saved
// state at the same object (cx.obj_k).  With one mesh in the list and no media
// (SceneView::mesh_obj >= 0) the objects before the mesh are simply tested again --
// pure functions of the ray and the closest-so-far, the same results -- and the
// objects a suspended lane meets after its mesh are tested for nothing (the wave
// tests them for its other lanes anyway; k_paths discards the suspended lane's
// result).  Otherwise ("skip" mode) the list state (object, closest-so-far, record so
// far) is saved beside the walk's, a resuming lane passes over the objects before
// its mesh and a suspended lane over the objects after it: a medium draws from the
// path's RNG (constant_medium.h:19-50), which must not be drawn twice, and another
// mesh walk would reuse the lane's traversal stack, which holds the suspended walk.
// The objects stay in list order for every lane, so the result is the same.
template <bool MEDIA, int TR>
SRR_D WorldHit world_hit(const SceneView& S, const Ray& r, Rng& rng, const TraceCtx& cx) {
  WorldHit w{-1, -1, 0};
  float closest = FLT_MAX;  // numeric_limits<float>::max(), Raytracing_n.cpp:58
  const float tmin = 0.001f;
  constexpr bool SUSP = (TR & TR_SUSP) != 0;
  const bool skip = MEDIA || S.mesh_obj < 0;  // (wave-uniform) the list state is saved, see above
  int k_res = -1;  // (SUSP, skip) the object whose walk this lane resumes
  if constexpr (SUSP) {
    if (skip && cx.resume) {
      const float4 v = *walk_save(cx, 2);
      k_res = __float_as_int(v.x);
      closest = v.y;
      w.obj = __float_as_int(v.z);
      w.prim = __float_as_int(v.w);
      w.t = closest;
    }
  }
  for (int k = 0; k < S.n_world; ++k) {
    const DObj ob = maybe_uni<SRR_UNIFORM != 0>(wload<TR>(S.objs, k));
    if constexpr (SUSP) {
      // (a per-lane skip, not a break: the object loop stays wave-uniform)
      if (skip && (cx.susp || k < k_res)) continue;
      cx.obj_k = k;
    }
    Ray lr = chain_in<TR, SRR_UNIFORM != 0>(S, ob, r);
    ObjHit h;
    bool hit;
    if (MEDIA && ob.kind == OBJ_MEDIUM) {
      hit = medium_hit<TR>(S, maybe_uni<SRR_UNIFORM != 0>(wload<TR>(S.media, ob.idx)), lr, tmin, closest, rng, h.t, cx);
      h.prim = -1;
    } else {
      hit = basic_hit<TR, SRR_UNIFORM != 0>(S, ob, lr, tmin, closest, false, h, cx);
    }
    if (SUSP && skip && cx.susp) {
      *walk_save(cx, 2) = make_float4(__int_as_float(k), closest, __int_as_float(w.obj), __int_as_float(w.prim));
      continue;
    }
    if (hit) {
      closest = h.t;
      w.obj = k;
      w.prim = h.prim;
      w.t = h.t;
    }
  }
  return w;
}

// The winning object's hit record (t, u, v, p, normal, mat), recomputed in its
// local frame with the same arithmetic as the test, then taken out through the
// instance chain.
struct HitRec {
  V3 p, n;
  float u, v;
  int mat;
};

#if SRR_XFAX
// prim_record's rect branch with the plane axis a compile-time constant: u, v by
// rect_hit's arithmetic (aarect.h:96-147), the normal along the axis
template <int KAX>
SRR_D void rect_rec(const DRect& q, const Ray& r, HitRec& h) {
  constexpr int A0 = KAX == 0 ? 1 : 0, A1 = KAX == 2 ? 1 : 2;
  const float tt = (q.k - r.o[KAX]) / r.d[KAX];
  const float x = r.o[A0] + tt * r.d[A0];
  const float y = r.o[A1] + tt * r.d[A1];
  h.u = (x - q.lo0) / (q.hi0 - q.lo0);
  h.v = (y - q.lo1) / (q.hi1 - q.lo1);
  h.n = v3(0.f);
  h.n.set(KAX, 1.f);
}
#endif

SRR_D void sphere_uv(V3 p, float& u, float& v) {  // hitable.h:10-15
  float phi = ratan2(p.z, p.x);
  float theta = rasin(p.y);
  u = 1 - (phi + kPi) / (2 * kPi);
  v = (theta + kPi / 2) / kPi;
}

// record of one primitive (or mesh triangle `prim`) hit at t, in its local frame
template <int TR = 0>
SRR_D void prim_record(const SceneView& S, const DObj& ob, const Ray& lr, float t, int prim, HitRec& h) {
  switch (ob.kind) {
    case OBJ_SPHERE:
    case OBJ_MSPHERE: {
      const DSphere& s = S.spheres[ob.idx];
      V3 c = sphere_center(s, lr.tm, ob.kind == OBJ_MSPHERE);
      h.p = lr.at(t);
      if (ob.kind == OBJ_SPHERE) sphere_uv((h.p - c) / s.r, h.u, h.v);
      h.n = (h.p - c) / s.r;
      h.mat = s.mat;
      break;
    }
    case OBJ_RECT: {
      const DRect& q = S.rects[ob.idx];
#if SRR_XFAX
      switch (q.kax) {
        case 0: rect_rec<0>(q, lr, h); break;
        case 1: rect_rec<1>(q, lr, h); break;
        default: rect_rec<2>(q, lr, h); break;
      }
#else
      float tt;
      rect_hit(q, lr, -FLT_MAX, FLT_MAX, tt, h.u, h.v);
      h.n = v3(0.f);
      h.n.set(q.kax, 1.f);
#endif
      h.p = lr.at(t);
      h.mat = q.mat;
      break;
    }
    case OBJ_TRI:
    case OBJ_MESH: {
      // (values, not a pointer into either table: a pointer that may be LDS or
      // global compiles to flat loads, whose waits drain both the vector-memory
      // and the LDS counters)
      V3 p0, p1, p2;
      TriShade shv;
      if (ob.kind == OBJ_TRI) {
        DStandaloneTri T;
        if constexpr ((TR & TR_WL) != 0) {  // world tables in LDS: LDS-space loads
          static_assert(sizeof(DStandaloneTri) == 25 * 4, "DStandaloneTri: 25 words");
          const __attribute__((address_space(3))) float* q =
              (const __attribute__((address_space(3))) float*)(S.stris + ob.idx);
          float* t = (float*)&T;
#pragma unroll
          for (int k = 0; k < 25; ++k) t[k] = q[k];
        } else {
          T = S.stris[ob.idx];
        }
        p0 = v3(T.p[0], T.p[1], T.p[2]);
        p1 = v3(T.p[3], T.p[4], T.p[5]);
        p2 = v3(T.p[6], T.p[7], T.p[8]);
        shv = T.sh;
      } else {
        const float4* tp = S.tri_pos + kTriStride * (size_t)prim;
        float4 a = tp[0], b = tp[1], c = tp[2];
        p0 = v3(a.x, a.y, a.z);
        p1 = v3(b.x, b.y, b.z);
        p2 = v3(c.x, c.y, c.z);
        shv = S.tri_shade[prim];
      }
      const TriShade* sh = &shv;
      V3 dir = lr.d / length(lr.d);
      float tt, u, v;
      tri_hit(p0, p1, p2, true, lr.o, dir, tt, u, v);  // world rays never take the back test
      float a0 = 1 - u - v;
      // triangle.h:172-184
      float uvx = a0 * sh->uv[0] + u * sh->uv[2] + v * sh->uv[4];
      float uvy = a0 * sh->uv[1] + u * sh->uv[3] + v * sh->uv[5];
      h.u = uvx;
      h.v = uvy;
      V3 n0 = v3(sh->n[0], sh->n[1], sh->n[2]), n1 = v3(sh->n[3], sh->n[4], sh->n[5]),
         n2 = v3(sh->n[6], sh->n[7], sh->n[8]);
      h.n = unit_vector(a0 * n0 + u * n1 + v * n2);
      h.p = a0 * p0 + u * p1 + v * p2;
      h.mat = sh->mat;
      break;
    }
    case OBJ_MEDIUM: {
      h.p = lr.at(t);
      h.n = v3(1, 0, 0);
      h.mat = S.media[ob.idx].phase_mat;
      break;
    }
  }
}

template <int TR = 0>  // TR & TR_WL: world tables in LDS (plain loads, never cload)
SRR_D HitRec world_record(const SceneView& S, const Ray& r, const WorldHit& w) {
  const DObj& ob = S.objs[w.obj];
  Ray lr = chain_in<TR>(S, ob, r);
  HitRec h;
  h.u = 0;  // moving_sphere / constant_medium leave u, v unset in the reference;
  h.v = 0;  // defined here as 0
  if (ob.kind == OBJ_OBVH || ob.kind == OBJ_SGROUP) {  // the primitive inside, then the node's chain
    const DObj& in = S.objs[ob.kind == OBJ_SGROUP ? S.sg_items[w.prim].obj : w.prim];
    prim_record<TR>(S, in, chain_in<TR>(S, in, lr), w.t, -1, h);
    chain_out(S, in, h.p, h.n);
  } else {
    prim_record<TR>(S, ob, lr, w.t, w.prim, h);
  }
  chain_out(S, ob, h.p, h.n);
  return h;
}

// Material families for the per-bounce sort: the trace kernel bins every ray
// into one list per family so each shade kernel carries only its family's
// code (and registers).  Only diffuse_light emits and it never scatters, so a
// scattering bounce always has emitted == 0 (material.h:89-92).
enum Family : int { FAM_TERM = 0, FAM_DIFF = 1, FAM_BECK = 2, FAM_SPEC = 3 };

SRR_D int family_of(int mat, int kind, int depth, int max_depth) {
  if (mat < 0 || kind == MAT_DIFFUSE_LIGHT || depth >= max_depth) return FAM_TERM;  // Raytracing_n.cpp:63
  if (kind == MAT_LAMBERTIAN || kind == MAT_ORENNAYAR) return FAM_DIFF;
  if (kind == MAT_BECKMANN) return FAM_BECK;
  return FAM_SPEC;
}

// Material of a world hit without building its record (the trace kernels bin
// rays by material family with it).
SRR_D int hit_material(const SceneView& S, const WorldHit& w) {
  DObj ob = S.objs[w.obj];
  if (ob.kind == OBJ_OBVH) ob = S.objs[w.prim];
  else if (ob.kind == OBJ_SGROUP) ob = S.objs[S.sg_items[w.prim].obj];
  switch (ob.kind) {
    case OBJ_SPHERE:
    case OBJ_MSPHERE: return S.spheres[ob.idx].mat;
    case OBJ_RECT: return S.rects[ob.idx].mat;
    case OBJ_TRI: return S.stris[ob.idx].sh.mat;
    case OBJ_MESH: return S.tri_shade[w.prim].mat;
    case OBJ_MEDIUM: return S.media[ob.idx].phase_mat;
  }
  return -1;
}

SRR_D void store_hit(const SceneView& S, const PathState& P, int p, const WorldHit& w, int max_depth, int& fam) {
  if (w.obj < 0) {
    nts(&P.hit_w[p], make_int4(-1, -1, 0, -1));
    fam = FAM_TERM;
    return;
  }
  const int mat = hit_material(S, w);
  nts(&P.hit_w[p], make_int4(w.obj, w.prim, __float_as_int(w.t), mat));
  fam = family_of(mat, mat >= 0 ? S.mats[mat].kind : -1, ntl(&P.depth[p]), max_depth);
}

// ================================================================ shading
// Attempts of one resampling loop `while (pdf_val == 0)` (Raytracing_n.cpp:79-83).
// The reference loops without bound, and a hit point in a light's own plane never
// leaves the loop (every light sample runs parallel to the light, the BSDF half is
// 0).  Build definition, shared with the oracle
// (oracle/restate.cpp kMixtureGuard): stop after kMixtureGuard attempts and keep
// the last attempt (pdf 0; the record's division then gives inf/NaN, de_nan'd).
constexpr int kMixtureGuard = 100000;
SRR_D V3 tex_value_slow(const SceneView& S, int ti, float u, float v, V3 p) {
  // checker_texture recursion (texture.h:13-19) unrolled to a few levels
  for (int guard = 0; guard < 8; ++guard) {
    const DTex& T = S.texs[ti];
    if (T.kind == TEX_CONST) return v3(T.c[0], T.c[1], T.c[2]);
    if (T.kind == TEX_IMAGE) {  // texture.h:58-70
      int i = (u) * T.nx;
      int j = (1 - v) * T.ny - 0.001;
      if (i < 0) i = 0;
      if (j < 0) j = 0;
      if (i > T.nx - 1) i = T.nx - 1;
      if (j > T.ny - 1) j = T.ny - 1;
      const uint8_t* px = S.images + T.off + 3 * (size_t)i + 3 * (size_t)T.nx * j;
      // int(px[c]) / 255.0 is a double quotient rounded to float; for each of the 256
      // byte values it equals the float quotient (float)x / 255.0f (tests/test_texture_quotient.py),
      // which saves three double divisions per lookup
      float r = (float)int(px[0]) / 255.0f;
      float g = (float)int(px[1]) / 255.0f;
      float b = (float)int(px[2]) / 255.0f;
      return v3(r, g, b);
    }
    if (T.kind == TEX_CHECKER) {
      float sines = rsin(10 * p.x) * rsin(10 * p.y) * rsin(10 * p.z);
      ti = sines < 0 ? T.odd : T.even;
      continue;
    }
    // noise_texture (texture.h:35-46) with perlin.h's turb()
    float scale = T.c[0];
    V3 tp = scale * p;
    float accum = 0, weight = 1.0f;
    for (int oct = 0; oct < 7; ++oct) {
      float fx = floorf(tp.x), fy = floorf(tp.y), fz = floorf(tp.z);
      float uu = tp.x - fx, vv = tp.y - fy, ww = tp.z - fz;
      int i = (int)fx, j = (int)fy, k = (int)fz;
      float hu = uu * uu * (3 - 2 * uu), hv = vv * vv * (3 - 2 * vv), hw = ww * ww * (3 - 2 * ww);
      float acc = 0;
      for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
          for (int c = 0; c < 2; c++) {
            int idx = S.perlin_perm[(i + a) & 255] ^ S.perlin_perm[256 + ((j + b) & 255)] ^
                      S.perlin_perm[512 + ((k + c) & 255)];
            V3 g = v3(S.perlin_ranvec[3 * idx], S.perlin_ranvec[3 * idx + 1], S.perlin_ranvec[3 * idx + 2]);
            V3 wv = v3(uu - a, vv - b, ww - c);
            acc += (a * hu + (1 - a) * (1 - hu)) * (b * hv + (1 - b) * (1 - hv)) * (c * hw + (1 - c) * (1 - hw)) *
                   dot(g, wv);
          }
      accum += weight * acc;
      weight *= 0.5f;
      tp = tp * 2.0f;
    }
    float turb = fabsf(accum);
    return v3(1, 1, 1) * 0.5f * (1 + rsin(scale * p.z + 5 * turb));
  }
  return v3(0.f);
}

SRR_D V3 tex_value(const SceneView& S, int ti, float u, float v, V3 p) {
  const DTex& T = S.texs[ti];
  if (T.kind == TEX_CONST) return v3(T.c[0], T.c[1], T.c[2]);
  return tex_value_slow(S, ti, u, v, p);
}

struct Onb {  // onb.h:21-30
  V3 u, v, w;
};
SRR_D Onb onb_from_w(V3 n) {
  Onb o;
  o.w = unit_vector(n);
  V3 a = (fabsf(o.w.x) >= kUp0p9) ? v3(0, 1, 0) : v3(1, 0, 0);  // fabs(w.x) > 0.9 (double)
  o.v = unit_vector(cross(o.w, a));
  o.u = cross(o.w, o.v);
  return o;
}
SRR_D V3 onb_local(const Onb& b, V3 a) { return a.x * b.u + a.y * b.v + a.z * b.w; }

// reflection.h:8-32
SRR_D float Cos2Theta(V3 w) { return w.z * w.z; }
SRR_D float AbsCosTheta(V3 w) { return fabsf(w.z); }
SRR_D float Sin2Theta(V3 w) { return fmaxf(0.0f, 1.0f - Cos2Theta(w)); }
SRR_D float SinTheta(V3 w) { return rsqrt_exact(Sin2Theta(w)); }
SRR_D float TanTheta(V3 w) { return SinTheta(w) / w.z; }
SRR_D float Tan2Theta(V3 w) { return Sin2Theta(w) / Cos2Theta(w); }
SRR_D float clamp11(float x) { return x < -1 ? -1.f : (x > 1 ? 1.f : x); }
SRR_D float CosPhi(V3 w) {
  float s = SinTheta(w);
  return (s == 0) ? 1 : clamp11(w.x / s);
}
SRR_D float SinPhi(V3 w) {
  float s = SinTheta(w);
  return (s == 0) ? 0 : clamp11(w.y / s);
}
SRR_D float Cos2Phi(V3 w) { return CosPhi(w) * CosPhi(w); }
SRR_D float Sin2Phi(V3 w) { return SinPhi(w) * SinPhi(w); }

// common.h:26-78
SRR_D float Erf(float x) {
  float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f, a5 = 1.061405429f;
  float p = 0.3275911f;
  int sign = 1;
  if (x < 0) sign = -1;
  x = fabsf(x);
  float t = 1 / (1 + p * x);
  float y = 1 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t + rexp(-x * x);
  return sign * y;
}
SRR_D float ErfInv(float x) {
  float w, p;
  x = x < -.99999f ? -.99999f : (x > .99999f ? .99999f : x);
  w = -rlog((1 - x) * (1 + x));
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
    w = rsqrt_exact(w) - 3;
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

// microfacet_distribution.h:137-211, sampleVisibleArea = true
struct Beck {
  float ax, ay;
  SRR_D float D(V3 wh) const {
    float tan2 = Tan2Theta(wh);
    if (isinf(tan2)) return 0.;
    float cos4 = Cos2Theta(wh) * Cos2Theta(wh);
    return rexp(-tan2 * (Cos2Phi(wh) / (ax * ax) + Sin2Phi(wh) / (ay * ay))) / (kPi * ax * ay * cos4);
  }
  SRR_D float Lambda(V3 w) const {
    float absTan = fabsf(TanTheta(w));
    if (isinf(absTan)) return 0;
    float alpha = rsqrt_exact(Cos2Phi(w) * ax * ax + Sin2Phi(w) * ay * ay);
    float a = 1 / (alpha * absTan);
    if (a > 1.6f) return 0;
    return (1 - 1.259f * a + 0.396f * a * a) / (3.535f * a + 2.181f * a * a);
  }
  SRR_D float G1(V3 w) const { return 1 / (1 + Lambda(w)); }
  SRR_D float G(V3 wo, V3 wi) const { return 1 / (1 + Lambda(wo) + Lambda(wi)); }
  SRR_D float Pdf(V3 wo, V3 wh) const { return D(wh) * G1(wo) * fabsf(dot(wo, wh)) / AbsCosTheta(wo); }
};

SRR_D void beckmann_sample11(float cosThetaI, float u1, float u2, float& sx, float& sy) {  // :34-107
  if (cosThetaI > .9999) {
    float r = rsqrt_exact(-rlog(1.0f - u1));
    float sinPhi = ::sin(2 * kPi * u2);
    float cosPhi = ::cos(2 * kPi * u2);
    sx = r * cosPhi;
    sy = r * sinPhi;
    return;
  }
  float sinThetaI = rsqrt_exact(fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI));
  float tanThetaI = sinThetaI / cosThetaI;
  float cotThetaI = 1 / tanThetaI;
  float a = -1, c = Erf(cosThetaI);
  float sample_x = fmaxf(u1, 1e-6f);
  float thetaI = racos(cosThetaI);
  float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
  float b = c - (1 + c) * rpow(1 - sample_x, fit);
  const float SQRT_PI_INV = (float)(1.f / ::sqrt(kPi));
  float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * rexp(-cotThetaI * cotThetaI));
  int it = 0;
  // (a loop that stops on |value| < 1e-5 has just computed ErfInv of the final b:
  // the reference's ErfInv(b) after the loop is that same value, so it is reused)
  float invErf = 0;
  bool fresh = false;
  while (++it < 10) {
    if (!(b >= a && b <= c)) b = 0.5f * (a + c);
    invErf = ErfInv(b);
    float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * (rexp(-invErf * invErf))) - sample_x;
    float derivative = normalization * (1 - invErf * tanThetaI);
    if (fabsf(value) < 1e-5f) {
      fresh = true;
      break;
    }
    if (value > 0) c = b;
    else a = b;
    b -= value / derivative;
  }
  sx = fresh ? invErf : ErfInv(b);
  sy = ErfInv(2.0f * fmaxf(u2, 1e-6f) - 1.0f);
}

SRR_D V3 beckmann_sample_wh(const Beck& d, V3 wo, float u1, float u2) {  // :12-32, :203-210
  bool flip = wo.z < 0;
  V3 wi = flip ? -wo : wo;
  V3 ws = unit_vector(v3(d.ax * wi.x, d.ay * wi.y, wi.z));
  float sx, sy;
  beckmann_sample11(ws.z, u1, u2, sx, sy);
  float tmp = CosPhi(ws) * sx - SinPhi(ws) * sy;
  sy = SinPhi(ws) * sx + CosPhi(ws) * sy;
  sx = tmp;
  sx = d.ax * sx;
  sy = d.ay * sy;
  V3 wh = unit_vector(v3(-sx, -sy, 1.f));
  if (flip) wh = -wh;
  return wh;
}

// The terms of one Beckmann sample that depend only on the incoming direction: computed
// once per scatter by bsdf_prepare<true>, where the reference recomputes them on every
// attempt of the resampling loop (pdf.h:136-152 -> :12-32, :34-107).  Same expressions,
// so the same values; the per-attempt part below takes them from here.
struct BeckPre {
  V3 wwo;            // the local unit -wo (pdf.h:140)
  V3 uw;             // unit_vector(wwo) (Reflect's)
  float cphi, sphi;  // CosPhi / SinPhi of the stretched direction ws
  float ct;          // ws.z: BeckmannSample11's cosThetaI
  float tan_t, c, fit, norm;  // its tanThetaI, Erf(cosThetaI), fit, normalization (ct <= .9999)
  float lam1;        // 1 + Lambda(wo): G(wo, wi)'s first two terms
  bool flip;         // wwo.z < 0
};

SRR_D void beckmann_pre(const Beck& d, const Onb& uvw, V3 wo, BeckPre& p) {
  const V3 mwo = -wo;
  p.wwo = unit_vector(v3(dot(mwo, uvw.u), dot(mwo, uvw.v), dot(mwo, uvw.w)));
  p.uw = unit_vector(p.wwo);
  p.flip = p.wwo.z < 0;
  const V3 wi = p.flip ? -p.wwo : p.wwo;
  const V3 ws = unit_vector(v3(d.ax * wi.x, d.ay * wi.y, wi.z));
  p.cphi = CosPhi(ws);
  p.sphi = SinPhi(ws);
  p.ct = ws.z;
  p.tan_t = p.c = p.fit = p.norm = 0;
  if (!(p.ct > .9999)) {
    const float cosThetaI = p.ct;
    float sinThetaI = rsqrt_exact(fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI));
    float tanThetaI = sinThetaI / cosThetaI;
    float cotThetaI = 1 / tanThetaI;
    p.c = Erf(cosThetaI);
    float thetaI = racos(cosThetaI);
    p.fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
    const float SQRT_PI_INV = (float)(1.f / ::sqrt(kPi));
    p.norm = 1 / (1 + p.c + SQRT_PI_INV * tanThetaI * rexp(-cotThetaI * cotThetaI));
    p.tan_t = tanThetaI;
  }
  p.lam1 = 1 + d.Lambda(wo);
}

// beckmann_sample11 with its direction terms from BeckPre
SRR_D void beckmann_sample11_pre(const BeckPre& p, float u1, float u2, float& sx, float& sy) {
  if (p.ct > .9999) {
    float r = rsqrt_exact(-rlog(1.0f - u1));
    float sinPhi = ::sin(2 * kPi * u2);
    float cosPhi = ::cos(2 * kPi * u2);
    sx = r * cosPhi;
    sy = r * sinPhi;
    return;
  }
  const float tanThetaI = p.tan_t, normalization = p.norm;
  float a = -1, c = p.c;
  float sample_x = fmaxf(u1, 1e-6f);
  float b = c - (1 + c) * rpow(1 - sample_x, p.fit);
  const float SQRT_PI_INV = (float)(1.f / ::sqrt(kPi));
  int it = 0;
  float invErf = 0;
  bool fresh = false;
  while (++it < 10) {
    if (!(b >= a && b <= c)) b = 0.5f * (a + c);
    invErf = ErfInv(b);
    float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * (rexp(-invErf * invErf))) - sample_x;
    float derivative = normalization * (1 - invErf * tanThetaI);
    if (fabsf(value) < 1e-5f) {
      fresh = true;
      break;
    }
    if (value > 0) c = b;
    else a = b;
    b -= value / derivative;
  }
  sx = fresh ? invErf : ErfInv(b);
  sy = ErfInv(2.0f * fmaxf(u2, 1e-6f) - 1.0f);
}

SRR_D V3 beckmann_sample_wh_pre(const Beck& d, const BeckPre& p, float u1, float u2) {
  float sx, sy;
  beckmann_sample11_pre(p, u1, u2, sx, sy);
  float tmp = p.cphi * sx - p.sphi * sy;
  sy = p.sphi * sx + p.cphi * sy;
  sx = tmp;
  sx = d.ax * sx;
  sy = d.ay * sy;
  V3 wh = unit_vector(v3(-sx, -sy, 1.f));
  if (p.flip) wh = -wh;
  return wh;
}

#ifndef SRR_SINCOS
#define SRR_SINCOS 1  // random_cosine_direction's sine and cosine from one sincosf_ (A/B: -DSRR_SINCOS=0)
#endif
// pdf.h:10-18
SRR_D V3 random_cosine_direction(Rng& rng) {
  float r1 = drand(rng);
  float r2 = drand(rng);
  float phi = 2 * kPi * r1;
  float z = rsqrt_exact(1 - r2);
#if SRR_SINCOS && !defined(SRR_LIBM_DOUBLE)
  float sp, cp;
  gm::sincosf_(phi, sp, cp);  // = sinf_(phi), cosf_(phi)
  float x = cp * 2 * rsqrt_exact(r2);
  float y = sp * 2 * rsqrt_exact(r2);
#else
  float x = rcos(phi) * 2 * rsqrt_exact(r2);  // cosf / sinf (glibc_mathf.h)
  float y = rsin(phi) * 2 * rsqrt_exact(r2);
#endif
  return v3(x, y, z);
}

// material.h:43-50: the three draws land in z, y, x (g++ argument order)
SRR_D V3 random_in_unit_sphere(Rng& rng) {
  V3 p;
  do {
    float z = (float)drand(rng);
    float y = (float)drand(rng);
    float x = (float)drand(rng);
    p = 2.0f * v3(x, y, z) - v3(1, 1, 1);
  } while (dot(p, p) >= 1.0);
  return p;
}

// light list (hitable_pdf over a hitable_list, hitable_list.h:54-67).  The sphere /
// triangle lights are out-of-line calls (rare kinds; inlined they bloat every
// variant), taking their tables, the light and the RNG state BY VALUE: a
// reference to the scene view or the Rng would give the caller's copies an
// address, and the path kernel would then keep them in scratch memory -- every
// RNG draw a scratch store (round 3's ALLFAM / MEDIA variants did).
__device__ __noinline__ float light_pdf_other(const DSphere* spheres, const DStandaloneTri* stris, DLight L, V3 o,
                                              V3 v);

SRR_D float light_pdf_one(const SceneView& S, const DLight& L, V3 o, V3 v) {
  Ray r{o, v, 0.0f};
  if (L.kind == LIGHT_XZRECT) {  // aarect.h:45-55
    const DRect& q = S.rects[L.idx];
    float t;
#if SRR_RECTAX
    if (rect_hit_t<1>(q, r, 0.001f, FLT_MAX, t)) {  // an xz_rect light (kax 1)
#else
    float u, vv;
    if (rect_hit(q, r, 0.001f, FLT_MAX, t, u, vv)) {
#endif
      float area = (q.hi0 - q.lo0) * (q.hi1 - q.lo1);
      float distance_square = t * t * squared_length(v);
      float cosine = fabsf(v.y / length(v));  // dot(v, (0,1,0)) / |v|
      return distance_square / (cosine * area);
    }
    return 0;
  }
  if (L.kind == LIGHT_NONE) return 0.0;
  return light_pdf_other(S.spheres, S.stris, L, o, v);
}

__device__ __noinline__ float light_pdf_other(const DSphere* spheres, const DStandaloneTri* stris, DLight L, V3 o,
                                              V3 v) {
  Ray r{o, v, 0.0f};
  if (L.kind == LIGHT_SPHERE) {  // sphere.h:69-78
    const DSphere& s = spheres[L.idx];
    float t;
    if (sphere_hit(s, false, r, 0.001f, FLT_MAX, t)) {
      V3 c = v3(s.c0[0], s.c0[1], s.c0[2]);
      float cos_theta_max = rsqrt_exact(1 - s.r * s.r / squared_length(c - o));
      float solid_angle = 2 * kPi * (1 - cos_theta_max);
      return 1 / solid_angle;
    }
    return 0;
  }
  if (L.kind == LIGHT_TRI) {  // triangle.h:70-87
    const DStandaloneTri& T = stris[L.idx];
    V3 p0 = v3(T.p[0], T.p[1], T.p[2]), p1 = v3(T.p[3], T.p[4], T.p[5]), p2 = v3(T.p[6], T.p[7], T.p[8]);
    float t, u, vv;
    if (tri_hit(p0, p1, p2, true, o, v / length(v), t, u, vv)) {
      const TriShade& sh = T.sh;
      float a0 = 1 - u - vv;
      V3 n = unit_vector(a0 * v3(sh.n[0], sh.n[1], sh.n[2]) + u * v3(sh.n[3], sh.n[4], sh.n[5]) +
                         vv * v3(sh.n[6], sh.n[7], sh.n[8]));
      V3 v01 = p1 - p0;
      V3 v01n = v01 / length(v01);
      V3 v02 = p2 - p0;
      V3 v02n = v02 / length(v02);
      float cos102 = dot(v01n, v02n);
      float sin102 = rsqrt_exact(1 - cos102 * cos102);
      float h = length(v02) * sin102;
      float area = 0.5 * length(v01) * h;
      float distance_square = t * t * squared_length(v);
      float cosine = fabsf(dot(v, n)) / length(v);
      return distance_square / (cosine * area);
    }
    return 0;
  }
  return 0.0;
}

SRR_D float lights_pdf(const SceneView& S, V3 o, V3 v) {
  const float weight = S.light_weight;  // 1.0 / n (a double division), made once on the host
  float sum = 0;
  for (int k = 0; k < S.n_lights; ++k) sum += weight * light_pdf_one(S, S.lights[k], o, v);
  return sum;
}

struct LightDraw {  // light_random_other's direction and the LCG state after its draws
  V3 d;
  uint64_t lcg;
};
__device__ __noinline__ LightDraw light_random_other(const DSphere* spheres, const DStandaloneTri* stris, DLight L,
                                                     V3 o, uint64_t lcg);

// one light's random() (aarect.h:57-60, sphere.h:80-86, triangle.h:89-94)
SRR_D V3 light_random_one(const SceneView& S, const DLight& L, V3 o, Rng& rng) {
  if (L.kind == LIGHT_XZRECT) {  // aarect.h:57-60: z drawn before x
    const DRect& q = S.rects[L.idx];
    float z = q.lo1 + drand(rng) * (q.hi1 - q.lo1);
    float x = q.lo0 + drand(rng) * (q.hi0 - q.lo0);
    return v3(x, q.k, z) - o;
  }
  if (L.kind == LIGHT_NONE) return v3(1, 0, 0);
  const LightDraw ld = light_random_other(S.spheres, S.stris, L, o, rng.lcg);
  rng.lcg = ld.lcg;
  return ld.d;
}

// hitable_list::random over the light list (hitable_list.h:63-67)
SRR_D V3 lights_random(const SceneView& S, V3 o, Rng& rng) {
  int index = int(drand(rng) * S.n_lights);
  return light_random_one(S, S.lights[index], o, rng);
}

__device__ __noinline__ LightDraw light_random_other(const DSphere* spheres, const DStandaloneTri* stris, DLight L,
                                                     V3 o, uint64_t lcg) {
  Rng rng{lcg, 0};  // (drand48 draws only: the PCG stream is not used here)
  if (L.kind == LIGHT_SPHERE) {  // sphere.h:7-15, 80-86
    const DSphere& s = spheres[L.idx];
    V3 dirc = v3(s.c0[0], s.c0[1], s.c0[2]) - o;
    float d2 = squared_length(dirc);
    Onb uvw = onb_from_w(dirc);
    float r1 = drand(rng);
    float r2 = drand(rng);
    float z = 1 + r2 * (rsqrt_exact(1 - s.r * s.r / d2) - 1);
    float phi = 2 * kPi * r1;
    float x = rcos(phi) * rsqrt_exact(1 - z * z);
    float y = rsin(phi) * rsqrt_exact(1 - z * z);
    return LightDraw{onb_local(uvw, v3(x, y, z)), rng.lcg};
  }
  if (L.kind == LIGHT_TRI) {  // triangle.h:89-94
    const DStandaloneTri& T = stris[L.idx];
    float u = drand(rng);
    float v = drand(rng) * (1 - u);
    V3 p0 = v3(T.p[0], T.p[1], T.p[2]), p1 = v3(T.p[3], T.p[4], T.p[5]), p2 = v3(T.p[6], T.p[7], T.p[8]);
    return LightDraw{p0 * (1 - u - v) + p1 * u + p2 * v - o, rng.lcg};
  }
  return LightDraw{v3(1, 0, 0), rng.lcg};
}

// The BSDF half of the mixture (pdf.h:30-156) for one non-specular hit.
struct Bsdf {
  int kind;
  Onb uvw;
  V3 n;
  float A, B;      // orennayar
  Beck dist;       // beckmann
  float beck_pdf;  // beckmann_pdf::pdf_value, set by generate (starts 0)
  // value()'s terms that depend only on the incoming direction, computed once per
  // bounce (bsdf_prepare) instead of once per resampling iteration
  float co;        // cosine_pdf: dot(unit_vector(wo), n)
  V3 lo;           // onrennayar_pdf: local unit(-wo)
  bool flip;       // cosine_pdf / onrennayar_pdf generate: dot(-wo, n) > 0
  BeckPre bp;      // beckmann: the sample's incoming-direction terms (bsdf_prepare<true>)
};

SRR_D V3 to_local_unit(const Onb& b, V3 d) {
  V3 ud = unit_vector(d);
  return unit_vector(v3(dot(ud, b.u), dot(ud, b.v), dot(ud, b.w)));
}

template <bool BECK>
SRR_D V3 bsdf_generate(Bsdf& f, V3 wo, Rng& rng) {
  if (BECK) {  // pdf.h:136-152
    (void)wo;  // (its terms are in f.bp, from bsdf_prepare<true>)
    float u1 = pcg_uniform(rng);
    float u2 = pcg_uniform(rng);
    const BeckPre& p = f.bp;
    V3 wh = beckmann_sample_wh_pre(f.dist, p, u1, u2);
    V3 wi = -p.uw + 2 * dot(p.uw, wh) * wh;  // Reflect (reflection.h:34-36)
    V3 wwi = unit_vector(wi.x * f.uvw.u + wi.y * f.uvw.v + wi.z * f.uvw.w);
    // D(wh) * G(wo, wi), G = 1 / (1 + Lambda(wo) + Lambda(wi))
    f.beck_pdf = f.dist.D(wh) * (1 / (p.lam1 + f.dist.Lambda(wi))) / (4 * AbsCosTheta(wi) * AbsCosTheta(p.wwo));
    if (!(wi.z * p.wwo.z > 0)) f.beck_pdf = 0;
    return wwi;
  }
  // cosine_pdf / onrennayar_pdf (pdf.h:47-56, 103-112)
  V3 g = random_cosine_direction(rng);
  if (f.flip) g.z *= -1;  // dot(-wo, n) > 0, computed by bsdf_prepare
  return onb_local(f.uvw, g);
}

template <bool BECK>
SRR_D void bsdf_prepare(Bsdf& f, V3 wo) {
  if (BECK) {
    beckmann_pre(f.dist, f.uvw, wo, f.bp);
    return;
  }
  f.flip = dot(-wo, f.n) > 0;
  // (both fields written on every path: one of them left unset kept f in scratch)
  float co = 0;
  V3 lo = v3(0.f);
  if (f.kind == MAT_LAMBERTIAN) co = dot(unit_vector(wo), f.n);
  else lo = to_local_unit(f.uvw, -wo);
  f.co = co;
  f.lo = lo;
}

template <bool BECK>
SRR_D float bsdf_value(const Bsdf& f, V3 wo, V3 wi) {  // after bsdf_prepare(f, wo)
  (void)wo;
  if (BECK) return f.beck_pdf;
  if (f.kind == MAT_LAMBERTIAN) {  // pdf.h:33-46
    const float co = f.co;
    float ci = dot(unit_vector(wi), f.n);
    if (ci * co < 0) return fabsf(ci) / kPi;
    return 0;
  }
  // onrennayar_pdf::value (pdf.h:64-101)
  const V3 lo = f.lo;
  V3 li = to_local_unit(f.uvw, wi);
  float sinThetaI = SinTheta(li), sinThetaO = SinTheta(lo);
  float maxCos = 0;
  if (sinThetaI > 1e-4 && sinThetaO > 1e-4) {
    float sinPhiI = SinPhi(li), cosPhiI = CosPhi(li);
    float sinPhiO = SinPhi(lo), cosPhiO = CosPhi(lo);
    float dCos = cosPhiI * cosPhiO + sinPhiI * sinPhiO;
    maxCos = ffmax(0.0f, dCos);
  }
  float sinAlpha, tanBeta;
  if (AbsCosTheta(li) > AbsCosTheta(lo)) {
    sinAlpha = sinThetaO;
    tanBeta = sinThetaI / AbsCosTheta(li);
  } else {
    sinAlpha = sinThetaI;
    tanBeta = sinThetaO / AbsCosTheta(lo);
  }
  float cosine = li.z;
  if (cosine < 0) cosine = 0;
  return cosine * (f.A + f.B * maxCos * sinAlpha * tanBeta) / kPi;
}

template <bool BECK>
SRR_D float scattering_pdf(const Bsdf& f, V3 n, V3 rin, V3 sc) {
  if (BECK) {  // material.h:160-185
    V3 wo = to_local_unit(f.uvw, -rin);
    V3 wi = to_local_unit(f.uvw, sc);
    V3 wh = unit_vector(wi + wo);
    return f.dist.Pdf(wo, wh) / (4 * dot(wo, wh));
  }
  float c = dot(n, unit_vector(sc));  // material.h:100-105, 134-138
  if (c < 0) c = 0;
  return c / kPi;
}

// ================================================================ kernels
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-aggregated append: one atomic per wave for the lanes with `pred`.
__device__ __forceinline__ void append(bool pred, int value, int* list, int* count) {
  uint64_t mask = __ballot(pred);
  if (!mask) return;
  int leader = __ffsll((unsigned long long)mask) - 1;
  int base = 0;
  if (lane_id() == leader) base = atomicAdd(count, __popcll(mask));
  base = __shfl(base, leader);
  if (pred) {
    int rank = __popcll(mask & ((1ull << lane_id()) - 1));
    list[base + rank] = value;
  }
}

// append() for the four material families at once: the four list counters are
// bumped by one atomic instruction (lanes 0-3), so a wave pays one round trip.
__device__ __forceinline__ void append4(int fam, int value, int* lists, int list_cap, int* counts) {
  const uint64_t m0 = __ballot(fam == 0), m1 = __ballot(fam == 1), m2 = __ballot(fam == 2), m3 = __ballot(fam == 3);
  if ((m0 | m1 | m2 | m3) == 0) return;
  const int l = lane_id();
  const uint64_t mine = l == 0 ? m0 : l == 1 ? m1 : l == 2 ? m2 : m3;
  int base = 0;
  if (l < 4 && mine) base = atomicAdd(counts + l, __popcll(mine));
  base = __shfl(base, fam >= 0 ? fam : 0);
  if (fam >= 0) {
    const uint64_t m = fam == 0 ? m0 : fam == 1 ? m1 : fam == 2 ? m2 : m3;
    lists[fam * list_cap + base + __popcll(m & ((1ull << l) - 1))] = value;
  }
}

// ---------------------------------------------- wave-cooperative mixture loop
// The resampling loop of a diffuse bounce (Raytracing_n.cpp:75-89: draw from the
// 50/50 light / BSDF mixture until its pdf is non-zero) needs ~2
// attempts per lane but a wave would run until its slowest lane is done (~7 for
// 64 lanes).  Instead the wave runs the loops of all its pending lanes together:
// per round every lane evaluates one attempt of some pending path, the k-th
// helper of a path taking attempt tries+k.  That attempt's LCG state is the
// path's state advanced over k attempts' draws, and an attempt's draw count is a
// function of the state alone (branch draw; light: index draw + 2 if the light
// samples, BSDF: 2), so skip_attempt() reaches it exactly.  Each path keeps its
// first successful attempt (direction, pdf, LCG state after it): bit for bit the
// sequential loop's result.  Only the LCG is drawn in a diffuse mixture loop.

// what one attempt of a path's mixture loop reads (plus its LCG state)
struct DiffSetup {
  V3 p;          // hit point (light sampling origin)
  V3 w, v;       // the bounce's onb (u = cross(w, v), exactly as onb_from_w)
  V3 nl;         // lambertian: n (bsdf value); orennayar: local unit(-wo)
  float c0, c1;  // lambertian: co; orennayar: A, B
  int flags;     // bit 0: orennayar, bit 1: flip (dot(-wo, n) > 0)
};

SRR_D DiffSetup diff_setup(const Bsdf& f, V3 p) {
  const bool on = f.kind != MAT_LAMBERTIAN;
  // (selected as values, not as one of two addresses in f)
  V3 nl = f.n;
  float c0 = f.co;
  if (on) {
    nl = f.lo;
    c0 = f.A;
  }
  return DiffSetup{p, f.uvw.w, f.uvw.v, nl, c0, f.B, (on ? 1 : 0) | (f.flip ? 2 : 0)};
}

SRR_D Bsdf bsdf_of(const DiffSetup& d) {
  Bsdf f;
  f.kind = (d.flags & 1) ? (int)MAT_ORENNAYAR : (int)MAT_LAMBERTIAN;
  f.uvw.w = d.w;
  f.uvw.v = d.v;
  f.uvw.u = cross(d.w, d.v);
  f.n = d.nl;
  f.lo = d.nl;
  f.co = d.c0;
  f.A = d.c0;
  f.B = d.c1;
  f.flip = (d.flags & 2) != 0;
  return f;
}

// one attempt of the loop body (Raytracing_n.cpp:76-88; pdf.h:183-192)
SRR_D float mixture_attempt(const SceneView& S, Bsdf& f, V3 hpt, Rng& rng, V3& ndir) {
  if (drand(rng) < 0.5) ndir = lights_random(S, hpt, rng);
  else ndir = bsdf_generate<false>(f, v3(0.f), rng);
  return 0.5 * lights_pdf(S, hpt, ndir) + 0.5 * bsdf_value<false>(f, v3(0.f), ndir);
}

SRR_D uint64_t lcg_step(uint64_t s) { return (0x5DEECE66DULL * s + 0xB16ULL) & 0xFFFFFFFFFFFFULL; }

// the LCG state after one attempt's draws, from the state before it
SRR_D uint64_t skip_attempt(const SceneView& S, uint64_t s) {
  s = lcg_step(s);                      // drand() < 0.5: the branch
  if ((s >> 47) == 0) {                 // light: hitable_list::random (hitable_list.h:63-67)
    s = lcg_step(s);                    // the light index
    const int idx = int((double)(uint32_t)(s >> 16) / 4294967296.0 * S.n_lights);
    if (S.lights[idx].kind != LIGHT_NONE) s = lcg_step(lcg_step(s));  // xz_rect / sphere / triangle: 2
  } else {
    s = lcg_step(lcg_step(s));          // random_cosine_direction: 2
  }
  return s;
}


#ifndef SRR_COOP_HELPERS
#define SRR_COOP_HELPERS 8
#endif
#ifndef SRR_COOP_ID0
#define SRR_COOP_ID0 0
#endif
constexpr int kMaxHelpers = SRR_COOP_HELPERS;  // attempts of one path per round

// Runs to completion the loops of every lane with `pend` (converged wave, all 64
// lanes active).  In: the lane's setup, its LCG state before attempt `tries`.
// Out: ndir, pdf and the LCG state after the first attempt with pdf != 0 (or the
// guard's last attempt).  The first round is each pending lane's own attempt
// (no exchange); later rounds spread the remaining paths over all 64 lanes.
// deep_tries: past this many failed attempts a path takes every free lane
// (PathWork::deep_tries, 32; SRR_DEEP_TRIES=0 forces it from the first round).
SRR_D int coop_mixture(const SceneView& S, const DiffSetup& me, bool& pend, int& tries, uint64_t& lcg, V3& ndir,
                       float& pdf, int deep_tries) {
  int rounds = 0;
  const int lane = lane_id();
  const uint64_t lt = (1ull << lane) - 1;
  uint64_t F = __ballot(pend);
  bool first = SRR_COOP_ID0 != 0;
  while (F) {
    const int nF = __popcll(F);
    // paths whose loop has failed kDeepTries times (e.g. a hit point in the light's
    // own plane: every light sample runs parallel to it) may need up to the guard's
    // 100,000 attempts; once every pending path is that deep, all 64 lanes help
    const int cap = __ballot(pend && tries < deep_tries) == 0 ? 64 : kMaxHelpers;
    const int rank = pend ? __popcll(F & lt) : nF + __popcll(~F & lt);
    DiffSetup d;
    int t0, k;
    uint64_t s;
    if (first) {
      d = me;
      t0 = tries;
      s = lcg;
      k = pend ? 0 : 64;
    } else {
      // lane r < nF learns the lane of the r-th pending path (a permutation of
      // all 64 lanes: pending lanes in order, then the others)
      const int owner_of = __builtin_amdgcn_ds_permute(rank << 2, lane);
      const int q = lane % nF;
      k = lane / nF;
      const int src = __builtin_amdgcn_ds_bpermute(q << 2, owner_of);
      d.p = v3(__shfl(me.p.x, src), __shfl(me.p.y, src), __shfl(me.p.z, src));
      d.w = v3(__shfl(me.w.x, src), __shfl(me.w.y, src), __shfl(me.w.z, src));
      d.v = v3(__shfl(me.v.x, src), __shfl(me.v.y, src), __shfl(me.v.z, src));
      d.nl = v3(__shfl(me.nl.x, src), __shfl(me.nl.y, src), __shfl(me.nl.z, src));
      d.c0 = __shfl(me.c0, src);
      d.c1 = __shfl(me.c1, src);
      d.flags = __shfl(me.flags, src);
      t0 = __shfl(tries, src);
      s = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(lcg >> 32), src) << 32) |
          (uint32_t)__shfl((int)(uint32_t)lcg, src);
    }
    const bool active = k < cap && t0 + k < kMixtureGuard;
    V3 nd = v3(0.f);
    float pv = 0;
    if (active) {
      for (int j = 0; j < k; ++j) s = skip_attempt(S, s);
      Rng rr{s, 0};
      Bsdf f = bsdf_of(d);
      pv = mixture_attempt(S, f, d.p, rr, nd);
      s = rr.lcg;
    }
    const uint64_t ok = __ballot(active && (pv != 0 || t0 + k + 1 >= kMixtureGuard));
    if (first) {  // every pending lane ran its own next attempt
      if (pend) {
        lcg = s;
        if ((ok >> lane) & 1) {
          ndir = nd;
          pdf = pv;
          pend = false;
        } else {
          tries += 1;
        }
      }
      first = false;
    } else {
      // owner: its first successful helper (k ascending), else its last one
      int win = lane, m = 0;
      if (pend) {
        m = min(cap, (63 - rank) / nF + 1);
        m = min(m, kMixtureGuard - tries);
        int j = 0;
        while (j < m - 1 && !((ok >> (rank + j * nF)) & 1)) ++j;
        win = rank + j * nF;
      }
      const float wx = __shfl(nd.x, win), wy = __shfl(nd.y, win), wz = __shfl(nd.z, win), wp = __shfl(pv, win);
      const uint64_t ws = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(s >> 32), win) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)s, win);
      if (pend) {
        lcg = ws;
        if ((ok >> win) & 1) {
          ndir = v3(wx, wy, wz);
          pdf = wp;
          pend = false;
        } else {
          tries += m;
        }
      }
    }
    F = __ballot(pend);
    ++rounds;
  }
  return rounds;
}

// camera::get_ray(s, t) (camera.h:51-59; random_in_unit_disk camera.h:8-14)
SRR_D void camera_get_ray(const DCamera& C, float u, float v, Rng& rng, V3& o, V3& dir, float& time) {
  V3 pd;
  do {  // random_in_unit_disk (camera.h:8-14): y drawn before x
    float y = drand(rng);
    float x = drand(rng);
    pd = 2.0f * v3(x, y, 0) - v3(1, 1, 0);
  } while (dot(pd, pd) >= 1.0);
  V3 rd = C.lens_radius * pd;
  V3 cu = v3(C.u[0], C.u[1], C.u[2]), cv = v3(C.v[0], C.v[1], C.v[2]);
  V3 offset = cu * rd.x + cv * rd.y;
  time = C.time0 + drand(rng) * (C.time1 - C.time0);
  V3 org = v3(C.origin[0], C.origin[1], C.origin[2]);
  dir = v3(C.llc[0], C.llc[1], C.llc[2]) + u * v3(C.horizontal[0], C.horizontal[1], C.horizontal[2]) +
        v * v3(C.vertical[0], C.vertical[1], C.vertical[2]) - org - offset;
  dir = unit_vector(dir);
  o = org + offset;
}

// ------------------------------------------- mixture loop with dead BSDF draws
// For most diffuse bounces no BSDF-branch sample of the mixture can have a
// non-zero pdf: the BSDF value of a cosine / Oren-Nayar sample is 0 (SURVEY Q1:
// the sample is put in the hemisphere opposite the viewer), and every light lies
// wholly on the far side of the tangent plane from that hemisphere, so the light
// pdf of the sample is 0 too.  bsdf_dead() proves this per bounce (with margins
// far above float rounding); the loop then passes over such attempts by their
// LCG draws alone -- the branch draw, and r1, r2 of random_cosine_direction,
// whose r2 <= 0.999 keeps the sample's w component >= 0.03, well clear of the
// tangent plane -- and evaluates exactly only light-branch attempts, near-tangent
// BSDF samples, and the guard's last attempt.  The attempts it evaluates and
// their results are the sequential loop's, bit for bit.
#ifndef SRR_MIXTURE_SKIP
#define SRR_MIXTURE_SKIP 2
#endif

SRR_D bool light_point_far(V3 c, V3 p, V3 w, float sgn, float m) { return sgn * dot(c - p, w) <= -m; }

SRR_D bool bsdf_dead(const SceneView& S, const Bsdf& f, V3 p) {
  // the BSDF value: lambertian |ci|/pi only when ci*co < 0, with sign(ci) the
  // sample's hemisphere (-1 flipped, +1 not); orennayar's cosine clamps a
  // flipped sample to 0
  if (f.kind == MAT_LAMBERTIAN) {
    if (f.flip ? !(f.co <= 0) : !(f.co >= 0)) return false;
  } else if (!f.flip) {
    return false;
  }
  const float sgn = f.flip ? -1.f : 1.f;
  const V3 w = f.uvw.w;
  const float ps = fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fabsf(p.z)) + 1.f;
  for (int k = 0; k < S.n_lights; ++k) {
    const DLight L = S.lights[k];
    if (L.kind == LIGHT_XZRECT) {
      const DRect q = S.rects[L.idx];
#if SRR_XFAX  // an xz_rect light: kax 1, a0 0, a1 2
      if (!(q.k != p.y)) return false;  // the hit point in the light's plane
#else
      if (!(q.k != p[q.kax])) return false;  // the hit point in the light's plane
#endif
      const float m = 1e-3f * (ps + fmaxf(fmaxf(fmaxf(fabsf(q.lo0), fabsf(q.hi0)), fmaxf(fabsf(q.lo1), fabsf(q.hi1))),
                                          fabsf(q.k)));
      for (int c = 0; c < 4; ++c) {
#if SRR_XFAX
        const V3 v = v3((c & 1) ? q.hi0 : q.lo0, q.k, (c & 2) ? q.hi1 : q.lo1);
#else
        V3 v = v3(0.f);
        v.set(q.kax, q.k);
        v.set(q.a0, (c & 1) ? q.hi0 : q.lo0);
        v.set(q.a1, (c & 2) ? q.hi1 : q.lo1);
#endif
        if (!light_point_far(v, p, w, sgn, m)) return false;
      }
    } else if (L.kind == LIGHT_SPHERE) {
      const DSphere sp = S.spheres[L.idx];
      const V3 c = v3(sp.c0[0], sp.c0[1], sp.c0[2]);
      const float r = fabsf(sp.r);
      const float m = 1e-3f * (ps + fmaxf(fmaxf(fabsf(c.x), fabsf(c.y)), fabsf(c.z)) + r);
      if (!light_point_far(c, p, w, sgn, r + m)) return false;
    } else if (L.kind == LIGHT_TRI) {
      const DStandaloneTri& T = S.stris[L.idx];  // (read in place: a copy indexed in a loop lived in scratch)
      float cs = 0;
#pragma unroll
      for (int k2 = 0; k2 < 9; ++k2) cs = fmaxf(cs, fabsf(T.p[k2]));
      const float m = 1e-3f * (ps + cs);
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (!light_point_far(v3(T.p[3 * c], T.p[3 * c + 1], T.p[3 * c + 2]), p, w, sgn, m)) return false;
    } else if (L.kind != LIGHT_NONE) {
      return false;
    }
  }
  return true;
}

// Runs to completion the loops of every lane with `pend`, each on its own path:
// pass over dead BSDF attempts, evaluate the next candidate attempt exactly,
// repeat while it fails.  In: the lane's setup and its LCG state before attempt
// `tries`.  Out: ndir, pdf and the LCG state after the first attempt with
// pdf != 0 (or the guard's last attempt).  Returns the wave's exact rounds.
SRR_D int skip_mixture(const SceneView& S, const DiffSetup& me, bool dead, bool& pend, int& tries, uint64_t& lcg,
                       V3& ndir, float& pdf, int max_rounds = 1 << 30) {
  int rounds = 0;
  while (rounds < max_rounds && __ballot(pend)) {
    if (pend) {
      uint64_t s = lcg;
      int t = tries;
      if (dead) {
        while (t + 1 < kMixtureGuard) {
          const uint64_t s1 = lcg_step(s);
          if ((s1 >> 47) == 0) break;  // light branch: a candidate
          const uint64_t s3 = lcg_step(lcg_step(s1));
          const float r2 = (float)((double)(uint32_t)(s3 >> 16) / 4294967296.0);
          if (!(r2 <= 0.999f)) break;  // near-tangent BSDF sample: evaluate it
          s = s3;
          ++t;
        }
      }
      Rng rr{s, 0};
      Bsdf f = bsdf_of(me);
      V3 nd;
      const float pv = mixture_attempt(S, f, me.p, rr, nd);
      lcg = rr.lcg;
      tries = t + 1;
      if (pv != 0 || tries >= kMixtureGuard) {
        ndir = nd;
        pdf = pv;
        pend = false;
      }
    }
    ++rounds;
  }
  return rounds;
}

// Point i of the reference's Sobol set for D = 2 (Raytracing_n.cpp:721-812, the
// Joe-Kuo generator with direction numbers "1" and "2 1 0 1"), computed instead
// of loaded: the generator's Gray-code recurrence X_i = X_{i-1} ^ V[c(i-1)] gives
// X_i = XOR of V[k] over the set bits k of gray(i) = i ^ (i >> 1); dimension 1 has
// V[k] = 2^(31-k) (so X = bit-reversed gray(i)), dimension 2 (s = 1, a = 0)
// V[0] = 2^31, V[k] = V[k-1] ^ (V[k-1] >> 1).  Both are exact in double after the
// division by 2^32.  Equal to the uploaded set point for point (the full-frame
// and golden parity tests use every point); it saves each path start a global load.
SRR_D void sobol2_point(uint32_t i, double& sx, double& sy) {
  const uint32_t g = i ^ (i >> 1);
  uint32_t y = 0, v = 0x80000000u;
  for (uint32_t t = g; t; t >>= 1, v ^= v >> 1)
    if (t & 1) y ^= v;
  sx = (double)__builtin_bitreverse32(g) / 4294967296.0;
  sy = (double)y / 4294967296.0;
}

// The camera ray of sample s_global of pixel `pix` with its per-path RNG streams
// (SURVEY §8(d) seeding; Raytracing_n.cpp:827-836; camera::get_ray, camera.h:51-59).
SRR_D uint32_t udiv31(uint32_t n, UDiv31 v) { return (uint32_t)(((uint64_t)n * v.m) >> v.p); }

SRR_D void camera_ray(const SceneView& S, int pix, int s_global, double sx, double sy, int nx, int ny,
                      uint64_t base_seed, V3& o, V3& dir, float& time, Rng& rng, const UDiv31* dnx = nullptr) {
  const int q = dnx ? (int)udiv31((uint32_t)pix, *dnx) : pix / nx;
  int i = pix - q * nx;   // pix % nx
  int j = ny - 1 - q;     // Raytracing_n.cpp:827-828 (SURVEY Q12 fix)
  uint64_t h = 0xcbf29ce484222325ULL ^ base_seed;
  uint32_t w[3] = {(uint32_t)i, (uint32_t)j, (uint32_t)s_global};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      h ^= (w[k] >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ULL;
    }
  rng.lcg = h & 0xFFFFFFFFFFFFULL;
  rng.pcg = 0x853c49e6748fea9bULL ^ (rng.lcg << 16);
  float u = float(sx + i) / float(nx);
  float v = float(sy + j) / float(ny);
  camera_get_ray(*S.cam, u, v, rng, o, dir, time);
}


__global__ void __launch_bounds__(256) k_raygen(SceneView S, PathState P, BatchInfo B) {
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B.n_paths) return;
  int lp = q / B.spp_batch;
  int s = B.s0 + q % B.spp_batch;
  int p = B.slot0 + q;
  if (q == 0) *B.count = B.act0 + B.n_paths;
  int pix = B.pixels[B.p0 + lp];
  Rng rng;
  V3 o, dir;
  float time;
  camera_ray(S, pix, B.s_base + s, B.sobol[2 * s], B.sobol[2 * s + 1], B.nx, B.ny, B.base_seed, o, dir, time, rng);
  nts(&P.ray_o[p], make_float4(o.x, o.y, o.z, time));
  nts(&P.ray_d[p], make_float4(dir.x, dir.y, dir.z, 0.f));
  nts(&P.lcg[p], rng.lcg);
  nts(&P.pcg[p], rng.pcg);
  nts(&P.depth[p], 0);
  nts(&P.spec[p], 0);
  B.active[B.act0 + q] = p;
  if (P.rays) P.rays[p] = 0;
}


template <bool MEDIA, int TR>
__global__ void __launch_bounds__(kTraceBlock) k_trace(SceneView S0, PathState P, const int* active, const int* count,
                                                       int* lists, int list_cap, int* fam_count, int max_depth,
                                                       unsigned long long* ctr) {
  const uint64_t t_start = tr_mode(TR) == TR_BVH4_TIMED ? __builtin_amdgcn_s_memtime() : 0;
  SceneView S = S0;
  if constexpr ((TR & TR_WL) != 0) {  // world tables -> LDS, once per block
    __shared__ uint4 s_world[kWorldLdsBytes / 16];
    for (int i = threadIdx.x; i < S0.world_words; i += blockDim.x) s_world[i] = S0.world_blob[i];
    __syncthreads();
    const char* b = (const char*)s_world;
    S.objs = (const DObj*)(b + S0.world_off[0]);
    S.xforms = (const DXform*)(b + S0.world_off[1]);
    S.spheres = (const DSphere*)(b + S0.world_off[2]);
    S.rects = (const DRect*)(b + S0.world_off[3]);
    S.stris = (const DStandaloneTri*)(b + S0.world_off[4]);
    S.meshes = (const DMesh*)(b + S0.world_off[5]);
    S.media = (const DMedium*)(b + S0.world_off[6]);
  }
  TraceCtx cx{ctr, nullptr, nullptr};
  if constexpr (tr_mode(TR) != TR_BVH2) {
    __shared__ int s_node[kStack * kTraceBlock];
    __shared__ float s_t[kStack * kTraceBlock];
    cx.st_node = to_lds(s_node + threadIdx.x);
    cx.st_t = to_lds(s_t + threadIdx.x);
  }
  const uint64_t t_staged = tr_mode(TR) == TR_BVH4_TIMED ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t t_ray = t_staged, t_hit = t_staged;
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  int n = *count;
  int p = -1, fam = -1;
  if (q < n) {
    p = active[q];
    float4 ro = ntl(&P.ray_o[p]), rdv = ntl(&P.ray_d[p]);
    Ray r{v3(ro.x, ro.y, ro.z), v3(rdv.x, rdv.y, rdv.z), ro.w};
    Rng rng{ntl(&P.lcg[p]), ntl(&P.pcg[p])};
    if (tr_mode(TR) == TR_BVH4_TIMED) {
      __builtin_amdgcn_s_waitcnt(0);  // diagnostics: ray loaded
      t_ray = __builtin_amdgcn_s_memtime();
    }
    WorldHit w = world_hit<MEDIA, TR>(S, r, rng, cx);
    if (tr_mode(TR) == TR_BVH4_TIMED) t_hit = __builtin_amdgcn_s_memtime();
    if (MEDIA) nts(&P.lcg[p], rng.lcg);
    store_hit(S, P, p, w, max_depth, fam);
  }
  append4(fam, p, lists, list_cap, fam_count);
  if (tr_mode(TR) == TR_BVH4_TIMED && ctr && n >= (1 << 20) && __lane_id() == 0) {  // diagnostics: one record per wave
    const unsigned long long k = atomicAdd(ctr, 1ull);
    if (k < kTimingCap) {
      unsigned long long* e = ctr + 1 + 8 * k;
      e[0] = __builtin_amdgcn_s_memtime() - t_start;
      e[1] = cx.mesh_cycles;
      e[2] = (unsigned long long)cx.mesh_steps;
      e[3] = t_staged - t_start;
      e[4] = t_ray - t_staged;
      e[5] = t_hit - t_ray;
      e[6] = __builtin_amdgcn_s_memtime() - t_hit;
    }
  }
}

// Hit records of the traced rays (world_record), kept out of the trace kernels
// so their register budget stays with the traversal.
__global__ void __launch_bounds__(256) k_record(SceneView S, PathState P, const int* active, const int* count) {
  const int n = *count;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int p = active[q];
    const int4 hw = ntl(&P.hit_w[p]);
    if (hw.x < 0 || hw.w < 0) continue;  // miss / null material: no record is read
    const float4 ro = ntl(&P.ray_o[p]), rdv = ntl(&P.ray_d[p]);
    const Ray r{v3(ro.x, ro.y, ro.z), v3(rdv.x, rdv.y, rdv.z), ro.w};
    const HitRec h = world_record(S, r, WorldHit{hw.x, hw.y, __int_as_float(hw.z)});
    nts(&P.hit_p[p], make_float4(h.p.x, h.p.y, h.p.z, h.u));
    nts(&P.hit_n[p], make_float4(h.n.x, h.n.y, h.n.z, h.v));
  }
}

// Diagnostic probes (SRR_PROBE=1, timing attribution only): the trace kernel's
// stages re-run over the same active rays with their results discarded.
// MODE 0: load the ray; 1: + world list without meshes; 4: + mesh instance
// transform and ray setup; 5: + the mesh's first node; 2: + meshes (the full
// closest-hit); 3: + hit record.
template <bool MEDIA, int TR, int MODE>
__global__ void __launch_bounds__(kTraceBlock) k_probe(SceneView S, PathState P, const int* active, const int* count,
                                                       int* sink) {
  TraceCtx cx{nullptr, nullptr, nullptr};
  if constexpr (TR != TR_BVH2) {
    __shared__ int s_node[kStack * kTraceBlock];
    __shared__ float s_t[kStack * kTraceBlock];
    cx.st_node = to_lds(s_node + threadIdx.x);
    cx.st_t = to_lds(s_t + threadIdx.x);
  }
  int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= *count) return;
  int p = active[q];
  float4 ro = ntl(&P.ray_o[p]), rdv = ntl(&P.ray_d[p]);
  Ray r{v3(ro.x, ro.y, ro.z), v3(rdv.x, rdv.y, rdv.z), ro.w};
  float acc = ro.x + rdv.y;
  if (MODE >= 1) {
    Rng rng{ntl(&P.lcg[p]), ntl(&P.pcg[p])};
    WorldHit w{-1, -1, 0};
    if (MODE == 1 || MODE == 4 || MODE == 5) {
      float closest = FLT_MAX;
      for (int k = 0; k < S.n_world; ++k) {
        const DObj ob = wload<TR>(S.objs, k);
        if (ob.kind == OBJ_MEDIUM) continue;
        if (ob.kind == OBJ_MESH) {
          if (MODE == 1) continue;
          const Ray lr = chain_in(S, ob, r);
          const DMesh m = wload<TR>(S.meshes, ob.idx);
          const V3 inv = v3(1.0f / lr.d.x, 1.0f / lr.d.y, 1.0f / lr.d.z);
          const float len = length(lr.d);
          const V3 dir = lr.d / len;
          acc += inv.x + inv.y + inv.z + dir.x + dir.y + dir.z + (float)m.node4_off;
          if (MODE == 5) {  // + the first 4-wide node and its leaf boxes
            const float4* N = S.node4 + 8 * (size_t)m.node4_off;
            float4 a = N[0], b = N[3], c = N[6];
            acc += (a.x - lr.o.x) * inv.x + (b.y - lr.o.y) * inv.y + c.z;
          }
          continue;
        }
        ObjHit h;
        if (basic_hit<TR>(S, ob, chain_in(S, ob, r), 0.001f, closest, false, h, cx)) { closest = h.t; w.obj = k; }
      }
      acc += closest;
    } else {
      w = world_hit<MEDIA, TR>(S, r, rng, cx);
      acc += w.t;
      if (MODE == 3 && w.obj >= 0) {
        HitRec h = world_record(S, r, w);
        acc += h.p.x + h.n.y + h.u;
      }
    }
    acc += (float)w.obj;
  }
  if (acc == 1234.5678f) sink[0] = p;  // keeps the work alive
}

// Folds the recorded bounces back to front exactly like the recursion returns
// (Raytracing_n.cpp:69 and :94), then de_nan and store the sample.
__device__ void finish_path(const PathState& P, int p, V3 C, int depth, uint64_t spec, int max_depth) {
  for (int k = depth - 1; k >= 0; --k) {
    float4 a = ntl(&P.rec_a[(size_t)p * max_depth + k]);
    V3 av = v3(a.x, a.y, a.z);
    if ((spec >> k) & 1) C = av * C;
    else C = v3(0.f) + (av * C) / a.w;  // emitted (== 0) + attenuation*pdf*color / pdf_val
  }
  if (P.raw) {
    P.raw[3 * (size_t)p] = C.x;
    P.raw[3 * (size_t)p + 1] = C.y;
    P.raw[3 * (size_t)p + 2] = C.z;
  }
  // de_nan (Raytracing_n.cpp:47-53)
  if (!(C.x == C.x)) C.x = 0;
  if (!(C.y == C.y)) C.y = 0;
  if (!(C.z == C.z)) C.z = 0;
  nts(&P.sample[3 * (size_t)p], C.x);
  nts(&P.sample[3 * (size_t)p + 1], C.y);
  nts(&P.sample[3 * (size_t)p + 2], C.z);
}

// emitted() of the hit's material toward the incoming ray (material.h:348-354):
// only diffuse_light emits, one-sided
SRR_D V3 hit_emitted(const SceneView& S, int mat, V3 rdir, V3 hpt, V3 nrm, float hu, float hv) {
  if (mat < 0) return v3(0.f);  // a null material* is UB in the reference: 0 here
  const DMat& M = S.mats[mat];
  if (M.kind == MAT_DIFFUSE_LIGHT && dot(nrm, rdir) < 0.0) return tex_value(S, M.tex, hu, hv, hpt);
  return v3(0.f);
}

// The pdf slot of a specular bounce's record: a signalling NaN, which no float
// arithmetic or conversion produces (their NaNs are quiet), so the path kernel's
// fold tells specular records from any diffuse pdf without a per-path bit mask.
constexpr uint32_t kSpecMark = 0x7f800001u;

// The scattering half of one color() bounce for family F (Raytracing_n.cpp:63-94,
// material.h): the next direction and time, and the bounce's record for the
// back-to-front fold: (attenuation * scattering_pdf, pdf) or, specular,
// (attenuation, kSpecMark) with `spec` set.
template <int F>
SRR_D void scatter(const SceneView& S, const DMat& M, V3 rdir, float rtime, V3 hpt, V3 nrm, float hu, float hv,
                   Rng& rng, float4& rec, bool& spec, V3& ndir, float& ntime, int* attempts = nullptr) {
  ntime = 0.0f;  // ray(a, b) defaults time to 0 (ray.h:10) for specular rays
  if (F == FAM_SPEC) {
    V3 atten;
    if (M.kind == MAT_METAL) {  // material.h:248-256
      V3 ud = unit_vector(rdir);
      V3 refl = ud - 2 * dot(ud, nrm) * nrm;
      ndir = refl + M.p[3] * random_in_unit_sphere(rng);
      atten = v3(M.p[0], M.p[1], M.p[2]);
    } else if (M.kind == MAT_DIELECTRIC) {  // material.h:285-324
      float ri = M.p[0];
      atten = v3(1.0f, 1.0f, 1.0f);
      V3 reflected = rdir - 2 * dot(rdir, nrm) * nrm;
      V3 outward;
      float ni_over_nt, cosine;
      if (dot(rdir, nrm) > 0) {
        outward = -nrm;
        ni_over_nt = ri;
        cosine = dot(rdir, nrm) / length(rdir);
      } else {
        outward = nrm;
        ni_over_nt = 1.0 / ri;
        cosine = -dot(rdir, nrm) / length(rdir);
      }
      V3 uv = unit_vector(rdir);  // refract (material.h:21-32)
      float dt = dot(uv, outward);
      float disc = 1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt);
      float reflect_prob;
      V3 refracted;
      if (disc > 0) {
        refracted = ni_over_nt * (uv - outward * dt) - outward * rsqrt_exact(disc);
        float r0 = (1 - ri) / (1 + ri);  // schlick (material.h:14-19), pow(float,int) in double
        r0 = r0 * r0;
        reflect_prob = r0 + (1 - r0) * ::pow((double)(1 - cosine), 5.0);
      } else {
        reflect_prob = 1.0;
      }
      float r01 = drand(rng);
      ndir = (r01 < reflect_prob) ? reflected : refracted;
    } else {  // isotropic (material.h:362-367)
      ndir = random_in_unit_sphere(rng);
      atten = tex_value(S, M.tex, hu, hv, hpt);
    }
    rec = make_float4(atten.x, atten.y, atten.z, __uint_as_float(kSpecMark));
    spec = true;
  } else {
    // lambertian / orennayar / beckmann: mixture(light, bsdf) (Raytracing_n.cpp:73-94)
    V3 atten = tex_value(S, M.tex, hu, hv, hpt);
    Bsdf f;
    f.kind = (F == FAM_BECK) ? (int)MAT_BECKMANN : M.kind;
    f.n = nrm;
    f.uvw = onb_from_w(nrm);
    f.A = M.p[0];
    f.B = M.p[1];
    f.dist.ax = M.p[0];
    f.dist.ay = M.p[1];
    f.beck_pdf = 0;
    bsdf_prepare<F == FAM_BECK>(f, rdir);
    float pdf_val = 0;
    if (S.n_lights > 0) {
      (void)drand(rng);  // mixture_pdf ctor (pdf.h:175)
      for (int guard = 0; pdf_val == 0 && guard < kMixtureGuard; ++guard) {
        if (attempts) ++*attempts;  // (diagnostics)
        if (drand(rng) < 0.5) ndir = lights_random(S, hpt, rng);
        else ndir = bsdf_generate<F == FAM_BECK>(f, rdir, rng);
        pdf_val = 0.5 * lights_pdf(S, hpt, ndir) + 0.5 * bsdf_value<F == FAM_BECK>(f, rdir, ndir);
      }
    } else {
      ndir = bsdf_generate<F == FAM_BECK>(f, rdir, rng);
      pdf_val = bsdf_value<F == FAM_BECK>(f, rdir, ndir);
    }
    float spdf = scattering_pdf<F == FAM_BECK>(f, nrm, rdir, ndir);
    V3 as = atten * spdf;
    rec = make_float4(as.x, as.y, as.z, pdf_val);
    spec = false;
    ntime = rtime;
  }
}

// One hit of family F (color(), Raytracing_n.cpp:55-106).  Returns true when the
// path continues with a new ray.
template <int F>
SRR_D bool shade_one(const SceneView& S, const PathState& P, int p, int max_depth) {
  float4 ro = ntl(&P.ray_o[p]), rdv = ntl(&P.ray_d[p]);
  V3 rdir = v3(rdv.x, rdv.y, rdv.z);
  int depth = ntl(&P.depth[p]);
  uint64_t spec = ntl(&P.spec[p]);
  if (P.rays) P.rays[p] += 1;
  const int mat = ntl(&P.hit_w[p]).w;
  if (F == FAM_TERM) {
    // miss -> vec3(0.0) (:104); no scatter (light) or depth limit -> emitted (:97-100)
    V3 emitted = v3(0.f);
    if (mat >= 0) {
      float4 hp = ntl(&P.hit_p[p]), hn = ntl(&P.hit_n[p]);
      emitted = hit_emitted(S, mat, rdir, v3(hp.x, hp.y, hp.z), v3(hn.x, hn.y, hn.z), hp.w, hn.w);
    }
    finish_path(P, p, emitted, depth, spec, max_depth);
    return false;
  }
  float4 hp = ntl(&P.hit_p[p]), hn = ntl(&P.hit_n[p]);
  V3 hpt = v3(hp.x, hp.y, hp.z), nrm = v3(hn.x, hn.y, hn.z);
  const DMat M = S.mats[mat];
  Rng rng{ntl(&P.lcg[p]), ntl(&P.pcg[p])};
  V3 ndir;
  float ntime;
  float4 rec;
  bool sp;
  scatter<F>(S, M, rdir, ro.w, hpt, nrm, hp.w, hn.w, rng, rec, sp, ndir, ntime);
  nts(&P.rec_a[(size_t)p * max_depth + depth], rec);
  if (sp) spec |= (1ull << depth);
  nts(&P.ray_o[p], make_float4(hpt.x, hpt.y, hpt.z, ntime));
  nts(&P.ray_d[p], make_float4(ndir.x, ndir.y, ndir.z, 0.f));
  nts(&P.lcg[p], rng.lcg);
  nts(&P.pcg[p], rng.pcg);
  nts(&P.depth[p], depth + 1);
  nts(&P.spec[p], spec);
  return true;
}

// ===================================================== path-resident engine
// One persistent kernel runs whole paths: each lane holds its path's ray, RNG
// streams, depth and specular mask in registers across bounces (trace over the
// LDS-staged world and the 4-wide BVH, hit record, material scatter), and when
// its path ends it folds the bounce records back to front exactly like the
// recursion returns, writes the sample and fetches the next (pixel, sample) from
// a global cursor (one wave-aggregated atomic per refill).  No path state goes
// through memory between bounces except the write-only bounce records.
// bounce records: plain stores keep the first bounces' records (a few MB per
// XCD) in L2 for the fold; nontemporal ones stream them to HBM
#ifndef SRR_REC_NT
#define SRR_REC_NT 0
#endif
#ifndef SRR_FOLD4
#define SRR_FOLD4 1  // the fold's record loads four at a time (A/B: -DSRR_FOLD4=0)
#endif
SRR_D void rec_store(float4* p, float4 v) {
  if (SRR_REC_NT) nts(p, v);
  else *p = v;
}
SRR_D float4 rec_load(const float4* p) { return SRR_REC_NT ? ntl(p) : *p; }

constexpr int kPathsBlock = 256;
constexpr unsigned long long kPoolChunk = 64;  // path indices a wave takes per cursor atomic

// Camera-ray ring (SRR_RAYRING, default on).  A lane whose path ended used to
// generate its next camera ray itself (pixel and sample from the path index,
// per-path seeds, Sobol point, lens disk, normalisation: a few hundred VALU
// instructions) while the wave's other lanes, still inside their paths, idled:
// about half the lanes refill per wave-iteration (C2 paths average 2.03 world
// rays), so the refill ran at ~50 % lane utilisation every iteration.  With the
// ring, the wave generates the camera rays of a whole 64-path chunk at once --
// lane k the ray of path chunk + k, every lane busy -- into its 64 LDS entries,
// and refilling lanes just read theirs: the chunk's rays cost one full-wave
// generation per ~2 iterations instead of a half-empty one per iteration.  Every
// path's ray is the same function of its index, so paths are unchanged.
#ifndef SRR_RAYRING
#define SRR_RAYRING 1
#endif
// diagnostics-only k_paths variants (phase timing, compressed nodes): `make diag`
#ifndef SRR_DIAG_VARIANTS
#define SRR_DIAG_VARIANTS 0
#endif
constexpr int kRingWords = 11;  // o.xyz, d.xyz, time, lcg (2 words), pcg (2 words)

// BS: lanes per block.  256 (4 blocks per CU) or 1,024 (one block per CU, the same
// 4 waves per SIMD): one LDS allocation per CU, whose 160 KB then cache
// kPathsLdsNodesBig BVH4 nodes (the top ~5 levels) instead of 96.
// 8 KB world + 8 B x kStack x 1,024 lanes of stacks + the camera-ray rings (44 B
// per lane) + the node cache <= 160 KB (344 nodes at kStack 8)
constexpr int kPathsLdsNodesBig =
    (160 * 1024 - 8192 - 8 * kPathsLdsStack * 1024 - 1024 - (SRR_RAYRING ? 4 * kRingWords * 1024 : 0)) / 128;
// 256-lane blocks (4 per CU, <= 40 KB each) of the LDS-world variant: the ring
// displaces the node cache.  These blocks serve mesh-free scenes by default
// (paths_block_lanes); mesh scenes reach them only with SRR_BIGBLOCK=0 (an A/B
// knob).  The two other 256-lane variants that serve mesh scenes keep the whole
// cache: the global-world one (world tables beyond kWorldLdsBytes) has the 8 KB
// of the LDS world to spare (16 KB stacks + 11 KB ring + 12 KB nodes), and the
// quad-cooperative one (SRR_QUAD) runs without the ring.
constexpr int kPathsLdsNodesSmall = SRR_RAYRING ? 8 : kPathsLdsNodes;

// The camera ray of path index idx of the window (pixel-major: idx = lp * spp_w + s)
// with its RNG streams, as k_paths' refill needs it.
SRR_D void path_camera_ray(const SceneView& S, const PathWork& W, uint32_t idx, Ray& r, Rng& rng) {
  const uint32_t lp = udiv31(idx, W.div_spp), s = idx - lp * (uint32_t)W.spp_w;
  if ((int)lp >= W.npix || (int)s >= W.spp_w) atomicOr(W.err, 1);
  const int pix = W.pixels ? W.pixels[lp] : lp;
  V3 o, d;
  float tm;
  double sx, sy;
  sobol2_point((uint32_t)(W.s_base + (int)s), sx, sy);  // = W.sobol[2 s], W.sobol[2 s + 1]
  camera_ray(S, pix, W.s_base + s, sx, sy, W.nx, W.ny, W.base_seed, o, d, tm, rng, &W.div_nx);
  r = Ray{o, d, tm};
}

template <int BS>
SRR_D void ring_put(lds_ptr<float> e, const Ray& r, const Rng& rng) {  // e: the entry's word 0
  e[0] = r.o.x;
  e[BS] = r.o.y;
  e[2 * BS] = r.o.z;
  e[3 * BS] = r.d.x;
  e[4 * BS] = r.d.y;
  e[5 * BS] = r.d.z;
  e[6 * BS] = r.tm;
  e[7 * BS] = __uint_as_float((uint32_t)rng.lcg);
  e[8 * BS] = __uint_as_float((uint32_t)(rng.lcg >> 32));
  e[9 * BS] = __uint_as_float((uint32_t)rng.pcg);
  e[10 * BS] = __uint_as_float((uint32_t)(rng.pcg >> 32));
}

template <int BS>
SRR_D void ring_get(lds_ptr<const float> e, Ray& r, Rng& rng) {
  r = Ray{v3(e[0], e[BS], e[2 * BS]), v3(e[3 * BS], e[4 * BS], e[5 * BS]), e[6 * BS]};
  rng.lcg = (uint64_t)__float_as_uint(e[7 * BS]) | ((uint64_t)__float_as_uint(e[8 * BS]) << 32);
  rng.pcg = (uint64_t)__float_as_uint(e[9 * BS]) | ((uint64_t)__float_as_uint(e[10 * BS]) << 32);
}

// k_paths' arguments, read through the kernel-argument segment pointer laundered
// by an empty asm (paths_args): the compiler can no longer prove two reads of a
// field equal, so each phase of the path loop (refill, world hit, record and
// scatter, mixture, fold) loads the fields it uses with scalar loads at its start
// and they die at its end.  With the arguments as one by-value SceneView /
// PathWork, every table pointer of the scene and the window (~40 64-bit values)
// stayed live in SGPRs across the whole loop, and 114-137 of them spilled to VGPR
// lanes: each reload a v_readlane on the VALU, and in the 128-VGPR ALLFAM / MEDIA
// variants those VGPRs spilled on to scratch memory.
struct PathsArgs {
  SceneView S;
  PathWork W;
};
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
using kptr = const __attribute__((address_space(4))) T*;
SRR_D kptr<PathsArgs> paths_args() {
  kptr<PathsArgs> p = (kptr<PathsArgs>)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
#else  // (the host pass parses kernel bodies but never compiles them)
SRR_D const PathsArgs* paths_args() { return nullptr; }
#endif

// SP: mesh walks may suspend (TR_SUSP; launched when PathWork::walk_q > 0): the 1,024-lane
// variants and the diagnostics (TIMED) one are built both ways
template <bool MEDIA, bool ALLFAM, int MINB, bool TIMED = false, bool WL = true, bool QUAD = false, bool CQ = false,
          int BS = kPathsBlock, bool SP = false>
#ifdef SRR_NUM_VGPR  // register-pressure study builds only: cap k_paths' VGPRs
#define SRR_PATHS_VGPR_ATTR __attribute__((amdgpu_num_vgpr(SRR_NUM_VGPR)))
#else
#define SRR_PATHS_VGPR_ATTR
#endif
__global__ void __launch_bounds__(BS, MINB) SRR_PATHS_VGPR_ATTR k_paths(PathsArgs A) {
  static_assert(BS == kPathsBlock || BS == 1024, "block size");
  (void)A;  // read through paths_args()
  // TIMED (diagnostics): per-wave cycles in refill / world hit (mesh part) / record+scatter / fold
  uint64_t tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // TIMED family diagnostics -> W.counters[16..35]: ticks in the BECK / SPEC / DIFF-set-up
  // branches of the per-lane scatter, iterations each branch ran, lanes it ran for;
  // lanes in a path; the longest walk's node steps, all lanes' steps, walking lanes (wave time
  // in the mesh is tp[2])
  uint64_t tf[20] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t it = 0;
  // WL: world tables staged in LDS (they fit in kWorldLdsBytes); otherwise read
  // from global memory (large object lists, e.g. random_scene's ~490 spheres)
  // QUAD: meshes traced by mesh_hit4_quad (large BVHs, SceneView::quad_trace)
  // (per-lane walks over 128-B nodes may suspend: TR_SUSP, PathWork::walk_q)
  constexpr int TR = TR_BVH4_PRUNE | (WL ? TR_WL : 0) | (QUAD ? TR_QUAD : 0) | (CQ ? TR_Q : 0) | (BS == 1024 ? TR_BIG : 0) |
                     ((SP && !QUAD && !CQ) ? TR_SUSP : 0);
  __shared__ uint4 s_world[WL ? kWorldLdsBytes / 16 : 1];
  // the scene as a phase reads it: scalar loads of the fields it uses, the world
  // tables re-pointed into LDS (WL)
  const auto view = [&]() {
    SceneView S = paths_args()->S;
    if constexpr (WL) {
      const char* b = (const char*)s_world;
      S.objs = (const DObj*)(b + S.world_off[0]);
      S.xforms = (const DXform*)(b + S.world_off[1]);
      S.spheres = (const DSphere*)(b + S.world_off[2]);
      S.rects = (const DRect*)(b + S.world_off[3]);
      S.stris = (const DStandaloneTri*)(b + S.world_off[4]);
      S.meshes = (const DMesh*)(b + S.world_off[5]);
      S.media = (const DMedium*)(b + S.world_off[6]);
      S.mats = (const DMat*)(b + S.world_off[7]);
      S.texs = (const DTex*)(b + S.world_off[8]);
      S.lights = (const DLight*)(b + S.world_off[9]);
    }
    return S;
  };
  const auto work = []() { return PathWork(paths_args()->W); };
  __shared__ int s_node[kStack * BS];
  __shared__ float s_t[kStack * BS];
  constexpr bool RING = SRR_RAYRING && !QUAD;
  constexpr int kNodesLds = BS == 1024 ? kPathsLdsNodesBig : ((WL && RING) ? kPathsLdsNodesSmall : kPathsLdsNodes);
  __shared__ float4 s_n4[kNodesLds * 8];
  // RING: the wave's camera-ray ring, SoA [kRingWords][BS]; the wave's 64 entries
  // are its own lanes' columns (entry e of wave v at column 64 v + e)
  __shared__ float s_ring[RING ? kRingWords * BS : 1];
  const lds_ptr<float> ringw = to_lds(s_ring + (RING ? (threadIdx.x & ~63u) : 0));
  uint32_t ring_base = 0;  // path index of the ring's entry 0 (wave-uniform)
  const uint32_t n_paths = (uint32_t)paths_args()->W.n_paths;
  const uint64_t t_start = paths_args()->W.wave_times ? __builtin_amdgcn_s_memrealtime() : 0;
  {
    const SceneView S0 = paths_args()->S;
    if constexpr (WL)
      for (int i = threadIdx.x; i < S0.world_words; i += blockDim.x) s_world[i] = S0.world_blob[i];
    // (CQ: the same LDS bytes hold twice as many 64-B nodes)
    const int n_lds_nodes = CQ ? min(S0.node4_total, 2 * kNodesLds) : min(S0.node4_total, kNodesLds);
    if (CQ)
      for (int i = threadIdx.x; i < n_lds_nodes * 4; i += blockDim.x) s_n4[i] = S0.node4q[i];
    else
      for (int i = threadIdx.x; i < n_lds_nodes * 8; i += blockDim.x) s_n4[i] = S0.node4[i];
  }
  __syncthreads();
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  // this lane's record column W.rec + slot, re-derived at each use: hoisted out of
  // the loop as a 64-bit address it was live (and spilled) across every phase
  const auto rec_at = [&](const PathWork& W, int k) -> float4* {
    int s = slot;
    asm volatile("" : "+v"(s));
    return W.rec + ((size_t)k * W.lanes + s);
  };
  int g = -1;  // path of this lane (a window numbers its paths below 2^31), -1 idle
  // the wave's unissued path indices [pool, pool_end): wave-uniform (scalar)
  uint32_t pool = 0, pool_end = 0;
  uint32_t nxt_lane0 = 0;  // lane 0: base of the armed next chunk
  bool nxt_armed = false;
  // the armed chunk's base, read once the world hit is done (nxt_ready): by then
  // the atomic has long returned, and no store of this iteration is yet in flight
  // (the wave's vector-memory counter is in issue order, so reading the atomic's
  // result right after the fold's sample stores would wait for those)
  uint32_t nxt_base = 0;
  bool nxt_ready = false;
  Ray r{};
  Rng rng{};
  int depth = 0;
  int walking = 0;  // (TR_SUSP) this lane's world hit is a suspended mesh walk
  uint32_t nrays = 0;
  // this lane's events, two counts in one register (each loop-carried VGPR is dear in the
  // ALLFAM variants): resampling loops stopped by kMixtureGuard in bits 0-11 (each costs
  // 100,000 attempts: a lane never reaches 4,096) and suspended mesh walks from bit 12
  uint32_t n_events = 0;
  constexpr uint32_t kCapped = 1, kSuspended = 1u << 12;
  uint32_t n_iter = 0, max_rounds = 0;  // wave-iterations, most mixture rounds (SRR_WAVE_TIMES diagnostics)
  for (;;) {
    ++n_iter;
    uint64_t tq = TIMED ? __builtin_amdgcn_s_memtime() : 0;
    // refill lanes whose path ended, from the wave's pool of path indices; the
    // pool is re-armed one chunk ahead (an atomic whose result is first read an
    // iteration later, so its latency hides behind that iteration's work)
    const bool need = g < 0;
    const uint64_t nm = __ballot(need);
    if (nm && pool < n_paths) {
      const SceneView S = view();
      const PathWork W = work();
      const uint32_t cnt = __popcll(nm);
      const uint32_t rank = __popcll(nm & ((1ull << lane_id()) - 1));
      const uint32_t avail = pool_end - pool;
      uint32_t idx = 0;
      if (RING) {
        // lanes whose path is in the ring's chunk take it first (before the chunk is replaced)
        if (need && rank < avail) {
          const uint32_t i0 = pool + rank;
          if (i0 < n_paths) {
            g = (int)i0;
            ring_get<BS>(ringw + (i0 - ring_base), r, rng);
            depth = 0;
          }
        }
        if (avail >= cnt) {
          pool += cnt;
        } else {
          uint32_t nb;
          if (nxt_armed) {
            nb = nxt_ready ? nxt_base : __builtin_amdgcn_readfirstlane(nxt_lane0);
            nxt_armed = false;
            nxt_ready = false;
          } else {
            uint32_t b = 0;
            if (lane_id() == 0) b = (uint32_t)atomicAdd(W.cursor, (unsigned long long)kPoolChunk);
            nb = __builtin_amdgcn_readfirstlane(b);
          }
          // the next chunk's camera rays, one per lane, every lane of the wave
          const uint32_t gi = nb + (uint32_t)lane_id();
          if (gi < n_paths) {
            Ray gr;
            Rng grng;
            path_camera_ray(S, W, gi, gr, grng);
            ring_put<BS>(ringw + lane_id(), gr, grng);
          }
          // (one wave writes and reads these entries: its LDS operations run in order;
          // the fence keeps the compiler from moving the reads above the writes)
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          ring_base = nb;
          if (need && rank >= avail) {
            const uint32_t i1 = nb + (rank - avail);
            if (i1 < n_paths) {
              g = (int)i1;
              ring_get<BS>(ringw + (i1 - nb), r, rng);
              depth = 0;
            }
          }
          pool = nb + (cnt - avail);
          pool_end = nb + (uint32_t)kPoolChunk;
        }
      } else if (avail >= cnt) {
        idx = pool + rank;
        pool += cnt;
      } else {
        uint32_t nb;
        if (nxt_armed) {
          nb = nxt_ready ? nxt_base : __builtin_amdgcn_readfirstlane(nxt_lane0);
          nxt_armed = false;
          nxt_ready = false;
        } else {
          uint32_t b = 0;
          if (lane_id() == 0) b = (uint32_t)atomicAdd(W.cursor, (unsigned long long)kPoolChunk);
          nb = __builtin_amdgcn_readfirstlane(b);
        }
        idx = rank < avail ? pool + rank : nb + (rank - avail);
        pool = nb + (cnt - avail);
        pool_end = nb + (uint32_t)kPoolChunk;
      }
      if (!RING && need && idx < n_paths) {
        g = (int)idx;
        path_camera_ray(S, W, idx, r, rng);
        depth = 0;
      }
    }
    if (!nxt_armed && pool_end < n_paths) {  // arm the next chunk
      if (lane_id() == 0) nxt_lane0 = (uint32_t)atomicAdd(paths_args()->W.cursor, (unsigned long long)kPoolChunk);
      nxt_armed = true;
    }
    if (__ballot(g >= 0) == 0) break;
    if (TIMED) tf[9] += __popcll(__ballot(g >= 0));
    if (TIMED) {
      __builtin_amdgcn_s_waitcnt(0);
      const uint64_t t = __builtin_amdgcn_s_memtime();
      tp[0] += t - tq;
      tq = t;
      ++it;
    }
    bool done = false;
    V3 C = v3(0.f);
    // a diffuse bounce with lights: set up here, its mixture loop runs below with
    // the whole wave (coop_mixture), then its record is written
    bool diff = false, pend = false;
    int natt = 0;  // (TIMED: mixture attempts of this lane's Beckmann scatter)
    uint64_t fam_dt[3] = {0, 0, 0};  // (TIMED: this lane's ticks in the BECK / SPEC / DIFF-set-up branch)
    DiffSetup ds{};
    V3 d_atten = v3(0.f), d_n = v3(0.f), d_dir = v3(0.f);
    float d_pdf = 0;
    int d_tries = 0;
    bool d_dead = false;
    WorldHit w{-1, -1, 0};
    if (g >= 0) {
      const SceneView S = view();
      const PathWork W = work();
      TraceCtx cx{nullptr, to_lds(s_node + threadIdx.x), to_lds(s_t + threadIdx.x)};
      cx.lds_nodes = (const __attribute__((address_space(3))) f32x4*)to_lds(s_n4);
      cx.lds_count = CQ ? min(S.node4_total, 2 * kNodesLds) : min(S.node4_total, kNodesLds);
      // (clamped: a host compiled with another SRR_KSTACK must not index past the
      // kernel's kStack LDS entries per lane)
      cx.st_cap = min(W.stack_cap, kStack);
      cx.ovf = W.counters + 11;
      cx.gst = W.gstack;
      cx.gst_cap = W.gstack ? W.gstack_cap : 0;
      cx.gst_stride = W.lanes;
      cx.slot = slot;
      if constexpr ((TR & TR_SUSP) != 0) {
        // suspend walks once at most walk_q / 64 of the wave's lanes in a path still walk
        // (the save area follows the global stack extension: none without it)
        // (walk_q 0: threshold 0, and a walk only stops when its lanes all finished)
        cx.walk_thr = vreg((int)((__popcll(__ballot(true)) * (uint32_t)paths_args()->W.walk_q) >> 6));
        cx.resume = walking;
        cx.susp = vreg(0);
      }
#ifdef SRR_SLOW_RAYS
      const uint64_t t_w0 = __builtin_amdgcn_s_memrealtime();
      cx.last_steps = 0;
      const Ray r_in = r;
#endif
      w = world_hit<MEDIA, TIMED ? (TR_BVH4_TIMED | (WL ? TR_WL : 0) | (SP ? TR_SUSP : 0)) : TR>(S, r, rng, cx);
      if constexpr ((TR & TR_SUSP) != 0) {
        walking = cx.susp;  // (its record, scatter and fold wait for the walk's end)
        if (walking) {
          w.obj = -1;
          n_events += kSuspended;
        }
      }
#ifdef SRR_SLOW_RAYS
      // diagnostics build: every lane of a world hit slower than SRR_SLOW_RAYS
      // ticks (100 MHz) records its ray: g, depth, o, d, time, ticks, steps, hit
      const uint64_t t_w = __builtin_amdgcn_s_memrealtime() - t_w0;
      if ((t_w > (uint64_t)SRR_SLOW_RAYS || (cx.last_steps & (1 << 28))) && W.slow_rays) {
        const unsigned q = atomicAdd(W.slow_count, 1u);
        if (q < 65536u) {
          float* e = W.slow_rays + 16 * (size_t)q;
          e[0] = __int_as_float(g);
          e[1] = __int_as_float(depth);
          e[2] = r_in.o.x; e[3] = r_in.o.y; e[4] = r_in.o.z;
          e[5] = r_in.d.x; e[6] = r_in.d.y; e[7] = r_in.d.z;
          e[8] = r_in.tm;
          e[9] = __int_as_float((int)t_w);
          e[10] = __int_as_float(cx.last_steps);
          e[11] = __int_as_float(w.obj);
          e[12] = __int_as_float(w.prim);
          e[13] = w.t;
          e[14] = __int_as_float(slot);
          e[15] = __int_as_float((int)(t_w0 & 0x7fffffff));
        }
      }
#endif
      if (TIMED) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        tp[1] += t - tq - cx.mesh_cycles;
        tp[2] += cx.mesh_cycles;
        tf[10] += cx.mesh_steps;
        tf[11] += cx.mesh_lane_steps;
        tf[12] += cx.mesh_walkers;
        tf[13] += cx.leaf_cycles;
        tf[14] += cx.leaf_passes;
        tf[15] += cx.step_parts[0];
        tf[16] += cx.step_parts[1];
        tf[17] += cx.step_parts[2];
        tq = t;
      }
      done = !walking;
    }
    if (nxt_armed && !nxt_ready) {  // (uniform: every lane of the wave is here)
      nxt_base = __builtin_amdgcn_readfirstlane(nxt_lane0);
      nxt_ready = true;
    }
    if (g >= 0) {
      if (w.obj >= 0) {
        const SceneView S = view();
        const PathWork W = work();
        const HitRec h = world_record<TR>(S, r, w);
        const int kind = h.mat >= 0 ? S.mats[h.mat].kind : -1;
        if (TIMED) {
          __builtin_amdgcn_s_waitcnt(0);
          const uint64_t t = __builtin_amdgcn_s_memtime();
          tp[5] += t - tq;
          tq = t;
        }
        const int fam = family_of(h.mat, kind, depth, W.max_depth);
        if (TIMED) {
          const uint64_t mb = __ballot(fam == FAM_BECK), ms = __ballot(fam == FAM_SPEC),
                         md = __ballot(fam == FAM_DIFF && S.n_lights > 0);
          tf[3] += mb != 0; tf[4] += ms != 0; tf[5] += md != 0;
          tf[6] += __popcll(mb); tf[7] += __popcll(ms); tf[8] += __popcll(md);
        }
        if (fam == FAM_TERM) {
          C = hit_emitted(S, h.mat, r.d, h.p, h.n, h.u, h.v);
        } else if ((!ALLFAM || fam == FAM_DIFF) && S.n_lights > 0) {
          // scatter<FAM_DIFF> up to its resampling loop (Raytracing_n.cpp:73-75)
          const DMat M = S.mats[h.mat];
          d_atten = tex_value(S, M.tex, h.u, h.v, h.p);
          Bsdf f;
          f.kind = M.kind;
          f.n = h.n;
          f.uvw = onb_from_w(h.n);
          f.A = M.p[0];
          f.B = M.p[1];
          bsdf_prepare<false>(f, r.d);
          ds = diff_setup(f, h.p);
          if (SRR_MIXTURE_SKIP) d_dead = bsdf_dead(S, f, h.p);
          (void)drand(rng);  // mixture_pdf ctor (pdf.h:175)
          d_n = h.n;
          diff = pend = true;
          done = false;
          if (TIMED) fam_dt[2] = __builtin_amdgcn_s_memtime() - tq;
        } else {
          const DMat M = S.mats[h.mat];
          float4 rec;
          bool sp;
          V3 nd;
          float nt;
          const uint64_t tb = TIMED ? __builtin_amdgcn_s_memtime() : 0;
          if (!ALLFAM || fam == FAM_DIFF) scatter<FAM_DIFF>(S, M, r.d, r.tm, h.p, h.n, h.u, h.v, rng, rec, sp, nd, nt);
          else if (fam == FAM_BECK) {
            scatter<FAM_BECK>(S, M, r.d, r.tm, h.p, h.n, h.u, h.v, rng, rec, sp, nd, nt, TIMED ? &natt : nullptr);
            if (TIMED) fam_dt[0] = __builtin_amdgcn_s_memtime() - tb;
          } else {
            scatter<FAM_SPEC>(S, M, r.d, r.tm, h.p, h.n, h.u, h.v, rng, rec, sp, nd, nt);
            if (TIMED) fam_dt[1] = __builtin_amdgcn_s_memtime() - tb;
          }
          if (depth >= W.max_depth || slot >= W.lanes) atomicOr(W.err, 2);
          else rec_store(rec_at(W, depth), rec);
          if (!sp && S.n_lights > 0 && rec.w == 0) n_events += kCapped;  // the loop reached kMixtureGuard
          r = Ray{h.p, nd, nt};
          ++depth;
          done = false;
        }
      }
    }
    if (TIMED) {  // Beckmann mixture attempts: the wave's sum and its slowest lane's
      int sum = natt, mx = natt;
      for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        mx = max(mx, __shfl_xor(mx, o));
      }
      tf[18] += sum;
      tf[19] += mx;
      // the family branches' wave time this iteration: the longest of their lanes' stamps
      // (lanes of one branch run it together; lanes outside it stamped 0)
      for (int q = 0; q < 3; ++q) {
        uint64_t m = fam_dt[q];
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint64_t)__shfl_xor((unsigned long long)m, o));
        tf[q] += m;
      }
    }
    if (__ballot(pend)) {
      const SceneView S = view();
      const uint64_t tc = TIMED ? __builtin_amdgcn_s_memtime() : 0;
      // SRR_MIXTURE_SKIP 1: per-lane loops passing over dead draws; 2: one such
      // round, then the wave-cooperative loop for what is left; 0: cooperative only
      int rounds = 0;
      if (SRR_MIXTURE_SKIP == 1) {
        rounds = skip_mixture(S, ds, d_dead, pend, d_tries, rng.lcg, d_dir, d_pdf);
      } else {
        if (SRR_MIXTURE_SKIP == 2) rounds = skip_mixture(S, ds, d_dead, pend, d_tries, rng.lcg, d_dir, d_pdf, 1);
        if (__ballot(pend)) rounds += coop_mixture(S, ds, pend, d_tries, rng.lcg, d_dir, d_pdf, paths_args()->W.deep_tries);
      }
      if (TIMED) {
        tp[6] += __builtin_amdgcn_s_memtime() - tc;
        tp[7] += rounds;
      }
      max_rounds = max(max_rounds, (uint32_t)rounds);
    }
    if (diff) {  // the rest of scatter<FAM_DIFF>: scattering_pdf and the record
      const PathWork W = work();
      if (d_pdf == 0) n_events += kCapped;  // the loop reached kMixtureGuard
      float c = dot(d_n, unit_vector(d_dir));  // material.h:100-105, 134-138
      if (c < 0) c = 0;
      const V3 as = d_atten * (c / kPi);
      if (depth >= W.max_depth || slot >= W.lanes) atomicOr(W.err, 2);
      else rec_store(rec_at(W, depth), make_float4(as.x, as.y, as.z, d_pdf));
      r = Ray{ds.p, d_dir, r.tm};
      ++depth;
    }
    if (g >= 0) {
      const PathWork W = work();
      if (TIMED) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        tp[3] += t - tq;
        tq = t;
      }
      if (done && (g >= W.n_paths || depth > W.max_depth)) {
        atomicOr(W.err, 4);
        g = -1;
        done = false;
      }
      if (done) {
        // fold the bounces back to front (Raytracing_n.cpp:69, :94), as finish_path
#if SRR_FOLD4
        // the last four records' loads issued together (one L2 round trip, not one
        // per bounce), then folded in the same order
        int k = depth - 1;
        for (; k >= 0; k -= 4) {
          float4 a[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = k - j >= 0 ? rec_load(rec_at(W, k - j)) : make_float4(0, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (k - j < 0) break;
            const V3 av = v3(a[j].x, a[j].y, a[j].z);
            if (__float_as_uint(a[j].w) == kSpecMark) C = av * C;  // specular: attenuation * color
            else C = v3(0.f) + (av * C) / a[j].w;
          }
        }
#else
        for (int k = depth - 1; k >= 0; --k) {
          const float4 a = rec_load(rec_at(W, k));
          const V3 av = v3(a.x, a.y, a.z);
          if (__float_as_uint(a.w) == kSpecMark) C = av * C;  // specular: attenuation * color
          else C = v3(0.f) + (av * C) / a.w;
        }
#endif
        if (W.raw) {  // kept paths: [pixel][sample of the frame]
          const size_t kq = (size_t)(g / W.spp_w) * W.keep_spp + W.keep_s0 + (size_t)(g % W.spp_w);
          W.raw[3 * kq] = C.x;
          W.raw[3 * kq + 1] = C.y;
          W.raw[3 * kq + 2] = C.z;
          W.rays[kq] = (uint8_t)(depth + 1);  // world rays of the path
        }
        if (!(C.x == C.x)) C.x = 0;  // de_nan (Raytracing_n.cpp:47-53)
        if (!(C.y == C.y)) C.y = 0;
        if (!(C.z == C.z)) C.z = 0;
        nts(&W.sample[3 * (size_t)g], C.x);
        nts(&W.sample[3 * (size_t)g + 1], C.y);
        nts(&W.sample[3 * (size_t)g + 2], C.z);
        nrays += depth + 1;
        g = -1;
      }
      if (TIMED) tp[4] += __builtin_amdgcn_s_memtime() - tq;
    }
  }
  const PathWork W = work();
  if (TIMED && lane_id() == 0) {  // per-wave totals -> W.counters[4..9]
    for (int q = 0; q < 5; ++q) atomicAdd(W.counters + 4 + q, (unsigned long long)tp[q]);
    atomicAdd(W.counters + 9, (unsigned long long)it);
    atomicAdd(W.counters + 10, (unsigned long long)tp[5]);
    atomicAdd(W.counters + 13, (unsigned long long)tp[6]);
    atomicAdd(W.counters + 14, (unsigned long long)tp[7]);
    for (int q = 0; q < 20; ++q) atomicAdd(W.counters + 16 + q, (unsigned long long)tf[q]);
  }

  unsigned long long tot = nrays;
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  if (lane_id() == 0 && tot) atomicAdd(W.counters, tot);
  if (__ballot(n_events != 0)) {
    unsigned long long cap = n_events & (kSuspended - 1), su = n_events / kSuspended;
    for (int o = 32; o > 0; o >>= 1) {
      cap += __shfl_xor(cap, o);
      su += __shfl_xor(su, o);
    }
    if (lane_id() == 0) {
      if (cap) atomicAdd(W.counters + 15, cap);
      if (su) atomicAdd(W.counters + 36, su);
    }
  }
  if (W.wave_times && lane_id() == 0) {  // diagnostics: start, exit, world rays, wave-iterations
    const size_t wv = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) / 64;
    W.wave_times[4 * wv] = t_start;
    W.wave_times[4 * wv + 1] = __builtin_amdgcn_s_memrealtime();
    W.wave_times[4 * wv + 2] = tot;
    W.wave_times[4 * wv + 3] = n_iter | ((unsigned long long)max_rounds << 32);
  }
}

// acc[pixel] += the window's samples in sample order (the sum order of
// k_accumulate, Raytracing_n.cpp:841).  Samples are [pixel][sample]; a block
// stages 256 pixels x 16 samples through LDS with coalesced loads, then each
// thread adds its own pixel's samples in order.
constexpr int kAccChunk = 16;
// init: the sums start from 0 (the frame's first window; no memset of acc).
// out (the frame's last window, else nullptr): also writes the pixel's output --
// the mean sum * (float)(1.0 / ns) of k_finish, or (scale_ns == 0) the raw sums.
struct AccOut {
  float* out;
  int scale_ns;
};
SRR_D void acc_write(float* acc, AccOut o, size_t a, float cx, float cy, float cz) {
  acc[a] = cx;
  acc[a + 1] = cy;
  acc[a + 2] = cz;
  if (o.out) {
    if (o.scale_ns) {
      const float k = 1.0 / (float)o.scale_ns;  // k_finish
      o.out[a] = cx * k;
      o.out[a + 1] = cy * k;
      o.out[a + 2] = cz * k;
    } else {
      o.out[a] = cx;
      o.out[a + 1] = cy;
      o.out[a + 2] = cz;
    }
  }
}

__global__ void __launch_bounds__(256) k_accumulate_window(const float* sample, int npix, int spp_w, float* acc,
                                                           int init, AccOut o) {
  __shared__ float tile[256 * (3 * kAccChunk + 1)];
  const int p0 = blockIdx.x * 256;
  const int lp = p0 + threadIdx.x;
  const int np = min(256, npix - p0);
  float cx = 0, cy = 0, cz = 0;
  if (lp < npix && !init) {
    cx = acc[3 * (size_t)lp];
    cy = acc[3 * (size_t)lp + 1];
    cz = acc[3 * (size_t)lp + 2];
  }
  for (int s0 = 0; s0 < spp_w; s0 += kAccChunk) {
    const int n = min(kAccChunk, spp_w - s0), row = 3 * n;
    for (int i = threadIdx.x; i < np * row; i += 256) {
      const int px = i / row, f = i - px * row;
      tile[px * (3 * kAccChunk + 1) + f] = ntl(&sample[((size_t)(p0 + px) * spp_w + s0) * 3 + f]);
    }
    __syncthreads();
    if (lp < npix) {
      const float* t = &tile[threadIdx.x * (3 * kAccChunk + 1)];
      for (int k = 0; k < n; ++k) {
        cx += t[3 * k];
        cy += t[3 * k + 1];
        cz += t[3 * k + 2];
      }
    }
    __syncthreads();
  }
  if (lp >= npix) return;
  acc_write(acc, o, 3 * (size_t)lp, cx, cy, cz);
}

// The same sums with 16-byte loads, for windows of a multiple of 4 samples: a pixel's
// row of 3 x spp_w floats is then 16-byte aligned and its chunk of 16 samples is 12
// contiguous float4, so a block fetches its 256 x 16 samples with 12 float4 loads per
// thread (no per-element division); a window's last 4, 8 or 12 samples (spp_w % 16:
// the 1080p windows are 344 samples) go through the same tile as one shorter chunk.
__global__ void __launch_bounds__(256) k_accumulate_window16(const float4* sample4, int npix, int spp_w, float* acc,
                                                             int init, AccOut o) {
  __shared__ float tile[256 * (3 * kAccChunk + 1)];
  constexpr int kQ = 3 * kAccChunk / 4;  // float4 per pixel chunk
  const int p0 = blockIdx.x * 256;
  const int lp = p0 + threadIdx.x;
  const int np = min(256, npix - p0);
  const int s_full = spp_w - spp_w % kAccChunk;  // samples in whole chunks
  float cx = 0, cy = 0, cz = 0;
  if (lp < npix && !init) {
    cx = acc[3 * (size_t)lp];
    cy = acc[3 * (size_t)lp + 1];
    cz = acc[3 * (size_t)lp + 2];
  }
  if (np == 256) {
    // full block: the 12 loads of chunk s0 + 16 are in flight while the block
    // sums chunk s0 out of LDS (same per-pixel order of additions)
    float4 v[kQ];
    const float4* base = sample4 + (size_t)p0 * spp_w * 3 / 4;
    auto fetch = [&](int s0) {
#pragma unroll
      for (int j = 0; j < kQ; ++j) {
        const int i = threadIdx.x + 256 * j, px = i / kQ, f4 = i - px * kQ;
        v[j] = ntl(&base[((size_t)px * spp_w + s0) * 3 / 4 + f4]);
      }
    };
    if (s_full > 0) fetch(0);
    for (int s0 = 0; s0 < s_full; s0 += kAccChunk) {
#pragma unroll
      for (int j = 0; j < kQ; ++j) {
        const int i = threadIdx.x + 256 * j, px = i / kQ, f4 = i - px * kQ;
        float* d = &tile[px * (3 * kAccChunk + 1) + 4 * f4];
        d[0] = v[j].x;
        d[1] = v[j].y;
        d[2] = v[j].z;
        d[3] = v[j].w;
      }
      __syncthreads();
      if (s0 + kAccChunk < s_full) fetch(s0 + kAccChunk);
      const float* t = &tile[threadIdx.x * (3 * kAccChunk + 1)];
#pragma unroll
      for (int k = 0; k < kAccChunk; ++k) {
        cx += t[3 * k];
        cy += t[3 * k + 1];
        cz += t[3 * k + 2];
      }
      __syncthreads();
    }
  } else {
    for (int s0 = 0; s0 < s_full; s0 += kAccChunk) {
      for (int i = threadIdx.x; i < np * kQ; i += 256) {
        const int px = i / kQ, f4 = i - px * kQ;
        const float4 v = ntl(&sample4[((size_t)(p0 + px) * spp_w + s0) * 3 / 4 + f4]);
        float* d = &tile[px * (3 * kAccChunk + 1) + 4 * f4];
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
      }
      __syncthreads();
      if (lp < npix) {
        const float* t = &tile[threadIdx.x * (3 * kAccChunk + 1)];
#pragma unroll
        for (int k = 0; k < kAccChunk; ++k) {
          cx += t[3 * k];
          cy += t[3 * k + 1];
          cz += t[3 * k + 2];
        }
      }
      __syncthreads();
    }
  }
  if (s_full < spp_w) {  // the last n = 4, 8 or 12 samples: 3n / 4 float4 per pixel
    const int n = spp_w - s_full, qn = 3 * n / 4;
    for (int i = threadIdx.x; i < np * qn; i += 256) {
      const int px = i / qn, f4 = i - px * qn;
      const float4 v = ntl(&sample4[((size_t)(p0 + px) * spp_w + s_full) * 3 / 4 + f4]);
      float* d = &tile[px * (3 * kAccChunk + 1) + 4 * f4];
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    __syncthreads();
    if (lp < npix) {
      const float* t = &tile[threadIdx.x * (3 * kAccChunk + 1)];
      for (int k = 0; k < n; ++k) {
        cx += t[3 * k];
        cy += t[3 * k + 1];
        cz += t[3 * k + 2];
      }
    }
  }
  if (lp >= npix) return;
  acc_write(acc, o, 3 * (size_t)lp, cx, cy, cz);
}

constexpr int kMaxRegions = 8;

// Grid-stride over family F's list (sized on the device: no host readback);
// survivors are compacted into `next` with one atomic per wave.
template <int F>
__global__ void __launch_bounds__(256) k_shade(SceneView S, PathState P, const int* lists, int list_cap,
                                               const int* fam_count, int* next, int* next_count, int* region_alive,
                                               int region_size, int max_depth) {
  __shared__ int hist[kMaxRegions];
  if (threadIdx.x < kMaxRegions) hist[threadIdx.x] = 0;
  __syncthreads();
  const int* list = lists + (size_t)F * list_cap;
  const int n = fam_count[F];
  for (int base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    int q = base + threadIdx.x;
    bool alive = false;
    int p = -1;
    if (q < n) {
      p = list[q];
      alive = shade_one<F>(S, P, p, max_depth);
    }
    if (F != FAM_TERM) {
      append(alive, p, next, next_count);
      // survivors per batch region, so the host knows when a batch has drained
      if (alive) atomicAdd(&hist[p / region_size], 1);
    }
  }
  if (F != FAM_TERM) {
    __syncthreads();
    if (threadIdx.x < kMaxRegions && hist[threadIdx.x]) atomicAdd(&region_alive[threadIdx.x], hist[threadIdx.x]);
  }
}

// acc[pixel] += samples in sample order (Raytracing_n.cpp:841), batch by batch
__global__ void __launch_bounds__(256) k_accumulate(PathState P, BatchInfo B, float* acc) {
  int lp = blockIdx.x * blockDim.x + threadIdx.x;
  if (lp >= B.n_paths / B.spp_batch) return;
  size_t a = 3 * (size_t)(B.p0 + lp);
  float cx = acc[a], cy = acc[a + 1], cz = acc[a + 2];
  for (int s = 0; s < B.spp_batch; ++s) {
    size_t q = 3 * ((size_t)B.slot0 + (size_t)lp * B.spp_batch + s);
    cx += ntl(&P.sample[q]);
    cy += ntl(&P.sample[q + 1]);
    cz += ntl(&P.sample[q + 2]);
  }
  acc[a] = cx;
  acc[a + 1] = cy;
  acc[a + 2] = cz;
}

// col /= float(ns): k = 1.0 / t in double, stored to float (vec3.h:160-167)
__global__ void k_finish(const float* acc, float* mean, int64_t n, int ns) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * n) return;
  float k = 1.0 / (float)ns;
  mean[i] = acc[i] * k;
}

// Multi-device frame assembly (multi.cpp): the gathered shard slabs, packed in
// shard order, scattered to their image pixels: image[index[i]] = packed[i]
// (float3).  One thread per channel word, so the packed reads coalesce.
__global__ void k_scatter_pixels(const float* __restrict__ packed, const int32_t* __restrict__ index, int64_t n,
                                 float* __restrict__ image) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * n) return;
  const int64_t px = i / 3;
  image[3 * (int64_t)index[px] + (i - 3 * px)] = packed[i];
}

// ------------------------------------------------------------ MERL lookup
// brdf::lookup_brdf_val (brdf.h:190-214) for n direction pairs: one query per
// thread, angles[4q..4q+3] = (theta_in, fi_in, theta_out, fi_out).
__global__ void __launch_bounds__(256) k_merl_lookup(const double* table, int64_t n, const double* angles,
                                                     double* rgb, int32_t* cell) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const double* a = angles + 4 * q;
  const int c = merl::cell_of(a[0], a[1], a[2], a[3]);
  double r, g, b;
  merl::rgb_of(table, c, r, g, b);
  rgb[3 * q] = r;
  rgb[3 * q + 1] = g;
  rgb[3 * q + 2] = b;
  if (cell) cell[q] = c;
}

// ------------------------------------------------- device known-answer tests
// Test infrastructure (srr_device_kat): the product's device functions on the
// reference's KAT records (tests/golden/kat_*.bin, layouts in oracle/ref/kat.inc):
// inputs are read from each record and the outputs written back in place, so a
// test can compare them bit for bit with the reference's outputs.
// aux: 4 host-computed floats per record (Beckmann alphas, Oren-Nayar A / B).
enum KatKind : int { KAT_ERF, KAT_BECK11, KAT_BECK_DIST, KAT_BECK_PDF, KAT_COSINE, KAT_ORENNAYAR, KAT_DIELECTRIC,
                     KAT_METAL, KAT_TRIANGLE, KAT_AABB, KAT_SQRT, KAT_CAMERA, KAT_LIGHTS, KAT_LIGHT_LIST };

SRR_D V3 kat3(const float* p) { return v3(p[0], p[1], p[2]); }
SRR_D void kat_put3(float* p, V3 v) { p[0] = v.x, p[1] = v.y, p[2] = v.z; }
SRR_D uint64_t kat_lcg(const float* p) { return (uint64_t)p[0] | ((uint64_t)p[1] << 24); }
SRR_D void kat_put_lcg(float* p, uint64_t s) { p[0] = (float)(s & 0xFFFFFF), p[1] = (float)((s >> 24) & 0xFFFFFF); }
SRR_D uint64_t kat_pcg(const float* p) {
  uint64_t s = 0;
  for (int k = 0; k < 4; ++k) s |= (uint64_t)p[k] << (16 * k);
  return s;
}
SRR_D void kat_put_pcg(float* p, uint64_t s) {
  for (int k = 0; k < 4; ++k) p[k] = (float)((s >> (16 * k)) & 0xFFFF);
}

__global__ void k_kat(int kind, int n, int w, float* rec, const float* aux, const DStandaloneTri* tris, KatTables kt) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  float* r = rec + (size_t)q * w;
  const float* a = aux + 4 * (size_t)q;
  switch (kind) {
    case KAT_ERF:
      r[1] = Erf(r[0]);
      r[2] = ErfInv(r[0]);
      break;
    case KAT_BECK11:
      beckmann_sample11(r[0], r[1], r[2], r[3], r[4]);
      break;
    case KAT_BECK_DIST: {
      const Beck d{a[0], a[1]};
      const V3 wo = kat3(r + 2);
      const V3 wh = beckmann_sample_wh(d, wo, r[5], r[6]);
      r[7] = d.ax;
      r[8] = d.ay;
      kat_put3(r + 9, wh);
      r[12] = d.D(wh);
      r[13] = d.G(wo, wh);
      r[14] = d.Pdf(wo, wh);
      r[15] = d.Lambda(wo);
      break;
    }
    case KAT_BECK_PDF: {
      Bsdf f;
      f.kind = MAT_BECKMANN;
      f.n = kat3(r + 2);
      f.uvw = onb_from_w(f.n);
      f.dist = Beck{a[0], a[1]};
      f.beck_pdf = 0;
      const V3 wo = kat3(r + 5);
      Rng rng{0, kat_pcg(r + 8)};
      bsdf_prepare<true>(f, wo);
      const V3 wi = bsdf_generate<true>(f, wo, rng);
      kat_put3(r + 12, wi);
      r[15] = bsdf_value<true>(f, wo, wi);
      r[16] = scattering_pdf<true>(f, f.n, wo, wi);
      kat_put_pcg(r + 17, rng.pcg);
      break;
    }
    case KAT_COSINE:
    case KAT_ORENNAYAR: {
      Bsdf f;
      f.kind = kind == KAT_COSINE ? MAT_LAMBERTIAN : MAT_ORENNAYAR;
      f.n = kat3(r + 1);
      f.uvw = onb_from_w(f.n);
      f.A = a[0];
      f.B = a[1];
      const V3 wo = kat3(r + 4);
      bsdf_prepare<false>(f, wo);
      Rng rng{kat_lcg(r + 7), 0};
      const V3 d = bsdf_generate<false>(f, wo, rng);
      r[9] = a[0];
      r[10] = a[1];
      kat_put3(r + 11, d);
      r[14] = bsdf_value<false>(f, wo, d);
      r[15] = bsdf_value<false>(f, wo, kat3(r + 16));
      kat_put_lcg(r + 19, rng.lcg);
      break;
    }
    case KAT_DIELECTRIC:
    case KAT_METAL: {
      DMat M{};
      if (kind == KAT_DIELECTRIC) {
        M.kind = MAT_DIELECTRIC;
        M.p[0] = r[0];
      } else {
        M.kind = MAT_METAL;
        M.p[0] = M.p[1] = M.p[2] = 0.5f;
        M.p[3] = r[0] < 1 ? r[0] : 1;
      }
      Rng rng{kat_lcg(r + 7), 0};
      float4 rc;
      bool sp;
      V3 nd;
      float nt;
      scatter<FAM_SPEC>(SceneView{}, M, kat3(r + 1), 0.25f, v3(1, 2, 3), kat3(r + 4), 0, 0, rng, rc, sp, nd, nt);
      kat_put3(r + 9, nd);
      kat_put_lcg(r + 12, rng.lcg);
      break;
    }
    case KAT_TRIANGLE: {
      SceneView S{};
      S.stris = tris;
      const DObj ob{OBJ_TRI, 0, 0, q};
      const Ray ray{kat3(r + 9), kat3(r + 12), 0.0f};
      float t = 0;
      const bool h = prim_hit<TR_WL>(S, ob, ray, 0.001f, FLT_MAX, r[15] != 0, t);
      HitRec hr;
      hr.u = hr.v = 0;
      hr.p = hr.n = v3(0.f);
      if (h) prim_record(S, ob, ray, t, -1, hr);
      r[16] = h ? 1.f : 0.f;
      r[17] = h ? t : 0;
      r[18] = hr.u;
      r[19] = hr.v;
      kat_put3(r + 20, hr.n);
      kat_put3(r + 23, hr.p);
      break;
    }
    case KAT_SQRT:
      r[1] = rsqrt_exact(r[0]);
      break;
    case KAT_CAMERA: {  // in: lookfrom lookat vfov aspect aperture focus s t lcg | out: origin dir time lcg
      Rng rng{kat_lcg(r + 12), 0};
      V3 o, d;
      float tm;
      camera_get_ray(kt.cams[q], r[10], r[11], rng, o, d, tm);
      kat_put3(r + 14, o);
      kat_put3(r + 17, d);
      r[20] = tm;
      kat_put_lcg(r + 21, rng.lcg);
      break;
    }
    case KAT_LIGHTS:        // in: o lcg | out: rect dir, pdf; sphere dir, pdf; lcg
    case KAT_LIGHT_LIST: {  // in: o lcg | out: list dir, list pdf; triangle dir, pdf; lcg
      SceneView S{};
      S.rects = kt.rects;
      S.spheres = kt.spheres;
      S.stris = kt.stris;
      S.lights = kt.lights;
      S.n_lights = kt.n_lights;
      S.light_weight = kt.n_lights > 0 ? (float)(1.0 / kt.n_lights) : 0.f;
      Rng rng{kat_lcg(r + 3), 0};
      const V3 o = kat3(r);
      V3 d1, d2;
      float p1, p2;
      if (kind == KAT_LIGHTS) {  // the list's first two lights on their own: flip(xz_rect), sphere
        d1 = light_random_one(S, kt.lights[0], o, rng);
        p1 = light_pdf_one(S, kt.lights[0], o, d1);
        d2 = light_random_one(S, kt.lights[1], o, rng);
        p2 = light_pdf_one(S, kt.lights[1], o, d2);
      } else {  // the whole list (hitable_list::random / pdf_value), then its triangle alone
        d1 = lights_random(S, o, rng);
        p1 = lights_pdf(S, o, d1);
        d2 = light_random_one(S, kt.lights[2], o, rng);
        p2 = light_pdf_one(S, kt.lights[2], o, d2);
      }
      kat_put3(r + 5, d1);
      r[8] = p1;
      kat_put3(r + 9, d2);
      r[12] = p2;
      kat_put_lcg(r + 13, rng.lcg);
      break;
    }
    case KAT_AABB: {
      const V3 d = kat3(r + 9);
      r[14] = slab(make_float4(r[0], r[1], r[2], 0), make_float4(r[3], r[4], r[5], 0), kat3(r + 6),
                   v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z), r[12], r[13]) ? 1.f : 0.f;
      break;
    }
  }
}

}  // namespace dev

// ------------------------------------------------------------ launch shims
void launch_raygen(const SceneView& S, const PathState& P, const BatchInfo& B, hipStream_t st) {
  int g = (B.n_paths + 255) / 256;
  hipLaunchKernelGGL(dev::k_raygen, dim3(g), dim3(256), 0, st, S, P, B);
}
static unsigned long long* g_timing = nullptr;

void dump_trace_timing() {  // SRR_TRAVERSAL=timed diagnostics
  if (!g_timing) return;
  std::vector<unsigned long long> v(1 + 8 * dev::kTimingCap);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(v.data(), g_timing, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  size_t n = std::min<unsigned long long>(v[0], dev::kTimingCap);
  std::vector<double> tot, mesh, steps, per, stg, ray, hit, tail;
  for (size_t k = 0; k < n; ++k) {
    const unsigned long long* e = &v[1 + 8 * k];
    stg.push_back((double)e[3]);
    ray.push_back((double)e[4]);
    hit.push_back((double)e[5]);
    tail.push_back((double)e[6]);
    tot.push_back((double)e[0]);
    mesh.push_back((double)e[1]);
    steps.push_back((double)e[2]);
    if (e[2] > 0) per.push_back((double)e[1] / (double)e[2]);
  }
  auto pct = [](std::vector<double> x, double q) {
    if (x.empty()) return 0.0;
    std::sort(x.begin(), x.end());
    return x[std::min(x.size() - 1, (size_t)(q * x.size()))];
  };
  auto mean = [](const std::vector<double>& x) {
    double a = 0;
    for (double y : x) a += y;
    return x.empty() ? 0.0 : a / x.size();
  };
  fprintf(stderr, "trace timing: %zu waves (s_memtime ticks)\n", n);
  for (auto [name, x] : {std::pair<const char*, std::vector<double>*>{"wave total", &tot}, {"mesh", &mesh},
                         {"mesh steps (wave max)", &steps}, {"ticks per step", &per}, {"LDS staging", &stg},
                         {"ray load", &ray}, {"world hit", &hit}, {"store+append", &tail}})
    fprintf(stderr, "  %-22s mean %10.1f  p10 %10.1f  p50 %10.1f  p90 %10.1f  p99 %10.1f\n", name, mean(*x), pct(*x, .1),
            pct(*x, .5), pct(*x, .9), pct(*x, .99));
}

void launch_trace(const SceneView& S, const PathState& P, const int* active, const int* count, int max_n,
                  int* lists, int list_cap, int* fam_count, int* fetch, int max_depth, unsigned long long* ctr,
                  hipStream_t st) {
  int g = (max_n + 255) / 256;
  // SRR_TRAVERSAL: bvh4prune (default) | bvh4 | bvh2 = one ray per thread over the
  // SAH 4-wide BVH (with / without closest-hit pruning) or the threaded reference
  // BVH2;
  // timed = bvh4prune with per-wave timing records (diagnostics)
  static const int tr = [] {
    const char* e = getenv("SRR_TRAVERSAL");
    if (e && !strcmp(e, "bvh2")) return (int)dev::TR_BVH2;
    if (e && !strcmp(e, "bvh4")) return (int)dev::TR_BVH4;
    if (e && !strcmp(e, "bvh4prune")) return (int)dev::TR_BVH4_PRUNE;
    if (e && !strcmp(e, "timed")) return (int)dev::TR_BVH4_TIMED;
    return (int)dev::TR_BVH4_PRUNE;
  }();
  const int grec = std::min(g, 2048);
  static unsigned long long* timing = nullptr;
  if (tr == dev::TR_BVH4_TIMED && !timing) {
    (void)hipMalloc((void**)&timing, (1 + 8 * dev::kTimingCap) * sizeof(unsigned long long));
    (void)hipMemset(timing, 0, (1 + 8 * dev::kTimingCap) * sizeof(unsigned long long));
    g_timing = timing;
  }
  unsigned long long* kctr = tr == dev::TR_BVH4_TIMED ? timing : ctr;
#define SRR_LAUNCH_TRACE(M, T)                                                                        \
  hipLaunchKernelGGL((dev::k_trace<M, T>), dim3(g), dim3(dev::kTraceBlock), 0, st, S, P, active, count, \
                     lists, list_cap, fam_count, max_depth, kctr)
  const bool wl = S.world_words * 16 <= dev::kWorldLdsBytes && !getenv("SRR_NO_WORLD_LDS");
#define SRR_LAUNCH_TRACE_W(M, T)                  \
  if (wl) SRR_LAUNCH_TRACE(M, (T) | dev::TR_WL); \
  else SRR_LAUNCH_TRACE(M, T);
#define SRR_LAUNCH_TRACE_M(M)                                                 \
  if (trm == dev::TR_BVH2) { SRR_LAUNCH_TRACE_W(M, dev::TR_BVH2) }            \
  else if (trm == dev::TR_BVH4) { SRR_LAUNCH_TRACE_W(M, dev::TR_BVH4) }       \
  else if (trm == dev::TR_BVH4_TIMED) { SRR_LAUNCH_TRACE_W(M, dev::TR_BVH4_TIMED) } \
  else { SRR_LAUNCH_TRACE_W(M, dev::TR_BVH4_PRUNE) }
  const int trm = tr;
  if (S.has_media) {
    SRR_LAUNCH_TRACE_M(true)
  } else {
    SRR_LAUNCH_TRACE_M(false)
  }
  hipLaunchKernelGGL(dev::k_record, dim3(grec), dim3(256), 0, st, S, P, active, count);
  static const bool probe = getenv("SRR_PROBE") && getenv("SRR_PROBE")[0] == '1';
  if (probe && !S.has_media) {
    static int* sink = nullptr;
    if (!sink) (void)hipMalloc((void**)&sink, 16);
#define SRR_PROBE(T, M) \
  hipLaunchKernelGGL((dev::k_probe<false, T, M>), dim3(g), dim3(dev::kTraceBlock), 0, st, S, P, active, count, sink)
#define SRR_PROBES(T) SRR_PROBE(T, 0); SRR_PROBE(T, 1); SRR_PROBE(T, 4); SRR_PROBE(T, 5); SRR_PROBE(T, 2);
    if (trm == dev::TR_BVH2) { SRR_PROBES(dev::TR_BVH2) }
    else if (trm == dev::TR_BVH4) { SRR_PROBES(dev::TR_BVH4) }
    else { SRR_PROBES(dev::TR_BVH4_PRUNE) }
#undef SRR_PROBES
#undef SRR_PROBE
  }
#undef SRR_LAUNCH_TRACE_M
#undef SRR_LAUNCH_TRACE_W
#undef SRR_LAUNCH_TRACE
}
void launch_shade(const SceneView& S, const PathState& P, const int* lists, int list_cap, const int* fam_count,
                  int* next, int* next_count, int* region_alive, int region_size, int max_n, int max_depth,
                  hipStream_t st) {
  // grid sized for the whole bounce; each family kernel strides over its own list
  int g = std::min((max_n + 255) / 256, 2048);
  hipLaunchKernelGGL(dev::k_shade<dev::FAM_DIFF>, dim3(g), dim3(256), 0, st, S, P, lists, list_cap, fam_count, next,
                     next_count, region_alive, region_size, max_depth);
  hipLaunchKernelGGL(dev::k_shade<dev::FAM_BECK>, dim3(g), dim3(256), 0, st, S, P, lists, list_cap, fam_count, next,
                     next_count, region_alive, region_size, max_depth);
  hipLaunchKernelGGL(dev::k_shade<dev::FAM_SPEC>, dim3(g), dim3(256), 0, st, S, P, lists, list_cap, fam_count, next,
                     next_count, region_alive, region_size, max_depth);
  hipLaunchKernelGGL(dev::k_shade<dev::FAM_TERM>, dim3(g), dim3(256), 0, st, S, P, lists, list_cap, fam_count, next,
                     next_count, region_alive, region_size, max_depth);
}
void launch_accumulate(const PathState& P, const BatchInfo& B, float* acc, hipStream_t st) {
  int np = B.n_paths / B.spp_batch;
  int g = (np + 255) / 256;
  hipLaunchKernelGGL(dev::k_accumulate, dim3(g), dim3(256), 0, st, P, B, acc);
}
void launch_finish(const float* acc, float* mean, int64_t n, int ns, hipStream_t st) {
  int64_t g = (3 * n + 255) / 256;
  hipLaunchKernelGGL(dev::k_finish, dim3((unsigned)g), dim3(256), 0, st, acc, mean, n, ns);
}

void launch_scatter_pixels(const float* packed, const int32_t* index, int64_t n, float* image, hipStream_t st) {
  if (n <= 0) return;
  const int64_t g = (3 * n + 255) / 256;
  hipLaunchKernelGGL(dev::k_scatter_pixels, dim3((unsigned)g), dim3(256), 0, st, packed, index, n, image);
}


// Occupancy of the path kernel: min resident 256-thread blocks per CU (2-6,
// SRR_PATHS_OCC).  The kernel's natural allocation is ~226 VGPRs (2 waves per
// SIMD); capping registers spills some cold state to scratch but hides more
// latency -- measured on C2: 2 -> 5.25, 3 -> 6.10, 4 -> 6.49 Gsamples/s.
constexpr int kPathsOccDefault = 4;
static int paths_min_blocks() {
  static const int v = [] {
    const char* e = getenv("SRR_PATHS_OCC");
    int x = e ? atoi(e) : kPathsOccDefault;
    return x >= 2 && x <= 6 ? x : kPathsOccDefault;
  }();
  return v;
}

// Lanes per k_paths block for this scene: 1,024 (SRR_BIGBLOCK, the default) when the
// launch would take the per-lane, LDS-world path, else 256.  render_paths rounds
// the window's lanes to it.
int paths_block_lanes(const SceneView& S) {
  static const bool big = [] {
    const char* e = getenv("SRR_BIGBLOCK");
    return !e || atoi(e) != 0;
  }();
  static const bool timed = SRR_DIAG_VARIANTS && getenv("SRR_PATHS_TIMING") != nullptr;
  static const bool force_global = getenv("SRR_WORLD_GLOBAL") != nullptr;
  const bool wl = !force_global && S.world_words * 16 <= dev::kWorldLdsBytes;
  // (a scene without meshes has no BVH4 nodes to cache: 256-lane blocks, which
  // free their CU slots at a finer grain when frames overlap -- C1 +1.6 %)
  return (big && wl && !timed && !S.quad_trace && S.node4_total > 0 &&
          paths_min_blocks() == kPathsOccDefault) ? 1024 : dev::kPathsBlock;
}

int paths_lanes_per_device(const SceneView& S, int device) {
  (void)S;
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)dev::k_paths<false, false, 4>,
                                                   dev::kPathsBlock, 0) != hipSuccess || per_cu <= 0)
    per_cu = 2;
  per_cu = std::max(per_cu, paths_min_blocks());
  return cus * per_cu * dev::kPathsBlock;
}

int launch_paths(const SceneView& S, const PathWork& W, int all_families, hipStream_t st) {
  // the kernels index kStack LDS entries per lane: a host built with a larger
  // SRR_KSTACK is refused here (round 4 ran such a mix once: an illegal address)
  if (W.stack_cap < 1 || W.stack_cap > dev::kStack) return -1;
  const dev::PathsArgs args{S, W};
  const int blocks = W.lanes / dev::kPathsBlock;
  static const bool force_global = getenv("SRR_WORLD_GLOBAL") != nullptr;  // A/B diagnostics
  if (force_global || S.world_words * 16 > dev::kWorldLdsBytes) {  // world tables too large for LDS: global reads
#define SRR_LAUNCH_PATHS_G(M, A)                                                                                      \
  if (S.quad_trace) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, false, true>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args); \
  else hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, false>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args)
    if (S.has_media) {
      if (all_families) SRR_LAUNCH_PATHS_G(true, true);
      else SRR_LAUNCH_PATHS_G(true, false);
    } else {
      if (all_families) SRR_LAUNCH_PATHS_G(false, true);
      else SRR_LAUNCH_PATHS_G(false, false);
    }
#undef SRR_LAUNCH_PATHS_G
    return 0;
  }
  const int bs = paths_block_lanes(S);
  const int blocks_b = W.lanes / bs;
  // suspendable mesh walks: the variant with them when the frame asks for them (walk_q > 0);
  // only the 1,024-lane (mesh scene) and diagnostics variants have one
  const bool sp = W.walk_q > 0;
#if SRR_DIAG_VARIANTS
  // diagnostics build (make diag): SRR_PATHS_TIMING=1 phase timing, SRR_CBVH=1 compressed nodes
  static const bool timed = getenv("SRR_PATHS_TIMING") != nullptr;
  const bool cq = S.use_q && !S.quad_trace && !timed;  // compressed nodes, per-lane walks
#define SRR_LAUNCH_PATHS_DIAG(M, A, B)                                                                                         \
  if (timed && sp) hipLaunchKernelGGL((dev::k_paths<M, A, 4, true, true, false, false, dev::kPathsBlock, true>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args); \
  else if (timed) hipLaunchKernelGGL((dev::k_paths<M, A, 4, true>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args);      \
  else if (bs == 1024 && B == 4 && cq) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, true, false, true, 1024>), dim3(blocks_b), dim3(1024), 0, st, args); \
  else if (cq && B == 4) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, true, false, true>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args); \
  else
#else
  if (S.use_q || getenv("SRR_PATHS_TIMING"))
    fprintf(stderr, "srr: SRR_CBVH / SRR_PATHS_TIMING need the diagnostics build (make diag); ignored\n");
#define SRR_LAUNCH_PATHS_DIAG(M, A, B)
#endif
#define SRR_LAUNCH_PATHS(M, A, B)                                                                      \
  SRR_LAUNCH_PATHS_DIAG(M, A, B)                                                                       \
  if (bs == 1024 && B == 4 && !S.quad_trace && sp) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, true, false, false, 1024, true>), dim3(blocks_b), dim3(1024), 0, st, args); \
  else if (bs == 1024 && B == 4 && !S.quad_trace) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, true, false, false, 1024>), dim3(blocks_b), dim3(1024), 0, st, args); \
  else if (S.quad_trace && B == 4) hipLaunchKernelGGL((dev::k_paths<M, A, 4, false, true, true>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args); \
  else hipLaunchKernelGGL((dev::k_paths<M, A, B>), dim3(blocks), dim3(dev::kPathsBlock), 0, st, args)
#ifdef SRR_OCC_VARIANTS  // occupancy A/B builds (SRR_PATHS_OCC): 2, 3, 5 and 6 blocks per CU
#define SRR_LAUNCH_PATHS_B(M, A)                          \
  switch (paths_min_blocks()) {                           \
    case 2: SRR_LAUNCH_PATHS(M, A, 2); break;             \
    case 3: SRR_LAUNCH_PATHS(M, A, 3); break;             \
    case 5: SRR_LAUNCH_PATHS(M, A, 5); break;             \
    case 6: SRR_LAUNCH_PATHS(M, A, 6); break;             \
    default: SRR_LAUNCH_PATHS(M, A, 4); break;            \
  }
#else
#define SRR_LAUNCH_PATHS_B(M, A) SRR_LAUNCH_PATHS(M, A, 4);
#endif
  if (S.has_media) {
    if (all_families) { SRR_LAUNCH_PATHS_B(true, true) }
    else { SRR_LAUNCH_PATHS_B(true, false) }
  } else {
    if (all_families) { SRR_LAUNCH_PATHS_B(false, true) }
    else { SRR_LAUNCH_PATHS_B(false, false) }
  }
#undef SRR_LAUNCH_PATHS_DIAG
#undef SRR_LAUNCH_PATHS_B
#undef SRR_LAUNCH_PATHS
  return 0;
}

int launch_merl_lookup(const double* table, int64_t n, const double* angles, double* rgb, int32_t* cell) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dev::k_merl_lookup, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, table, n, angles, rgb,
                     cell);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_kat(int kind, int n, int w, float* d_rec, const float* d_aux, const DStandaloneTri* d_tris,
               const KatTables& kt) {
  hipLaunchKernelGGL(dev::k_kat, dim3((n + 63) / 64), dim3(64), 0, 0, kind, n, w, d_rec, d_aux, d_tris, kt);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

void launch_accumulate_window(const float* sample, int npix, int spp_w, float* acc, hipStream_t st, bool init,
                              float* out, int scale_ns) {
  static const bool scalar = getenv("SRR_ACC_SCALAR") != nullptr;  // A/B diagnostics
  const dev::AccOut o{out, scale_ns};
  if (spp_w % 4 == 0 && ((uintptr_t)sample & 15) == 0 && !scalar)
    hipLaunchKernelGGL(dev::k_accumulate_window16, dim3((npix + 255) / 256), dim3(256), 0, st, (const float4*)sample,
                       npix, spp_w, acc, init ? 1 : 0, o);
  else
    hipLaunchKernelGGL(dev::k_accumulate_window, dim3((npix + 255) / 256), dim3(256), 0, st, sample, npix, spp_w, acc,
                       init ? 1 : 0, o);
}

}  // namespace srr

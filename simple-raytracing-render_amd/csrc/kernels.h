// Device-side views of the uploaded scene and of the per-path wavefront state,
// plus the kernel launch shims (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_scene.h"

namespace srr {

struct SceneView {  // device pointers into the flattened tables (device_scene.h)
  const DObj* objs;
  int n_world;
  int has_media;
  const DXform* xforms;
  const DSphere* spheres;
  const DRect* rects;
  const DStandaloneTri* stris;
  const DMesh* meshes;
  const float4* nodes;  // 2 float4 per BVH2 node: lo (min.xyz, skip), hi (max.xyz, leaf)
  const float4* node4;  // 8 float4 per 4-wide node (device_scene.h), breadth-first per mesh
  int node4_lds;        // leading nodes the path kernel keeps in LDS (<= kPathsLdsNodes)
  int node4_total;      // BVH4 nodes of all meshes (the LDS caches take a prefix)
  const float4* node4q; // the same nodes compressed to 64 B (device_scene.h kNode4qWords), or nullptr
  int node4_lds_q;      // ...and how many of those the path kernel keeps in LDS (<= 2 kPathsLdsNodes)
  int use_q;            // k_paths traces meshes over node4q (SRR_CBVH)
  int quad_trace;       // k_paths traces meshes quad-cooperatively (BVH4 larger than an XCD's L2)
  int quad_max;         // ...when at most this many lanes of the wave enter the mesh (else per lane)
  int mesh_obj;         // the world list's one top-level mesh object, else -1 (kernels.hip world_hit: walk suspension's list mode)
  const float4* tri_pos;  // 4 float4 per triangle: p0, p1, p2, pad
  const float4* tri_edge;  // 8 float4 per triangle i: p0, e1, e2 of i and i+1 packed (renderer.cpp)
  const TriShade* tri_shade;
  const DMedium* media;
  const DObvh* obvhs;                 // object BVHs (global memory)
  const DObvhChild* obvh_children;
  const DSGroup* sgroups;             // sphere runs behind a BVH (global memory)
  const DSGItem* sg_items;
  const DMat* mats;
  const DTex* texs;
  const uint8_t* images;
  const float* perlin_ranvec;
  const int32_t* perlin_perm;
  const DLight* lights;
  int n_lights;
  float light_weight;  // hitable_list::pdf_value's weight, (float)(1.0 / n_lights) (hitable_list.h:55)
  const DCamera* cam;
  // the world traversal's and shading's small tables packed in one blob (16-B
  // aligned pieces) that the kernels copy to LDS: byte offsets of objs, xforms,
  // spheres, rects, stris, meshes, media, mats, texs, lights
  const uint4* world_blob;
  int world_words;  // 16-B words
  int world_off[10];
};

// Struct-of-arrays state of the paths of one batch (capacity N).
struct PathState {
  float4* ray_o;    // origin.xyz, time
  float4* ray_d;    // direction.xyz
  uint64_t* lcg;    // 48-bit LCG state (mathf.h:12), per path
  uint64_t* pcg;    // PCG32 state (pdf.h:20), per path
  int32_t* depth;   // the reference's *depth
  uint64_t* spec;   // bit k: bounce k was specular
  int4* hit_w;      // closest hit: object (-1 miss), primitive, t (float bits), material (-1 null)
  float4* hit_p;    // its record (k_record): p.xyz, u
  float4* hit_n;    //   normal.xyz, v
  float4* rec_a;    // [path][max_depth]: attenuation*scattering_pdf (or attenuation), pdf
  float* sample;    // [path][3] de_nan'd radiance
  float* raw;       // [path][3] radiance before de_nan (optional)
  uint8_t* rays;    // [path] world rays traced (optional)
};

struct BatchInfo {
  int32_t* active;        // active list the batch's paths are appended to
  int32_t* count;         // device count of that list, set to act0 + n_paths
  int act0;               // ... at this offset
  int slot0;              // first path-state slot of the batch's region
  const int32_t* pixels;  // shard pixel list (PPM-order indices)
  const double* sobol;    // [spp][2], already offset to global sample s_base
  int p0;                 // first shard pixel of the batch
  int n_paths;            // pixels_in_batch * spp_batch
  int s0, spp_batch;      // sample range [s0, s0 + spp_batch) of this render
  int s_base;             // global index of this render's sample 0 (sample sharding)
  int nx, ny;
  uint64_t base_seed;
};

// floor(n / d) for 0 <= n < 2^31 as (n * m) >> p with m = ceil(2^p / d),
// p = 31 + ceil(log2 d) (Granlund-Montgomery: exact for every 31-bit n; m < 2^32)
struct UDiv31 {
  uint32_t m, p;
};
inline UDiv31 make_udiv31(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint32_t p = 31 + l;
  return UDiv31{(uint32_t)(((1ull << p) + d - 1) / d), p};
}

// One window of a frame for the path-resident persistent kernel (k_paths):
// every (pixel, sample) of pixels x [0, spp_w) is a path, numbered pixel-major
// g = lp * spp_w + s (a wave's lanes take samples of one pixel: coherent first
// bounces); lanes fetch g from `cursor` as their paths finish.
struct PathWork {
  const int32_t* pixels;  // shard pixel list (PPM-order indices), nullptr = identity
  const double* sobol;    // [spp_w][2], window sample 0 first
  int npix, spp_w;
  int s_base;             // global sample index of window sample 0 (per-path seeds)
  int nx, ny;
  UDiv31 div_spp, div_nx;  // invariant divisors spp_w and nx (path index -> pixel, pixel -> i, j)
  uint64_t base_seed;
  int64_t n_paths;        // npix * spp_w
  int max_depth;
  unsigned long long* cursor;  // next path to start (device, zeroed per window)
  unsigned long long* counters;  // [0] += world rays traced
  float* sample;          // [n_paths][3] de_nan'd radiance, index g
  float* raw;             // optional kept paths [npix][keep_spp][3] before de_nan
  uint8_t* rays;          // optional kept [npix][keep_spp] world rays per path
  int keep_spp, keep_s0;  // frame spp and this window's first sample in them
  float4* rec;            // bounce records [max_depth][lanes]
  int lanes;              // persistent lanes (grid * block)
  int* err;               // guard bits set on an out-of-range index (never expected)
  int stack_cap;          // BVH4 traversal stack entries (kStack = 8; fewer forces the exact re-walk)
  int2* gstack;           // the stack's global extension [gstack_cap][lanes] (deep meshes), or nullptr
  int gstack_cap;
  unsigned long long* wave_times;  // diagnostics (SRR_WAVE_TIMES): per wave [start, exit] s_memrealtime, or nullptr
  int deep_tries;         // coop_mixture: failed attempts after which a path takes every free lane (32)
  float* slow_rays;       // diagnostics build (-DSRR_SLOW_RAYS=ticks): [65536][16] records of slow world hits
  unsigned* slow_count;
  // suspendable mesh walks (kernels.hip TraceCtx::walk_thr): a lane's walk, after a node
  // step, stops for this wave-iteration once at most walk_q / 64 of the wave's lanes in a
  // path are still walking (0: never); its state goes to the [3][lanes] float4 save area
  // that follows gstack's gstack_cap x lanes entries (so walks suspend only with gstack)
  int walk_q;
};
#ifndef SRR_KSTACK
#define SRR_KSTACK 8
#endif
constexpr int kPathsLdsStack = SRR_KSTACK;  // LDS traversal stack entries per lane (kernels.hip kStack)
constexpr int kPathsGlobalStack = 56;  // global stack entries per lane beyond the LDS ones

constexpr int kPathsWorldLdsBytes = 8192;  // == kernels.hip kWorldLdsBytes
#ifndef SRR_LDS_NODES
#define SRR_LDS_NODES 96
#endif
constexpr int kPathsLdsNodes = SRR_LDS_NODES;  // BVH4 nodes cached in LDS by k_paths (128 B each)
void dump_trace_timing();
int paths_lanes_per_device(const SceneView& S, int device);  // persistent grid capacity
int paths_block_lanes(const SceneView& S);  // k_paths lanes per block for this scene (256 or 1,024)
// 0, or -1 (nothing launched) when W.stack_cap exceeds the kernels' LDS stack (kStack)
int launch_paths(const SceneView& S, const PathWork& W, int all_families, hipStream_t st);
// device known-answer tests (srr_device_kat); kind = dev::KatKind
// device tables of the camera / light KATs (srr_device_kat builds them with the
// host scene code: one camera per record, one light list for all records)
struct KatTables {
  const DCamera* cams;
  const DRect* rects;
  const DSphere* spheres;
  const DStandaloneTri* stris;
  const DLight* lights;
  int n_lights;
};
int launch_kat(int kind, int n, int w, float* d_rec, const float* d_aux, const DStandaloneTri* d_tris,
               const KatTables& kt);
// MERL table lookup (merl.h) for n queries; device pointers
int launch_merl_lookup(const double* table, int64_t n, const double* angles, double* rgb, int32_t* cell);
// acc[pixel] (+)= the window's samples in order; init: acc starts at 0 (no
// memset); out != nullptr (the last window): also out = acc * (float)(1.0 / scale_ns)
// (k_finish), or the raw sums when scale_ns == 0
void launch_accumulate_window(const float* sample, int npix, int spp_w, float* acc, hipStream_t st, bool init = false,
                              float* out = nullptr, int scale_ns = 0);
void launch_raygen(const SceneView& S, const PathState& P, const BatchInfo& B, hipStream_t st);
void launch_trace(const SceneView& S, const PathState& P, const int* active, const int* count, int max_n,
                  int* lists, int list_cap, int* fam_count, int* fetch, int max_depth, unsigned long long* ctr,
                  hipStream_t st);
void launch_shade(const SceneView& S, const PathState& P, const int* lists, int list_cap, const int* fam_count,
                  int* next, int* next_count, int* region_alive, int region_size, int max_n, int max_depth,
                  hipStream_t st);
void launch_accumulate(const PathState& P, const BatchInfo& B, float* acc, hipStream_t st);
void launch_finish(const float* acc, float* mean, int64_t n, int ns, hipStream_t st);
// image[index[i]] = packed[i] (float3 per pixel) for i < n: multi-device frame assembly
void launch_scatter_pixels(const float* packed, const int32_t* index, int64_t n, float* image, hipStream_t st);

}  // namespace srr

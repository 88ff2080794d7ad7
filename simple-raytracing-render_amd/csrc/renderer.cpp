// Renderer: scene upload and the multi-lane wavefront driver (renderer.h).
#include "renderer.h"

#include "multi.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <cstdio>

namespace srr {

constexpr int kCtrWords = 40;  // FrameSlot::ctr: world rays, cursor, error, overflow and diagnostics counters
constexpr int kVisitWords = 3 + 2 * 64;  // SRR_FLAG_COUNT_VISITS: sums + two histograms

#define RCHK(x)                                                        \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      err = std::string(#x) + ": " + hipGetErrorString(e_);            \
      return SRR_EIO;                                                  \
    }                                                                  \
  } while (0)

template <class T>
static hipError_t upload(T** dst, const std::vector<T>& v, std::vector<void*>& keep) {
  size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  hipError_t e = hipMalloc((void**)dst, bytes);
  if (e != hipSuccess) return e;
  keep.push_back(*dst);
  if (!v.empty()) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return e;
}

int renderer_create(const Scene& sc, int device, srr_renderer** out, std::string& err) {
  Flat F;
  int rc = flatten(sc, F, err);
  if (rc < 0) return rc;
  return renderer_create_flat(F, device, out, err);
}

int renderer_create_flat(const Flat& F, int device, srr_renderer** out, std::string& err) {
  std::unique_ptr<srr_renderer> r(new srr_renderer());
  r->device = device;
  if (const char* e = getenv("SRR_LANES")) r->n_lanes = std::max(1, std::min(kMaxLanes, atoi(e)));
  RCHK(hipSetDevice(device));
  std::vector<void*>& K = r->scene_bufs;
  DObj* objs; DXform* xf; DSphere* sph; DRect* rct; DStandaloneTri* st; DMesh* me; float* nodes; float* n4;
  float* tp; TriShade* ts; DMedium* md; DMat* mt; DTex* tx; uint8_t* im; float* pr; int32_t* pp; DLight* li;
  DCamera* cm;
  DObvh* ob;
  DObvhChild* oc;
  DSGroup* sg;
  DSGItem* sgi;
  std::vector<DCamera> cam{F.cam};
  RCHK(upload(&objs, F.objs, K));
  RCHK(upload(&xf, F.xforms, K));
  RCHK(upload(&sph, F.spheres, K));
  RCHK(upload(&rct, F.rects, K));
  RCHK(upload(&st, F.stris, K));
  RCHK(upload(&me, F.meshes, K));
  RCHK(upload(&nodes, F.nodes, K));
  RCHK(upload(&n4, F.node4, K));
  float* n4q;
  RCHK(upload(&n4q, F.node4q, K));
  RCHK(upload(&tp, F.tri_pos, K));
  // the walk's leaf-pair records (kernels.h SceneView::tri_edge): record i (128 B) holds
  // p0, e1 = p1 - p0, e2 = p2 - p0 of triangles i and i+1 (the last repeats itself), the
  // float differences tri_hit's front test forms -- computed here, they round the same
  float* tedge;
  {
    const size_t nt = F.tri_pos.size() / 16;
    std::vector<float> pr(32 * nt, 0.f);
    for (size_t i = 0; i < nt; ++i)
      for (int j = 0; j < 2; ++j) {
        const float* q = &F.tri_pos[16 * std::min(i + j, nt - 1)];
        float* o = &pr[32 * i + 9 * j];
        for (int c = 0; c < 3; ++c) {
          o[c] = q[c];
          o[3 + c] = q[4 + c] - q[c];
          o[6 + c] = q[8 + c] - q[c];
        }
      }
    RCHK(upload(&tedge, pr, K));
  }
  RCHK(upload(&ts, F.tri_shade, K));
  RCHK(upload(&md, F.media, K));
  RCHK(upload(&ob, F.obvhs, K));
  RCHK(upload(&oc, F.obvh_children, K));
  RCHK(upload(&sg, F.sgroups, K));
  RCHK(upload(&sgi, F.sg_items, K));
  RCHK(upload(&mt, F.mats, K));
  RCHK(upload(&tx, F.texs, K));
  RCHK(upload(&im, F.images, K));
  RCHK(upload(&pr, F.perlin_ranvec, K));
  RCHK(upload(&pp, F.perlin_perm, K));
  RCHK(upload(&li, F.lights, K));
  RCHK(upload(&cm, cam, K));
  // world-traversal tables packed for LDS staging (kernels.h SceneView::world_blob)
  std::vector<uint8_t> blob;
  int off[10];
  auto put = [&](int k, const void* data, size_t bytes) {
    off[k] = (int)blob.size();
    blob.insert(blob.end(), (const uint8_t*)data, (const uint8_t*)data + bytes);
    blob.resize((blob.size() + 15) & ~(size_t)15, 0);
  };
  put(0, F.objs.data(), F.objs.size() * sizeof(DObj));
  put(1, F.xforms.data(), F.xforms.size() * sizeof(DXform));
  put(2, F.spheres.data(), F.spheres.size() * sizeof(DSphere));
  put(3, F.rects.data(), F.rects.size() * sizeof(DRect));
  put(4, F.stris.data(), F.stris.size() * sizeof(DStandaloneTri));
  put(5, F.meshes.data(), F.meshes.size() * sizeof(DMesh));
  put(6, F.media.data(), F.media.size() * sizeof(DMedium));
  put(7, F.mats.data(), F.mats.size() * sizeof(DMat));
  put(8, F.texs.data(), F.texs.size() * sizeof(DTex));
  put(9, F.lights.data(), F.lights.size() * sizeof(DLight));
  uint8_t* wb;
  RCHK(upload(&wb, blob, K));
  SceneView& V = r->view;
  V.world_blob = (const uint4*)wb;
  V.world_words = (int)(blob.size() / 16);
  for (int k = 0; k < 10; ++k) V.world_off[k] = off[k];
  V.objs = objs;
  V.n_world = F.n_world;
  V.has_media = F.media.empty() ? 0 : 1;
  V.xforms = xf;
  V.spheres = sph;
  V.rects = rct;
  V.stris = st;
  V.meshes = me;
  V.nodes = (const float4*)nodes;
  V.node4 = (const float4*)n4;
  V.node4_lds = (int)std::min<size_t>(kPathsLdsNodes, F.node4.size() / 32);
  V.node4_total = (int)(F.node4.size() / 32);
  V.node4q = F.node4q_ok && !F.node4q.empty() ? (const float4*)n4q : nullptr;
  V.node4_lds_q = (int)std::min<size_t>(2 * kPathsLdsNodes, F.node4q.size() / kNode4qWords);
  {  // compressed 64-B nodes for the per-lane mesh walks (SRR_CBVH=0/1)
    const char* e = getenv("SRR_CBVH");
    V.use_q = V.node4q && e && atoi(e) != 0;
  }
  // Quad-cooperative mesh traversal (SRR_QUAD=1; off by default).  In round 2 it
  // paid on the 640,000-triangle teapot (1,054 -> 1,573 Msamples/s), but most of
  // that came from sharing the whole-tree walks of NaN-bound rays over a quad;
  // with those folded cooperatively (kernels.hip mesh_scan_nan) the per-lane walk
  // is faster there too: 5,384 vs 5,170 Msamples/s.
  {
    const char* e = getenv("SRR_QUAD");
    V.quad_trace = e ? (atoi(e) != 0) : false;
    const char* q = getenv("SRR_QUAD_MAX");
    V.quad_max = q ? atoi(q) : 32;  // 640k-tri teapot: 16 -> 1,569, 32 -> 1,598, 64 -> 1,552 Msamples/s
  }
  {  // one mesh at the top of the world list: k_paths compacts its traversals block-wide
    int n_mesh = 0;
    V.mesh_obj = -1;
    for (int k = 0; k < F.n_world; ++k)
      if (F.objs[k].kind == OBJ_MESH) {
        ++n_mesh;
        V.mesh_obj = k;
      }
    if (n_mesh != 1) V.mesh_obj = -1;
  }
  V.tri_pos = (const float4*)tp;
  V.tri_edge = (const float4*)tedge;
  V.tri_shade = ts;
  V.media = md;
  V.obvhs = ob;
  V.obvh_children = oc;
  V.sgroups = sg;
  V.sg_items = sgi;
  V.mats = mt;
  V.texs = tx;
  V.images = im;
  V.perlin_ranvec = pr;
  V.perlin_perm = pp;
  V.lights = li;
  V.n_lights = (int)F.lights.size();
  V.light_weight = V.n_lights > 0 ? (float)(1.0 / V.n_lights) : 0.f;
  V.cam = cm;
  r->has_meshes = !F.meshes.empty() || !F.obvhs.empty();
  r->diffuse_only = true;
  for (const DMat& m : F.mats)
    if (m.kind != MAT_LAMBERTIAN && m.kind != MAT_ORENNAYAR && m.kind != MAT_DIFFUSE_LIGHT) r->diffuse_only = false;
  // suspendable mesh walks by default (SRR_WALK_Q unset) where they were
  // measured to pay: specular / microfacet materials or media (walks from surfaces inside
  // the mesh's box run long: C3 +2 %, C4 +4 %, C4_real +3 %, C5 +6 %) or a large mesh (the
  // 640,000-triangle teapot +3 %); not for a diffuse-only scene with a small mesh, whose
  // walks are short (C2: the suspension check costs 0.5-1 % and gains nothing)
  {
    int max_tris = 0;
    for (const DMesh& m : F.meshes) max_tris = std::max(max_tris, (int)m.n_tris);
    r->walk_q_default = (!F.meshes.empty() && (!r->diffuse_only || V.has_media || max_tris >= 20000)) ? 8 : 0;
  }
  RCHK(hipStreamCreateWithFlags(&r->acc_st, hipStreamNonBlocking));
  RCHK(hipEventCreate(&r->ev_beg));
  RCHK(hipEventCreate(&r->ev_end));
  RCHK(hipEventCreateWithFlags(&r->ev_async_in, hipEventDisableTiming));
  for (int l = 0; l < kMaxLanes; ++l) {
    Lane& L = r->lanes[l];
    RCHK(hipStreamCreateWithFlags(&L.st, hipStreamNonBlocking));
    RCHK(hipEventCreate(&L.ev_t0));
    RCHK(hipEventCreate(&L.ev_t1));
    RCHK(hipEventCreate(&L.ev_s1));
    RCHK(hipEventCreateWithFlags(&L.ev_rb, hipEventDisableTiming));
    for (int k = 0; k < kRegionsPerLane; ++k) {
      RCHK(hipEventCreateWithFlags(&L.done_ev[k], hipEventDisableTiming));
      RCHK(hipEventCreateWithFlags(&L.acc_ev[k], hipEventDisableTiming));
    }
    RCHK(hipMalloc((void**)&L.cnt, 16 * sizeof(int32_t)));
    RCHK(hipHostMalloc((void**)&L.rb, 16 * sizeof(int32_t)));
  }
  *out = r.release();
  return 0;
}

static void free_lane_paths(Lane& L) {
  for (void* p : L.bufs) (void)hipFree(p);
  L.bufs.clear();
  L.cap = 0;
  L.P = PathState{};
  L.act[0] = L.act[1] = nullptr;
  L.lists = nullptr;
}

template <class T>
static hipError_t lane_alloc(Lane& L, T** p, size_t n) {
  hipError_t e = hipMalloc((void**)p, std::max<size_t>(n * sizeof(T), 16));
  if (e == hipSuccess) L.bufs.push_back(*p);
  return e;
}

static int ensure_lane(Lane& L, size_t n, int depth, bool keep, std::string& err) {
  int d = std::max(depth, 1);
  if (n <= L.cap && d <= L.cap_depth && (!keep || L.has_raw)) return 0;
  free_lane_paths(L);
  PathState& P = L.P;
  RCHK(lane_alloc(L, &P.ray_o, n));
  RCHK(lane_alloc(L, &P.ray_d, n));
  RCHK(lane_alloc(L, &P.lcg, n));
  RCHK(lane_alloc(L, &P.pcg, n));
  RCHK(lane_alloc(L, &P.depth, n));
  RCHK(lane_alloc(L, &P.spec, n));
  RCHK(lane_alloc(L, &P.hit_w, n));
  RCHK(lane_alloc(L, &P.hit_p, n));
  RCHK(lane_alloc(L, &P.hit_n, n));
  RCHK(lane_alloc(L, &P.rec_a, n * d));
  RCHK(lane_alloc(L, &P.sample, 3 * n));
  RCHK(lane_alloc(L, &L.lists, 4 * n));
  RCHK(lane_alloc(L, &L.act[0], n));
  RCHK(lane_alloc(L, &L.act[1], n));
  L.has_raw = keep;
  if (keep) {
    RCHK(lane_alloc(L, &P.raw, 3 * n));
    RCHK(lane_alloc(L, &P.rays, n));
  }
  L.cap = n;
  L.cap_depth = d;
  return 0;
}

// Per-pixel running sums: zeroed by a render without SRR_FLAG_CONTINUE; a render
// with it adds its samples to them, so consecutive sample ranges accumulate in
// sample order -- bitwise the sums of one render of all of them.
static void accum_key(const srr_params* p, int key[5]) {
  const bool whole = p->shard_count <= 1;
  key[0] = p->nx;
  key[1] = p->ny;
  key[2] = whole ? 0 : p->shard_index;
  key[3] = whole ? 1 : p->shard_count;
  key[4] = whole ? 0 : p->tile;
}

// zero_pending (optional): the caller zeroes the sums itself (its first
// accumulation starts from 0) instead of a memset here
static int begin_accum(srr_renderer* r, const srr_params* p, int64_t npix, hipStream_t st, std::string& err,
                       bool* zero_pending = nullptr) {
  if (zero_pending) *zero_pending = false;
  int key[5];
  accum_key(p, key);
  if (p->flags & SRR_FLAG_CONTINUE) {
    if (r->acc_npix != npix) {
      err = "SRR_FLAG_CONTINUE: no running sums for this shard (render without the flag or srr_accum_set first)";
      return SRR_EINVAL;
    }
    if (p->sample_begin != r->acc_samples) {
      err = "SRR_FLAG_CONTINUE: sample_begin " + std::to_string(p->sample_begin) + " != the " +
            std::to_string(r->acc_samples) + " samples already in the running sums";
      return SRR_EINVAL;
    }
    if (r->acc_key[0] >= 0 && !std::equal(key, key + 5, r->acc_key)) {
      err = "SRR_FLAG_CONTINUE: the running sums belong to another frame or shard";
      return SRR_EINVAL;
    }
    std::copy(key, key + 5, r->acc_key);
    return 0;
  }
  if (zero_pending) *zero_pending = true;
  else RCHK(hipMemsetAsync(r->acc, 0, 3 * npix * sizeof(float), st));
  r->acc_npix = npix;
  r->acc_samples = 0;
  std::copy(key, key + 5, r->acc_key);
  return 0;
}

// Stages a shard's pixel list on the device (with the frame accumulator sized
// to it); an identity list is not uploaded (the path engine does not read it).
static hipError_t stage_pixels(srr_renderer* r, const int32_t* pix, int64_t npix, bool identity) {
  r->pix_key[0] = -1;  // srr_render_device sets the key once the render succeeds
  if ((size_t)npix > r->pix_cap) {
    (void)hipFree(r->pixels);
    (void)hipFree(r->acc);
    r->pixels = nullptr;
    r->acc = nullptr;
    r->pix_cap = 0;
    // the running sums went with the old buffer: nothing may continue them
    r->acc_npix = 0;
    r->acc_samples = 0;
    std::fill(r->acc_key, r->acc_key + 5, -1);
    hipError_t e = hipMalloc((void**)&r->pixels, npix * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&r->acc, 3 * npix * sizeof(float));
    if (e != hipSuccess) return e;
    r->pix_cap = npix;
  }
  r->pix_identity = identity;
  return identity ? hipSuccess : hipMemcpy(r->pixels, pix, npix * sizeof(int32_t), hipMemcpyHostToDevice);
}

// The device Sobol set holds the first sobol_n points; the set is a
// prefix-stable sequence (tests/test_dist_gloo.py), so it is generated and
// uploaded only when a render needs more points than it holds.
static hipError_t ensure_sobol(srr_renderer* r, int n_sobol) {
  if (n_sobol <= r->sobol_n) return hipSuccess;
  (void)hipFree(r->sobol);
  r->sobol = nullptr;
  r->sobol_n = 0;
  hipError_t e = hipMalloc((void**)&r->sobol, 2 * (size_t)n_sobol * sizeof(double));
  if (e != hipSuccess) return e;
  std::vector<double> sp(2 * (size_t)n_sobol);
  sobol2((unsigned)n_sobol, sp.data());
  e = hipMemcpy(r->sobol, sp.data(), sp.size() * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) r->sobol_n = n_sobol;
  return e;
}

// Invalidates the running sums unless the render that began them committed:
// a failed render leaves partial sums that no SRR_FLAG_CONTINUE may build on.
struct AccCommit {
  srr_renderer* r;
  bool ok = false;
  ~AccCommit() {
    if (!ok) r->acc_npix = 0;
  }
};

// The stream, buffers and events of one path-engine frame (renderer.h FrameSlot):
// created on first use, grown as frames need.
static int slot_init(FrameSlot& F, hipStream_t shared_st, std::string& err) {
  if (F.ev_beg) return 0;
  if (shared_st) {
    F.st = shared_st;
  } else {
    RCHK(hipStreamCreateWithFlags(&F.st, hipStreamNonBlocking));
    F.own_stream = true;
  }
  RCHK(hipEventCreate(&F.ev_beg));
  RCHK(hipEventCreate(&F.ev_end));
  RCHK(hipMalloc((void**)&F.ctr, kCtrWords * sizeof(unsigned long long)));
  RCHK(hipHostMalloc((void**)&F.ctr_host, kCtrWords * sizeof(unsigned long long)));
  return 0;
}

void slot_free(FrameSlot& F) {
  (void)hipFree(F.rec);
  (void)hipFree(F.gstack);
  (void)hipFree(F.sample);
  (void)hipFree(F.ctr);
  (void)hipFree(F.acc);
  if (F.ctr_host) (void)hipHostFree(F.ctr_host);
  for (hipEvent_t e : F.win_ev) (void)hipEventDestroy(e);
  if (F.ev_beg) (void)hipEventDestroy(F.ev_beg);
  if (F.ev_end) (void)hipEventDestroy(F.ev_end);
  if (F.own_stream && F.st) (void)hipStreamDestroy(F.st);
  F = FrameSlot{};
}

// frees a slot's sample window (the largest per-frame buffer); the next frame
// on the slot allocates it again
static void release_window(FrameSlot& F) {
  if (!F.sample) return;
  (void)hipFree(F.sample);
  F.sample = nullptr;
  F.sample_cap = 0;
}

// Path-resident engine (kernels.hip k_paths): one persistent kernel per window
// of samples; samples land in a [pixel][sample] buffer that k_accumulate_window
// sums per pixel in sample order, so the image is bitwise the wavefront engine's.
// paths_enqueue puts a whole frame on slot F's stream (sums in `acc`, zeroed by
// the first window when `zero_pending`); paths_finish waits for it and reads its
// counters.  The caller has staged the pixel list and the Sobol set.
static int paths_enqueue(srr_renderer* r, FrameSlot& F, const srr_params* p, bool identity, int64_t npix,
                         float* acc, bool zero_pending, int64_t acc_total, float* d_mean, bool diagnostics,
                         std::string& err) {
  const bool keep = (p->flags & SRR_FLAG_KEEP_PATHS) != 0;
  hipStream_t st = F.st;
  // persistent lanes and their bounce records
  if (!r->pw_lanes) r->pw_lanes = paths_lanes_per_device(r->view, r->device);
  const size_t rec_need = (size_t)r->pw_lanes * std::max(1, p->max_depth);
  if (rec_need > F.rec_cap) {
    (void)hipFree(F.rec);
    F.rec = nullptr;
    F.rec_cap = 0;
    RCHK(hipMalloc((void**)&F.rec, rec_need * sizeof(float4)));
    F.rec_cap = rec_need;
  }
  // global extension of the BVH4 traversal stack, for meshes deep enough to need it
  // (SRR_GSTACK=0 disables it: every deeper traversal then re-walks the BVH2)
  const char* gs_env = getenv("SRR_GSTACK");
  const int gst_cap = (r->has_meshes && !(gs_env && !atoi(gs_env))) ? kPathsGlobalStack : 0;
  // ... followed by the save area of suspended mesh walks (3 float4 per lane)
  if (gst_cap && !F.gstack)
    RCHK(hipMalloc((void**)&F.gstack, (size_t)gst_cap * r->pw_lanes * sizeof(int2) + 3 * (size_t)r->pw_lanes * sizeof(float4)));
  // suspendable mesh walks: a walk still running when at most SRR_WALK_Q / 64
  // of its wave's lanes walk continues in the next wave-iteration (default: the scene's
  // walk_q_default, 8 or 0); SRR_WALK_Q=0 never suspends and launches the kernel variant
  // without the feature (read per frame: tests switch it between renders)
  const char* wq_env = getenv("SRR_WALK_Q");
  const int walk_q = wq_env ? std::max(0, std::min(64, atoi(wq_env))) : r->walk_q_default;
  // sample window: all pixels x W samples, buffer within SRR_WINDOW_MB (default 16384: a
  // 1080p frame of 1,024 spp in 2 windows, not 3 -- one drain and one serial accumulation
  // fewer)
  size_t budget = (size_t)16384 << 20;
  if (const char* e = getenv("SRR_WINDOW_MB")) budget = (size_t)std::max(1, atoi(e)) << 20;
  budget /= (size_t)std::max(1, r->window_share);
  // (k_paths numbers a window's paths in 32 bits: npix * W < 2^31)
  const int64_t w_max = std::max<int64_t>(1, (((int64_t)1 << 31) - 1) / std::max<int64_t>(1, npix));
  int W = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::min<int64_t>(p->spp, w_max), (int64_t)(budget / (12 * (size_t)npix))));
  // a window of a multiple of 4 samples is summed with 16-byte loads (k_accumulate_window16;
  // 1080p: 345 -> 344 samples, still 3 windows of 1,024); the sums do not depend on W
  if (W < p->spp && W >= 16) W &= ~3;
  if ((int64_t)npix * W >= ((int64_t)1 << 31)) {
    err = "frame too large for one sample window (npix >= 2^31)";
    return SRR_EINVAL;
  }
  const size_t win_paths = (size_t)npix * W;
  if (win_paths > F.sample_cap) {
    (void)hipFree(F.sample);
    F.sample = nullptr;
    F.sample_cap = 0;
    hipError_t e = hipMalloc((void**)&F.sample, win_paths * 3 * sizeof(float));
    if (e == hipErrorOutOfMemory) {
      // the synchronous slot and the two async slots each keep their window across
      // mode switches (at most 3 x SRR_WINDOW_MB of the 288 GB); only when the device
      // runs out are the other mode's windows given back
      (void)hipGetLastError();
      if (&F == &r->sync_slot) {
        drain_async(r);
        for (FrameSlot& A : r->async_slots) release_window(A);
      } else {
        release_window(r->sync_slot);
      }
      e = hipMalloc((void**)&F.sample, win_paths * 3 * sizeof(float));
    }
    RCHK(e);
    F.sample_cap = win_paths;
  }
  RCHK(hipMemsetAsync(F.ctr, 0, kCtrWords * sizeof(unsigned long long), st));
  const bool want_sums = (p->flags & SRR_FLAG_SUMS) != 0;
  // per-window HIP events around k_paths, read once the frame is done (no host
  // round trip between windows)
  const int n_windows = (p->spp + W - 1) / W;
  while ((int)F.win_ev.size() < 2 * n_windows) {
    hipEvent_t e;
    RCHK(hipEventCreate(&e));
    F.win_ev.push_back(e);
  }
  F.n_windows = n_windows;
  const bool all_fam = !r->diffuse_only;
  // diagnostics (SRR_WAVE_TIMES=1): per-wave start / exit times of each k_paths launch
  static const bool want_wave_times = getenv("SRR_WAVE_TIMES") != nullptr;
  unsigned long long* wave_times = nullptr;
  const int n_waves = (r->pw_lanes + 63) / 64;
  if (want_wave_times && diagnostics) {  // owned by the renderer (freed in ~srr_renderer), so no early return leaks it
    if (!r->pw_wave_times) RCHK(hipMalloc((void**)&r->pw_wave_times, 4 * (size_t)n_waves * sizeof(unsigned long long)));
    wave_times = r->pw_wave_times;
    RCHK(hipMemsetAsync(wave_times, 0, 4 * (size_t)n_waves * sizeof(unsigned long long), st));
  }
  // attempts after which a pending resampling loop takes every free lane of its
  // wave (kernels.hip coop_mixture); SRR_DEEP_TRIES=0 forces that branch (tests)
  const char* dt_env = getenv("SRR_DEEP_TRIES");
  const int deep_tries = dt_env ? std::max(0, atoi(dt_env)) : 32;
#ifdef SRR_SLOW_RAYS
  if (!r->pw_slow) RCHK(hipMalloc((void**)&r->pw_slow, (16 * 65536 + 16) * sizeof(float)));
  RCHK(hipMemsetAsync(r->pw_slow + 16 * 65536, 0, 16 * sizeof(float), st));
#endif
  RCHK(hipEventRecord(F.ev_beg, st));
  for (int s0 = 0; s0 < p->spp; s0 += W) {
    const int Wn = std::min(W, p->spp - s0);
    PathWork w{};
    w.pixels = identity ? nullptr : r->pixels;
    w.sobol = r->sobol + 2 * (size_t)(p->sample_begin + s0);
    w.npix = (int)npix;
    w.spp_w = Wn;
    w.s_base = p->sample_begin + s0;
    w.nx = p->nx;
    w.ny = p->ny;
    w.div_spp = make_udiv31((uint32_t)Wn);
    w.div_nx = make_udiv31((uint32_t)p->nx);
    w.base_seed = p->base_seed;
    w.n_paths = (int64_t)npix * Wn;
    w.max_depth = p->max_depth;
    w.cursor = F.ctr + 1;
    w.counters = F.ctr;
    w.sample = F.sample;
    w.raw = keep ? r->raw_all : nullptr;
    w.rays = keep ? r->rays_all : nullptr;
    w.keep_spp = p->spp;
    w.keep_s0 = s0;
    w.rec = F.rec;
    w.err = (int*)(F.ctr + 2);
    const int64_t bl = paths_block_lanes(r->view);  // whole blocks of the launch's size
    w.lanes = (int)std::min<int64_t>(r->pw_lanes, ((w.n_paths + bl - 1) / bl) * bl);
    w.stack_cap = kPathsLdsStack;  // kernels.hip kStack
    if (const char* e = getenv("SRR_STACK_CAP")) w.stack_cap = std::max(1, std::min(kPathsLdsStack, atoi(e)));
    w.gstack = gst_cap ? F.gstack : nullptr;
    w.gstack_cap = gst_cap;
    w.wave_times = wave_times;
    w.deep_tries = deep_tries;
    w.walk_q = gst_cap ? walk_q : 0;  // (the save area follows the global stack extension)
    w.slow_rays = diagnostics ? r->pw_slow : nullptr;
    w.slow_count = w.slow_rays ? (unsigned*)(r->pw_slow + 16 * 65536) : nullptr;
    const int wi = s0 / W;
    if (wi > 0) RCHK(hipMemsetAsync(w.cursor, 0, sizeof(unsigned long long), st));  // window 0: zeroed with ctr
    RCHK(hipEventRecord(F.win_ev[2 * wi], st));
    if (launch_paths(r->view, w, all_fam ? 1 : 0, st) != 0) {
      err = "k_paths refused: stack_cap " + std::to_string(w.stack_cap) +
            " exceeds the kernel build's LDS stack (a host and kernels built with different SRR_KSTACK)";
      return SRR_EINVAL;
    }
    RCHK(hipEventRecord(F.win_ev[2 * wi + 1], st));
    // the last window also writes the output (k_finish fused): means, or raw sums (SRR_FLAG_SUMS)
    const bool last = s0 + Wn >= p->spp;
    launch_accumulate_window(F.sample, (int)npix, Wn, acc, st, wi == 0 && zero_pending, last ? d_mean : nullptr,
                             want_sums ? 0 : (int)acc_total);
    if (wave_times) {  // realtime clock: 100 MHz (10 ns ticks)
      RCHK(hipEventSynchronize(F.win_ev[2 * wi + 1]));
      float ms = 0;
      RCHK(hipEventElapsedTime(&ms, F.win_ev[2 * wi], F.win_ev[2 * wi + 1]));
      std::vector<unsigned long long> wt(4 * (size_t)n_waves);
      RCHK(hipMemcpy(wt.data(), wave_times, wt.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      std::vector<std::pair<double, int>> ex;
      unsigned long long t0 = ~0ull;
      for (int i = 0; i < n_waves; ++i)
        if (wt[4 * i + 1]) t0 = std::min(t0, wt[4 * i]);
      for (int i = 0; i < n_waves; ++i)
        if (wt[4 * i + 1]) ex.push_back({(wt[4 * i + 1] - t0) * 1e-5, i});  // ms
      std::sort(ex.begin(), ex.end());
      if (!ex.empty()) {
        auto q = [&](double f) { return ex[std::min(ex.size() - 1, (size_t)(f * ex.size()))].first; };
        fprintf(stderr, "k_paths wave exits (ms after the first wave start, %zu waves, kernel %.3f ms): "
                "min %.3f p10 %.3f p50 %.3f p90 %.3f p99 %.3f max %.3f\n", ex.size(), ms, ex.front().first, q(0.1),
                q(0.5), q(0.9), q(0.99), ex.back().first);
        // per wave: start, exit, world rays, wave-iterations, most mixture rounds in one iteration
        auto show = [&](const char* what, int i) {
          fprintf(stderr, "  %s wave %d: start %.3f exit %.3f rays %llu iterations %llu max mixture rounds %llu\n", what,
                  i, (wt[4 * i] - t0) * 1e-5, (wt[4 * i + 1] - t0) * 1e-5, wt[4 * i + 2], wt[4 * i + 3] & 0xffffffffull,
                  wt[4 * i + 3] >> 32);
        };
        show("median", ex[ex.size() / 2].second);
        for (size_t k = ex.size() - std::min<size_t>(4, ex.size()); k < ex.size(); ++k) show("late", ex[k].second);
      }
      RCHK(hipMemsetAsync(wave_times, 0, wt.size() * sizeof(unsigned long long), st));
    }
  }
  if (n_windows == 0) {  // spp 0: nothing rendered, the output is the sums as they stand
    if (want_sums)
      RCHK(hipMemcpyAsync(d_mean, acc, 3 * (size_t)npix * sizeof(float), hipMemcpyDeviceToDevice, st));
    else
      launch_finish(acc, d_mean, npix, (int)acc_total, st);
  }
  RCHK(hipMemcpyAsync(F.ctr_host, F.ctr, kCtrWords * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  RCHK(hipEventRecord(F.ev_end, st));
  F.npix = npix;
  F.paths = npix * p->spp;
  return 0;
}

static int paths_finish(srr_renderer* r, FrameSlot& F, const srr_params* p, srr_stats* stats, std::string& err) {
  RCHK(hipStreamSynchronize(F.st));
  RCHK(hipGetLastError());
  srr_stats s{};
  double kernel_ms = 0;
  for (int wi = 0; wi < F.n_windows; ++wi) {
    float ms = 0;
    RCHK(hipEventElapsedTime(&ms, F.win_ev[2 * wi], F.win_ev[2 * wi + 1]));
    kernel_ms += ms;
  }
  unsigned long long ctr[kCtrWords];
  std::memcpy(ctr, F.ctr_host, sizeof(ctr));
  if (getenv("SRR_PATHS_TIMING") && ctr[9]) {
    const double it = (double)ctr[9];
    fprintf(stderr, "k_paths per wave-iteration (ticks): refill %.0f  world %.0f  mesh %.0f  record %.0f  scatter %.0f  fold %.0f  (%llu wave-iterations)\n",
            ctr[4] / it, ctr[5] / it, ctr[6] / it, ctr[10] / it, (ctr[7] - ctr[10]) / it, ctr[8] / it, ctr[9]);
    fprintf(stderr, "  scatter: mixture loop %.0f ticks, %.2f rounds per wave-iteration\n", ctr[13] / it, ctr[14] / it);
    auto per = [](unsigned long long a, unsigned long long b) { return b ? (double)a / (double)b : 0.0; };
    fprintf(stderr, "  families: beck %.0f ticks/it (runs in %.1f %% of its, %.1f lanes/run), spec %.0f (%.1f %%, %.1f), "
                    "diff set-up %.0f (%.1f %%, %.1f); lanes in a path %.1f of 64\n",
            ctr[16] / it, 100 * ctr[19] / it, per(ctr[22], ctr[19]), ctr[17] / it, 100 * ctr[20] / it,
            per(ctr[23], ctr[20]), ctr[18] / it, 100 * ctr[21] / it, per(ctr[24], ctr[21]), ctr[25] / it);
    fprintf(stderr, "  mesh: longest walk %.1f node steps/it, %.1f lane steps/it over %.1f walking lanes, "
                    "%.0f ticks per step of the longest walk\n",
            ctr[26] / it, ctr[27] / it, ctr[28] / it, per(ctr[6], ctr[26]));
    fprintf(stderr, "  mesh leaf queue: %.0f ticks/it, %.1f passes/it (%.0f ticks per pass)\n", ctr[29] / it,
            ctr[30] / it, per(ctr[29], ctr[30]));
    fprintf(stderr, "  mesh step parts (ticks/it): node fetch %.0f  slab + queue %.0f  order + push + pop %.0f\n",
            ctr[31] / it, ctr[32] / it, ctr[33] / it);
    fprintf(stderr, "  beckmann mixture: %.2f attempts per Beckmann scatter, %.2f for the wave's slowest lane per run\n",
            per(ctr[34], ctr[22]), per(ctr[35], ctr[19]));
    fprintf(stderr, "  suspended walks: %.2f lanes per wave-iteration\n", ctr[36] / it);
  }
#ifdef SRR_SLOW_RAYS
  if (r->pw_slow) {  // diagnostics build: dump the slow world hits' records (one line per lane, JSON)
    unsigned n = 0;
    RCHK(hipMemcpy(&n, r->pw_slow + 16 * 65536, sizeof(unsigned), hipMemcpyDeviceToHost));
    n = std::min(n, 65536u);
    std::vector<float> v(16 * (size_t)n);
    if (n) RCHK(hipMemcpy(v.data(), r->pw_slow, v.size() * sizeof(float), hipMemcpyDeviceToHost));
    auto I = [&](size_t k) { int x; memcpy(&x, &v[k], 4); return x; };
    for (unsigned i = 0; i < n; ++i) {
      const size_t b = 16 * (size_t)i;
      fprintf(stderr, "SLOWRAY {\"g\": %d, \"depth\": %d, \"o\": [%.9g, %.9g, %.9g], \"d\": [%.9g, %.9g, %.9g], "
              "\"tm\": %.9g, \"ticks\": %d, \"steps\": %d, \"obj\": %d, \"prim\": %d, \"t\": %.9g, \"slot\": %d, "
              "\"t0\": %d, \"spp_w\": %d}\n", I(b), I(b + 1), v[b + 2], v[b + 3], v[b + 4], v[b + 5], v[b + 6], v[b + 7], v[b + 8],
              I(b + 9), I(b + 10), I(b + 11), I(b + 12), v[b + 13], I(b + 14), I(b + 15), p->spp);
    }
  }
#else
  (void)r;
  (void)p;
#endif
  if (ctr[2]) {
    err = "k_paths index guard tripped (bits " + std::to_string(ctr[2]) + ")";
    return SRR_EIO;
  }
  float total = 0;
  RCHK(hipEventElapsedTime(&total, F.ev_beg, F.ev_end));
  s.world_rays = (int64_t)ctr[0];
  s.stack_overflows = (int64_t)ctr[11];
  s.deep_traversals = (int64_t)ctr[12];
  s.mixture_capped = (int64_t)ctr[15];
  s.walks_suspended = (int64_t)ctr[36];
  s.paths = F.paths;
  s.trace_ms = kernel_ms;
  s.total_ms = total;
  s.trace_launches = F.n_windows;
  if (stats) *stats = s;
  return 0;
}

static void finish_slot(srr_renderer* r, FrameSlot& F) {
  F.busy = false;
  srr_params none{};
  F.rc = paths_finish(r, F, &none, &F.stats, F.err);
  r->done_tickets.push_back({F.ticket, F.rc, F.stats, F.err});
}

// Frames in flight read the shard's pixel list and the Sobol set: anything that
// reallocates them waits for those frames first (their stats stay for srr_render_wait).
void drain_async(srr_renderer* r) {
  for (FrameSlot& F : r->async_slots)
    if (F.busy) finish_slot(r, F);
}

static int paths_stage(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, bool& identity,
                       std::string& err) {
  identity = r->pix_identity;
  if (pix != nullptr || p->sample_begin + p->spp > r->sobol_n) drain_async(r);
  if (pix) {  // a new pixel list (else the renderer holds this shard's already)
    identity = p->shard_count <= 1;
    for (int64_t i = 0; identity && i < npix; i += std::max<int64_t>(1, npix / 64)) identity = pix[i] == i;
    RCHK(stage_pixels(r, pix, npix, identity));
  }
  RCHK(ensure_sobol(r, p->sample_begin + p->spp));
  return 0;
}

static int render_paths(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, float* d_mean,
                        srr_stats* stats, std::string& err) {
  const bool keep = (p->flags & SRR_FLAG_KEEP_PATHS) != 0;
  bool identity = false;
  {
    const int rc = paths_stage(r, p, pix, npix, identity, err);
    if (rc < 0) return rc;
  }
  if (keep) {
    size_t need = (size_t)npix * p->spp;
    if (need > r->keep_cap) {
      (void)hipFree(r->raw_all);
      (void)hipFree(r->rays_all);
      RCHK(hipMalloc((void**)&r->raw_all, need * 3 * sizeof(float)));
      RCHK(hipMalloc((void**)&r->rays_all, need));
      r->keep_cap = need;
    }
    r->kept_paths = (int64_t)need;
  }
  FrameSlot& F = r->sync_slot;
  {
    const int rc = slot_init(F, r->acc_st, err);
    if (rc < 0) return rc;
  }
  // the sums of a fresh frame are zeroed by the first window's accumulation (init)
  bool zero_pending = false;
  {
    const int rc = begin_accum(r, p, npix, F.st, err, p->spp > 0 ? &zero_pending : nullptr);
    if (rc < 0) return rc;
  }
  AccCommit commit{r};
  const int64_t acc_total = r->acc_samples + p->spp;
  {
    const int rc = paths_enqueue(r, F, p, identity, npix, r->acc, zero_pending, acc_total, d_mean, true, err);
    if (rc < 0) {
      (void)hipStreamSynchronize(F.st);  // windows already enqueued must not outlive the error
      return rc;
    }
  }
  {
    const int rc = paths_finish(r, F, p, stats, err);
    if (rc < 0) return rc;
  }
  r->acc_samples = acc_total;
  commit.ok = true;
  return 0;
}

// srr_render_device_async: a fresh frame (no CONTINUE, KEEP_PATHS, COUNT_VISITS or
// wavefront engine) on one of the renderer's two frame slots, each with its own
// stream, sums and buffers, so the next frame's persistent blocks take the CUs
// the previous frame's drain frees.  Returns at once; srr_render_wait reads it.
int render_device_async(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, float* d_mean,
                        int64_t* ticket, std::string& err) {
  if (p->flags & (SRR_FLAG_CONTINUE | SRR_FLAG_KEEP_PATHS | SRR_FLAG_COUNT_VISITS | SRR_FLAG_WAVEFRONT)) {
    err = "srr_render_device_async: fresh path-engine frames only (no CONTINUE, KEEP_PATHS, COUNT_VISITS, WAVEFRONT)";
    return SRR_EINVAL;
  }
  if (const char* e = getenv("SRR_ENGINE"); e && !strcmp(e, "wave")) {
    err = "srr_render_device_async: SRR_ENGINE=wave is synchronous only";
    return SRR_EINVAL;
  }
  RCHK(hipSetDevice(r->device));
  FrameSlot& F = r->async_slots[r->next_ticket % 2];
  if (F.busy) finish_slot(r, F);  // the slot's previous frame has not been waited for: finish it now
  bool identity = false;
  {
    const int rc = paths_stage(r, p, pix, npix, identity, err);
    if (rc < 0) return rc;
  }
  {
    const int rc = slot_init(F, nullptr, err);
    if (rc < 0) return rc;
  }
  if ((size_t)npix > F.acc_cap) {
    (void)hipFree(F.acc);
    F.acc = nullptr;
    F.acc_cap = 0;
    RCHK(hipMalloc((void**)&F.acc, 3 * (size_t)npix * sizeof(float)));
    F.acc_cap = npix;
  }
  // the caller's stream order: the frame starts after what the legacy stream holds
  RCHK(hipEventRecord(r->ev_async_in, nullptr));
  RCHK(hipStreamWaitEvent(F.st, r->ev_async_in, 0));
  {
    const int rc = paths_enqueue(r, F, p, identity, npix, F.acc, true, p->spp, d_mean, false, err);
    if (rc < 0) {
      // windows already on F.st read the slot's buffers: drain them before the slot is reused
      (void)hipStreamSynchronize(F.st);
      return rc;
    }
  }
  F.ticket = r->next_ticket++;
  F.busy = true;
  *ticket = F.ticket;
  return 0;
}

hipEvent_t render_ticket_event(srr_renderer* r, int64_t ticket) {
  for (FrameSlot& F : r->async_slots)
    if (F.busy && F.ticket == ticket) return F.ev_end;
  return nullptr;
}

int render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats, std::string& err) {
  RCHK(hipSetDevice(r->device));
  for (size_t k = 0; k < r->done_tickets.size(); ++k)
    if (r->done_tickets[k].ticket == ticket) {
      const DoneTicket d = r->done_tickets[k];
      r->done_tickets.erase(r->done_tickets.begin() + k);
      if (stats) *stats = d.stats;
      err = d.err;
      return d.rc;
    }
  for (FrameSlot& F : r->async_slots)
    if (F.busy && F.ticket == ticket) {
      F.busy = false;
      srr_params none{};
      return paths_finish(r, F, &none, stats, err);
    }
  err = "srr_render_wait: unknown or already waited ticket " + std::to_string(ticket);
  return SRR_EINVAL;
}

int render_device(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, float* d_mean,
                  srr_stats* stats, std::string& err) {
  static const bool wave_env = [] {
    const char* e = getenv("SRR_ENGINE");
    return e && !strcmp(e, "wave");
  }();
  const bool wave_engine = wave_env || (p->flags & SRR_FLAG_WAVEFRONT);
  // every buffer either engine allocates belongs to the renderer's device,
  // whatever device the caller has current
  RCHK(hipSetDevice(r->device));
  // the path engine stages the world tables in LDS when they fit
  // (kernels.hip kWorldLdsBytes) and reads them from global memory otherwise
  if (!wave_engine && !(p->flags & SRR_FLAG_COUNT_VISITS))
    return render_paths(r, p, pix, npix, d_mean, stats, err);
  drain_async(r);  // the wavefront engine restages the pixel list
  const bool keep = (p->flags & SRR_FLAG_KEEP_PATHS) != 0;
  const int R = kRegionsPerLane;
  hipStream_t ast = r->acc_st;
  unsigned long long* visits = nullptr;
  if (p->flags & SRR_FLAG_COUNT_VISITS) {
    if (!r->visits) RCHK(hipMalloc((void**)&r->visits, kVisitWords * sizeof(unsigned long long)));
    RCHK(hipMemset(r->visits, 0, kVisitWords * sizeof(unsigned long long)));
    visits = r->visits;
  }
  // frame buffers
  if (pix) RCHK(stage_pixels(r, pix, npix, false));
  else if (r->pix_identity) {  // the path engine skipped the upload of an identity list
    std::vector<int32_t> id((size_t)npix);
    for (int64_t i = 0; i < npix; ++i) id[i] = (int32_t)i;
    RCHK(stage_pixels(r, id.data(), npix, false));
  }
  // Sobol points of the global sample range [sample_begin, sample_begin + spp):
  // the set is a prefix-stable sequence, so a sample shard reads its own slice.
  RCHK(ensure_sobol(r, p->sample_begin + p->spp));
  if (keep) {
    size_t need = (size_t)npix * p->spp;
    if (need > r->keep_cap) {
      (void)hipFree(r->raw_all);
      (void)hipFree(r->rays_all);
      RCHK(hipMalloc((void**)&r->raw_all, need * 3 * sizeof(float)));
      RCHK(hipMalloc((void**)&r->rays_all, need));
      r->keep_cap = need;
    }
    r->kept_paths = (int64_t)need;
  }
  // Batches: (pixel chunk, sample chunk) in the order every pixel must see its
  // samples accumulated.
  int64_t N = p->batch_paths > 0 ? p->batch_paths : (int64_t)1 << 20;
  int64_t pix_chunk = std::min<int64_t>(npix, N);
  int S = (int)std::max<int64_t>(1, std::min<int64_t>(p->spp, N / pix_chunk));
  const int64_t region = pix_chunk * S;
  std::vector<BatchInfo> batches;
  for (int64_t p0 = 0; p0 < npix; p0 += pix_chunk) {
    int np = (int)std::min<int64_t>(pix_chunk, npix - p0);
    for (int s0 = 0; s0 < p->spp; s0 += S) {
      BatchInfo B{};
      B.pixels = r->pixels;
      B.sobol = r->sobol + 2 * (size_t)p->sample_begin;
      B.s_base = p->sample_begin;
      B.p0 = (int)p0;
      B.spp_batch = std::min(S, p->spp - s0);
      B.n_paths = np * B.spp_batch;
      B.s0 = s0;
      B.nx = p->nx;
      B.ny = p->ny;
      B.base_seed = p->base_seed;
      batches.push_back(B);
    }
  }
  const size_t nb = batches.size();
  // lanes: enough paths in flight to fill the GPU, without idle lanes on small frames
  int lanes = (int)std::min<size_t>(nb, (size_t)r->n_lanes);
  lanes = std::max(1, lanes);
  size_t cap = (size_t)region * R;
  if (cap > (size_t)INT32_MAX / 4) {
    err = "batch_paths too large";
    return SRR_EINVAL;
  }
  for (int l = 0; l < lanes; ++l) {
    int rc = ensure_lane(r->lanes[l], cap, p->max_depth, keep, err);
    if (rc < 0) return rc;
  }
  RCHK(hipDeviceSynchronize());
  {
    const int rc = begin_accum(r, p, npix, ast, err);
    if (rc < 0) return rc;
  }
  AccCommit commit{r};
  RCHK(hipEventRecord(r->ev_beg, ast));
  for (int l = 0; l < lanes; ++l) {
    Lane& L = r->lanes[l];
    L.n = 0;
    L.cur = 0;
    L.pending = false;
    L.trace_ms = L.shade_ms = 0;
    for (int k = 0; k < R; ++k) {
      L.reg_batch[k] = -1;
      L.acc_pending[k] = false;
    }
    if (!keep) {
      L.P.raw = nullptr;
      L.P.rays = nullptr;
    }
    RCHK(hipStreamWaitEvent(L.st, r->ev_beg, 0));
  }
  std::vector<int> b_lane(nb, -1), b_reg(nb, -1);
  std::vector<char> b_done(nb, 0);
  srr_stats s{};
  size_t next_batch = 0, acc_head = 0;
  const int64_t target = std::max<int64_t>(region, (int64_t)3 << 20) / 2;  // paths in flight per lane

  while (acc_head < nb) {
    bool progress = false;
    for (int l = 0; l < lanes; ++l) {
      Lane& L = r->lanes[l];
      if (L.pending) {
        hipError_t q = hipEventQuery(L.ev_rb);
        if (q == hipErrorNotReady) continue;
        RCHK(q);
        L.pending = false;
        progress = true;
        float ms = 0;
        RCHK(hipEventElapsedTime(&ms, L.ev_t0, L.ev_t1));
        L.trace_ms += ms;
        RCHK(hipEventElapsedTime(&ms, L.ev_t1, L.ev_s1));
        L.shade_ms += ms;
        L.n = L.rb[R];
        for (int k = 0; k < R; ++k)
          if (L.reg_batch[k] >= 0 && !b_done[L.reg_batch[k]] && L.rb[k] == 0) {
            b_done[L.reg_batch[k]] = 1;
            RCHK(hipEventRecord(L.done_ev[k], L.st));
          }
      }
      // refill free regions with new batches
      while (next_batch < nb && L.n < target) {
        int fr = -1;
        for (int k = 0; k < R; ++k)
          if (L.reg_batch[k] < 0) {
            fr = k;
            break;
          }
        if (fr < 0) break;
        if (L.acc_pending[fr]) {  // the region's previous batch is still being accumulated
          RCHK(hipStreamWaitEvent(L.st, L.acc_ev[fr], 0));
          L.acc_pending[fr] = false;
        }
        BatchInfo& B = batches[next_batch];
        B.active = L.act[L.cur];
        B.act0 = L.n;
        B.slot0 = (int)(fr * region);
        B.count = L.cnt + L.cur;
        launch_raygen(r->view, L.P, B, L.st);
        L.n += B.n_paths;
        L.reg_batch[fr] = (int)next_batch;
        b_lane[next_batch] = l;
        b_reg[next_batch] = fr;
        s.paths += B.n_paths;
        ++next_batch;
        progress = true;
      }
      if (L.n > 0) {
        int n = L.n, cur = L.cur;
        int* alive = L.cnt + 2;
        int* fam = alive + R;
        RCHK(hipMemsetAsync(L.cnt + (cur ^ 1), 0, sizeof(int), L.st));
        int* fetch = alive + R + 4;  // persistent trace's ray cursor
        RCHK(hipMemsetAsync(alive, 0, (R + 5) * sizeof(int), L.st));
        RCHK(hipEventRecord(L.ev_t0, L.st));
        launch_trace(r->view, L.P, L.act[cur], L.cnt + cur, n, L.lists, (int)L.cap, fam, fetch, p->max_depth, visits,
                     L.st);
        RCHK(hipEventRecord(L.ev_t1, L.st));
        launch_shade(r->view, L.P, L.lists, (int)L.cap, fam, L.act[cur ^ 1], L.cnt + (cur ^ 1), alive, (int)region,
                     n, p->max_depth, L.st);
        RCHK(hipEventRecord(L.ev_s1, L.st));
        RCHK(hipMemcpyAsync(L.rb, alive, R * sizeof(int), hipMemcpyDeviceToHost, L.st));
        RCHK(hipMemcpyAsync(L.rb + R, L.cnt + (cur ^ 1), sizeof(int), hipMemcpyDeviceToHost, L.st));
        RCHK(hipEventRecord(L.ev_rb, L.st));
        L.pending = true;
        L.cur ^= 1;
        s.world_rays += n;
        s.trace_launches += 1;
        s.bounces += 1;
        progress = true;
      }
    }
    // accumulate finished batches strictly in batch order, on the acc stream
    while (acc_head < next_batch && b_done[acc_head]) {
      Lane& L = r->lanes[b_lane[acc_head]];
      int rg = b_reg[acc_head];
      BatchInfo& B = batches[acc_head];
      RCHK(hipStreamWaitEvent(ast, L.done_ev[rg], 0));
      launch_accumulate(L.P, B, r->acc, ast);
      if (keep) {  // region paths are [pixel][sample-in-batch]; the frame keeps [pixel][spp]
        int np = B.n_paths / B.spp_batch, Sb = B.spp_batch;
        RCHK(hipMemcpy2DAsync(r->raw_all + 3 * ((size_t)B.p0 * p->spp + B.s0), 3 * sizeof(float) * p->spp,
                              L.P.raw + 3 * (size_t)B.slot0, 3 * sizeof(float) * Sb, 3 * sizeof(float) * Sb, np,
                              hipMemcpyDeviceToDevice, ast));
        RCHK(hipMemcpy2DAsync(r->rays_all + ((size_t)B.p0 * p->spp + B.s0), p->spp, L.P.rays + B.slot0, Sb, Sb, np,
                              hipMemcpyDeviceToDevice, ast));
      }
      RCHK(hipEventRecord(L.acc_ev[rg], ast));
      L.acc_pending[rg] = true;
      L.reg_batch[rg] = -1;
      ++acc_head;
      progress = true;
    }
    if (!progress) std::this_thread::yield();
  }
  const int64_t acc_total = r->acc_samples + p->spp;
  if (p->flags & SRR_FLAG_SUMS)
    RCHK(hipMemcpyAsync(d_mean, r->acc, 3 * (size_t)npix * sizeof(float), hipMemcpyDeviceToDevice, ast));
  else
    launch_finish(r->acc, d_mean, npix, (int)acc_total, ast);
  RCHK(hipEventRecord(r->ev_end, ast));
  RCHK(hipStreamSynchronize(ast));
  RCHK(hipGetLastError());
  r->acc_samples = acc_total;
  commit.ok = true;
  float total = 0;
  RCHK(hipEventElapsedTime(&total, r->ev_beg, r->ev_end));
  s.total_ms = total;
  for (int l = 0; l < lanes; ++l) {
    s.trace_ms += r->lanes[l].trace_ms;
    s.shade_ms += r->lanes[l].shade_ms;
  }
  if (getenv("SRR_TIMING")) dump_trace_timing();
  if (visits) {
    unsigned long long v[kVisitWords];
    RCHK(hipDeviceSynchronize());
    RCHK(hipMemcpy(v, visits, sizeof(v), hipMemcpyDeviceToHost));
    if (getenv("SRR_HIST")) {  // diagnostics: node steps per ray / per wave
      for (int h = 0; h < 2; ++h) {
        fprintf(stderr, h ? "steps per wave (max):" : "steps per ray:");
        for (int b = 0; b < 64; ++b)
          if (v[3 + 64 * h + b]) fprintf(stderr, " %d:%llu", b, v[3 + 64 * h + b]);
        fprintf(stderr, "\n");
      }
    }
    s.box_tests = (int64_t)v[0];
    s.tri_tests = (int64_t)v[1];
    s.stack_overflows = (int64_t)v[2];
  }
  if (stats) *stats = s;
  return 0;
}

}  // namespace srr

srr_renderer::~srr_renderer() {
  if (multi) {
    srr::multi_destroy(multi);
    multi = nullptr;
  }
  (void)hipSetDevice(device);
  (void)hipDeviceSynchronize();
  for (void* p : scene_bufs) (void)hipFree(p);
  if (visits) (void)hipFree(visits);
  srr::slot_free(sync_slot);
  for (auto& F : async_slots) srr::slot_free(F);
  if (ev_async_in) (void)hipEventDestroy(ev_async_in);
  (void)hipFree(pw_wave_times);
  (void)hipFree(pw_slow);
  for (auto& L : lanes) {
    srr::free_lane_paths(L);
    (void)hipFree(L.cnt);
    if (L.rb) (void)hipHostFree(L.rb);
    for (hipEvent_t e : {L.ev_t0, L.ev_t1, L.ev_s1, L.ev_rb})
      if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < srr::kRegionsPerLane; ++k) {
      if (L.done_ev[k]) (void)hipEventDestroy(L.done_ev[k]);
      if (L.acc_ev[k]) (void)hipEventDestroy(L.acc_ev[k]);
    }
    if (L.st) (void)hipStreamDestroy(L.st);
  }
  (void)hipFree(acc);
  (void)hipFree(pixels);
  (void)hipFree(sobol);
  (void)hipFree(raw_all);
  (void)hipFree(rays_all);
  if (ev_beg) (void)hipEventDestroy(ev_beg);
  if (ev_end) (void)hipEventDestroy(ev_end);
  if (acc_st) (void)hipStreamDestroy(acc_st);
}

// The device-resident renderer behind srr_renderer_* (include/srr_capi.h):
// uploaded scene tables plus the wavefront path pools.
//
// Work is organised in LANES: each lane owns a HIP stream and a pool of path
// slots split into regions; a region holds one batch (a pixel chunk x sample
// chunk).  A lane runs trace -> shade (material-sorted) bounces over all its live
// paths, refilling freed regions with new batches, so a batch's tail of long
// paths overlaps the next batches' first bounces; several lanes run
// concurrently so one lane's straggler waves overlap other lanes' kernels.
// Finished batches are accumulated on a separate stream strictly in batch order
// (per-pixel sums stay in sample order, hence bitwise reproducible).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/srr_capi.h"
#include "kernels.h"
#include "scene.h"

namespace srr {

constexpr int kRegionsPerLane = 3;  // <= kernels.hip kMaxRegions
constexpr int kMaxLanes = 4;

struct Lane {
  hipStream_t st = nullptr;
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr, ev_s1 = nullptr, ev_rb = nullptr;
  hipEvent_t done_ev[kRegionsPerLane] = {};  // batch in region finished (lane stream)
  hipEvent_t acc_ev[kRegionsPerLane] = {};   // batch in region accumulated (acc stream)
  bool acc_pending[kRegionsPerLane] = {};    // region reuse must wait for acc_ev
  PathState P{};
  int32_t* act[2] = {nullptr, nullptr};
  int32_t* lists = nullptr;  // 4 material-family lists
  int32_t* cnt = nullptr;    // [0..1] active counts, [2..2+R) region survivors, [2+R..6+R) families
  int32_t* rb = nullptr;     // pinned host mirror of region survivors + next count
  size_t cap = 0;
  int cap_depth = 0;
  bool has_raw = false;
  std::vector<void*> bufs;
  // per-frame state
  int n = 0, cur = 0;
  bool pending = false;
  int reg_batch[kRegionsPerLane];
  double trace_ms = 0, shade_ms = 0;
};

// One frame of the path engine: its stream, bounce records, traversal-stack
// extension, sample window, counters and events (renderer.cpp paths_enqueue);
// the synchronous path owns one, srr_render_device_async alternates two.
struct FrameSlot {
  hipStream_t st = nullptr;
  bool own_stream = false;
  hipEvent_t ev_beg = nullptr, ev_end = nullptr;
  std::vector<hipEvent_t> win_ev;  // per sample window: k_paths start / end
  float4* rec = nullptr;
  size_t rec_cap = 0;
  // [kPathsGlobalStack][pw_lanes] int2 (kernels.h), then [3][pw_lanes] float4 of suspended
  // mesh walks (kernels.h PathWork::walk_q)
  int2* gstack = nullptr;
  float* sample = nullptr;
  size_t sample_cap = 0;
  unsigned long long* ctr = nullptr;       // [0] world rays, [1] path cursor, ...
  unsigned long long* ctr_host = nullptr;  // pinned mirror, read after the frame's stream sync
  float* acc = nullptr;                    // async slots: the frame's own per-pixel sums
  size_t acc_cap = 0;
  // a frame in flight (async slots)
  bool busy = false;
  int64_t ticket = -1, npix = 0, paths = 0;
  int n_windows = 0;
  int rc = 0;
  srr_stats stats{};
  std::string err;
};
void slot_free(FrameSlot& F);

struct DoneTicket {  // an async frame finished before its srr_render_wait
  int64_t ticket;
  int rc;
  srr_stats stats;
  std::string err;
};

struct Multi;  // multi.h
}  // namespace srr

struct srr_renderer {
  int device = 0;
  // srr_renderer_create_multi: this handle renders over several devices through
  // their own renderers (multi.cpp); its single-device state below stays unused
  srr::Multi* multi = nullptr;
  srr::SceneView view{};
  std::vector<void*> scene_bufs;
  int n_lanes = 2;
  srr::Lane lanes[srr::kMaxLanes];
  hipStream_t acc_st = nullptr;
  hipEvent_t ev_beg = nullptr, ev_end = nullptr;
  // frame buffers
  float* acc = nullptr;
  int64_t acc_npix = 0;     // pixels the running sums cover (SRR_FLAG_CONTINUE)
  int64_t acc_samples = 0;  // samples per pixel accumulated in them
  // the frame and shard the running sums belong to: {nx, ny, shard_index,
  // shard_count, tile}; all -1 after srr_accum_set (only npix is known then)
  int acc_key[5] = {-1, -1, -1, -1, -1};
  unsigned long long* visits = nullptr;  // SRR_FLAG_COUNT_VISITS counters (3)
  // path-resident engine (render_paths)
  int pw_lanes = 0;
  bool diffuse_only = false;  // no beckmann / specular materials: lean kernel variant
  int walk_q_default = 0;     // suspendable mesh walks unless SRR_WALK_Q says otherwise (renderer.cpp)
  bool has_meshes = false;
  srr::FrameSlot sync_slot;         // srr_render_device (stream acc_st, sums in acc)
  srr::FrameSlot async_slots[2];    // srr_render_device_async, alternating
  int64_t next_ticket = 0;
  std::vector<srr::DoneTicket> done_tickets;
  hipEvent_t ev_async_in = nullptr;  // orders an async frame after the caller's legacy-stream work
  // renderers sharing this device under one multi-device handle (multi.cpp): each takes
  // 1/window_share of the sample-window budget (SRR_WINDOW_MB)
  int window_share = 1;
  unsigned long long* pw_wave_times = nullptr;  // SRR_WAVE_TIMES diagnostics, 4 words per wave
  float* pw_slow = nullptr;  // diagnostics build (-DSRR_SLOW_RAYS): slow world-hit records + count
  int32_t* pixels = nullptr;
  size_t pix_cap = 0;
  // the shard whose pixel list (srr_shard_pixels) the renderer holds: {nx, ny,
  // shard_index, shard_count, tile}, its pixel count, and whether it is the
  // identity (then `pixels` is not read); key[0] = -1: none.  srr_render_device
  // passes pix = nullptr to render_device when the shard is this one.
  int pix_key[5] = {-1, -1, -1, -1, -1};
  int64_t pix_n = 0;
  bool pix_identity = false;
  double* sobol = nullptr;
  int sobol_n = 0;
  float* raw_all = nullptr;
  uint8_t* rays_all = nullptr;
  size_t keep_cap = 0;
  int64_t kept_paths = 0;
  ~srr_renderer();
};

namespace srr {
int renderer_create(const Scene& s, int device, srr_renderer** out, std::string& err);
// the same from an already flattened scene (a multi-device renderer flattens once)
int renderer_create_flat(const Flat& F, int device, srr_renderer** out, std::string& err);
// pix: the shard's npix pixel indices, or nullptr when the renderer already holds
// them (srr_renderer::pix_key)
int render_device(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, float* d_mean,
                  srr_stats* stats, std::string& err);
int render_device_async(srr_renderer* r, const srr_params* p, const int32_t* pix, int64_t npix, float* d_mean,
                        int64_t* ticket, std::string& err);
int render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats, std::string& err);
void drain_async(srr_renderer* r);  // finish every async frame in flight (results kept for render_wait)
// the event recorded after async frame `ticket`'s last operation (its slot's frame end),
// or nullptr when that frame is no longer in flight (multi.cpp orders its exchange by it)
hipEvent_t render_ticket_event(srr_renderer* r, int64_t ticket);
}  // namespace srr

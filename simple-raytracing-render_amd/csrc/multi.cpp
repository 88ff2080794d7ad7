// Multi-device renderer: one host process, N GPUs, one frame-end gather over
// RCCL (multi.h).
//
// The reference renders a frame with 8 renderthreads in one process
// (Raytracing_n.cpp:932-941), all sharing one scene.  Here one renderer handle
// owns N per-device renderers (the scene flattened once, uploaded N times).  A
// frame is split into the same rotated round-robin tile shards the torch path
// uses (srr_shard_pixels, srr/dist.py): shard k renders on device k, all shards
// concurrently -- one host thread per device for a synchronous frame, or each
// device's srr_render_device_async for a pipelined one -- and then
//   * RCCL: one ncclGroupStart / ncclSend (every shard, device 0's own to itself)
//     / ncclRecv (device 0, into the packed frame) / ncclGroupEnd over a
//     communicator from ncclCommInitAll;
//   * device 0 scatters the packed slabs to their pixels (k_scatter_pixels).
// Every path is seeded by its (pixel, sample), so the frame is bitwise the
// one-device frame.  When device_ids repeats a device (a rehearsal on one GPU)
// or SRR_MULTI_TRANSPORT=copy, the gather is peer / device copies instead.
//
// librccl is opened with dlopen at the first multi-device renderer, not linked:
// a process that already holds an RCCL (torch's) shares it, and libsrr.so
// itself loads without one.
#include "multi.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <thread>

#include "kernels.h"
#include "renderer.h"

namespace srr {

namespace {

#define MCHK(x)                                                        \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      err = std::string(#x) + ": " + hipGetErrorString(e_);            \
      return SRR_EIO;                                                  \
    }                                                                  \
  } while (0)

struct Rccl {
  void* so = nullptr;
  std::string why;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*ErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
};

const Rccl& rccl() {
  static const Rccl R = [] {
    Rccl r;
    // the soname first (an RCCL already in the process is reused), then ROCm's
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.so) break;
    }
    if (!r.so) {
      const char* e = dlerror();
      r.why = std::string("dlopen librccl.so.1: ") + (e ? e : "not found");
      return r;
    }
    auto sym = [&](const char* n) { return dlsym(r.so, n); };
    r.CommInitAll = (decltype(r.CommInitAll))sym("ncclCommInitAll");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.ErrorString = (decltype(r.ErrorString))sym("ncclGetErrorString");
    r.GetVersion = (decltype(r.GetVersion))sym("ncclGetVersion");
    if (!r.CommInitAll || !r.CommDestroy || !r.GroupStart || !r.GroupEnd || !r.Send || !r.Recv || !r.ErrorString) {
      r.why = "librccl.so.1 lacks the ncclCommInitAll / ncclSend / ncclRecv / ncclGroup* entry points";
      r.so = nullptr;
    }
    return r;
  }();
  return R;
}

struct PendingFrame {
  int64_t ticket = -1;
  int buf = 0;
  float* d_image = nullptr;
  std::vector<int64_t> tickets;  // each device's srr_render_device_async ticket
};



}  // namespace

struct Multi {
  std::vector<int> devs;
  std::vector<srr_renderer*> peers;  // peers[k] renders shard k on devs[k] (owned)
  bool use_rccl = false;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> xst;  // per-device exchange stream
  // per buffer set (frames in flight each have their own): on devs[0] the exchange's
  // start / end and the caller's legacy-stream work it follows; per device the end of
  // its send (RCCL)
  hipEvent_t ev_x0[2] = {nullptr, nullptr}, ev_x1[2] = {nullptr, nullptr}, ev_in[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> ev_sent[2];
  // the frame plan: {nx, ny, tile}; shard pixel lists and offsets in the packed frame
  int key[3] = {-1, -1, -1};
  std::vector<std::vector<int32_t>> shard_pix;
  std::vector<int64_t> off;
  int64_t npix = 0;
  int32_t* d_index = nullptr;  // devs[0]: packed entry -> image pixel
  // two buffer sets (frames in flight): the packed frame on devs[0]; per device the
  // shard's output (RCCL: every device's, sent to device 0; copies: k >= 1 only,
  // shard 0 renders into the packed frame)
  float* packed[2] = {nullptr, nullptr};
  std::vector<float*> slab[2];
  std::vector<size_t> slab_cap[2];
  size_t packed_cap[2] = {0, 0};
  std::deque<PendingFrame> pending;
  std::vector<DoneTicket> done;
  int64_t next_ticket = 0;

  ~Multi() {
    for (size_t k = 0; k < devs.size(); ++k) {
      (void)hipSetDevice(devs[k]);
      (void)hipDeviceSynchronize();
    }
    if (use_rccl)
      for (ncclComm_t c : comms)
        if (c) rccl().CommDestroy(c);
    for (size_t k = 0; k < devs.size(); ++k) {
      (void)hipSetDevice(devs[k]);
      for (int b = 0; b < 2; ++b) {
        if (k < slab[b].size() && slab[b][k]) (void)hipFree(slab[b][k]);
        if (k < ev_sent[b].size() && ev_sent[b][k]) (void)hipEventDestroy(ev_sent[b][k]);
      }
      if (k < xst.size() && xst[k]) (void)hipStreamDestroy(xst[k]);
    }
    if (!devs.empty()) {
      (void)hipSetDevice(devs[0]);
      for (float* p : packed) (void)hipFree(p);
      (void)hipFree(d_index);
      for (int b = 0; b < 2; ++b)
        for (hipEvent_t e : {ev_x0[b], ev_x1[b], ev_in[b]})
          if (e) (void)hipEventDestroy(e);
    }
    for (srr_renderer* r : peers) srr_renderer_destroy(r);
  }
};

int64_t multi_plan(const srr_params* p, int n, std::vector<std::vector<int32_t>>* shard_pix, int32_t* index,
                   int64_t* off, std::string& err) {
  if (!p || n < 1 || p->nx <= 0 || p->ny <= 0) {
    err = "multi_plan: bad params";
    return SRR_EINVAL;
  }
  if (p->shard_count > 1) {
    err = "a multi-device renderer shards the frame itself: shard_count must be 0 or 1";
    return SRR_EINVAL;
  }
  int64_t total = 0;
  if (shard_pix) shard_pix->assign(n, {});
  for (int k = 0; k < n; ++k) {
    srr_params q = *p;
    q.shard_index = k;
    q.shard_count = n;
    const int64_t nk = srr_shard_pixels(&q, nullptr);
    if (nk < 0) {
      err = "srr_shard_pixels failed";
      return nk;
    }
    std::vector<int32_t> pix((size_t)nk);
    srr_shard_pixels(&q, pix.data());
    if (off) off[k] = total;
    if (index) std::copy(pix.begin(), pix.end(), index + total);
    total += nk;
    if (shard_pix) (*shard_pix)[k] = std::move(pix);
  }
  if (off) off[n] = total;
  if (total != (int64_t)p->nx * p->ny) {
    err = "multi_plan: shards do not cover the frame";
    return SRR_EIO;
  }
  return total;
}

int multi_create(const Scene& sc, int n, const int* ids, srr_renderer** out, std::string& err) {
  if (n < 1 || !ids) {
    err = "srr_renderer_create_multi: n_devices >= 1 and device_ids needed";
    return SRR_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    err = "no HIP device (the srr renderer has no CPU fallback)";
    return SRR_ENODEV;
  }
  for (int k = 0; k < n; ++k)
    if (ids[k] < 0 || ids[k] >= ndev) {
      err = "device index " + std::to_string(ids[k]) + " out of range (" + std::to_string(ndev) + " devices)";
      return SRR_ENODEV;
    }
  Flat F;
  int rc = flatten(sc, F, err);
  if (rc < 0) return rc;
  std::unique_ptr<srr_renderer> shell(new srr_renderer());
  shell->device = ids[0];
  shell->multi = new Multi();
  Multi& M = *shell->multi;
  M.devs.assign(ids, ids + n);
  for (int k = 0; k < n; ++k) {
    srr_renderer* r = nullptr;
    rc = renderer_create_flat(F, ids[k], &r, err);
    if (rc < 0) return rc;  // (the shell's destructor frees the peers made so far)
    M.peers.push_back(r);
  }
  bool distinct = true;
  for (int a = 0; a < n; ++a)
    for (int b = a + 1; b < n; ++b) distinct = distinct && ids[a] != ids[b];
  const char* tr = getenv("SRR_MULTI_TRANSPORT");
  const bool want_copy = tr && !strcmp(tr, "copy");
  if (tr && !want_copy && strcmp(tr, "rccl")) {
    err = std::string("SRR_MULTI_TRANSPORT must be rccl or copy, not ") + tr;
    return SRR_EINVAL;
  }
  if (tr && !strcmp(tr, "rccl") && !distinct) {
    err = "SRR_MULTI_TRANSPORT=rccl needs distinct devices (RCCL wants one GPU per rank)";
    return SRR_EINVAL;
  }
  M.use_rccl = distinct && !want_copy;
  M.xst.assign(n, nullptr);
  for (int k = 0; k < n; ++k) {
    MCHK(hipSetDevice(ids[k]));
    MCHK(hipStreamCreateWithFlags(&M.xst[k], hipStreamNonBlocking));
  }
  for (int b = 0; b < 2; ++b) {
    M.ev_sent[b].assign(n, nullptr);
    for (int k = 0; k < n; ++k) {
      MCHK(hipSetDevice(ids[k]));
      MCHK(hipEventCreateWithFlags(&M.ev_sent[b][k], hipEventDisableTiming));
    }
    MCHK(hipSetDevice(ids[0]));
    MCHK(hipEventCreate(&M.ev_x0[b]));
    MCHK(hipEventCreate(&M.ev_x1[b]));
    MCHK(hipEventCreateWithFlags(&M.ev_in[b], hipEventDisableTiming));
  }
  // peers sharing a device (a one-GPU rehearsal) split the sample-window budget, so
  // the device holds what one renderer would (renderer.cpp paths_enqueue)
  for (int k = 0; k < n; ++k)
    M.peers[k]->window_share = (int)std::count(ids, ids + n, ids[k]);
  if (M.use_rccl) {
    const Rccl& R = rccl();
    if (!R.so) {
      err = R.why;
      return SRR_ENOTSUP;
    }
    M.comms.assign(n, nullptr);
    const ncclResult_t e = R.CommInitAll(M.comms.data(), n, ids);
    if (e != ncclSuccess) {
      M.comms.clear();
      err = std::string("ncclCommInitAll: ") + R.ErrorString(e);
      return SRR_EIO;
    }
  }
  for (int b = 0; b < 2; ++b) {
    M.slab[b].assign(n, nullptr);
    M.slab_cap[b].assign(n, 0);
  }
  *out = shell.release();
  return 0;
}

void multi_destroy(Multi* m) { delete m; }

int multi_devices(const Multi* m, int* ids, int cap) {
  const int n = (int)m->devs.size();
  for (int k = 0; ids && k < std::min(n, cap); ++k) ids[k] = m->devs[k];
  return n;
}

const char* multi_transport(const Multi* m) { return m->use_rccl ? "rccl" : "copy"; }

namespace {

int check_params(const srr_params* p, std::string& err) {
  if (p->flags & (SRR_FLAG_KEEP_PATHS | SRR_FLAG_CONTINUE)) {
    err = "a multi-device renderer renders fresh frames (no KEEP_PATHS / CONTINUE: use one device's renderer)";
    return SRR_EINVAL;
  }
  if (p->shard_count > 1) {
    err = "a multi-device renderer shards the frame itself: shard_count must be 0 or 1";
    return SRR_EINVAL;
  }
  return 0;
}

int finish_oldest(Multi& M);

// the frame plan and buffer set b for p (host lists once per {nx, ny, tile})
int stage(Multi& M, const srr_params* p, int b, std::string& err) {
  const int n = (int)M.devs.size();
  const int key[3] = {p->nx, p->ny, p->tile};
  if (!std::equal(key, key + 3, M.key)) {
    while (!M.pending.empty()) finish_oldest(M);  // frames in flight exchange by the current plan
    std::vector<int32_t> index((size_t)p->nx * p->ny);
    std::vector<int64_t> off(n + 1);
    const int64_t total = multi_plan(p, n, &M.shard_pix, index.data(), off.data(), err);
    if (total < 0) return (int)total;
    MCHK(hipSetDevice(M.devs[0]));
    // the plan is invalid from here until its index is staged: a failure below leaves
    // no key that a later frame could take for the staged one
    M.key[0] = -1;
    if (total > M.npix) {
      (void)hipFree(M.d_index);
      M.d_index = nullptr;
      M.npix = 0;
      if (const char* e = getenv("SRR_MULTI_FAIL_INDEX"); e && atoi(e)) {  // tests: a failed allocation
        err = "SRR_MULTI_FAIL_INDEX: the pixel index allocation fails (test hook)";
        return SRR_ENOMEM;
      }
      MCHK(hipMalloc((void**)&M.d_index, total * sizeof(int32_t)));
      M.npix = total;
    }
    MCHK(hipMemcpy(M.d_index, index.data(), total * sizeof(int32_t), hipMemcpyHostToDevice));
    M.off = off;
    std::copy(key, key + 3, M.key);
  }
  const int64_t total = M.off[n];
  MCHK(hipSetDevice(M.devs[0]));
  if ((size_t)total > M.packed_cap[b]) {
    (void)hipFree(M.packed[b]);
    M.packed[b] = nullptr;
    M.packed_cap[b] = 0;
    MCHK(hipMalloc((void**)&M.packed[b], 3 * (size_t)total * sizeof(float)));
    M.packed_cap[b] = total;
  }
  for (int k = M.use_rccl ? 0 : 1; k < n; ++k) {
    const size_t nk = (size_t)(M.off[k + 1] - M.off[k]);
    if (nk > M.slab_cap[b][k]) {
      MCHK(hipSetDevice(M.devs[k]));
      (void)hipFree(M.slab[b][k]);
      M.slab[b][k] = nullptr;
      M.slab_cap[b][k] = 0;
      MCHK(hipMalloc((void**)&M.slab[b][k], 3 * std::max<size_t>(nk, 1) * sizeof(float)));
      M.slab_cap[b][k] = nk;
    }
  }
  return 0;
}

// where shard k writes its pixels in buffer set b
float* shard_out(Multi& M, int b, int k) {
  if (!M.use_rccl && k == 0) return M.packed[b];
  return M.slab[b][k];
}

srr_params shard_params(const Multi& M, const srr_params* p, int k) {
  srr_params q = *p;
  q.shard_index = k;
  q.shard_count = (int)M.devs.size();
  return q;
}

void merge(srr_stats& s, const srr_stats& t) {
  s.world_rays += t.world_rays;
  s.paths += t.paths;
  s.trace_launches += t.trace_launches;
  s.trace_ms += t.trace_ms;
  s.shade_ms += t.shade_ms;
  s.total_ms = std::max(s.total_ms, t.total_ms);
  s.bounces += t.bounces;
  s.box_tests += t.box_tests;
  s.tri_tests += t.tri_tests;
  s.stack_overflows += t.stack_overflows;
  s.deep_traversals += t.deep_traversals;
  s.mixture_capped += t.mixture_capped;
  s.walks_suspended += t.walks_suspended;
}

// The frame-end exchange of buffer set b, enqueued on the exchange streams without
// a host wait: the shards' slabs into the packed frame on device 0 (RCCL send /
// recv, or copies), then the scatter into d_image.  Each shard's part waits on
// done[k] (its frame's end event; nullptr: the shard already finished on the host),
// and device 0's part also on the caller's legacy-stream work queued before it
// (the image's producers).  wait_exchange reads the result.
int enqueue_exchange(Multi& M, int b, float* d_image, const std::vector<hipEvent_t>& done, std::string& err) {
  const int n = (int)M.devs.size();
  MCHK(hipSetDevice(M.devs[0]));
  MCHK(hipEventRecord(M.ev_in[b], nullptr));
  MCHK(hipStreamWaitEvent(M.xst[0], M.ev_in[b], 0));
  for (int k = 0; k < n; ++k) {
    if (!done[k]) continue;
    // RCCL: shard k's send runs on its device's exchange stream; copies: device 0's
    // stream reads every slab (an event of another device may be waited on)
    MCHK(hipSetDevice(M.use_rccl ? M.devs[k] : M.devs[0]));
    MCHK(hipStreamWaitEvent(M.use_rccl ? M.xst[k] : M.xst[0], done[k], 0));
  }
  MCHK(hipSetDevice(M.devs[0]));
  MCHK(hipEventRecord(M.ev_x0[b], M.xst[0]));
  if (M.use_rccl) {
    const Rccl& R = rccl();
    ncclResult_t e = R.GroupStart();
    for (int k = 0; e == ncclSuccess && k < n; ++k) {
      const size_t cnt = 3 * (size_t)(M.off[k + 1] - M.off[k]);
      if (cnt) e = R.Send(M.slab[b][k], cnt, ncclFloat32, 0, M.comms[k], M.xst[k]);
    }
    for (int k = 0; e == ncclSuccess && k < n; ++k) {
      const size_t cnt = 3 * (size_t)(M.off[k + 1] - M.off[k]);
      if (cnt) e = R.Recv(M.packed[b] + 3 * M.off[k], cnt, ncclFloat32, k, M.comms[0], M.xst[0]);
    }
    const ncclResult_t e2 = R.GroupEnd();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) {
      err = std::string("RCCL gather: ") + R.ErrorString(e);
      return SRR_EIO;
    }
    for (int k = 1; k < n; ++k) {  // the senders' ends (their slabs are reused by a later frame)
      MCHK(hipSetDevice(M.devs[k]));
      MCHK(hipEventRecord(M.ev_sent[b][k], M.xst[k]));
    }
  } else {
    for (int k = 1; k < n; ++k) {
      const size_t bytes = 3 * (size_t)(M.off[k + 1] - M.off[k]) * sizeof(float);
      if (bytes)
        MCHK(hipMemcpyPeerAsync(M.packed[b] + 3 * M.off[k], M.devs[0], M.slab[b][k], M.devs[k], bytes, M.xst[0]));
    }
  }
  MCHK(hipSetDevice(M.devs[0]));
  launch_scatter_pixels(M.packed[b], M.d_index, M.off[n], d_image, M.xst[0]);
  MCHK(hipGetLastError());
  MCHK(hipEventRecord(M.ev_x1[b], M.xst[0]));
  return 0;
}

// waits for buffer set b's exchange (the host's only wait on it); its device time in *ms
int wait_exchange(Multi& M, int b, double* ms, std::string& err) {
  const int n = (int)M.devs.size();
  MCHK(hipSetDevice(M.devs[0]));
  MCHK(hipEventSynchronize(M.ev_x1[b]));
  if (M.use_rccl)
    for (int k = 1; k < n; ++k) {
      MCHK(hipSetDevice(M.devs[k]));
      MCHK(hipEventSynchronize(M.ev_sent[b][k]));
    }
  MCHK(hipSetDevice(M.devs[0]));
  float t = 0;
  MCHK(hipEventElapsedTime(&t, M.ev_x0[b], M.ev_x1[b]));
  *ms = t;
  return 0;
}

// finish the oldest frame in flight: every shard's stats, then its exchange (enqueued
// when the frame was submitted)
int finish_oldest(Multi& M) {
  PendingFrame f = M.pending.front();
  M.pending.pop_front();
  DoneTicket d{f.ticket, 0, srr_stats{}, ""};
  for (size_t k = 0; k < M.devs.size(); ++k) {
    if (f.tickets[k] < 0) continue;
    srr_stats s{};
    const int rc = srr_render_wait(M.peers[k], f.tickets[k], &s);
    if (rc < 0 && d.rc == 0) {
      d.rc = rc;
      d.err = std::string("device ") + std::to_string(M.devs[k]) + ": " + srr_last_error();
    }
    merge(d.stats, s);
  }
  double ms = 0;
  std::string xerr;
  const int xrc = wait_exchange(M, f.buf, &ms, xerr);  // (also after a shard error: the buffers are reused)
  if (d.rc == 0 && xrc < 0) {
    d.rc = xrc;
    d.err = xerr;
  }
  if (d.rc == 0) d.stats.total_ms += ms;
  M.done.push_back(d);
  return d.rc;
}

}  // namespace

int multi_render_device(srr_renderer* r, const srr_params* p, float* d_image, srr_stats* stats, std::string& err) {
  Multi& M = *r->multi;
  int rc = check_params(p, err);
  if (rc < 0) return rc;
  while (!M.pending.empty()) finish_oldest(M);  // (their results stay for srr_render_wait)
  rc = stage(M, p, 0, err);
  if (rc < 0) return rc;
  const int n = (int)M.devs.size();
  std::vector<int> rcs(n, 0);
  std::vector<srr_stats> st(n);
  std::vector<std::string> errs(n);
  auto shard = [&](int k) {
    const srr_params q = shard_params(M, p, k);
    if (M.off[k + 1] == M.off[k]) return;  // an empty shard (fewer pixels than devices)
    rcs[k] = srr_render_device(M.peers[k], &q, shard_out(M, 0, k), &st[k]);
    if (rcs[k] < 0) errs[k] = srr_last_error();
  };
  std::vector<std::thread> th;
  for (int k = 1; k < n; ++k) th.emplace_back(shard, k);
  shard(0);
  for (std::thread& t : th) t.join();
  srr_stats s{};
  for (int k = 0; k < n; ++k) {
    if (rcs[k] < 0) {
      err = "device " + std::to_string(M.devs[k]) + ": " + errs[k];
      return rcs[k];
    }
    merge(s, st[k]);
  }
  double ms = 0;
  // (the shards finished on the host: no events to wait on)
  rc = enqueue_exchange(M, 0, d_image, std::vector<hipEvent_t>(n, nullptr), err);
  if (rc < 0) return rc;
  rc = wait_exchange(M, 0, &ms, err);
  if (rc < 0) return rc;
  s.total_ms += ms;
  if (stats) *stats = s;
  return 0;
}

int multi_render_device_async(srr_renderer* r, const srr_params* p, float* d_image, int64_t* ticket,
                              std::string& err) {
  Multi& M = *r->multi;
  int rc = check_params(p, err);
  if (rc < 0) return rc;
  const int n = (int)M.devs.size();
  if (M.pending.size() >= 2) finish_oldest(M);  // a third frame: the oldest finishes first
  PendingFrame f;
  f.ticket = M.next_ticket;
  f.buf = (int)(f.ticket % 2);
  // the frame of this buffer set before this one must have finished
  for (;;) {
    bool clash = false;
    for (const PendingFrame& g : M.pending) clash = clash || g.buf == f.buf;
    if (!clash) break;
    finish_oldest(M);
  }
  rc = stage(M, p, f.buf, err);
  if (rc < 0) return rc;
  f.d_image = d_image;
  f.tickets.assign(n, -1);
  for (int k = 0; k < n; ++k) {
    if (M.off[k + 1] == M.off[k]) continue;
    const srr_params q = shard_params(M, p, k);
    rc = srr_render_device_async(M.peers[k], &q, shard_out(M, f.buf, k), &f.tickets[k]);
    if (rc < 0) {
      err = "device " + std::to_string(M.devs[k]) + ": " + srr_last_error();
      for (int j = 0; j < k; ++j)  // the shards already enqueued finish before the error returns
        if (f.tickets[j] >= 0) (void)srr_render_wait(M.peers[j], f.tickets[j], nullptr);
      return rc;
    }
  }
  // the exchange goes on the GPU now, behind each shard's frame end: the host waits
  // for nothing until srr_render_wait
  std::vector<hipEvent_t> done(n, nullptr);
  for (int k = 0; k < n; ++k)
    if (f.tickets[k] >= 0) done[k] = render_ticket_event(M.peers[k], f.tickets[k]);
  rc = enqueue_exchange(M, f.buf, d_image, done, err);
  if (rc < 0) {
    for (int k = 0; k < n; ++k)
      if (f.tickets[k] >= 0) (void)srr_render_wait(M.peers[k], f.tickets[k], nullptr);
    for (int k = 0; k < n; ++k) {  // what was enqueued of the exchange ends before its buffers are reused
      (void)hipSetDevice(M.devs[k]);
      (void)hipStreamSynchronize(M.xst[k]);
    }
    return rc;
  }
  M.next_ticket++;
  M.pending.push_back(f);
  *ticket = f.ticket;
  return 0;
}

int multi_render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats, std::string& err) {
  Multi& M = *r->multi;
  for (;;) {
    for (size_t k = 0; k < M.done.size(); ++k)
      if (M.done[k].ticket == ticket) {
        const DoneTicket d = M.done[k];
        M.done.erase(M.done.begin() + k);
        if (stats) *stats = d.stats;
        err = d.err;
        return d.rc;
      }
    bool in_flight = false;
    for (const PendingFrame& f : M.pending) in_flight = in_flight || f.ticket == ticket;
    if (!in_flight) {
      err = "srr_render_wait: unknown or already waited ticket " + std::to_string(ticket);
      return SRR_EINVAL;
    }
    finish_oldest(M);  // frames finish in order
  }
}

}  // namespace srr

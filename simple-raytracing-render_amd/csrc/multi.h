// Multi-device renderer (srr_renderer_create_multi, include/srr_capi.h): one
// process drives N GPUs, the replacement for the reference's 8 renderthreads in
// one process (Raytracing_n.cpp:932-941) at node scale.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/srr_capi.h"
#include "scene.h"

namespace srr {

struct Multi;

// Shard bookkeeping of an N-device frame (host only): shard k renders the pixels
// srr_shard_pixels gives for {shard_index k, shard_count n} (p->tile tiles dealt
// round-robin, each tile row rotated by one); the gather packs the shards' slabs
// in shard order, so packed entry i is image pixel index[i] and shard k's slab
// starts at off[k].  Returns the frame's pixel count or a negative code.
int64_t multi_plan(const srr_params* p, int n, std::vector<std::vector<int32_t>>* shard_pix, int32_t* index,
                   int64_t* off, std::string& err);

// A renderer handle whose srr_render* calls render over every device: the scene
// is flattened once and uploaded to each device; device_ids may repeat a device
// (rehearsal on one GPU: the gather then copies instead of using RCCL).
int multi_create(const Scene& sc, int n, const int* device_ids, srr_renderer** out, std::string& err);
void multi_destroy(Multi* m);
int multi_devices(const Multi* m, int* ids, int cap);
const char* multi_transport(const Multi* m);
int multi_render_device(srr_renderer* r, const srr_params* p, float* d_image, srr_stats* stats, std::string& err);
int multi_render_device_async(srr_renderer* r, const srr_params* p, float* d_image, int64_t* ticket,
                              std::string& err);
int multi_render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats, std::string& err);

}  // namespace srr

/* The reference's program, main() (Raytracing_n.cpp:882-952), over srr, in C++:
 * pick a scene builder by sceneid (:893-919), build it with the reference's
 * builder signature `void f(hitable** scene, camera** cam, hitable** hlist, float
 * aspect)` against include/srr/ref_api.h, render nx x ny x ns with maxDepth on
 * the GPU(s) (the 8 render threads of :923-932 become one srr_render, over
 * --gpus N devices of the node with one RCCL gather at frame end), print the
 * elapsed milliseconds (:934-937) and write the ASCII P3 image (:848-886).
 *
 *     int main(int argc, char** argv) {
 *       static const srr::ref::scene_entry scenes[] = {{2, "ball_scenes", ball_scenes}, ...};
 *       return srr::ref::render_main(argc, argv, scenes, sizeof scenes / sizeof scenes[0]);
 *     }
 *
 * Options (defaults are the reference's globals, Raytracing_n.cpp:39-43):
 *   --sceneid N | --scene NAME   which builder (default sceneid 2)
 *   --scene-text FILE            instead of a builder: an srr scene description
 *                                (srr_scene_from_text), e.g. one of the reference's
 *                                builders written by python -m srr.ref_scenes
 *   --nx 1000 --ny 1000 --ns 50 --max-depth 50 --device 0 --out out.ppm
 *   --gpus N                     render on devices device .. device+N-1
 *                                (srr_renderer_create_multi: tiles of --tile
 *                                pixels, default 1, dealt round-robin, one RCCL
 *                                gather to the first device); bitwise the 1-GPU image
 *   --devices 0,1,2,3            the same with an explicit device list (a list of
 *                                one device still goes through the RCCL gather)
 *   --dry-run                    build the scene and print its digest
 *                                (srr_scene_digest), no GPU
 * Differences, all forced by the reference: its render threads race on shared
 * state and its pixel mapping scrambles non-square frames (Q12);
 * srr renders every (pixel, sample) path with its per-path seed.  Exit codes:
 * 0, 1 on an srr error (message on stderr), 2 on bad arguments. */
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "ref_api.h"

namespace srr {
namespace ref {

using builder_fn = void (*)(hitable** scene, camera** cam, hitable** hlist, float aspect);

struct scene_entry {
  int sceneid;
  const char* name;
  builder_fn build;
};

inline int render_main(int argc, char** argv, const scene_entry* scenes, int n_scenes) {
  int nx = 1000, ny = 1000, ns = 50, max_depth = 50, sceneid = 2, device = 0;  // Raytracing_n.cpp:39-43
  int gpus = 1, tile = 1;
  std::vector<int> devices;
  std::string name, out = "out.ppm", text_path;
  bool dry = false;
  auto usage = [&]() {
    std::fprintf(stderr, "usage: %s [--sceneid N | --scene NAME] [--nx N] [--ny N] [--ns N] [--max-depth N] "
                         "[--device N] [--gpus N | --devices a,b,..] [--tile N] [--out FILE] [--dry-run]\nscenes:",
                 argv[0]);
    for (int k = 0; k < n_scenes; ++k) std::fprintf(stderr, " %d:%s", scenes[k].sceneid, scenes[k].name);
    std::fprintf(stderr, "\n");
    return 2;
  };
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto num = [&](int& v) {
      if (i + 1 >= argc) return false;
      v = std::atoi(argv[++i]);
      return true;
    };
    bool ok = true;
    if (a == "--sceneid") ok = num(sceneid);
    else if (a == "--scene" && i + 1 < argc) name = argv[++i];
    else if (a == "--scene-text" && i + 1 < argc) text_path = argv[++i];
    else if (a == "--nx") ok = num(nx);
    else if (a == "--ny") ok = num(ny);
    else if (a == "--ns") ok = num(ns);
    else if (a == "--max-depth") ok = num(max_depth);
    else if (a == "--device") ok = num(device);
    else if (a == "--gpus") ok = num(gpus) && gpus >= 1;
    else if (a == "--tile") ok = num(tile) && tile >= 1;
    else if (a == "--devices" && i + 1 < argc) {
      std::stringstream ds(argv[++i]);
      for (std::string t; std::getline(ds, t, ',');) devices.push_back(std::atoi(t.c_str()));
      ok = !devices.empty();
    }
    else if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (a == "--dry-run") dry = true;
    else ok = false;
    if (!ok) return usage();
  }
  const scene_entry* e = nullptr;
  for (int k = 0; k < n_scenes; ++k)
    if (name.empty() ? scenes[k].sceneid == sceneid : name == scenes[k].name) e = &scenes[k];
  if ((!e && text_path.empty()) || nx < 1 || ny < 1 || ns < 1) return usage();
  const char* scene_name = text_path.empty() ? e->name : text_path.c_str();

  srr_scene* s = nullptr;
  if (!text_path.empty()) {
    std::ifstream f(text_path);
    std::stringstream ss;
    ss << f.rdbuf();
    if (!f || srr_scene_from_text(ss.str().c_str(), &s) < 0) {
      std::fprintf(stderr, "%s: %s\n", text_path.c_str(), f ? srr_last_error() : "cannot read");
      return 1;
    }
  } else {
    s = srr_scene_create();
    if (!s) return 1;
    hitable *world = nullptr, *hlist = nullptr;
    camera* cam = nullptr;
    try {
      scene_scope scope(s);
      e->build(&world, &cam, &hlist, float(nx) / float(ny));  // :894-919
      if (!world) throw error(SRR_EINVAL, "the builder set no world");
      capture(world, hlist);
    } catch (const error& x) {
      std::fprintf(stderr, "%s\n", x.what());
      srr_scene_destroy(s);
      return 1;
    }
  }
  if (dry) {
    uint64_t d = 0;
    if (srr_scene_digest(s, &d, nullptr) < 0) {
      std::fprintf(stderr, "%s\n", srr_last_error());
      srr_scene_destroy(s);
      return 1;
    }
    std::printf("%s %016llx\n", scene_name, (unsigned long long)d);
    srr_scene_destroy(s);
    return 0;
  }
  const bool multi = !devices.empty() || gpus > 1;  // an explicit --devices list: multi even for one device
  if (devices.empty())
    for (int k = 0; k < gpus; ++k) devices.push_back(device + k);
  srr_renderer* r = nullptr;
  const int rc0 = multi ? srr_renderer_create_multi(s, (int)devices.size(), devices.data(), &r)
                        : srr_renderer_create(s, devices[0], &r);
  if (rc0 < 0) {
    std::fprintf(stderr, "%s\n", srr_last_error());
    srr_scene_destroy(s);
    return 1;
  }
  srr_params p{};
  p.nx = nx;
  p.ny = ny;
  p.spp = ns;
  p.max_depth = max_depth;
  p.tile = tile;
  p.shard_count = 1;
  std::vector<unsigned char> rgb8(3 * (size_t)nx * ny);
  srr_stats st{};
  const auto t0 = std::chrono::steady_clock::now();
  int rc = srr_render(r, &p, nullptr, rgb8.data(), &st);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (rc == 0) rc = srr_write_ppm(out.c_str(), nx, ny, rgb8.data());
  if (rc < 0) std::fprintf(stderr, "%s\n", srr_last_error());
  else {
    std::printf("%dms\n", (int)ms);  // :934-937
    std::fprintf(stderr, "%s: %dx%dx%d, %lld world rays, %.1f Msamples/s on %d GPU(s) (%s) -> %s\n", scene_name, nx,
                 ny, ns, (long long)st.world_rays, st.world_rays / (ms * 1e3), (int)devices.size(),
                 srr_renderer_transport(r), out.c_str());
  }
  srr_renderer_destroy(r);
  srr_scene_destroy(s);
  return rc < 0 ? 1 : 0;
}

}  // namespace ref
}  // namespace srr

// INTEGRATION.md §1 worked example: the reference's Cornell-box + teapot builder
// (Raytracing_n.cpp:216-304 style; scene S2 of SURVEY.md §8(d)) written against the
// C-ABI, rendered with srr_render (the renderthread/main replacement) and written as
// the reference's P3 PPM.  tests/test_integration_example.py builds it (CPU) and
// checks its image against the Python-built S2 render (GPU).
//
//   cornell_teapot NX NY SPP OUT.ppm [OUT_MEAN.f32]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "srr_capi.h"

static int check(int rc) {
  if (rc < 0) {
    std::fprintf(stderr, "srr error %d: %s\n", rc, srr_last_error());
    std::exit(1);
  }
  return rc;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s NX NY SPP OUT.ppm [OUT_MEAN.f32]\n", argv[0]);
    return 2;
  }
  srr_scene* s = srr_scene_create();
  int red = check(srr_lambertian(s, check(srr_constant_texture(s, .65f, .05f, .05f))));
  int white = check(srr_lambertian(s, check(srr_constant_texture(s, .73f, .73f, .73f))));
  int green = check(srr_lambertian(s, check(srr_constant_texture(s, .12f, .45f, .15f))));
  int light = check(srr_diffuse_light(s, check(srr_constant_texture(s, 15.f, 15.f, 15.f))));
  std::vector<int> list;
  list.push_back(check(srr_flip_normals(s, check(srr_yz_rect(s, 0, 555, 0, 555, 555, green)))));
  list.push_back(check(srr_yz_rect(s, 0, 555, 0, 555, 0, red)));
  list.push_back(check(srr_flip_normals(s, check(srr_xz_rect(s, 0, 555, 0, 555, 555, white)))));
  list.push_back(check(srr_xz_rect(s, 0, 555, 0, 555, 0, white)));
  list.push_back(check(srr_flip_normals(s, check(srr_xy_rect(s, 0, 555, 0, 555, 555, white)))));
  list.push_back(check(srr_flip_normals(s, check(srr_xz_rect(s, 213, 343, 227, 332, 554, light)))));
  const float c[3] = {190, 90, 190};
  list.push_back(check(srr_sphere(s, c, 90, white)));
  // teapot(60, white) with divs 10 (teapot.h:16), bvh_node(tris, n, 0, 1) (bvh.h:96),
  // rotate_x(.., 90) and translate(.., (330, 0, 300)) (hitable.h)
  int first = 0;
  int ntri = check(srr_teapot(s, 60.f, 10, white, &first));
  std::vector<int> tris(ntri);
  for (int k = 0; k < ntri; ++k) tris[k] = first + k;
  int bvh = check(srr_bvh_node(s, tris.data(), ntri, 0.f, 1.f));
  const float off[3] = {330, 0, 300};
  list.push_back(check(srr_translate(s, check(srr_rotate_x(s, bvh, 90.f)), off)));
  check(srr_scene_set_world(s, check(srr_hitable_list(s, list.data(), (int)list.size()))));
  const float from[3] = {278, 278, -800}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
  check(srr_camera(s, from, at, up, 40.f, 1.f, 0.f, 10.f, 0.f, 1.f));
  int lshape = check(srr_flip_normals(s, check(srr_xz_rect(s, 213, 343, 227, 332, 554, -1))));
  check(srr_scene_set_lights(s, check(srr_hitable_list(s, &lshape, 1))));  // hlist

  srr_renderer* r = nullptr;
  check(srr_renderer_create(s, /*device*/ 0, &r));
  srr_params p{};
  p.nx = std::atoi(argv[1]);
  p.ny = std::atoi(argv[2]);
  p.spp = std::atoi(argv[3]);
  p.max_depth = 50;
  p.tile = 32;
  p.shard_count = 1;
  std::vector<float> mean(3 * (size_t)p.nx * p.ny);
  std::vector<unsigned char> rgb8(mean.size());
  srr_stats st{};
  check(srr_render(r, &p, mean.data(), rgb8.data(), &st));
  check(srr_write_ppm(argv[4], p.nx, p.ny, rgb8.data()));
  if (argc > 5) {
    FILE* f = std::fopen(argv[5], "wb");
    if (!f || std::fwrite(mean.data(), sizeof(float), mean.size(), f) != mean.size()) return 1;
    std::fclose(f);
  }
  std::printf("world rays %lld in %.1f ms\n", (long long)st.world_rays, st.total_ms);
  srr_renderer_destroy(r);
  srr_scene_destroy(s);
  return 0;
}

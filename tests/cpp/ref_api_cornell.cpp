// A scene builder written the way the reference writes them
// (Raytracing_n.cpp:216-304: `void f(hitable** scene, camera** cam, hitable**
// hlist, float aspect)`), compiled against srr's reference-compatible classes
// (include/srr/ref_api.h) instead of the reference's headers, then rendered
// through the C-ABI.  tests/test_integration_example.py checks its image against
// the Python-built S2 scene bitwise.
//
//   ref_api_cornell NX NY SPP OUT_MEAN.f32 [MESH_FILE]
//
// With MESH_FILE the teapot is replaced by model(MESH_FILE, ...).genhitablemodel()
// (model.h:28-91), the way the reference's soldier_scene loads its mesh.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "srr/ref_api.h"

using namespace srr::ref;

static const char* g_mesh = nullptr;

void cornell_teapot(hitable** scene, camera** cam, hitable** hlist, float aspect) {
  int i = 0;
  hitable** list = new hitable*[9];
  material* red = new lambertian(new constant_texture(vec3(0.65f, 0.05f, 0.05f)));
  material* white = new lambertian(new constant_texture(vec3(0.73f, 0.73f, 0.73f)));
  material* green = new lambertian(new constant_texture(vec3(0.12f, 0.45f, 0.15f)));
  material* light = new diffuse_light(new constant_texture(vec3(15, 15, 15)));
  list[i++] = new flip_normals(new yz_rect(0, 555, 0, 555, 555, green));
  list[i++] = new yz_rect(0, 555, 0, 555, 0, red);
  list[i++] = new flip_normals(new xz_rect(0, 555, 0, 555, 555, white));
  list[i++] = new xz_rect(0, 555, 0, 555, 0, white);
  list[i++] = new flip_normals(new xy_rect(0, 555, 0, 555, 555, white));
  list[i++] = new flip_normals(new xz_rect(213, 343, 227, 332, 554, light));
  list[i++] = new sphere(vec3(190, 90, 190), 90, white);
  hitable** tris;
  int ntris;
  if (g_mesh) {
    model* m = new model(g_mesh, true, true, white, vec3(1, 1, 1));
    tris = m->genhitablemodel();
    ntris = m->gettrianglecount();
  } else {
    teapot* tp = new teapot(60, white, 10);
    tris = tp->createPloyTeapot();
    ntris = tp->getTriangleCount();
  }
  list[i++] = new translate(new rotate_x(new bvh_node(tris, ntris, 0, 1), 90), vec3(330, 0, 300));
  *scene = new hitable_list(list, i);
  *cam = new camera(vec3(278, 278, -800), vec3(278, 278, 0), vec3(0, 1, 0), 40, aspect, 0.0f, 10.0f, 0.0f, 1.0f);
  hitable** lights = new hitable*[1];
  lights[0] = new flip_normals(new xz_rect(213, 343, 227, 332, 554, nullptr));
  *hlist = new hitable_list(lights, 1);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s NX NY SPP OUT_MEAN.f32 [MESH_FILE]\n", argv[0]);
    return 2;
  }
  if (argc > 5) g_mesh = argv[5];
  srr_scene* s = srr_scene_create();
  hitable *world = nullptr, *hlist = nullptr;
  camera* cam = nullptr;
  try {
    scene_scope scope(s);
    cornell_teapot(&world, &cam, &hlist, 1.0f);
    capture(world, hlist);
  } catch (const error& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  srr_renderer* r = nullptr;
  if (srr_renderer_create(s, 0, &r) < 0) {
    std::fprintf(stderr, "%s\n", srr_last_error());
    return 1;
  }
  srr_params p{};
  p.nx = std::atoi(argv[1]);
  p.ny = std::atoi(argv[2]);
  p.spp = std::atoi(argv[3]);
  p.max_depth = 50;
  p.tile = 32;
  p.shard_count = 1;
  std::vector<float> mean(3 * (size_t)p.nx * p.ny);
  if (srr_render(r, &p, mean.data(), nullptr, nullptr) < 0) {
    std::fprintf(stderr, "%s\n", srr_last_error());
    return 1;
  }
  FILE* f = std::fopen(argv[4], "wb");
  if (!f || std::fwrite(mean.data(), sizeof(float), mean.size(), f) != mean.size()) return 1;
  std::fclose(f);
  srr_renderer_destroy(r);
  srr_scene_destroy(s);
  return 0;
}

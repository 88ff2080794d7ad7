// render_main: the reference's program (Raytracing_n.cpp:882-952) as a C++
// binary over srr (include/srr/render_main.h), with the BASELINE configs'
// scenes written as reference-style builders against include/srr/ref_api.h.
// They mirror srr/scenes.py call for call (tests/test_render_main.py checks the
// scene digests against the Python-built scenes, and on the GPU the images).
//
//   render_main --scene s2 --nx 512 --ny 512 --ns 1024 --out c2.ppm
//   render_main --scene-text FILE ...   (any srr scene description, e.g. one of
//                                        the reference's own builders written by
//                                        python -m srr.ref_scenes --sceneid N)
//
// The reference's own builders (cornell_box, ball_scenes, final, ...) compile
// unchanged against ref_api.h; a program that links them passes its own table
// to srr::ref::render_main with the reference's sceneids (:893-919).
#include "srr/render_main.h"

using namespace srr::ref;

namespace {

const vec3 kRed(0.65f, 0.05f, 0.05f), kWhite(0.73f, 0.73f, 0.73f), kGreen(0.12f, 0.45f, 0.15f);

// the Cornell box of SURVEY §8(d) S1: five walls, the ceiling light, a sphere
int cornell(hitable** list, material** white_out, material* sphere_mat) {
  int i = 0;
  material* red = new lambertian(new constant_texture(kRed));
  material* white = new lambertian(new constant_texture(kWhite));
  material* green = new lambertian(new constant_texture(kGreen));
  material* light = new diffuse_light(new constant_texture(vec3(15.0f)));
  list[i++] = new flip_normals(new yz_rect(0, 555, 0, 555, 555, green));
  list[i++] = new yz_rect(0, 555, 0, 555, 0, red);
  list[i++] = new flip_normals(new xz_rect(0, 555, 0, 555, 555, white));
  list[i++] = new xz_rect(0, 555, 0, 555, 0, white);
  list[i++] = new flip_normals(new xy_rect(0, 555, 0, 555, 555, white));
  list[i++] = new flip_normals(new xz_rect(213, 343, 227, 332, 554, light));
  list[i++] = new sphere(vec3(190, 90, 190), 90, sphere_mat ? sphere_mat : white);
  *white_out = white;
  return i;
}

void cornell_camera_and_lights(camera** cam, hitable** hlist, float aspect) {
  *cam = new camera(vec3(278, 278, -800), vec3(278, 278, 0), vec3(0, 1, 0), 40, aspect, 0.0f, 10.0f, 0.0f, 1.0f);
  hitable** lights = new hitable*[1];
  lights[0] = new flip_normals(new xz_rect(213, 343, 227, 332, 554, nullptr));
  *hlist = new hitable_list(lights, 1);
}

// translate(rotate_x(bvh_node(teapot), 90), at): the teapot of S2-S5 (z-up, Q6)
hitable* teapot_instance(material* m, int divs, const vec3& at) {
  teapot* tp = new teapot(60, m, divs);
  hitable** tris = tp->createPloyTeapot();
  return new translate(new rotate_x(new bvh_node(tris, tp->getTriangleCount(), 0, 1), 90), at);
}

// C1: Cornell box, lambertian only (aarect + sphere), 256x256x64
void s1_cornell(hitable** scene, camera** cam, hitable** hlist, float aspect) {
  hitable** list = new hitable*[8];
  material* white;
  const int n = cornell(list, &white, nullptr);
  *scene = new hitable_list(list, n);
  cornell_camera_and_lights(cam, hlist, aspect);
}

// C2: + the 6,400-triangle Utah teapot, lambertian 0.73, 512x512x1024
void s2_cornell_teapot(hitable** scene, camera** cam, hitable** hlist, float aspect) {
  hitable** list = new hitable*[8];
  material* white;
  int n = cornell(list, &white, nullptr);
  list[n++] = teapot_instance(white, 10, vec3(330, 0, 300));
  *scene = new hitable_list(list, n);
  cornell_camera_and_lights(cam, hlist, aspect);
}

// C3: microfacet (beckmann 0.01 / 0.05, gold) or metal teapot, dielectric sphere
void s3_teapot(hitable** scene, camera** cam, hitable** hlist, float aspect, bool metal_pot) {
  material* glass = new dielectric(1.5f);
  hitable** list = new hitable*[8];
  material* white;
  int n = cornell(list, &white, glass);
  material* tm = metal_pot ? (material*)new metal(vec3(0.9f), 0.0f)
                           : (material*)new beckmann(new constant_texture(vec3(0.945f, 0.75f, 0.336f)), 0.01f, 0.05f);
  list[n++] = teapot_instance(tm, 10, vec3(330, 0, 300));
  *scene = new hitable_list(list, n);
  cornell_camera_and_lights(cam, hlist, aspect);
}
void s3_beckmann(hitable** s, camera** c, hitable** h, float a) { s3_teapot(s, c, h, a, false); }
void s3_metal(hitable** s, camera** c, hitable** h, float a) { s3_teapot(s, c, h, a, true); }

// C4 / C5: soldier_scene's geometry with a 102,400-triangle
// teapot for the soldier and generated textures; C5 adds the fog
void s4_soldier(hitable** scene, camera** cam, hitable** hlist, float aspect, bool fog) {
  const vec3 lookfrom(300, 500, -800);
  material* light = new diffuse_light(new constant_texture(vec3(35.0f)));
  texture* floor_tex = new generated_texture(256, 256, 1234, 1);
  texture* env_tex = new generated_texture(1024, 512, 1234, 0);
  material* floor_mat = new orennayar(floor_tex, 0.5f);
  material* glass = new dielectric(1.4f);
  hitable** list = new hitable*[6];
  int i = 0;
  list[i++] = new flip_normals(new xz_rect(203, 353, 17, 167, 800, light));
  list[i++] = new box(vec3(0, -0.1f, 0), vec3(600, 0.1f, 600), floor_mat);
  list[i++] = new box(vec3(0, -1, 0), vec3(600, 1, 600), glass);
  list[i++] = new flip_normals(new sphere(lookfrom, 10000, new diffuse_light(env_tex)));
  material* tm = new beckmann(new constant_texture(vec3(0.8f, 0.85f, 0.88f)), 0.9f, 0.85f);
  list[i++] = teapot_instance(tm, 40, vec3(300, 0, 300));
  if (fog) {
    hitable* boundary = new sphere(vec3(0, 0, 0), 5000, new dielectric(1.5f));
    list[i++] = new constant_medium(boundary, 0.0001f, new constant_texture(vec3(1.0f)));
  }
  *scene = new hitable_list(list, i);
  *cam = new camera(lookfrom, vec3(300, 278, 200), vec3(0, 1, 0), 40, aspect, 10.0f, 1000.0f, 0.0f, 1.0f);
  hitable** lights = new hitable*[1];
  lights[0] = new flip_normals(new xz_rect(203, 353, 17, 167, 800, nullptr));
  *hlist = new hitable_list(lights, 1);
}
void s4_soldier_standin(hitable** s, camera** c, hitable** h, float a) { s4_soldier(s, c, h, a, false); }
void s5_soldier_fog(hitable** s, camera** c, hitable** h, float a) { s4_soldier(s, c, h, a, true); }

const scene_entry kScenes[] = {
    {1, "s1", s1_cornell},         {2, "s2", s2_cornell_teapot},      {3, "s3", s3_beckmann},
    {4, "s3_metal", s3_metal},     {5, "s4", s4_soldier_standin},     {6, "s5", s5_soldier_fog},
};

}  // namespace

int main(int argc, char** argv) { return render_main(argc, argv, kScenes, (int)(sizeof kScenes / sizeof kScenes[0])); }

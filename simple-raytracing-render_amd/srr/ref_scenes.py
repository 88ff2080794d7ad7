"""The reference's own scene builders (Raytracing_n.cpp:108-711), restated over
the reference-named builder API of ``scene.py`` with the reference's assets.

``main()`` (Raytracing_n.cpp:882-952) picks one with ``sceneid`` (:43): 0
cornell_box, 1 teapot_scene, 2 ball_scenes (the as-shipped default), 3
ball_orennayar_scenes, 4 jadebunny_scene, 5 final, 6 soldier_scene, 7
flatnormal_bunny; ``random_scene`` (:108) is the remaining builder.  Each
function here issues the same constructor calls in the same order -- including
every ``drand48()`` draw, in the order g++ evaluates the arguments (pinned by tests/test_ref_scenes.py against the reference's own builders
run by oracle/ref's harness) -- so the scene LCG reaches every ``bvh_node`` in
the state the reference's does.

Assets are read from ``contents`` (default ``$SRR_CONTENTS`` or
/root/reference/contents): images through srr's stb-exact decoder
(Scene.image_texture_file), meshes through srr's PLY / FBX loaders
(Scene.model).  Deviations, each forced by the reference itself:

* teapot_scene loads ``contents/models/dragon.ply``, which the reference does
  not ship (assimp returns no scene and the reference dereferences it): the
  dragon is left out unless ``dragon=`` names a file.
* flatnormal_bunny never assigns ``*hlist`` (uninitialised pointer, :659-689):
  build definition ``hlist = hitable_list([light_shape])`` (its ``a[0]``).
* teapots built by ``teapot::createPloyTeapot`` get face normals.
"""
from __future__ import annotations

import os

import numpy as np

from .scene import Scene

CONTENTS = os.environ.get("SRR_CONTENTS", "/root/reference/contents")


def _f32(x):
    return np.float32(x)


def _size_t_f32(x: int) -> float:
    """An unsigned 64-bit (size_t) expression converted to float, as C++ does."""
    return float(np.float32(float(x % (1 << 64))))


def _asset(contents, *parts):
    return os.path.join(contents or CONTENTS, *parts)


def _env_sphere(sc: Scene, lookfrom, image_path):
    """flip_normals(sphere(lookfrom, 10000, diffuse_light(image_texture(...))))"""
    return sc.flip_normals(sc.sphere(lookfrom, 10000, sc.diffuse_light(sc.image_texture_file(image_path))))


def random_scene(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:108-182: checker ground, 22x22 grid of small moving
    lambertian / metal / glass spheres, three large spheres, a 6-rect sky box."""
    sc = Scene()
    lookfrom = (-10, 6, -15)
    sc.camera(lookfrom, (0, 0, 0), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    checker = sc.checker_texture(sc.constant_texture((0.2, 0.3, 0.1)), sc.constant_texture((0.9, 0.9, 0.9)))
    objs = [sc.sphere((0, -1000, 0), 1000, sc.lambertian(checker))]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose_mat = sc.drand48()
            dz = sc.drand48()  # center(a + 0.9*drand48(), 0.2, b + drand48()): last argument first
            dx = sc.drand48()
            center = np.array([_f32(a + 0.9 * dx), _f32(0.2), _f32(b + dz)], np.float32)
            d = center - np.array([4, 0.2, 0], np.float32)
            if float(np.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])) > 0.9:
                if choose_mat < 0.8:
                    dy = sc.drand48()
                    c1 = center + np.array([0, _f32(0.5 * dy), 0], np.float32)
                    objs.append(sc.moving_sphere(center.tolist(), c1.tolist(), 0.0, 1.0, 0.2,
                                                 sc.lambertian(sc.constant_texture(0.5))))
                elif choose_mat < 0.95:
                    # metal(vec3(0.5*(1+d), 0.5*(1+d), 0.5*(1+d)), 0.5*d): the vec3 temporary
                    # (its arguments last to first), then the fuzz argument
                    bz, by, bx = sc.drand48(), sc.drand48(), sc.drand48()
                    fuzz = 0.5 * sc.drand48()
                    objs.append(sc.sphere(center.tolist(), 0.2,
                                          sc.metal((0.5 * (1 + bx), 0.5 * (1 + by), 0.5 * (1 + bz)), fuzz)))
                else:
                    objs.append(sc.sphere(center.tolist(), 0.2, sc.dielectric(1.5)))
    objs.append(sc.sphere((0, 1, 0), 1.0, sc.dielectric(1.5)))
    objs.append(sc.sphere((-4, 1, 0), 1.0, sc.lambertian(sc.constant_texture((0.4, 0.2, 0.1)))))
    objs.append(sc.sphere((4, 1, 0), 1.0, sc.metal((0.7, 0.6, 0.5), 0.0)))
    sky = lambda f: sc.diffuse_light(sc.image_texture_file(_asset(contents, "environment_map", "sky_1", f)))  # noqa: E731
    env = [
        sc.xy_rect(-100, 100, -100, 100, -100, sky("Front.jpg")),
        sc.flip_normals(sc.xy_rect(-100, 100, -100, 100, 100, sky("Back.jpg"))),
        sc.yz_rect(-100, 100, -100, 100, 100, sky("Left.jpg")),
        sc.flip_normals(sc.yz_rect(-100, 100, -100, 100, -100, sky("Right.jpg"))),
        sc.flip_normals(sc.xz_rect(-100, 100, -100, 100, 100, sky("Top.jpg"))),
        sc.xz_rect(-100, 100, -100, 100, -100, sky("Bottom.jpg")),
    ]
    objs += env
    sc.set_lights(sc.hitable_list(env))
    sc.set_world(sc.hitable_list(objs))
    return sc


def _bunny(sc: Scene, contents, flip_winding, mat, scale, at):
    tris = sc.model(_asset(contents, "models", "bunny.ply"), False, flip_winding, mat, (scale,) * 3)
    return sc.translate(sc.rotate_y(sc.bvh_node(tris, 0, 1), 180), at)


def cornell_box(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:216-304 (sceneid 0): Oren-Nayar floor, light at y=800,
    sky_2 environment sphere, Oren-Nayar bunny (assimp PLY, scale 2000)."""
    sc = Scene()
    lookfrom = (300, 500, -800)
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(45))
    orennayar_white_0 = sc.orennayar(sc.constant_texture(0.7), 0)
    orennayar_white_10 = sc.orennayar(sc.constant_texture(0.7), 10)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800, light)),
        sc.xz_rect(0, 555, 0, 555, 0, orennayar_white_0),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
        _bunny(sc, contents, True, orennayar_white_10, 2000, (250, -70, 400)),
    ]
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800))]))
    return sc


def teapot_scene(aspect: float, contents: str | None = None, divs: int = 100, dragon: str | None = None) -> Scene:
    """Raytracing_n.cpp:306-377 (sceneid 1): two 640,000-triangle teapots (metal,
    beckmann gold), Oren-Nayar bunny, glass sphere wrapped in blue fog, sky_2."""
    sc = Scene()
    lookfrom = (100, 800, -400)
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(40))
    beckmann_gold = sc.beckmann(sc.constant_texture((0.945, 0.75, 0.336)), 0.01, 0.05)
    beckmann_silver = sc.beckmann(sc.constant_texture((0.8, 0.85, 0.88)), 0.1, 0.1)
    lambertian_brow = sc.lambertian(sc.constant_texture((0.426, 0.3, 0.254)))
    orennayar_white = sc.orennayar(sc.constant_texture(1), 10)
    objs = [
        sc.flip_normals(sc.xz_rect(3, 153, 217, 343, 800, light)),
        sc.xz_rect(0, 555, 0, 555, 0, lambertian_brow),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
    ]
    t1 = sc.teapot(40, divs, sc.metal(0.9, 0.0))
    objs.append(sc.translate(sc.rotate_x(sc.bvh_node(t1, 0, 1), 90), (200, 0, 250)))
    t2 = sc.teapot(40, divs, beckmann_gold)
    objs.append(sc.translate(sc.rotate_x(sc.bvh_node(t2, 0, 1), 90), (360, 0, 150)))
    objs.append(_bunny(sc, contents, True, orennayar_white, 2000, (180, -70, 450)))
    c = sc.sphere((280, 30, 70), 30, sc.dielectric(1.5))
    objs.append(c)
    objs.append(sc.constant_medium(c, 0.2, sc.constant_texture((0.2, 0.4, 0.9))))
    if dragon:
        tris = sc.model(dragon, False, True, beckmann_silver, (500, 500, 500))
        objs.append(sc.translate(sc.rotate_y(sc.bvh_node(tris, 0, 1), 180), (140, -20, 120)))
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(3, 153, 217, 343, 800))]))
    return sc


def ball_scenes(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:379-425 (sceneid 2, the as-shipped default): 11x11
    white Beckmann spheres with roughness (j%11)/11, (j/11)/11."""
    sc = Scene()
    lookfrom = (300, 600, -100)
    sc.camera(lookfrom, (300, 20, 250), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(20))
    sc.orennayar(sc.constant_texture(0.7), 10)  # orennayar_white_10 (constructed, unused)
    orennayar_brow = sc.orennayar(sc.constant_texture((0.426, 0.3, 0.254)), 0)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800, light)),
        sc.xz_rect(-100, 655, -100, 655, 0, orennayar_brow),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
    ]
    for j in range(121):
        m = sc.beckmann(sc.constant_texture(1), float(_f32(j % 11) / _f32(11)), float(_f32(j // 11) / _f32(11)))
        # j is a size_t (Raytracing_n.cpp:400): 450 - 50*(j/11) wraps for the last
        # row (j >= 110) to 2^64 - 50, which the vec3 float rounds to 2^64
        objs.append(sc.sphere((_size_t_f32(550 - (j % 11) * 50), 20, _size_t_f32(450 - 50 * (j // 11))), 20, m))
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800))]))
    return sc


def ball_orennayar_scenes(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:427-473 (sceneid 3): 21 white Oren-Nayar spheres with
    sigma 0..20 degrees."""
    sc = Scene()
    lookfrom = (300, 800, -100)
    sc.camera(lookfrom, (300, 20, 450), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(20))
    sc.orennayar(sc.constant_texture(0.7), 10)  # orennayar_white_10 (constructed, unused)
    orennayar_brow = sc.orennayar(sc.constant_texture((0.426, 0.3, 0.254)), 0)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800, light)),
        sc.xz_rect(-100, 655, -100, 655, 0, orennayar_brow),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
    ]
    for j in range(21):
        objs.append(sc.sphere((550 - (j % 7) * 70, 30, 450 - 70 * (j // 7)), 30,
                              sc.orennayar(sc.constant_texture(1), j)))
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800))]))
    return sc


def final(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:475-533 (sceneid 5): "The Next Week" final scene -- BVH
    of 400 random-height boxes, moving sphere, glass, metal, blue fog ball,
    global thin fog, earth-map sphere, Perlin sphere, BVH of 1,000 spheres."""
    sc = Scene()
    white = sc.lambertian(sc.constant_texture((0.73, 0.73, 0.73)))
    ground = sc.lambertian(sc.constant_texture((0.48, 0.83, 0.53)))
    boxes = []
    for i in range(20):
        for j in range(20):
            w = 100.0
            x0 = -1000 + i * w
            z0 = -1000 + j * w
            y1 = float(_f32(100 * (sc.drand48() + 0.01)))
            boxes.append(sc.box((x0, 0, z0), (x0 + w, y1, z0 + w), ground))
    objs = [sc.bvh_node(boxes, 0, 1)]
    light = sc.diffuse_light(sc.constant_texture((7, 7, 7)))
    objs.append(sc.flip_normals(sc.xz_rect(123, 423, 147, 412, 554, light)))
    objs.append(sc.moving_sphere((400, 400, 200), (430, 400, 200), 0, 1, 50,
                                 sc.lambertian(sc.constant_texture((0.7, 0.3, 0.1)))))
    objs.append(sc.sphere((260, 150, 45), 50, sc.dielectric(1.5)))
    objs.append(sc.sphere((0, 150, 145), 50, sc.metal((0.8, 0.8, 0.9), 1.0)))
    boundary = sc.sphere((360, 150, 145), 70, sc.dielectric(1.5))
    objs.append(boundary)
    objs.append(sc.constant_medium(boundary, 0.2, sc.constant_texture((0.2, 0.4, 0.9))))
    boundary = sc.sphere((0, 0, 0), 5000, sc.dielectric(1.5))
    objs.append(sc.constant_medium(boundary, 0.0001, sc.constant_texture((1.0, 1.0, 1.0))))
    emat = sc.lambertian(sc.image_texture_file(_asset(contents, "textures", "earthmap.jpg")))
    objs.append(sc.sphere((400, 200, 400), 100, emat))
    objs.append(sc.sphere((220, 280, 300), 80, sc.lambertian(sc.noise_texture(0.1))))
    spheres = []
    for _ in range(1000):
        z, y, x = sc.drand48(), sc.drand48(), sc.drand48()  # vec3(165*d, 165*d, 165*d): last first
        spheres.append(sc.sphere((165 * x, 165 * y, 165 * z), 10, white))
    objs.append(sc.translate(sc.rotate_y(sc.bvh_node(spheres, 0.0, 1.0), 15), (-100, 270, 395)))
    sc.set_world(sc.hitable_list(objs))
    sc.camera((478, 278, -600), (278, 278, 0), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(123, 423, 147, 412, 554))]))
    return sc


def jadebunny_scene(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:535-583 (sceneid 4): glass bunny around a slightly
    smaller blue Oren-Nayar bunny."""
    sc = Scene()
    lookfrom = (300, 500, -800)
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(45))
    glass = sc.dielectric(1.2)
    orennayar_white_0 = sc.orennayar(sc.constant_texture(0.7), 0)
    orennayar_blue = sc.orennayar(sc.constant_texture((0.2, 0.4, 0.9)), 0)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 17, 543, 800, light)),
        sc.xz_rect(0, 555, 0, 555, 0, orennayar_white_0),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
        _bunny(sc, contents, False, glass, 2000, (250, -70, 400)),
        _bunny(sc, contents, True, orennayar_blue, 1990, (250, -70, 400)),
    ]
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 217, 343, 800))]))
    return sc


def soldier_scene(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:585-657 (sceneid 6): the FBX soldier (mesh 0, scale 8,
    textured Beckmann), wooden Oren-Nayar floor box inside a glass slab, sky4
    environment, depth of field (aperture 10, focus 1000)."""
    sc = Scene()
    lookfrom = (300, 500, -800)
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 10.0, 1000.0, 0.0, 1.0)
    light_1 = sc.diffuse_light(sc.constant_texture(35))
    roughx, roughy = 0.9, 0.85
    floor_tex = sc.image_texture_file(_asset(contents, "textures", "TexturesCom_Wood_Wenge_1K_albedo.png"))
    glass = sc.dielectric(1.4)
    imaged_bottom = sc.orennayar(floor_tex, 0.5)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800, light_1)),
        sc.box((0, -0.1, 0), (600, 0.1, 600), imaged_bottom),
        sc.box((0, -1, 0), (600, 1, 600), glass),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky4.jpg")),
    ]
    skin = sc.image_texture_file(_asset(contents, "textures", "NPC_YuanChengBing_A.png"))
    beckmann_tex = sc.beckmann(skin, roughx, roughy)
    tris = sc.model(_asset(contents, "models", "Soilder.FBX"), False, True, beckmann_tex, (8, 8, 8))
    objs.append(sc.translate(sc.rotate_y(sc.bvh_node(tris, 0, 1), 180), (250, 0, 300)))
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800))]))
    return sc


def flatnormal_bunny(aspect: float, contents: str | None = None) -> Scene:
    """Raytracing_n.cpp:659-689 (sceneid 7): light, Oren-Nayar floor, sky_2.
    The reference builds a Beckmann bunny but never adds it to the list, and
    never assigns ``*hlist`` (build definition: its ``a[0]``, the light shape)."""
    sc = Scene()
    lookfrom = (300, 500, -800)
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light = sc.diffuse_light(sc.constant_texture(45))
    orennayar_white = sc.orennayar(sc.constant_texture(0.7), 0.1)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800, light)),
        sc.xz_rect(0, 600, 0, 600, 0, orennayar_white),
        _env_sphere(sc, lookfrom, _asset(contents, "environment_map", "sky_2.png")),
    ]
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800))]))
    return sc


# main()'s sceneid switch (Raytracing_n.cpp:894-919)
BY_SCENEID = {0: cornell_box, 1: teapot_scene, 2: ball_scenes, 3: ball_orennayar_scenes, 4: jadebunny_scene,
              5: final, 6: soldier_scene, 7: flatnormal_bunny}
BUILDERS = {f.__name__: f for f in list(BY_SCENEID.values()) + [random_scene]}


def main(argv=None) -> int:
    """Write one of the reference's scenes as an srr scene description, for
    programs that take one (render_main --scene-text, srr_scene_from_text):

        python -m srr.ref_scenes --sceneid 2 [--aspect 1.0] [--contents DIR] > balls.scene
    """
    import argparse
    import sys
    ap = argparse.ArgumentParser(prog="python -m srr.ref_scenes")
    ap.add_argument("--sceneid", type=int, choices=sorted(BY_SCENEID))
    ap.add_argument("--builder", choices=sorted(BUILDERS))
    ap.add_argument("--aspect", type=float, default=1.0)
    ap.add_argument("--contents", default=None)
    a = ap.parse_args(argv)
    if (a.sceneid is None) == (a.builder is None):
        ap.error("give one of --sceneid / --builder")
    f = BY_SCENEID[a.sceneid] if a.builder is None else BUILDERS[a.builder]
    sys.stdout.write(f(a.aspect, contents=a.contents).text())
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

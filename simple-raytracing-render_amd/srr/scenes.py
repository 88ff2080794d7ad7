"""Synthetic benchmark scenes S1-S5 (SURVEY.md §8(d) "Synthetic inputs"),
written against the reference-named builder API in ``scene.py`` in the style of
the reference's own builders (``Raytracing_n.cpp:216-657``).  No file from the
reference's ``contents/`` is needed: textures are generated in code (seed 1234)
and the soldier mesh is replaced by a tessellated Utah teapot.

Each function returns ``(Scene, render_defaults)``.
"""
from __future__ import annotations

from .scene import Scene

RED = (0.65, 0.05, 0.05)
WHITE = (0.73, 0.73, 0.73)
GREEN = (0.12, 0.45, 0.15)


def _cornell(sc: Scene, light_level: float = 15.0, sphere_mat=None):
    red = sc.lambertian(sc.constant_texture(RED))
    white = sc.lambertian(sc.constant_texture(WHITE))
    green = sc.lambertian(sc.constant_texture(GREEN))
    light = sc.diffuse_light(sc.constant_texture(light_level))
    objs = [
        sc.flip_normals(sc.yz_rect(0, 555, 0, 555, 555, green)),
        sc.yz_rect(0, 555, 0, 555, 0, red),
        sc.flip_normals(sc.xz_rect(0, 555, 0, 555, 555, white)),
        sc.xz_rect(0, 555, 0, 555, 0, white),
        sc.flip_normals(sc.xy_rect(0, 555, 0, 555, 555, white)),
        sc.flip_normals(sc.xz_rect(213, 343, 227, 332, 554, light)),
        sc.sphere((190, 90, 190), 90, sphere_mat if sphere_mat is not None else white),
    ]
    return objs, white


def _cornell_camera_and_lights(sc: Scene, aspect: float = 1.0):
    sc.camera((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0)
    light_shape = sc.flip_normals(sc.xz_rect(213, 343, 227, 332, 554))
    sc.set_lights(sc.hitable_list([light_shape]))


def s1_cornell() -> tuple[Scene, dict]:
    """C1: Cornell box, lambertian only (aarect + sphere)."""
    sc = Scene()
    objs, _ = _cornell(sc)
    sc.set_world(sc.hitable_list(objs))
    _cornell_camera_and_lights(sc)
    return sc, dict(nx=256, ny=256, spp=64, max_depth=50)


def _teapot_instance(sc: Scene, mat, divs: int, scale: float = 60.0, at=(330, 0, 300)):
    tp = sc.teapot(scale, divs, mat)
    return sc.translate(sc.rotate_x(sc.bvh_node(tp, 0, 1), 90), at)


def s2_cornell_teapot(divs: int = 10) -> tuple[Scene, dict]:
    """C2: Cornell box + Utah teapot (6,400 tris at divs=10), lambertian 0.73."""
    sc = Scene()
    objs, white = _cornell(sc)
    objs.append(_teapot_instance(sc, white, divs))
    sc.set_world(sc.hitable_list(objs))
    _cornell_camera_and_lights(sc)
    return sc, dict(nx=512, ny=512, spp=1024, max_depth=50)


def s3_cornell_teapot_microfacet(variant: str = "beckmann", divs: int = 10) -> tuple[Scene, dict]:
    """C3: C2 with a microfacet (beckmann 0.01/0.05 gold, as Raytracing_n.cpp:324)
    or metal(0.9, 0) (as :348) teapot and a dielectric(1.5) sphere."""
    sc = Scene()
    glass = sc.dielectric(1.5)
    objs, _ = _cornell(sc, sphere_mat=glass)
    if variant == "beckmann":
        tm = sc.beckmann(sc.constant_texture((0.945, 0.75, 0.336)), 0.01, 0.05)
    elif variant == "metal":
        tm = sc.metal(0.9, 0.0)
    else:
        raise ValueError(variant)
    objs.append(_teapot_instance(sc, tm, divs))
    sc.set_world(sc.hitable_list(objs))
    _cornell_camera_and_lights(sc)
    return sc, dict(nx=512, ny=512, spp=1024, max_depth=50)


def s4_soldier_standin(divs: int = 40, fog: bool = False, aspect: float = 1920 / 1080) -> tuple[Scene, dict]:
    """C4 stand-in: soldier_scene geometry (Raytracing_n.cpp:585-657) with the
    soldier replaced by a 102,400-tri teapot; generated env/floor textures.
    ``fog`` adds C5's constant_medium (as Raytracing_n.cpp:506-507)."""
    sc = Scene()
    lookfrom = (300, 500, -800)
    light = sc.diffuse_light(sc.constant_texture(35))
    floor_tex = sc.image_texture_gen(256, 256, 1234, "wood")
    env_tex = sc.image_texture_gen(1024, 512, 1234, "sky")
    floor = sc.orennayar(floor_tex, 0.5)
    glass = sc.dielectric(1.4)
    objs = [
        sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800, light)),
        sc.box((0, -0.1, 0), (600, 0.1, 600), floor),
        sc.box((0, -1, 0), (600, 1, 600), glass),
        sc.flip_normals(sc.sphere(lookfrom, 10000, sc.diffuse_light(env_tex))),
    ]
    tm = sc.beckmann(sc.constant_texture((0.8, 0.85, 0.88)), 0.9, 0.85)
    objs.append(_teapot_instance(sc, tm, divs, at=(300, 0, 300)))
    if fog:
        boundary = sc.sphere((0, 0, 0), 5000, sc.dielectric(1.5))
        objs.append(sc.constant_medium(boundary, 0.0001, sc.constant_texture(1.0)))
    sc.set_world(sc.hitable_list(objs))
    sc.camera(lookfrom, (300, 278, 200), (0, 1, 0), 40.0, aspect, 10.0, 1000.0, 0.0, 1.0)
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(203, 353, 17, 167, 800))]))
    return sc, dict(nx=1920, ny=1080, spp=4096 if fog else 1024, max_depth=50)


def s5_soldier_fog(divs: int = 40) -> tuple[Scene, dict]:
    return s4_soldier_standin(divs=divs, fog=True)


def s6_mixed_lights() -> tuple[Scene, dict]:
    """Cornell box lit by its ceiling rect, an emissive sphere and an emissive
    triangle, all three in the light list (hlist): exercises hitable_list's light
    selection (hitable_list.h:54-67) and the sphere and triangle light pdfs
    (sphere.h:69-86, triangle.h:70-94) next to the xz_rect's (aarect.h:45-60)."""
    sc = Scene()
    objs, _ = _cornell(sc)
    glow = sc.diffuse_light(sc.constant_texture(8.0))
    tri_p = ((150, 500, 150), (400, 520, 180), (260, 540, 420))
    objs.append(sc.sphere((420, 380, 380), 45, glow))
    objs.append(sc.triangle(*tri_p, glow))
    sc.set_world(sc.hitable_list(objs))
    sc.camera((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, 1.0, 0.0, 10.0, 0.0, 1.0)
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(213, 343, 227, 332, 554)),
                                   sc.sphere((420, 380, 380), 45), sc.triangle(*tri_p)]))
    return sc, dict(nx=256, ny=256, spp=64, max_depth=50)


def s7_coplanar_light() -> tuple[Scene, dict]:
    """The resampling loop's attempt cap (DESIGN §2 build definitions): the
    Cornell box (its ceiling light in the world) whose light list (hlist) holds
    only a small triangle lying in the floor's plane y = 0 (where the barycentric
    light samples of ``triangle::random`` stay exactly in the plane).  From a
    floor hit point at y >= 0 every light sample runs in (or just below) the
    triangle's plane, so ``triangle::hit`` rejects it (det < 1e-4,
    triangle.h:146-148) and the lambertian value of that direction is 0
    (pdf.h:40-45); BSDF samples have a zero value too (Q1) and meet the triangle's
    plane at the hit point itself, outside the triangle.  The reference's
    ``while (pdf_val == 0)`` (Raytracing_n.cpp:79-83) never ends there; srr and
    the restatement stop after 100,000 attempts."""
    sc = Scene()
    objs, _ = _cornell(sc)
    sc.set_world(sc.hitable_list(objs))
    sc.camera((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, 1.0, 0.0, 10.0, 0.0, 1.0)
    tri_p = ((500, 0, 500), (500.5, 0, 500), (500.25, 0, 500.5))
    sc.set_lights(sc.hitable_list([sc.triangle(*tri_p)]))
    return sc, dict(nx=12, ny=12, spp=2, max_depth=50)


SCENES = {
    "s1": s1_cornell,
    "s2": s2_cornell_teapot,
    "s3": s3_cornell_teapot_microfacet,
    "s3_metal": lambda: s3_cornell_teapot_microfacet("metal"),
    "s4": s4_soldier_standin,
    "s5": s5_soldier_fog,
    "s6": s6_mixed_lights,
    "s7": s7_coplanar_light,
}

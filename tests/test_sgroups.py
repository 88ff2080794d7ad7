"""Sphere runs behind a BVH (device_scene.h DSGroup, kernels.hip sgroup_hit): a
run of >= 8 consecutive plain spheres of a hitable_list -- random_scene's ~480,
ball_scenes' 121 (Raytracing_n.cpp:108-182, :379-425) -- is tested through a BVH
instead of one by one, and must give the list's answer bit for bit
(hitable_list.h:21-33: the smallest first root below the closest-so-far, ties
to the earliest sphere).  GPU paths against the CPU restatement (which keeps the
reference's linear list), on the reference's two sphere-list scenes and on a
scene built to hit the edge cases: duplicated spheres with different materials
(exact ties), concentric spheres (origins inside), far tiny spheres
(near-tangent rays), moving spheres, a huge ground sphere."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_bind as ob
import parity
from srr import capi, ref_scenes
from srr.scene import Scene

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def edge_scene() -> Scene:
    sc = Scene()
    sc.camera((0, 3, -12), (0, 1, 0), (0, 1, 0), 50.0, 1.0, 0.0, 10.0, 0.0, 1.0)
    white = sc.lambertian(sc.constant_texture((0.73, 0.73, 0.73)))
    red = sc.lambertian(sc.constant_texture((0.65, 0.05, 0.05)))
    steel = sc.metal((0.8, 0.8, 0.9), 0.1)
    glass = sc.dielectric(1.5)
    light = sc.diffuse_light(sc.constant_texture(8.0))
    lamp = sc.xz_rect(-3, 3, -3, 3, 9, light)
    objs = [sc.flip_normals(lamp), sc.sphere((0, -1000, 0), 1000, white)]
    rng = np.random.default_rng(7)
    for k in range(24):
        c = (float(rng.uniform(-4, 4)), float(rng.uniform(0.2, 2.5)), float(rng.uniform(-3, 5)))
        r = float(rng.uniform(0.2, 0.8))
        objs.append(sc.sphere(c, r, [white, red, steel, glass][k % 4]))
        if k % 5 == 0:  # the same sphere again with another material: exact ties
            objs.append(sc.sphere(c, r, steel if k % 2 else red))
        if k % 7 == 0:  # a concentric shell around it
            objs.append(sc.sphere(c, 1.5 * r, glass))
    for k in range(12):  # far tiny spheres: near-tangent camera and bounce rays
        objs.append(sc.sphere((float(rng.uniform(-40, 40)), float(rng.uniform(0, 20)), 60.0), 0.02, white))
    for k in range(10):  # moving spheres
        c0 = (float(rng.uniform(-4, 4)), 0.3, float(rng.uniform(-2, 2)))
        objs.append(sc.moving_sphere(c0, (c0[0], c0[1] + 0.6, c0[2]), 0.0, 1.0, 0.3, red))
    objs.append(sc.xy_rect(-20, 20, -1, 20, 30, white))
    sc.set_world(sc.hitable_list(objs))
    sc.set_lights(sc.hitable_list([sc.flip_normals(sc.xz_rect(-3, 3, -3, 3, 9))]))
    return sc


def _digest(text, sgroup):
    code = ("import sys; sys.path.insert(0, %r); from srr import capi; print(capi.scene_digest(sys.stdin.read()))"
            % os.path.join(ROOT, "simple-raytracing-render_amd"))
    out = subprocess.run([sys.executable, "-c", code], input=text, capture_output=True, text=True,
                         env=dict(os.environ, SRR_SGROUP=sgroup), check=True)
    return out.stdout.strip()


def _contents():
    if os.path.isdir("/root/reference/contents"):
        return "/root/reference/contents"
    import ref_fixtures
    return ref_fixtures.contents_dir()


def test_runs_are_grouped_only_where_long_enough():
    """SRR_SGROUP=0 keeps the plain list: the flattened scene changes for the
    sphere-list scenes and the edge scene, not for C2 (no run of 8 spheres)."""
    from srr import scenes
    for text, grouped in [(edge_scene().text(), True), (ref_scenes.random_scene(1.0, _contents()).text(), True),
                          (scenes.s2_cornell_teapot()[0].text(), False)]:
        assert (_digest(text, "1") != _digest(text, "0")) == grouped


def _check(text, nx, ny, spp):
    out = capi.Renderer(text).render(nx, ny, spp, 50, keep_paths=True)
    ref = ob.render(text, nx, ny, spp, 50, threads=os.cpu_count() or 4)
    pc = parity.compare_paths(out["paths"], ref["paths"])
    print(pc, "world rays", out["stats"]["world_rays"])
    assert pc["bitexact"] == 1.0, pc
    assert (out["rays"] == ref["rays"]).all()
    assert out["stats"]["world_rays"] == int(ref["stats"][0])


@pytest.mark.gpu
def test_edge_scene_is_the_linear_list():
    _check(edge_scene().text(), 64, 64, 16)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ball_scenes", "random_scene"])
def test_reference_sphere_list_scenes_are_the_linear_list(name):
    """The reference's own builders (the as-shipped default ball_scenes, and
    random_scene with its moving spheres) at 80x80x8: every path bit-exact
    against the restatement's linear list."""
    _check(ref_scenes.BUILDERS[name](1.0, _contents()).text(), 80, 80, 8)

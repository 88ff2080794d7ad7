"""The reference's own scene builders (Raytracing_n.cpp:108-711)
restated in srr/ref_scenes.py.

* CPU (needs the reference's assets, /root/reference/contents): the scene built
  by srr/ref_scenes.py -- images through srr's stb-exact decoder, meshes
  through srr's PLY/FBX loaders -- rendered by the CPU restatement must equal
  the goldens the REFERENCE made (tests/golden/make_scenes.py): refb_* from the
  reference's builder functions themselves, reft_* from the reference's classes
  built from the same scene text.
* GPU (no reference files on the box): all nine goldens from the committed
  fixtures (tests/ref_fixtures.py: flattened scenes, or the builders run on the
  reference's asset files from tests/golden/ref_assets.npz), the HIP path bit
  for bit against the reference's paths; and every builder with stand-in assets
  of the same names and sizes against the CPU restatement.
"""
import json
import os

import numpy as np
import pytest

import meshfiles as mf
import oracle_bind as ob
import parity
import ref_fixtures
from srr import capi, ref_scenes

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
META = json.load(open(os.path.join(GOLD, "ref_scenes.json")))
CONTENTS = "/root/reference/contents"


def _golden(key, m):
    n = m["nx"] * m["ny"]
    paths = np.fromfile(os.path.join(GOLD, key + ".paths.f32"), np.float32).reshape(n, m["spp"], 3)
    rays = np.fromfile(os.path.join(GOLD, key + ".rays.u8"), np.uint8).reshape(n, m["spp"])
    return paths, rays


@pytest.mark.parametrize("key", sorted(META))
def test_restated_builder_matches_reference(key):
    if not os.path.isdir(CONTENTS):
        pytest.skip("reference assets not present")
    m = META[key]
    sc = ref_scenes.BUILDERS[m["builder"]](m["nx"] / m["ny"], CONTENTS, **m["kwargs"])
    got = ob.render(sc.text(), m["nx"], m["ny"], m["spp"], m["max_depth"])
    want_paths, want_rays = _golden(key, m)
    pc = parity.compare_paths(got["paths"], want_paths)
    assert pc["bitexact"] == 1.0, pc  # every path, bit for bit
    assert (got["rays"].reshape(want_rays.shape) == want_rays).all()  # and every path's world rays
    assert int(got["rays"].sum()) == m["world_rays"] == int(want_rays.sum())


# ------------------------------------------- the goldens without /root/reference
@pytest.mark.parametrize("key", ref_fixtures.KEYS)
def test_fixture_scenes_render_the_reference_goldens(key):
    """The committed fixture scenes (tests/ref_fixtures.py) through the CPU
    restatement equal the REFERENCE's goldens: pins the fixtures the GPU test
    below renders, on any host."""
    m = META[key]
    got = ob.render(ref_fixtures.scene_text(key), m["nx"], m["ny"], m["spp"], m["max_depth"])
    want_paths, want_rays = _golden(key, m)
    pc = parity.compare_paths(got["paths"], want_paths)
    assert pc["bitexact"] == 1.0, pc
    assert (got["rays"].reshape(want_rays.shape) == want_rays).all()


@pytest.mark.gpu
@pytest.mark.parametrize("key", ref_fixtures.KEYS)
def test_gpu_renders_the_reference_goldens(key):
    """The HIP path against the goldens the REFERENCE rendered from its own builder
    functions (refb_*) or classes (reft_*): every path and its world rays bit for
    bit (the reference goldens had never run on the GPU)."""
    m = META[key]
    out = capi.Renderer(ref_fixtures.scene_text(key), device=0).render(m["nx"], m["ny"], m["spp"], m["max_depth"],
                                                                       keep_paths=True)
    want_paths, want_rays = _golden(key, m)
    pc = parity.compare_paths(out["paths"].reshape(want_paths.shape), want_paths)
    print(key, pc)
    assert pc["bitexact"] == 1.0, (key, pc)
    assert (out["rays"].reshape(want_rays.shape) == want_rays).all()
    assert int(out["stats"]["world_rays"]) == m["world_rays"]


def test_sceneid_table():
    assert [ref_scenes.BY_SCENEID[i].__name__ for i in range(8)] == [
        "cornell_box", "teapot_scene", "ball_scenes", "ball_orennayar_scenes", "jadebunny_scene", "final",
        "soldier_scene", "flatnormal_bunny"]


# ------------------------------------------------------------ stand-in assets
IMAGES = {  # name -> (w, h, gen kind) with the reference assets' sizes
    "environment_map/sky_2.png": (2000, 1000, "sky"),
    "environment_map/sky4.jpg": (4096, 2048, "sky"),
    "textures/earthmap.jpg": (2048, 1024, "checker"),
    "textures/TexturesCom_Wood_Wenge_1K_albedo.png": (1024, 1024, "wood"),
    "textures/NPC_YuanChengBing_A.png": (1024, 1024, "checker"),
}
for _f in ("Front", "Back", "Left", "Right", "Top", "Bottom"):
    IMAGES[f"environment_map/sky_1/{_f}.jpg"] = (2048, 2048, "sky")


def gen_rgb(w, h, kind, seed):
    """integer image like srr_text::gen_image (any deterministic bytes do)."""
    y, x = np.mgrid[0:h, 0:w]
    n = (x * 73856093 ^ y * 19349663 ^ seed * 83492791) & 0xFFFF
    if kind == "sky":
        t = (y * 255) // max(h - 1, 1)
        img = np.stack([90 + t * 120 // 255 + (n & 15), 140 + t * 90 // 255 + ((n >> 4) & 15),
                        235 - t * 60 // 255 + ((n >> 8) & 15)], -1)
    elif kind == "wood":
        band = ((x * 7 + ((n >> 3) & 7)) // 13) & 15
        img = np.stack([110 + band * 6 + (n & 7), 70 + band * 4 + ((n >> 5) & 7), 40 + band * 2 + ((n >> 9) & 7)], -1)
    else:
        c = ((x >> 5) ^ (y >> 5)) & 1
        img = np.stack([np.where(c, 230, 25), np.where(c, 200, 40), np.where(c, 60, 180)], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


def sphere_mesh(n_lat=12, n_lon=18, r=0.05, c=(0.0, 0.1, 0.0)):
    verts = []
    for i in range(n_lat + 1):
        th = np.pi * i / n_lat
        for j in range(n_lon):
            ph = 2 * np.pi * j / n_lon
            verts.append([c[0] + r * np.sin(th) * np.cos(ph), c[1] + r * np.cos(th), c[2] + r * np.sin(th) * np.sin(ph)])
    faces = []
    for i in range(n_lat):
        for j in range(n_lon):
            a, b = i * n_lon + j, i * n_lon + (j + 1) % n_lon
            faces.append([a, b + n_lon, a + n_lon] if i else [a, b + n_lon, a + n_lon])
            faces.append([a, b, b + n_lon])
    return np.array(verts, np.float32), faces


def make_standin_contents(root):
    """stand-in for the reference's contents/: same file names and image sizes;
    images are generated and written as PNG (srr's decoder reads by content, not
    extension); bunny.ply is a small generated sphere mesh (no normals, like the
    real one) and Soilder.FBX a generated FBX with normals and UVs."""
    for k, (name, (w, h, kind)) in enumerate(sorted(IMAGES.items())):
        p = os.path.join(root, name)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        capi.write_png(p, w, h, gen_rgb(w, h, kind, k))
    os.makedirs(os.path.join(root, "models"), exist_ok=True)
    v, f = sphere_mesh()
    mf.write_ply(os.path.join(root, "models", "bunny.ply"), v, f)
    v2, f2 = sphere_mesh(10, 14, r=30.0, c=(0.0, 40.0, 0.0))
    polys = [list(fc) for fc in f2]
    nrm = []
    uv = []
    for fc in polys:
        for i in fc:
            d = v2[i] - np.array([0, 40, 0], np.float32)
            nrm.append(d / np.linalg.norm(d))
            uv.append([(np.arctan2(d[2], d[0]) / (2 * np.pi)) % 1.0, 0.5 + d[1] / 60.0])
    geo = mf.fbx_geometry(1001, v2, polys, normals_pv=np.array(nrm, np.float32), uv=np.array(uv, np.float32),
                           uv_index=list(range(len(uv))))
    mf.write_fbx(os.path.join(root, "models", "Soilder.FBX"),
                 mf.fbx_scene([geo, mf.fbx_model(2001, "soldier")], [(1001, 2001)]))
    return root


@pytest.fixture(scope="module")
def standin(tmp_path_factory):
    return make_standin_contents(str(tmp_path_factory.mktemp("contents")))


def test_standin_contents_build(standin):
    """Host side only: every builder builds and parses on the stand-in assets."""
    for name, f in ref_scenes.BUILDERS.items():
        kw = {"divs": 4} if name == "teapot_scene" else {}
        text = f(4 / 3, standin, **kw).text()
        capi.Scene(text)  # the C-ABI parses and validates it


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ref_scenes.BUILDERS))
def test_gpu_reference_builders(standin, name):
    kw = {"divs": 10} if name == "teapot_scene" else {}
    nx, ny, spp = 24, 18, 4
    text = ref_scenes.BUILDERS[name](nx / ny, standin, **kw).text()
    out = capi.Renderer(text, device=0).render(nx, ny, spp, 50, keep_paths=True)
    ref = ob.render(text, nx, ny, spp, 50)
    pc = parity.compare_paths(out["paths"], ref["paths"])
    print(name, pc)
    assert pc["match"] >= parity.MIN_MATCH, (name, pc)
    assert pc["bitexact"] >= parity.MIN_BITEXACT, (name, pc)
    assert int(out["stats"]["world_rays"]) == int(ref["stats"][0])


@pytest.mark.gpu
def test_render_main_writes_the_reference_ppm(standin, tmp_path):
    """srr.render_main, the reference's main() (Raytracing_n.cpp:882-952): sceneid
    -> builder -> GPU render -> P3 PPM, byte-equal to tone-mapping the same
    render by hand."""
    from srr import capi, render_main
    out = str(tmp_path / "main.ppm")
    assert render_main.main(["--sceneid", "5", "--nx", "24", "--ny", "18", "--ns", "4", "--contents", standin,
                             "--out", out]) == 0
    sc = ref_scenes.BY_SCENEID[5](24 / 18, standin)
    img8 = capi.tonemap(capi.Renderer(sc.text()).render(24, 18, 4, 50)["mean"])
    want = str(tmp_path / "want.ppm")
    capi.write_ppm(want, 24, 18, img8)
    assert open(out, "rb").read() == open(want, "rb").read()
    assert open(out, "rb").read().startswith(b"P3\n24 18\n255\n")

"""the C++ worked example (tests/cpp/cornell_teapot.cpp) builds
S2 through the C-ABI.  CPU: it compiles and links against libsrr.so.  GPU: its
image equals, bitwise, the Python-built S2 render (same scene, same builder
order, same scene-build LCG draws), and its PPM is the reference's P3 format."""
import os
import subprocess

import numpy as np
import pytest

from srr import capi, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "simple-raytracing-render_amd")
SRC = os.path.join(ROOT, "tests", "cpp", "cornell_teapot.cpp")
REF_API_SRC = os.path.join(ROOT, "tests", "cpp", "ref_api_cornell.cpp")


def build(tmpdir, src=SRC, name="cornell_teapot"):
    exe = os.path.join(str(tmpdir), name)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src,
                    "-o", exe, "-L", LIBDIR, "-lsrr", f"-Wl,-rpath,{LIBDIR}"], check=True)
    return exe


def test_example_compiles_and_links(tmp_path):
    exe = build(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 2 and "usage" in out.stderr


@pytest.mark.gpu
def test_example_renders_the_python_built_scene(tmp_path):
    exe = build(tmp_path)
    nx, ny, spp = 48, 32, 4
    ppm, meanf = str(tmp_path / "o.ppm"), str(tmp_path / "o.f32")
    subprocess.run([exe, str(nx), str(ny), str(spp), ppm, meanf], check=True, timeout=300)
    got = np.fromfile(meanf, np.float32).reshape(nx * ny, 3)
    sc, _ = scenes.s2_cornell_teapot()
    want = capi.Renderer(sc.text()).render(nx, ny, spp, 50)
    np.testing.assert_array_equal(got.view(np.uint32), want["mean"].view(np.uint32))
    head = open(ppm, "rb").read(32).split(b"\n")
    assert head[0] == b"P3" and head[1].split() == [str(nx).encode(), str(ny).encode()]


def test_reference_style_builder_compiles(tmp_path):
    """include/srr/ref_api.h: a builder in the reference's own style (new sphere,
    new bvh_node(list, n, 0, 1), teapot::createPloyTeapot, camera) compiles."""
    exe = build(tmp_path, REF_API_SRC, "ref_api_cornell")
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 2 and "usage" in out.stderr


@pytest.mark.gpu
def test_reference_style_builder_renders_the_python_built_scene(tmp_path):
    exe = build(tmp_path, REF_API_SRC, "ref_api_cornell")
    nx, ny, spp = 40, 24, 4
    meanf = str(tmp_path / "m.f32")
    subprocess.run([exe, str(nx), str(ny), str(spp), meanf], check=True, timeout=300)
    got = np.fromfile(meanf, np.float32).reshape(nx * ny, 3)
    sc, _ = scenes.s2_cornell_teapot()
    want = capi.Renderer(sc.text()).render(nx, ny, spp, 50)
    np.testing.assert_array_equal(got.view(np.uint32), want["mean"].view(np.uint32))


@pytest.mark.gpu
def test_reference_style_model_loader_renders_the_python_built_scene(tmp_path):
    """model(file, flipUVs, flipWindingOrder, mat, scale).genhitablemodel() from
    C++ (include/srr/ref_api.h -> srr_model) and Scene.model from Python read the
    same PLY file and give bitwise the same image."""
    import meshfiles as mf
    import oracle_bind as ob
    exe = build(tmp_path, REF_API_SRC, "ref_api_cornell")
    tp = ob.teapot(60.0, 6).reshape(-1, 12)
    n_t = len(tp)
    path = str(tmp_path / "teapot.ply")
    mf.write_ply(path, tp[:, :9].reshape(-1, 3), [[3 * t, 3 * t + 1, 3 * t + 2] for t in range(n_t)],
                 np.repeat(tp[:, 9:12], 3, axis=0), np.zeros((3 * n_t, 2), np.float32), fmt="binary_little_endian")
    nx, ny, spp = 40, 24, 4
    meanf = str(tmp_path / "m.f32")
    subprocess.run([exe, str(nx), str(ny), str(spp), meanf, path], check=True, timeout=300)
    got = np.fromfile(meanf, np.float32).reshape(nx * ny, 3)
    from srr.scene import Scene
    sc = Scene()
    objs, white = scenes._cornell(sc)
    tris = sc.model(path, True, True, white, (1.0, 1.0, 1.0))
    objs.append(sc.translate(sc.rotate_x(sc.bvh_node(tris, 0, 1), 90), (330, 0, 300)))
    sc.set_world(sc.hitable_list(objs))
    scenes._cornell_camera_and_lights(sc)
    want = capi.Renderer(sc.text()).render(nx, ny, spp, 50)
    np.testing.assert_array_equal(got.view(np.uint32), want["mean"].view(np.uint32))

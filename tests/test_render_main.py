"""The reference's program main() (Raytracing_n.cpp:882-952) as a C++ binary:
include/srr/render_main.h (the sceneid switch, render, ms print, P3 output) and
simple-raytracing-render_amd/csrc/render_main.cpp (the BASELINE configs' scenes
written as reference-style builders against include/srr/ref_api.h).

CPU: it builds; each built-in builder makes byte-for-byte the scene srr/scenes.py
makes (srr_scene_digest); --scene-text renders any scene description (here the
reference's ball_scenes, restated by srr/ref_scenes.py); and, where the reference
is present, its OWN builder functions compiled against ref_api.h and dispatched
by render_main.h's sceneid switch make the restated scenes.  GPU: its PPM equals
the Python-rendered one byte for byte."""
import glob
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from srr import capi, ref_scenes, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simple-raytracing-render_amd")
EXE = os.path.join(PKG, "render_main")
REF_SRC = os.path.join("/root/reference", "Raytracing_n", "Raytracing_n.cpp")
SIZES = {"s1": (256, 256), "s2": (512, 512), "s3": (512, 512), "s3_metal": (512, 512), "s4": (1920, 1080),
         "s5": (1920, 1080)}


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-C", PKG, "render_main"], check=True, capture_output=True)
    return EXE


def _dry(exe, *args):
    r = subprocess.run([exe, *args, "--dry-run"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout.split()[-1]


@pytest.mark.parametrize("name", sorted(SIZES))
def test_builtin_builder_makes_the_python_scene(exe, name):
    nx, ny = SIZES[name]
    sc, cfg = scenes.SCENES[name]()
    assert (cfg["nx"], cfg["ny"]) == (nx, ny)
    assert _dry(exe, "--scene", name, "--nx", str(nx), "--ny", str(ny)) == capi.scene_digest(sc.text())


def test_sceneid_and_usage(exe):
    assert _dry(exe, "--sceneid", "2", "--nx", "512", "--ny", "512") == \
        capi.scene_digest(scenes.s2_cornell_teapot()[0].text())
    r = subprocess.run([exe, "--sceneid", "99"], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_scene_text_of_a_reference_builder(exe, tmp_path):
    text = ref_scenes.random_scene(1.0).text()
    f = tmp_path / "random.scene"
    f.write_text(text)
    assert _dry(exe, "--scene-text", str(f), "--nx", "64", "--ny", "64") == capi.scene_digest(text)


@pytest.mark.skipif(not os.path.exists(REF_SRC) or shutil.which("g++") is None,
                    reason="needs /root/reference (development container)")
def test_reference_builders_through_render_main(tmp_path):
    """The reference's own random_scene and ball_scenes (read from /root/reference
    at test time, nothing committed) linked into render_main.h's main."""
    from test_ref_builders_compile import extract
    raw = open(REF_SRC, "rb").read()
    text = raw.decode("utf-16") if raw[:2] in (b"\xff\xfe", b"\xfe\xff") else raw.decode("utf-8", "replace")
    text = text.replace("\r\n", "\n")
    names = ["random_scene", "ball_scenes"]
    body = "\n\n".join(extract(text, n) for n in names)
    cpp = tmp_path / "ref_main.cpp"
    cpp.write_text('#include "srr/render_main.h"\nusing namespace srr::ref;\n\n' + body +
                   '\nint main(int argc, char** argv) {\n'
                   '  static const scene_entry t[] = {{2, "ball_scenes", ball_scenes}, {9, "random_scene", random_scene}};\n'
                   '  return render_main(argc, argv, t, 2);\n}\n')
    exe = tmp_path / "ref_main"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-w", "-I", os.path.join(ROOT, "include"), str(cpp), "-o",
                        str(exe), "-L", PKG, "-lsrr", f"-Wl,-rpath,{PKG}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # the builders open their assets by relative Windows paths ("..\\contents\\...")
    ref = "/root/reference"
    for f in glob.glob(os.path.join(ref, "contents", "**", "*"), recursive=True):
        if os.path.isfile(f):
            os.symlink(f, os.path.join(tmp_path, "..\\" + os.path.relpath(f, ref).replace("/", "\\")))
    for sid, name in ((2, "ball_scenes"), (9, "random_scene")):
        got = subprocess.run([str(exe), "--sceneid", str(sid), "--nx", "300", "--ny", "200", "--dry-run"],
                             capture_output=True, text=True, cwd=tmp_path, timeout=300)
        assert got.returncode == 0, got.stderr
        want = capi.scene_digest(ref_scenes.BUILDERS[name](300 / 200).text())
        assert got.stdout.split()[-1] == want, name


@pytest.mark.gpu
def test_render_main_image_is_the_python_render(exe, tmp_path):
    nx, ny, ns = 40, 40, 4  # square: scenes.s2_cornell_teapot's camera has aspect 1
    out = str(tmp_path / "o.ppm")
    r = subprocess.run([exe, "--scene", "s2", "--nx", str(nx), "--ny", str(ny), "--ns", str(ns), "--out", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert re.fullmatch(r"\d+ms", r.stdout.strip())
    sc, _ = scenes.s2_cornell_teapot()
    want = capi.Renderer(sc.text()).render(nx, ny, ns, 50)
    ref = str(tmp_path / "want.ppm")
    capi.write_ppm(ref, nx, ny, want["img8"])
    assert open(out, "rb").read() == open(ref, "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("devs", ["0", "0,0,0"])
def test_render_main_multi_device_image_is_the_one_device_image(exe, tmp_path, devs):
    """render_main --devices (C++ host, srr_renderer_create_multi): "0" gathers
    through a real RCCL communicator of one GPU, "0,0,0" deals three shards on the
    leased GPU (device copies); the PPM is byte-identical to the one-device run."""
    nx, ny, ns = 48, 40, 4
    args = ["--scene", "s2", "--nx", str(nx), "--ny", str(ny), "--ns", str(ns)]
    one, multi = str(tmp_path / "one.ppm"), str(tmp_path / "multi.ppm")
    r = subprocess.run([exe, *args, "--out", one], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe, *args, "--devices", devs, "--out", multi], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert ("(rccl)" if devs == "0" else "(copy)") in r.stderr, r.stderr
    assert open(multi, "rb").read() == open(one, "rb").read()

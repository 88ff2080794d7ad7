"""GPU parity: the HIP path, called through the C-ABI (libsrr.so), against
(1) the REFERENCE's own per-path outputs (tests/golden/, made by
oracle/ref from /root/reference), (2) the CPU restatement oracle at larger
sizes, and (3) size-independent properties (shard / batch invariance).
Tolerances: tests/parity.py."""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
import parity
from srr import capi, scenes

pytestmark = pytest.mark.gpu
META = json.load(open(os.path.join(ob.GOLDEN, "golden.json")))["renders"]


def golden(name):
    m = META[name]
    n = m["nx"] * m["ny"]
    text = open(os.path.join(ob.GOLDEN, f"{name}.scene")).read()
    paths = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.paths.f32"), np.float32).reshape(n, m["spp"], 3)
    rays = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.rays.u8"), np.uint8).reshape(n, m["spp"])
    img = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.img.f32"), np.float32).reshape(n, 3)
    return m, text, paths, rays, img


ENGINES = {"paths": 0, "wavefront": capi.FLAG_WAVEFRONT}


@pytest.mark.parametrize("engine", sorted(ENGINES))
@pytest.mark.parametrize("name", sorted(META))
def test_paths_match_reference(name, engine):
    m, text, gp, gr, gi = golden(name)
    out = capi.Renderer(text).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True,
                                     flags=ENGINES[engine])
    pc = parity.compare_paths(out["paths"], gp)
    ic = parity.compare_images(out["mean"], gi)
    rays_eq = float((out["rays"] == gr).mean())
    print(f"{name}: {pc} rays_eq={rays_eq:.5f} world_rays={out['stats']['world_rays']} "
          f"(ref {m['world_rays']}) img={ic}")
    assert pc["match"] >= parity.MIN_MATCH, pc
    # the device rounds like the reference (correctly rounded sqrt, glibc's float
    # libm algorithms): paths are bit-identical, not just within tolerance
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert rays_eq == 1.0
    assert out["stats"]["world_rays"] == m["world_rays"]
    assert ic["mean_rel"] <= 0.005, ic


@pytest.mark.parametrize("name", sorted(META))
def test_quad_traversal_matches_reference(name, monkeypatch):
    """The quad-cooperative mesh traversal (kernels.hip mesh_hit4_quad; the
    default only for BVHs larger than an XCD's L2) forced on every golden scene:
    the same paths, bit for bit, and the same world rays as the reference."""
    monkeypatch.setenv("SRR_QUAD", "1")
    m, text, gp, gr, gi = golden(name)
    out = capi.Renderer(text).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    pc = parity.compare_paths(out["paths"], gp)
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert (out["rays"] == gr).all()
    assert out["stats"]["world_rays"] == m["world_rays"]


@pytest.mark.parametrize("factory", [scenes.s2_cornell_teapot, lambda: scenes.s3_cornell_teapot_microfacet("metal")])
def test_engines_render_identical_images(factory):
    """The path-resident and wavefront engines run the same per-path arithmetic
    and sum each pixel's samples in the same order: bitwise equal images."""
    sc, _ = factory()
    r = capi.Renderer(sc.text())
    a = r.render(40, 32, 12, 50)["mean"]
    b = r.render(40, 32, 12, 50, flags=capi.FLAG_WAVEFRONT)["mean"]
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_shards_assemble_to_the_same_image():
    """Tile sharding: per-path seeds do not depend on the shard,
    so the assembled image is bitwise the single-renderer image."""
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    nx, ny, spp = 48, 40, 8
    full = r.render(nx, ny, spp, 50)["mean"]
    asm = np.zeros_like(full)
    for k in range(3):
        part = r.render(nx, ny, spp, 50, shard=(k, 3), tile=16)["mean"]
        px = capi.shard_pixels(capi.make_params(nx, ny, spp, shard=(k, 3), tile=16))
        asm[px] = part
    np.testing.assert_array_equal(asm.view(np.uint32), full.view(np.uint32))


def test_sample_shards_are_slices_of_the_full_render():
    """Sample sharding (srr/dist.py plan "samples"): a render of samples
    [b, b + n) is bitwise the same paths as that slice of the full render."""
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    nx, ny, spp = 32, 24, 6
    full = r.render(nx, ny, spp, 50, keep_paths=True)
    for b, n in ((0, 2), (2, 3), (5, 1)):
        part = r.render(nx, ny, n, 50, keep_paths=True, sample_begin=b)
        np.testing.assert_array_equal(part["paths"].view(np.uint32), full["paths"][:, b:b + n].view(np.uint32))
        np.testing.assert_array_equal(part["rays"], full["rays"][:, b:b + n])


def test_batch_size_does_not_change_the_image():
    """Wavefront engine: ragged (pixel chunk, sample chunk) batches give the
    path engine's image bit for bit (batch_paths only steers the wavefront
    engine's batching)."""
    sc, _ = scenes.s3_cornell_teapot_microfacet()
    r = capi.Renderer(sc.text())
    a = r.render(40, 40, 12, 50)["mean"]
    b = r.render(40, 40, 12, 50, batch_paths=997, flags=capi.FLAG_WAVEFRONT)["mean"]
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_sample_windows_do_not_change_the_frame(monkeypatch):
    """Path engine: a frame cut into several sample windows (SRR_WINDOW_MB, read
    per call) gives the one-window frame bit for bit -- Sobol offsets, sample
    bases, kept-path placement and the running sums carried between windows."""
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    nx, ny, spp = 256, 256, 24
    one = r.render(nx, ny, spp, 50, keep_paths=True)
    monkeypatch.setenv("SRR_WINDOW_MB", "1")  # 1 MiB / (12 B x 65,536 px) -> 1 sample per window
    many = r.render(nx, ny, spp, 50, keep_paths=True)
    assert many["stats"]["trace_launches"] == spp and one["stats"]["trace_launches"] == 1
    np.testing.assert_array_equal(many["mean"].view(np.uint32), one["mean"].view(np.uint32))
    np.testing.assert_array_equal(many["paths"].view(np.uint32), one["paths"].view(np.uint32))
    np.testing.assert_array_equal(many["rays"], one["rays"])


@pytest.mark.parametrize("nx,ny,spp,window_mb,launches", [
    # 16 MiB / (12 B x 65,536 px) = 21 -> windows of 20, 20, 20, 4: 16-sample chunks, then a
    # 4-sample tail chunk; the last window is a tail chunk alone
    (256, 256, 64, "16", 4),
    # 32,500 px (the last block holds 244): 37 -> windows of 36 (two chunks + a tail of 4) and 4
    (250, 130, 40, "14", 2),
    # 29 -> 28: a chunk and a tail of 12; the last window (8) a tail chunk alone
    (256, 256, 64, "22", 3),
    # 58 -> 56: three chunks and a tail of 8; the last window (38) takes the scalar kernel
    (128, 128, 150, "11", 3),
])
def test_windows_of_a_multiple_of_four_samples(monkeypatch, nx, ny, spp, window_mb, launches):
    """Path engine: windows of >= 16 samples are cut to a multiple of 4 and summed with
    16-byte loads (k_accumulate_window16), including a last chunk of 4, 8 or 12 samples;
    the frame is the one-window frame bit for bit (the running sums keep sample order)."""
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    one = r.render(nx, ny, spp, 50)
    monkeypatch.setenv("SRR_WINDOW_MB", window_mb)
    many = r.render(nx, ny, spp, 50)
    assert one["stats"]["trace_launches"] == 1
    assert many["stats"]["trace_launches"] == launches, many["stats"]
    np.testing.assert_array_equal(many["mean"].view(np.uint32), one["mean"].view(np.uint32))


@pytest.mark.parametrize("factory,nx,ny,spp", [
    (scenes.s2_cornell_teapot, 256, 256, 16),
    (lambda: scenes.s3_cornell_teapot_microfacet("beckmann"), 256, 256, 16),
    (lambda: scenes.s4_soldier_standin(divs=20, fog=True), 192, 108, 8),
    # the reference's as-shipped teapot (teapot.h:77: 640,000 triangles)
    (lambda: scenes.s2_cornell_teapot(divs=100), 512, 512, 8),
    # C4 / C5 at their configured frame and mesh (1920x1080, 102,400 triangles)
    (lambda: scenes.s4_soldier_standin(divs=40), 1920, 1080, 4),
    (lambda: scenes.s4_soldier_standin(divs=40, fog=True), 1920, 1080, 2),
])
def test_larger_renders_match_oracle_on_sampled_pixels(factory, nx, ny, spp):
    sc, _ = factory()
    text = sc.text()
    out = capi.Renderer(text).render(nx, ny, spp, 50, keep_paths=True)
    rng = np.random.default_rng(7)
    pix = np.sort(rng.choice(nx * ny, size=300, replace=False)).astype(np.int32)
    ref = ob.render(text, nx, ny, spp, 50, pixels=pix, threads=8)
    pc = parity.compare_paths(out["paths"][pix], ref["paths"])
    print(pc)
    assert pc["match"] >= parity.MIN_MATCH, pc
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc


def _nan_panel_scene():
    """Cornell box + a BVH'd panel of 128 triangles, half of them with zero vertex
    normals: their shading normal is NaN (unit_vector of 0), so rays scattered off
    them have NaN directions and pass every slab test (as in the reference)."""
    from srr.scene import Scene
    sc = Scene()
    objs, white = scenes._cornell(sc)
    tris = []
    for a in range(8):
        for b in range(8):
            x0, x1 = 120 + 40 * a, 160 + 40 * a
            y0, y1 = 100 + 40 * b, 140 + 40 * b
            z0, z1 = 250 + 5 * a, 260 + 5 * b
            n = ((0, 0, 0),) * 3 if (a + b) % 2 == 0 else ((0, 0, -1),) * 3
            tris.append(sc.triangle((x0, y0, z0), (x1, y0, z1), (x1, y1, z0), white, normals=n))
            tris.append(sc.triangle((x0, y0, z0), (x1, y1, z0), (x0, y1, z1), white, normals=n))
    objs.append(sc.bvh_node(tris, 0, 1))
    sc.set_world(sc.hitable_list(objs))
    scenes._cornell_camera_and_lights(sc)
    return sc


def test_nan_rays_through_meshes_match_oracle():
    text = _nan_panel_scene().text()
    nx, ny, spp = 24, 24, 8
    out = capi.Renderer(text).render(nx, ny, spp, 50, keep_paths=True)
    ref = ob.render(text, nx, ny, spp, 50, threads=8)
    pc = parity.compare_paths(out["paths"], ref["paths"])
    print("nan panel:", pc, out["stats"]["world_rays"], int(ref["stats"][0]))
    assert pc["match"] >= parity.MIN_MATCH, pc
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert out["stats"]["world_rays"] == int(ref["stats"][0])


def test_depth_limit_zero_and_one():
    """maxDepth edge cases (Raytracing_n.cpp:63): depth 0 returns emitted only."""
    sc, _ = scenes.s1_cornell()
    text = sc.text()
    for md in (0, 1):
        out = capi.Renderer(text).render(16, 16, 4, md, keep_paths=True)
        ref = ob.render(text, 16, 16, 4, md)
        pc = parity.compare_paths(out["paths"], ref["paths"])
        assert pc["match"] >= parity.MIN_MATCH, (md, pc)
        assert pc["bitexact"] >= parity.MIN_BITEXACT, (md, pc)


def test_model_file_scene_matches_oracle(tmp_path):
    """A mesh read from a file (model.h path): the teapot written
    as a binary PLY with per-vertex normals and UVs, loaded through Scene.model
    (srr's PLY loader), rendered on the GPU and by the oracle from the same text."""
    import meshfiles as mf
    from srr.scene import Scene
    tp = ob.teapot(60.0, 6).reshape(-1, 12)
    n_t = len(tp)
    verts = tp[:, :9].reshape(-1, 3)
    rng = np.random.default_rng(11)
    nrm = np.repeat(tp[:, 9:12], 3, axis=0) + 0.2 * rng.standard_normal((3 * n_t, 3)).astype(np.float32)
    uvs = rng.random((3 * n_t, 2)).astype(np.float32)
    path = str(tmp_path / "teapot.ply")
    mf.write_ply(path, verts, [[3 * t, 3 * t + 1, 3 * t + 2] for t in range(n_t)], nrm, uvs,
                 fmt="binary_little_endian")
    sc = Scene()
    objs, white = scenes._cornell(sc)
    tris = sc.model(path, True, True, white, (1.0, 1.0, 1.0))
    objs.append(sc.translate(sc.rotate_x(sc.bvh_node(tris, 0, 1), 90), (330, 0, 300)))
    sc.set_world(sc.hitable_list(objs))
    scenes._cornell_camera_and_lights(sc)
    text = sc.text()
    nx, ny, spp = 32, 32, 8
    out = capi.Renderer(text).render(nx, ny, spp, 50, keep_paths=True)
    ref = ob.render(text, nx, ny, spp, 50, threads=8)
    pc = parity.compare_paths(out["paths"], ref["paths"])
    print("model scene:", pc)
    assert pc["match"] >= parity.MIN_MATCH, pc
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc


@pytest.mark.parametrize("quad", ["0", "1"])
@pytest.mark.parametrize("gstack", ["0", "1"])
@pytest.mark.parametrize("name", ["s4_d40", "s5_d40", "s2_d100"])
def test_stack_overflow_rewalk_matches_reference(name, gstack, quad, monkeypatch):
    """The BVH4 traversal's LDS stack holds kStack = 8 entries, extended in global
    memory by kPathsGlobalStack more; a ray that needs more re-walks the mesh with
    the exact stackless BVH2 (kernels.hip mesh_hit4).  SRR_STACK_CAP=1 (read per
    render call) sends most mesh rays of the 102,400- and 640,000-triangle goldens
    through the global extension (SRR_GSTACK=1) or, without it (SRR_GSTACK=0),
    through the re-walk: every path still bit-identical to the reference, and the
    counters show that path really ran.  SRR_QUAD (read when the scene is
    uploaded) runs both the per-lane and the quad-cooperative traversal."""
    m, text, gp, gr, gi = golden(name)
    monkeypatch.setenv("SRR_QUAD", quad)
    monkeypatch.setenv("SRR_STACK_CAP", "1")
    monkeypatch.setenv("SRR_GSTACK", gstack)
    out = capi.Renderer(text).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    pc = parity.compare_paths(out["paths"], gp)
    st = out["stats"]
    print(name, pc, "overflows:", st["stack_overflows"], "deep:", st["deep_traversals"])
    if gstack == "1":
        assert st["deep_traversals"] > 0
    else:
        assert st["stack_overflows"] > 0 and st["deep_traversals"] == 0
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert (out["rays"] == gr).all()
    assert out["stats"]["world_rays"] == m["world_rays"]


@pytest.mark.parametrize("walk", [("0", "0"), ("64", "0"), ("64", "2"), ("8", "0"), ("24", "0")])
@pytest.mark.parametrize("name", ["s2", "s3", "s4_d40", "s5_d40", "s2_d100"])
def test_suspended_walks_match_reference(name, walk, monkeypatch):
    """Suspendable mesh walks (kernels.hip TraceCtx::walk_thr): a walk
    may stop part-way and continue in a later wave-iteration from its saved state
    (next node, stack top and depth, best hit, bound; the list's object and
    closest-so-far).  SRR_WALK_Q=64 suspends every walk after each node step -- the
    most resumes the kernel can make -- and with SRR_STACK_CAP=2 the suspended
    stacks also reach into the global extension; SRR_WALK_Q=0 never suspends.
    Every path bit-identical to the reference's, the same world rays, and the
    counter shows the walks suspended."""
    q, cap = walk
    m, text, gp, gr, gi = golden(name)
    monkeypatch.setenv("SRR_WALK_Q", q)
    if cap != "0":
        monkeypatch.setenv("SRR_STACK_CAP", cap)
    out = capi.Renderer(text).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    pc = parity.compare_paths(out["paths"], gp)
    st = out["stats"]
    print(name, walk, pc, "suspended:", st["walks_suspended"], "deep:", st["deep_traversals"])
    if q == "0":
        assert st["walks_suspended"] == 0
    elif q == "64":
        assert st["walks_suspended"] > 0
    if cap != "0" and name != "s2":
        assert st["deep_traversals"] > 0
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert (out["rays"] == gr).all()
    assert st["world_rays"] == m["world_rays"]


def _multi_mesh_scene(fog: bool):
    """Cornell box with three meshes in the world list: one teapot BVH placed twice
    (two instances of the same mesh, different transforms) and a second teapot mesh;
    with fog, a constant_medium ahead of them in the list (its RNG draws must not be
    repeated when a walk resumes)."""
    from srr.scene import Scene
    sc = Scene()
    objs, white = scenes._cornell(sc)
    if fog:
        objs.insert(0, sc.constant_medium(sc.sphere((278, 278, 278), 2000, white), 0.0004,
                                          sc.constant_texture((1.0, 1.0, 1.0))))
    metal = sc.metal(0.9, 0.0)
    shared = sc.bvh_node(sc.teapot(45.0, 6, metal), 0, 1)
    objs.append(sc.translate(sc.rotate_x(shared, 90), (360, 0, 330)))
    objs.append(sc.translate(sc.rotate_x(shared, 90), (170, 180, 300)))
    objs.append(scenes._teapot_instance(sc, white, 5, scale=35.0, at=(300, 300, 200)))
    sc.set_world(sc.hitable_list(objs))
    scenes._cornell_camera_and_lights(sc)
    return sc


@pytest.mark.parametrize("fog", [False, True])
def test_suspended_walks_with_several_meshes_match_oracle(fog, monkeypatch):
    """Walk suspension with several meshes in one world list (kernels.hip world_hit:
    a walk resumes at the object it stopped in, TraceCtx::obj_k; a lane suspended in
    one mesh does not start a later one) and with a medium in the list (the
    list-state save, so the medium's draws are not repeated): every path of the most
    resuming setting (SRR_WALK_Q=64) and of the plain one (0) bit-identical to the
    CPU restatement."""
    text = _multi_mesh_scene(fog).text()
    nx, ny, spp = 24, 24, 8
    ref = ob.render(text, nx, ny, spp, 50, threads=8)
    for q in ("64", "0"):
        monkeypatch.setenv("SRR_WALK_Q", q)
        out = capi.Renderer(text).render(nx, ny, spp, 50, keep_paths=True)
        pc = parity.compare_paths(out["paths"], ref["paths"])
        print("multi-mesh fog" if fog else "multi-mesh", q, pc, "suspended", out["stats"]["walks_suspended"])
        if q == "64":
            assert out["stats"]["walks_suspended"] > 0
        assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
        assert out["stats"]["world_rays"] == int(ref["stats"][0])

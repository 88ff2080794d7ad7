"""Mesh loaders: srr's PLY and binary-FBX readers behind
srr_mesh_file_triangles / srr_model, with the reference model loader's
semantics (model.h:28-102, geometry.h:24-90): mesh 0 only, per-component scale,
FlipUVs (v -> 1 - v), FlipWindingOrder (corner order reversed), polygons
triangulated as a fan.  Parity unpinned: the reference's assimp is Win32-only,
so expectations are computed here from the polygons written into the files
(tests/meshfiles.py)."""
import ctypes
import os

import numpy as np
import pytest

import meshfiles as mf
from srr import capi
from srr.scene import Scene

VERTS = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0.5, 0.5, 2.0]], np.float32)
NRMS = np.array([[0, 0, 1], [0, 0.6, 0.8], [0.6, 0, 0.8], [0, 0, -1], [1, 0, 0]], np.float32)
UVS = np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0.25, 0.75]], np.float32)
FACES = [[0, 1, 2, 3], [0, 1, 4], [1, 2, 4, 3, 0]]


def expected(faces, per_corner, flip_uvs=False, flip_winding=False, scale=(1, 1, 1)):
    """per_corner(face_index, corner_index) -> (p, n, uv3); fan from corner 0,
    then the post-processing the reference asks assimp for."""
    sc = np.asarray(scale, np.float32)
    P, N, U = [], [], []
    for fi, fc in enumerate(faces):
        for k in range(1, len(fc) - 1):
            cs = [0, k, k + 1]
            if flip_winding:
                cs = cs[::-1]
            tri = [per_corner(fi, c) for c in cs]
            P.append([np.float32(t[0]) * sc for t in tri])
            N.append([t[1] for t in tri])
            uv = [np.array(t[2], np.float32) for t in tri]
            if flip_uvs:
                for u in uv:
                    u[1] = np.float32(1.0) - u[1]
            U.append(uv)
    return (np.array(P, np.float32).reshape(-1, 3, 3), np.array(N, np.float32).reshape(-1, 3, 3),
            np.array(U, np.float32).reshape(-1, 3, 3))


def ply_corner(fi, c):
    v = FACES[fi][c]
    return VERTS[v], NRMS[v], [UVS[v][0], UVS[v][1], 0.0]


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
@pytest.mark.parametrize("flips", [(False, False), (True, False), (False, True), (True, True)])
def test_ply_matches_polygons(tmp_path, fmt, flips):
    path = str(tmp_path / "m.ply")
    mf.write_ply(path, VERTS, FACES, NRMS, UVS, fmt=fmt)
    scale = (2.0, 0.5, 3.0)
    pos, uv, nrm, has_n, has_uv = capi.mesh_file_triangles(path, *flips, scale=scale)
    assert has_n and has_uv
    P, N, U = expected(FACES, ply_corner, *flips, scale=scale)
    assert pos.shape == (2 + 1 + 3, 3, 3)
    np.testing.assert_array_equal(pos, P)
    np.testing.assert_array_equal(nrm, N)
    np.testing.assert_array_equal(uv, U)


def test_ply_without_normals_or_uvs(tmp_path):
    path = str(tmp_path / "m.ply")
    mf.write_ply(path, VERTS, FACES, fmt="binary_little_endian")
    pos, uv, nrm, has_n, has_uv = capi.mesh_file_triangles(path)
    assert not has_n and not has_uv
    assert not nrm.any() and not uv.any()
    P, _, _ = expected(FACES, ply_corner)
    np.testing.assert_array_equal(pos, P)


def test_ply_errors(tmp_path):
    with pytest.raises(capi.SrrError, match="cannot open"):
        capi.mesh_file_triangles(str(tmp_path / "missing.ply"))
    bad = str(tmp_path / "bad.ply")
    mf.write_ply(bad, VERTS, [[0, 1, 7]])
    with pytest.raises(capi.SrrError, match="out of range"):
        capi.mesh_file_triangles(bad)
    with open(str(tmp_path / "m.obj"), "w") as f:
        f.write("v 0 0 0\n")
    with pytest.raises(capi.SrrError, match="unsupported"):
        capi.mesh_file_triangles(str(tmp_path / "m.obj"))
    trunc = str(tmp_path / "t.ply")
    mf.write_ply(trunc, VERTS, FACES, fmt="binary_little_endian")
    data = open(trunc, "rb").read()
    open(trunc, "wb").write(data[:-5])
    with pytest.raises(capi.SrrError, match="truncated"):
        capi.mesh_file_triangles(trunc)


# ------------------------------------------------------------------------ FBX
# Polygons of the FBX geometry and their per-polygon-vertex attributes.
FBX_POLYS = [[0, 1, 2, 3], [0, 1, 4], [1, 2, 4]]
FBX_MATS = [1, 0, 0]  # polygon 0 uses material 1 -> assimp's mesh 1, not loaded


def _fbx_attrs():
    nc = sum(len(p) for p in FBX_POLYS)
    rng = np.random.default_rng(5)
    nrm = rng.standard_normal((nc, 3)).astype(np.float64)
    uvd = rng.random((7, 2)).astype(np.float64)
    uvi = rng.integers(0, 7, nc)
    return nrm, uvd, uvi


def _fbx_corner_fn():
    nrm, uvd, uvi = _fbx_attrs()
    starts = np.cumsum([0] + [len(p) for p in FBX_POLYS])

    def corner(fi, c):
        k = starts[fi] + c
        u = uvd[uvi[k]]
        return VERTS[FBX_POLYS[fi][c]], nrm[k].astype(np.float32), [np.float32(u[0]), np.float32(u[1]), 0.0]
    return corner


def _write_two_model_fbx(path, version, compress, decoy_first):
    nrm, uvd, uvi = _fbx_attrs()
    geo = mf.fbx_geometry(100, VERTS.astype(np.float64), FBX_POLYS, nrm, uvd, uvi, FBX_MATS)
    decoy = mf.fbx_geometry(200, VERTS.astype(np.float64) + 10, [[0, 1, 2]])
    objs = [decoy, geo] if decoy_first else [geo, decoy]
    objs += [mf.fbx_model(10, "first"), mf.fbx_model(20, "second")]
    # root -> model 10 -> geometry 100; root -> model 20 -> geometry 200
    con = [(10, 0), (20, 0), (100, 10), (200, 20)]
    mf.write_fbx(path, mf.fbx_scene(objs, con), version=version, compress=compress)


@pytest.mark.parametrize("version,compress", [(7400, False), (7400, True), (7500, False), (7700, True)])
def test_fbx_mesh0_by_material(tmp_path, version, compress):
    path = str(tmp_path / "m.fbx")
    _write_two_model_fbx(path, version, compress, decoy_first=True)
    pos, uv, nrm, has_n, has_uv = capi.mesh_file_triangles(path, False, False, (1.0, 1.0, 1.0))
    assert has_n and has_uv
    keep = [i for i, m in enumerate(FBX_MATS) if m == min(FBX_MATS)]
    corner = _fbx_corner_fn()
    P, N, U = expected([FBX_POLYS[i] for i in keep], lambda fi, c: corner(keep[fi], c))
    np.testing.assert_array_equal(pos, P)
    np.testing.assert_array_equal(nrm, N)
    np.testing.assert_array_equal(uv, U)


def test_fbx_flips_and_scale(tmp_path):
    path = str(tmp_path / "m.fbx")
    _write_two_model_fbx(path, 7400, False, decoy_first=False)
    pos, uv, nrm, _, _ = capi.mesh_file_triangles(path, True, True, (0.5, 2.0, -1.0))
    keep = [i for i, m in enumerate(FBX_MATS) if m == min(FBX_MATS)]
    corner = _fbx_corner_fn()
    P, N, U = expected([FBX_POLYS[i] for i in keep], lambda fi, c: corner(keep[fi], c), True, True, (0.5, 2.0, -1.0))
    np.testing.assert_array_equal(pos, P)
    np.testing.assert_array_equal(nrm, N)
    np.testing.assert_array_equal(uv, U)


def test_fbx_errors(tmp_path):
    p = str(tmp_path / "a.fbx")
    open(p, "wb").write(b"; FBX 7.4.0 project file\n")
    with pytest.raises(capi.SrrError, match="not a binary FBX"):
        capi.mesh_file_triangles(p)
    _write_two_model_fbx(p, 7400, True, False)
    data = open(p, "rb").read()
    open(p, "wb").write(data[:200])
    with pytest.raises(capi.SrrError):
        capi.mesh_file_triangles(p)


# -------------------------------------------------------- scene integration


def test_srr_model_creates_triangle_handles(tmp_path):
    path = str(tmp_path / "m.ply")
    mf.write_ply(path, VERTS, FACES, NRMS, UVS)
    L = capi.lib()
    L.srr_scene_create.restype = ctypes.c_void_p
    L.srr_scene_destroy.argtypes = [ctypes.c_void_p]
    L.srr_constant_texture.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float]
    L.srr_lambertian.argtypes = [ctypes.c_void_p, ctypes.c_int]
    h = L.srr_scene_create()
    mat = L.srr_lambertian(h, L.srr_constant_texture(h, 0.5, 0.5, 0.5))
    assert mat >= 0
    L.srr_model.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                            ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    first = ctypes.c_int(-1)
    sc3 = np.array([1, 1, 1], np.float32)
    n = L.srr_model(h, path.encode(), 0, 0, mat, sc3.ctypes.data, ctypes.byref(first))
    assert n == 6 and first.value >= 0
    assert L.srr_model(h, str(tmp_path / "nope.ply").encode(), 0, 0, mat, sc3.ctypes.data, None) < 0
    L.srr_scene_destroy(h)


def test_scene_model_records_explicit_triangles(tmp_path):
    path = str(tmp_path / "m.ply")
    mf.write_ply(path, VERTS, FACES, NRMS, UVS, fmt="binary_little_endian")
    s = Scene()
    m = s.lambertian(s.constant_texture((0.5, 0.5, 0.5)))
    tris = s.model(path, True, False, m, (1.0, 2.0, 1.0))
    assert len(tris) == 6
    assert sum(l.split()[2] == "triangle_uvn" for l in s.lines if l.startswith("obj")) == 6
    s.set_world(s.bvh_node(tris, 0, 1))
    s.set_lights(tris[0])
    s.camera((0, 0, 5), (0, 0, 0), (0, 1, 0), 40, 1.0, 0.0, 5.0)
    capi.Scene(s.text())  # the C-ABI parses the recorded text


REF_MODELS = "/root/reference/contents/models"


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference checkout absent (development container only)")
@pytest.mark.parametrize("name,n_tris,has_n,has_uv", [("bunny.ply", 69451, False, False),
                                                      ("Soilder.FBX", 3971, True, True),
                                                      ("hero01.FBX", 14268, True, True)])
def test_reference_content_models_load(name, n_tris, has_n, has_uv):
    """The mesh files the reference's scenes name (Raytracing_n.cpp:273, :637)
    load with the expected mesh-0 triangle counts (bunny: the PLY header's 69,451
    faces; Soilder: SURVEY §8 C4's 3,971) and finite vertices."""
    pos, uv, nrm, hn, hu = capi.mesh_file_triangles(os.path.join(REF_MODELS, name), False, True, (8.0, 8.0, 8.0))
    assert pos.shape == (n_tris, 3, 3) and (hn, hu) == (has_n, has_uv)
    assert np.isfinite(pos).all() and np.isfinite(uv).all()

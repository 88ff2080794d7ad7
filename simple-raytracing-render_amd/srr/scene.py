"""Python mirror of the reference's scene-building API.

The reference builds scenes as C++ object graphs with ``new`` (builders at
``Raytracing_n.cpp:108-711``): textures (``texture.h``), materials
(``material.h``), hitables (``sphere.h``, ``aarect.h``, ``box.h``,
``triangle.h``, ``hitable.h`` instance wrappers, ``bvh.h``,
``hitable_list.h``, ``constant_medium.h``) and a ``camera`` (``camera.h``).
This module offers the same constructors by the same names and records each
call, in call order, as one line of the srr scene description v1 (DESIGN.md
§3).  The text is what the C-ABI (``srr_scene_from_text``) and the test
oracles consume, so one scene definition drives every consumer.
"""
from __future__ import annotations

import hashlib
import os
import struct
import tempfile
from dataclasses import dataclass

# State of the reference's global 48-bit LCG after perlin.h's static
# initialisers took 1,533 draws from seed 1 (mathf.h:12, perlin.h:94-97).
POST_PERLIN_SEED = 24561125610955


def f32(x: float) -> str:
    """Round to float32 (the reference's constructors take ``float``) and print
    with enough digits to round-trip exactly."""
    v = struct.unpack("<f", struct.pack("<f", float(x)))[0]
    return repr(v) if v == v else "nan"


@dataclass(frozen=True)
class Tex:
    id: int


@dataclass(frozen=True)
class Mat:
    id: int


@dataclass(frozen=True)
class Obj:
    id: int


@dataclass(frozen=True)
class Group:
    id: int
    count: int


NULL_MAT = Mat(-1)


def _bvh_draws(n: int) -> int:
    """Number of drand48 draws bvh_node(l, n, ...) takes: one axis pick per node
    (bvh.h:97), recursing while n > 2 (bvh.h:104-113)."""
    if n <= 2:
        return 1
    return 1 + _bvh_draws(n // 2) + _bvh_draws(n - n // 2)


class Scene:
    def __init__(self) -> None:
        self.lines: list[str] = ["srr_scene 1"]
        self._n = {"tex": 0, "mat": 0, "obj": 0, "grp": 0}
        self.lcg = POST_PERLIN_SEED
        self._consumer_lcg = POST_PERLIN_SEED  # state a text consumer will have
        self.world: Obj | None = None
        self.lights: Obj | None = None
        self.has_camera = False

    def _id(self, ns: str) -> int:
        i = self._n[ns]
        self._n[ns] += 1
        return i

    def _emit(self, *tok) -> None:
        self.lines.append(" ".join(str(t) for t in tok))

    @staticmethod
    def _v(v) -> list[str]:
        return [f32(v[0]), f32(v[1]), f32(v[2])]

    # ------------------------------------------------------------ textures
    def constant_texture(self, c) -> Tex:
        if isinstance(c, (int, float)):
            c = (c, c, c)
        t = Tex(self._id("tex"))
        self._emit("tex", t.id, "const", *self._v(c))
        return t

    def image_texture_gen(self, w: int, h: int, seed: int, kind: str) -> Tex:
        """Synthetic RGB8 image (stands in for stbi_load'ed assets)."""
        k = {"sky": 0, "wood": 1, "checker": 2}[kind]
        t = Tex(self._id("tex"))
        self._emit("tex", t.id, "image_gen", w, h, seed, k)
        return t

    def image_texture_file(self, path: str) -> Tex:
        """``image_texture(stbi_load(path, &tx, &ty, &tn, 0), tx, ty)`` -- the
        builders' idiom (Raytracing_n.cpp:269-270, :614-616, :631-632).  The file
        is decoded now by srr's stb-exact decoder (srr_image_load) and recorded as
        an ``image_raw`` texture: the 3 bytes per texel image_texture addresses
        (texture.h:58-70), cached under $SRR_IMAGE_CACHE (default
        <tmp>/srr_images) by content hash."""
        from .capi import image_load  # the decoder lives in libsrr
        px, _ = image_load(path, 0)
        h, w, ch = px.shape
        if ch < 3:
            raise ValueError(f"{path}: image_texture needs 3 or 4 channels, file has {ch}")
        raw = px.reshape(-1)[: w * h * 3].tobytes()
        cache = os.environ.get("SRR_IMAGE_CACHE") or os.path.join(tempfile.gettempdir(), "srr_images")
        os.makedirs(cache, exist_ok=True)
        fn = os.path.join(cache, f"{hashlib.sha256(raw).hexdigest()[:24]}_{w}x{h}.rgb")
        if not (os.path.exists(fn) and os.path.getsize(fn) == len(raw)):
            tmp = f"{fn}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(raw)
            os.replace(tmp, fn)
        t = Tex(self._id("tex"))
        self._emit("tex", t.id, "image_raw", w, h, fn)
        return t

    def checker_texture(self, t0: Tex, t1: Tex) -> Tex:
        t = Tex(self._id("tex"))
        self._emit("tex", t.id, "checker", t0.id, t1.id)
        return t

    def noise_texture(self, scale: float) -> Tex:
        t = Tex(self._id("tex"))
        self._emit("tex", t.id, "noise", f32(scale))
        return t

    # ----------------------------------------------------------- materials
    def _mat(self, *tok) -> Mat:
        m = Mat(self._id("mat"))
        self._emit("mat", m.id, *tok)
        return m

    def lambertian(self, a: Tex) -> Mat:
        return self._mat("lambertian", a.id)

    def orennayar(self, a: Tex, sigma: float) -> Mat:
        return self._mat("orennayar", a.id, f32(sigma))

    def beckmann(self, a: Tex, roughx: float, roughy: float) -> Mat:
        return self._mat("beckmann", a.id, f32(roughx), f32(roughy))

    def metal(self, albedo, fuzz: float) -> Mat:
        if isinstance(albedo, (int, float)):
            albedo = (albedo,) * 3
        return self._mat("metal", *self._v(albedo), f32(fuzz))

    def dielectric(self, ri: float) -> Mat:
        return self._mat("dielectric", f32(ri))

    def diffuse_light(self, a: Tex) -> Mat:
        return self._mat("diffuse_light", a.id)

    def isotropic(self, a: Tex) -> Mat:
        return self._mat("isotropic", a.id)

    # ------------------------------------------------------------ hitables
    def _obj(self, *tok) -> Obj:
        o = Obj(self._id("obj"))
        self._emit("obj", o.id, *tok)
        return o

    def sphere(self, center, radius: float, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("sphere", *self._v(center), f32(radius), mat.id)

    def moving_sphere(self, c0, c1, t0, t1, radius, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("moving_sphere", *self._v(c0), *self._v(c1), f32(t0), f32(t1), f32(radius), mat.id)

    def xy_rect(self, x0, x1, y0, y1, k, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("xy_rect", f32(x0), f32(x1), f32(y0), f32(y1), f32(k), mat.id)

    def xz_rect(self, x0, x1, z0, z1, k, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("xz_rect", f32(x0), f32(x1), f32(z0), f32(z1), f32(k), mat.id)

    def yz_rect(self, y0, y1, z0, z1, k, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("yz_rect", f32(y0), f32(y1), f32(z0), f32(z1), f32(k), mat.id)

    def box(self, p0, p1, mat: Mat = NULL_MAT) -> Obj:
        return self._obj("box", *self._v(p0), *self._v(p1), mat.id)

    def triangle(self, p0, p1, p2, mat: Mat = NULL_MAT, uvs=None, normals=None) -> Obj:
        tok = [*self._v(p0), *self._v(p1), *self._v(p2), mat.id]
        if uvs is None and normals is None:
            return self._obj("triangle", *tok)
        uvs = uvs or ((0, 0, 0),) * 3
        tok += [*self._v(uvs[0]), *self._v(uvs[1]), *self._v(uvs[2])]
        if normals is None:
            return self._obj("triangle_uv", *tok)
        tok += [*self._v(normals[0]), *self._v(normals[1]), *self._v(normals[2])]
        return self._obj("triangle_uvn", *tok)

    def flip_normals(self, child: Obj) -> Obj:
        return self._obj("flip", child.id)

    def translate(self, child: Obj, offset) -> Obj:
        return self._obj("translate", child.id, *self._v(offset))

    def rotate_y(self, child: Obj, angle: float) -> Obj:
        return self._obj("rotate_y", child.id, f32(angle))

    def rotate_x(self, child: Obj, angle: float) -> Obj:
        return self._obj("rotate_x", child.id, f32(angle))

    def constant_medium(self, boundary: Obj, density: float, a: Tex) -> Obj:
        return self._obj("constant_medium", boundary.id, f32(density), a.id)

    def hitable_list(self, children) -> Obj:
        if isinstance(children, Group):
            return self._obj("list_group", children.id)
        children = list(children)
        return self._obj("list", len(children), *[c.id for c in children])

    def bvh_node(self, children, time0: float = 0.0, time1: float = 1.0) -> Obj:
        if self._consumer_lcg != self.lcg:  # script-level draws happened since
            self._emit("lcg", self.lcg)
        if isinstance(children, Group):
            n = children.count
            o = self._obj("bvh_group", f32(time0), f32(time1), children.id)
        else:
            children = list(children)
            n = len(children)
            o = self._obj("bvh", f32(time0), f32(time1), n, *[c.id for c in children])
        self._advance_lcg(_bvh_draws(n))
        self._consumer_lcg = self.lcg
        return o

    def teapot(self, scale: float, divs: int, mat: Mat = NULL_MAT) -> Group:
        """Utah teapot tessellated like teapot::createPloyTeapot (teapot.h:76-166)
        but with a chosen ``divs`` (the reference hard-codes 100); each
        triangle carries its face normal (SURVEY Q5 build definition)."""
        g = Group(self._id("grp"), 32 * divs * divs * 2)
        self._emit("grp", g.id, "teapot", f32(scale), int(divs), mat.id)
        return g

    def model(self, filename: str, flip_uvs: bool, flip_winding: bool, mat: Mat = NULL_MAT,
              scale=(1.0, 1.0, 1.0)) -> list[Obj]:
        """``model(filename, flipUVs, flipWindingOrder, mat, scale).genhitablemodel()``
        (model.h:28-59, :75-91; geometry.h:24-90): the triangles of the file's first
        mesh, read now by srr's PLY / binary-FBX loader (assimp replaced) and
        recorded as explicit triangles, so every consumer of the text sees the same
        vertices.  Triangles carry the file's normals when it has them, else their
        face normal (SURVEY Q19 build definition); corners without UVs get (0,0,0)."""
        from .capi import mesh_file_triangles  # the loader lives in libsrr
        pos, uv, nrm, has_n, _ = mesh_file_triangles(filename, flip_uvs, flip_winding, scale)
        out = []
        for t in range(len(pos)):
            out.append(self.triangle(*pos[t].tolist(), mat=mat, uvs=uv[t].tolist(),
                                     normals=nrm[t].tolist() if has_n else None))
        return out

    # -------------------------------------------------------------- camera
    def camera(self, lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, t0=0.0, t1=1.0) -> None:
        self._emit("camera", *self._v(lookfrom), *self._v(lookat), *self._v(vup), f32(vfov), f32(aspect),
                   f32(aperture), f32(focus_dist), f32(t0), f32(t1))
        self.has_camera = True

    def set_world(self, o: Obj) -> None:
        self.world = o
        self._emit("world", o.id)

    def set_lights(self, o: Obj) -> None:
        self.lights = o
        self._emit("lights", o.id)

    # ------------------------------------------------------- scene LCG state
    def set_lcg(self, state: int) -> None:
        self.lcg = state & 0xFFFFFFFFFFFF
        self._consumer_lcg = self.lcg
        self._emit("lcg", self.lcg)

    def drand48(self) -> float:
        """The reference's global LCG (mathf.h:14-19), for builders that draw
        scene parameters (e.g. random_scene); keeps the state bvh_node sees."""
        self.lcg = (0x5DEECE66D * self.lcg + 0xB16) & 0xFFFFFFFFFFFF
        return (self.lcg >> 16) / 4294967296.0

    def _advance_lcg(self, n: int) -> None:
        for _ in range(n):
            self.lcg = (0x5DEECE66D * self.lcg + 0xB16) & 0xFFFFFFFFFFFF

    def text(self) -> str:
        if self.world is None or self.lights is None or not self.has_camera:
            raise ValueError("scene needs world, lights and a camera")
        return "\n".join(self.lines) + "\n"

"""ctypes binding of libsrr.so (include/srr_capi.h) -- the host-side mirror of
the reference's render driver (``renderthread``/``main``,
Raytracing_n.cpp:815-952) over the C-ABI.  The HIP path is the only path:
if libsrr.so is missing or no GPU is visible, calls fail loudly."""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SRR_LIB") or os.path.join(PKG, "libsrr.so")  # SRR_LIB: A/B builds
_LIB = None

FLAG_SORT_MATERIALS = 1
FLAG_KEEP_PATHS = 2
FLAG_COUNT_VISITS = 4
FLAG_WAVEFRONT = 8
FLAG_CONTINUE = 16
FLAG_SUMS = 32


class SrrError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int), ("ny", ctypes.c_int), ("spp", ctypes.c_int), ("max_depth", ctypes.c_int),
                ("tile", ctypes.c_int), ("shard_index", ctypes.c_int), ("shard_count", ctypes.c_int),
                ("batch_paths", ctypes.c_int), ("base_seed", ctypes.c_uint64), ("flags", ctypes.c_int),
                ("sample_begin", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("world_rays", ctypes.c_int64), ("paths", ctypes.c_int64), ("trace_launches", ctypes.c_int64),
                ("trace_ms", ctypes.c_double), ("shade_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("bounces", ctypes.c_int64), ("box_tests", ctypes.c_int64), ("tri_tests", ctypes.c_int64),
                ("stack_overflows", ctypes.c_int64), ("deep_traversals", ctypes.c_int64),
                ("mixture_capped", ctypes.c_int64), ("walks_suspended", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise SrrError(f"{LIB_PATH} not built (run __graft_entry__.build() or make -C simple-raytracing-render_amd)")
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 (the same SONAME
        # as /opt/rocm's, which libsrr.so's RUNPATH names), and whichever is loaded first
        # serves both.  Loaded first, /opt/rocm's left torch unable to initialise the GPU
        # afterwards ("No HIP GPUs are available", tools/torch_after_render.py), so when
        # torch is installed its runtime is loaded before libsrr.so.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, ip, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
        L.srr_last_error.restype = cp
        L.srr_version.restype = cp
        L.srr_scene_from_text.argtypes = [cp, ctypes.POINTER(vp)]
        L.srr_scene_destroy.argtypes = [vp]
        L.srr_renderer_create.argtypes = [vp, ip, ctypes.POINTER(vp)]
        L.srr_renderer_destroy.argtypes = [vp]
        L.srr_renderer_create_multi.argtypes = [vp, ip, vp, ctypes.POINTER(vp)]
        L.srr_renderer_devices.argtypes = [vp, vp, ip]
        L.srr_renderer_transport.argtypes = [vp]
        L.srr_renderer_transport.restype = cp
        L.srr_multi_plan.restype = ctypes.c_int64
        L.srr_multi_plan.argtypes = [ctypes.POINTER(Params), ip, vp, vp]
        L.srr_shard_pixels.restype = ctypes.c_int64
        L.srr_shard_pixels.argtypes = [ctypes.POINTER(Params), vp]
        L.srr_render_device.argtypes = [vp, ctypes.POINTER(Params), vp, ctypes.POINTER(Stats)]
        L.srr_render_device_async.argtypes = [vp, ctypes.POINTER(Params), vp, ctypes.POINTER(ctypes.c_int64)]
        L.srr_render_wait.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(Stats)]
        L.srr_merl_load.argtypes = [cp, ip, ctypes.POINTER(vp)]
        L.srr_merl_create.argtypes = [vp, ctypes.c_int64, ip, ctypes.POINTER(vp)]
        L.srr_merl_destroy.argtypes = [vp]
        L.srr_merl_lookup.argtypes = [vp, ctypes.c_int64, vp, vp, vp]
        L.srr_render.argtypes = [vp, ctypes.POINTER(Params), vp, vp, ctypes.POINTER(Stats)]
        L.srr_copy_paths.argtypes = [vp, vp, vp]
        L.srr_tonemap.argtypes = [vp, ctypes.c_int64, vp]
        L.srr_write_ppm.argtypes = [cp, ip, ip, vp]
        L.srr_sobol_points.argtypes = [ip, vp]
        L.srr_mesh_file_triangles.argtypes = [cp, ip, ip, vp, vp, vp, vp, ctypes.POINTER(ip)]
        u8p = ctypes.POINTER(ctypes.c_ubyte)
        L.srr_image_load.argtypes = [cp, ip, ctypes.POINTER(ip), ctypes.POINTER(ip), ctypes.POINTER(ip),
                                     ctypes.POINTER(u8p)]
        L.srr_image_free.argtypes = [u8p]
        L.srr_image_free.restype = None
        L.srr_write_png.argtypes = [cp, ip, ip, vp]
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.srr_accum_get.argtypes = [vp, vp, i64p, i64p]
        L.srr_accum_set.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int64]
        _LIB = L
    return _LIB


def _check(rc):
    if rc < 0:
        raise SrrError(f"srr error {rc}: {lib().srr_last_error().decode()}")
    return rc


def _ptr(a):
    return None if a is None else a.ctypes.data


def make_params(nx, ny, spp, max_depth=50, shard=(0, 1), tile=32, batch_paths=0, base_seed=0, flags=0,
                sample_begin=0):
    return Params(nx, ny, spp, max_depth, tile, shard[0], shard[1], batch_paths, base_seed, flags, sample_begin)


def shard_pixels(p: Params) -> np.ndarray:
    n = _check(lib().srr_shard_pixels(ctypes.byref(p), None))
    out = np.zeros(n, np.int32)
    lib().srr_shard_pixels(ctypes.byref(p), _ptr(out))
    return out


def multi_plan(p: Params, n_devices: int) -> tuple[np.ndarray, np.ndarray]:
    """srr_multi_plan (host only): the packed-frame order of an n-device frame --
    (gather_index[nx*ny]: image pixel of each packed entry, shard_offsets[n+1])."""
    total = _check(lib().srr_multi_plan(ctypes.byref(p), n_devices, None, None))
    index = np.zeros(total, np.int32)
    off = np.zeros(n_devices + 1, np.int64)
    _check(lib().srr_multi_plan(ctypes.byref(p), n_devices, _ptr(index), _ptr(off)))
    return index, off


def sobol_points(n: int) -> np.ndarray:
    out = np.zeros((n, 2), np.float64)
    _check(lib().srr_sobol_points(n, _ptr(out)))
    return out


class Scene:
    """A scene parsed from srr scene description v1 text."""

    def __init__(self, text: str):
        h = ctypes.c_void_p()
        _check(lib().srr_scene_from_text(text.encode(), ctypes.byref(h)))
        self.h = h
        self.text = text

    def __del__(self):
        if getattr(self, "h", None):
            lib().srr_scene_destroy(self.h)
            self.h = None


MERL_CELLS = 90 * 90 * 180  # doubles per channel of a MERL table (brdf.h:7-9)


class Merl:
    """A MERL measured-BRDF table on the GPU: the reference's ``brdf`` class
    (brdf.h).  ``Merl.load(path)`` is brdf::read_brdf, ``Merl(table)`` takes the
    3 * 90*90*180 doubles directly, ``lookup`` is brdf::lookup_brdf_val for a
    batch of (theta_in, fi_in, theta_out, fi_out) rows."""

    def __init__(self, table=None, device: int = 0, _handle=None):
        self.h = _handle
        if self.h is None:
            t = np.ascontiguousarray(table, dtype=np.float64).ravel()
            h = ctypes.c_void_p()
            _check(lib().srr_merl_create(t.ctypes.data, t.size, device, ctypes.byref(h)))
            self.h = h

    @classmethod
    def load(cls, path: str, device: int = 0) -> "Merl":
        h = ctypes.c_void_p()
        _check(lib().srr_merl_load(path.encode(), device, ctypes.byref(h)))
        return cls(_handle=h)

    def lookup(self, angles) -> tuple[np.ndarray, np.ndarray]:
        """angles: [n, 4] (theta_in, fi_in, theta_out, fi_out) -> (rgb [n, 3] f64, cell [n] int32)."""
        a = np.ascontiguousarray(angles, dtype=np.float64).reshape(-1, 4)
        rgb = np.zeros((a.shape[0], 3), np.float64)
        cell = np.zeros(a.shape[0], np.int32)
        _check(lib().srr_merl_lookup(self.h, a.shape[0], a.ctypes.data, rgb.ctypes.data, cell.ctypes.data))
        return rgb, cell

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.srr_merl_destroy(self.h)
            self.h = None


class Renderer:
    """Flattened scene resident on HIP device `device` (srr_renderer_create), or
    on every device of `devices` (srr_renderer_create_multi: the whole frame
    rendered over all of them, gathered to devices[0] over RCCL)."""

    def __init__(self, scene, device: int = 0, devices=None):
        if isinstance(scene, str):
            scene = Scene(scene)
        self.scene = scene
        h = ctypes.c_void_p()
        if devices is None:
            _check(lib().srr_renderer_create(scene.h, device, ctypes.byref(h)))
        else:
            ids = np.ascontiguousarray(devices, np.int32)
            _check(lib().srr_renderer_create_multi(scene.h, ids.size, _ptr(ids), ctypes.byref(h)))
        self.h = h

    def devices(self) -> list:
        n = _check(lib().srr_renderer_devices(self.h, None, 0))
        ids = np.zeros(n, np.int32)
        lib().srr_renderer_devices(self.h, _ptr(ids), n)
        return ids.tolist()

    @property
    def transport(self) -> str:
        """"rccl" / "copy" (multi-device frame-end gather) or "none" (one device)."""
        return lib().srr_renderer_transport(self.h).decode()

    def __del__(self):
        if getattr(self, "h", None):
            lib().srr_renderer_destroy(self.h)
            self.h = None

    def render(self, nx, ny, spp, max_depth=50, keep_paths=False, **kw):
        """Whole image (or shard); returns dict(mean[n,3], img8[n,3], stats,
        paths[n,spp,3], rays[n,spp] when keep_paths)."""
        flags = kw.pop("flags", 0) | (FLAG_KEEP_PATHS if keep_paths else 0)
        p = make_params(nx, ny, spp, max_depth, flags=flags, **kw)
        n = nx * ny if self.transport != "none" else shard_pixels(p).size
        mean = np.zeros((n, 3), np.float32)
        img8 = np.zeros((n, 3), np.uint8)
        st = Stats()
        _check(lib().srr_render(self.h, ctypes.byref(p), _ptr(mean), _ptr(img8), ctypes.byref(st)))
        out = dict(mean=mean, img8=img8, stats=st.as_dict())
        if keep_paths:
            paths = np.zeros((n, spp, 3), np.float32)
            rays = np.zeros((n, spp), np.uint8)
            _check(lib().srr_copy_paths(self.h, _ptr(paths), _ptr(rays)))
            out.update(paths=paths, rays=rays)
        return out

    def render_device(self, params: Params, d_mean_ptr: int) -> dict:
        """Render into a device buffer (e.g. a torch tensor's data_ptr())."""
        st = Stats()
        _check(lib().srr_render_device(self.h, ctypes.byref(params), ctypes.c_void_p(d_mean_ptr), ctypes.byref(st)))
        return st.as_dict()

    def render_device_async(self, params: Params, d_mean_ptr: int) -> int:
        """Enqueue a fresh frame (srr_render_device_async); returns its ticket.
        d_mean is written when wait(ticket) returns."""
        t = ctypes.c_int64()
        _check(lib().srr_render_device_async(self.h, ctypes.byref(params), ctypes.c_void_p(d_mean_ptr),
                                             ctypes.byref(t)))
        return t.value

    def wait(self, ticket: int) -> dict:
        """Wait for an async frame (srr_render_wait); returns its stats."""
        st = Stats()
        _check(lib().srr_render_wait(self.h, ctypes.c_int64(ticket), ctypes.byref(st)))
        return st.as_dict()


def tonemap(mean: np.ndarray) -> np.ndarray:
    mean = np.ascontiguousarray(mean, np.float32)
    out = np.zeros(mean.shape, np.uint8)
    _check(lib().srr_tonemap(_ptr(mean), mean.size // 3, _ptr(out)))
    return out


def scene_digest(text: str) -> str:
    """srr_scene_digest of a scene description: the FNV-1a digest of its
    flattened device tables (hex), equal for byte-identical scenes."""
    L = lib()
    L.srr_scene_digest.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    h = ctypes.c_void_p()
    _check(L.srr_scene_from_text(text.encode(), ctypes.byref(h)))
    d = ctypes.c_uint64()
    try:
        _check(L.srr_scene_digest(h, ctypes.byref(d), None))
    finally:
        L.srr_scene_destroy(h)
    return f"{d.value:016x}"


def write_ppm(path: str, nx: int, ny: int, img8: np.ndarray) -> None:
    img8 = np.ascontiguousarray(img8, np.uint8)
    _check(lib().srr_write_ppm(path.encode(), nx, ny, _ptr(img8)))


def image_load(path: str, req_comp: int = 0) -> tuple[np.ndarray, int]:
    """stbi_load(path, &x, &y, &comp, req_comp) (stb_image v2.19, as the
    reference's builders call it): returns ``(pixels[y, x, channels], comp)``
    with comp the file's own channel count."""
    x, y, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    p = ctypes.POINTER(ctypes.c_ubyte)()
    ch = _check(lib().srr_image_load(path.encode(), req_comp, ctypes.byref(x), ctypes.byref(y), ctypes.byref(n),
                                     ctypes.byref(p)))
    try:
        px = np.ctypeslib.as_array(p, shape=(y.value, x.value, ch)).copy()
    finally:
        lib().srr_image_free(p)
    return px, n.value


def write_png(path: str, nx: int, ny: int, img8: np.ndarray) -> None:
    img8 = np.ascontiguousarray(img8, np.uint8)
    if img8.size != nx * ny * 3:
        raise SrrError("write_png needs nx*ny*3 bytes")
    _check(lib().srr_write_png(path.encode(), nx, ny, _ptr(img8)))


def mesh_file_triangles(path: str, flip_uvs: bool = False, flip_winding: bool = False, scale=(1.0, 1.0, 1.0)):
    """Mesh 0 of a PLY / binary FBX file as the reference's model loader builds it
    (model.h:28-59, geometry.h:24-79): returns ``(pos, uv, nrm, has_normals,
    has_uvs)`` with arrays of shape (n_tris, 3 corners, 3)."""
    sc = np.ascontiguousarray(scale, np.float32)
    fl = ctypes.c_int(0)
    n = _check(lib().srr_mesh_file_triangles(path.encode(), int(flip_uvs), int(flip_winding), _ptr(sc), None, None,
                                             None, ctypes.byref(fl)))
    pos, uv, nrm = (np.zeros((n, 3, 3), np.float32) for _ in range(3))
    _check(lib().srr_mesh_file_triangles(path.encode(), int(flip_uvs), int(flip_winding), _ptr(sc), _ptr(pos),
                                         _ptr(uv), _ptr(nrm), None))
    return pos, uv, nrm, bool(fl.value & 1), bool(fl.value & 2)

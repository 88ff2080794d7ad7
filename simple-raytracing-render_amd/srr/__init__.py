"""srr -- MI355X-native path tracer with the reference renderer's scene API.

* ``srr.scene``  -- reference-named scene builder (emits scene description v1)
* ``srr.scenes`` -- benchmark scenes S1-S5
* ``srr.capi``   -- ctypes binding of libsrr.so (include/srr_capi.h), the HIP path
"""
from . import capi, scene, scenes  # noqa: F401

__all__ = ["scene", "scenes", "capi"]

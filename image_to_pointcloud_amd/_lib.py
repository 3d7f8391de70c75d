"""ctypes binding of libi2pc.so (the C ABI declared in include/i2pc.h).

The library is built in-tree by `python -m image_to_pointcloud_amd.build`.
There is NO fallback: if the library is missing, or a compute entry point is
called without a HIP device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("I2PC_LIB") or os.path.join(_PKG, "libi2pc.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "i2pc.h")

c_int = ctypes.c_int
c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_size_t = ctypes.c_size_t
c_double = ctypes.c_double
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p


class UnprojectParams(ctypes.Structure):
    _fields_ = [
        ("step", c_int32),
        ("invert", c_int32),
        ("depth_scale", c_double),
        ("fov_deg", c_double),
        ("smooth", c_int32),
        ("smooth_ksize", c_int32),
        ("projection", c_int32),     # 0 pinhole, 1 equirectangular
        ("reserved", c_int32),
    ]


class I2PCError(RuntimeError):
    pass


# name -> (restype, argtypes)
_SIGNATURES = {
    "i2pc_abi_version": (c_int, []),
    "i2pc_last_error": (c_char_p, []),
    "i2pc_unproject_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "i2pc_unproject": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                               ctypes.POINTER(UnprojectParams), c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_size_t, c_void_p]),
    "i2pc_gather_stride": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "i2pc_profile_enable": (c_int, [c_int]),
    "i2pc_profile_unproject_ms": (c_float, []),
    "i2pc_sor_workspace_bytes": (c_size_t, [c_int64]),
    "i2pc_sor": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "i2pc_clock_probe": (c_int, [c_int, c_int, c_void_p, c_void_p]),
}

_lib = None


def declared_symbols() -> list[str]:
    """Every function name declared in include/i2pc.h."""
    with open(HEADER_PATH) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(i2pc_[a-z0-9_]+)\s*\(", text)))


def load() -> ctypes.CDLL:
    """Load libi2pc.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise I2PCError(f"{LIB_PATH} is missing: build it with `python -m image_to_pointcloud_amd.build` "
                        "(hipcc, gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def register(name: str, restype, argtypes) -> None:
    """Add a signature (used by modules that bind further entry points)."""
    _SIGNATURES[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def call(name: str, *args) -> int:
    """Call an entry point whose signature is registered (without argtypes, ctypes would pass a
    device pointer as a 32-bit int: a truncated address and a memory fault on the GPU)."""
    lib = load()
    fn = getattr(lib, name)
    if fn.argtypes is None:
        raise I2PCError(f"{name}: no ctypes signature registered (_lib.register)")
    rc = fn(*args)
    if isinstance(rc, int) and rc != 0:
        msg = lib.i2pc_last_error().decode(errors="replace")
        raise I2PCError(f"{name} failed ({rc}): {msg}")
    return rc

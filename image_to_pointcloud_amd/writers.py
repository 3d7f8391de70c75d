"""Point-cloud artefact writers: the host-side mirror of save_point_cloud
(backend/app.py:310-389) over the native writers of libi2pc.so (csrc/writers.cpp).

`save_point_cloud(points, colors, format, filename)` has the reference's
signature, output paths (outputs/<filename>.<ext>) and error behaviour (ValueError
for an unsupported format, logged and re-raised). Points may be numpy arrays or
device tensors; colours may be float (0..255 integers, the reference's dtype)
or uint8.
"""
from __future__ import annotations

import ctypes
import logging
import os
from pathlib import Path

import numpy as np

from . import _lib

logger = logging.getLogger(__name__)

_lib.register("i2pc_write_xyz", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_int])
_lib.register("i2pc_write_ply", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64])
_lib.register("i2pc_write_las", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_double])

OUTPUT_DIR = "outputs"


def _host(points, colors):
    if hasattr(points, "detach"):
        points = points.detach().cpu().numpy()
    if colors is not None and hasattr(colors, "detach"):
        colors = colors.detach().cpu().numpy()
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    cols = None
    # batched [B, N, 3] buffers flatten to the points' row-major order before the count check
    c = None if colors is None else np.asarray(colors).reshape(-1, 3)
    if c is not None and len(c) == len(pts) and len(c) > 0:
        if c.dtype != np.uint8:
            c = np.clip(c, 0, 255).astype(np.uint8)      # integers 0..255 in the reference (app.py:239-244)
        cols = np.ascontiguousarray(c).reshape(-1, 3)
    return pts, cols


def _ptr(a):
    return None if a is None else a.ctypes.data


def write_xyz(path: str, points, colors, threads: int = 0) -> str:
    pts, cols = _host(points, colors)
    threads = threads or min(16, os.cpu_count() or 1)
    _lib.call("i2pc_write_xyz", path.encode(), _ptr(pts), _ptr(cols), len(pts), threads)
    return path


def write_ply(path: str, points, colors) -> str:
    pts, cols = _host(points, colors)
    _lib.call("i2pc_write_ply", path.encode(), _ptr(pts), _ptr(cols), len(pts))
    return path


def write_las(path: str, points, colors, scale: float = 0.01) -> str:
    pts, cols = _host(points, colors)
    if len(pts) == 0:
        raise ValueError("No points to write to LAS")                  # app.py:360-361
    _lib.call("i2pc_write_las", path.encode(), _ptr(pts), _ptr(cols), len(pts), float(scale))
    return path


def save_point_cloud(points, colors, format: str, filename: str) -> str:
    """Drop-in for app.py:310-331."""
    try:
        Path(OUTPUT_DIR).mkdir(exist_ok=True)
        fmt = format.lower()
        if fmt == "ply":
            return write_ply(f"{OUTPUT_DIR}/{filename}.ply", points, colors)
        if fmt in ("las", "laz"):
            return write_las(f"{OUTPUT_DIR}/{filename}.las", points, colors)
        if fmt == "xyz":
            return write_xyz(f"{OUTPUT_DIR}/{filename}.xyz", points, colors)
        raise ValueError(f"Unsupported format: {format}")
    except Exception as e:
        logger.error(f"Error saving point cloud: {str(e)}")
        raise

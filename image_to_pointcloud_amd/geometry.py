"""Depth -> point cloud on the GPU: the host-side mirror of the reference interface.

`depth_to_point_cloud` keeps the signature, argument meaning, return types and
error behaviour of backend/app.py:174-250 (numpy in, numpy out, raises on bad
input); `generate_gis_bounds` mirrors app.py:393-400.  Both run the HIP
kernels of libi2pc.so through the C ABI (include/i2pc.h); there is no CPU path.

`unproject_batch` is the batched device API the pipeline uses: torch CUDA
tensors in, torch CUDA tensors out, stream-ordered on the current stream.
"""
from __future__ import annotations

import ctypes
import logging
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib

logger = logging.getLogger(__name__)

DENSITY_STEP = {"low": 4, "medium": 2, "high": 1}   # app.py:226
# camera model of the back-projection: the reference's pinhole (app.py:216-238), or an
# equirectangular panorama (C4's 360-degree images; not in the reference, see i2pc.h)
PROJECTION = {"pinhole": 0, "equirect": 1}


def _torch():
    import torch
    return torch


def require_device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise _lib.I2PCError("image_to_pointcloud_amd needs a HIP device (MI355X); no CPU fallback exists")
    return torch.device("cuda", torch.cuda.current_device())


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream_handle():
    return _torch().cuda.current_stream().cuda_stream


_WS = {}


def workspace_bytes(batch: int, height: int, width: int, smooth: bool = False) -> int:
    """Device workspace one i2pc_unproject call of this shape needs (SelState + histograms + tap tables)."""
    return int(_lib.load().i2pc_unproject_workspace_bytes(batch, height, width, int(bool(smooth))))


def _workspace(nbytes: int, device):
    """Per-device scratch for one-off calls.  It is REPLACED when a call needs more bytes, so a
    caller that records launches into a HIP graph must own its workspace instead (pass
    `workspace=` to unproject_batch / unproject_band; PointCloudPipeline does)."""
    torch = _torch()
    key = (device.index if device.index is not None else torch.cuda.current_device())
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


@dataclass
class PointBatch:
    xyz: "object"     # torch.float32 [B, N, 3] on device
    rgb: "object"     # torch.uint8   [B, N, 3] on device
    bbox: "object"    # torch.float64 [B, 6]   minX maxX minY maxY minZ maxZ
    stats: "object"   # torch.float64 [B, 4]   p2 p98 branch median


def point_count(h: int, w: int, step: int) -> int:
    return ((h + step - 1) // step) * ((w + step - 1) // step)


def unproject_batch(depth, images, density: str = "medium", invert: bool = True,
                    depth_scale: float = 10.0, smooth: bool = False, smooth_ksize: int = 5,
                    fov: Optional[float] = None, out: Optional[PointBatch] = None,
                    workspace=None, projection: str = "pinhole") -> PointBatch:
    """Batched GPU depth_to_point_cloud.

    depth    : torch.float32 [B, h, w] (model resolution) on the device
    images   : torch.uint8 [B, H, W, C] BGR on the device
    workspace: optional caller-owned device uint8 buffer of >= workspace_bytes(B, H, W, smooth)
               bytes (required for graph capture: the shared per-device one may be reallocated)
    projection: "pinhole" (the reference's camera) or "equirect" (360-degree panoramas)
    """
    torch = _torch()
    if density not in DENSITY_STEP:
        raise KeyError(density)            # the reference's dict lookup raises KeyError (app.py:226)
    step = DENSITY_STEP[density]
    if depth.dim() == 2:
        depth = depth.unsqueeze(0)
    if images.dim() == 3:
        images = images.unsqueeze(0) if images.shape[-1] in (3, 4) else images.unsqueeze(-1).unsqueeze(0)
    if images.dim() == 2:
        images = images.unsqueeze(0).unsqueeze(-1)
    B, H, W, C = images.shape
    if depth.shape[0] != B:
        raise ValueError(f"batch mismatch: depth {tuple(depth.shape)} vs images {tuple(images.shape)}")
    if not depth.is_cuda or not images.is_cuda:
        raise _lib.I2PCError("unproject_batch expects device tensors")
    depth = depth.contiguous().to(torch.float32)
    images = images.contiguous()
    if images.dtype != torch.uint8:
        raise TypeError("images must be uint8")
    N = point_count(H, W, step)
    dev = depth.device
    if out is None:
        out = PointBatch(
            xyz=torch.empty((B, N, 3), dtype=torch.float32, device=dev),
            rgb=torch.empty((B, N, 3), dtype=torch.uint8, device=dev),
            bbox=torch.empty((B, 6), dtype=torch.float64, device=dev),
            stats=torch.empty((B, 4), dtype=torch.float64, device=dev),
        )
    lib = _lib.load()
    ws_bytes = lib.i2pc_unproject_workspace_bytes(B, H, W, int(bool(smooth)))
    if workspace is not None:
        if workspace.dtype != torch.uint8 or not workspace.is_cuda or workspace.numel() < ws_bytes:
            raise ValueError(f"workspace must be a device uint8 buffer of >= {ws_bytes} bytes")
        ws = workspace
    else:
        ws = _workspace(ws_bytes, dev)
    p = _lib.UnprojectParams(step=step, invert=int(bool(invert)), depth_scale=float(depth_scale),
                             fov_deg=float(fov) if fov else 0.0, smooth=int(bool(smooth)),
                             smooth_ksize=int(smooth_ksize), projection=PROJECTION[projection])
    _lib.call("i2pc_unproject", _ptr(depth), depth.shape[1], depth.shape[2], _ptr(images), C, B, H, W,
              ctypes.byref(p), _ptr(out.xyz), _ptr(out.rgb), _ptr(out.bbox), _ptr(out.stats),
              _ptr(ws), ws.numel(), _stream_handle())
    return out


def depth_to_point_cloud(image: np.ndarray, depth: np.ndarray, density: str = "medium",
                         invert: bool = True, depth_scale: float = 10.0, smooth: bool = False,
                         smooth_ksize: int = 5, fov: Optional[float] = None) -> tuple:
    """Drop-in for backend/app.py:174 -- same arguments, (points f32 Nx3, colors f32 Nx3)."""
    torch = _torch()
    try:
        dev = require_device()
        img = np.ascontiguousarray(image)
        if img.ndim == 2:
            img = img[:, :, None]
        timg = torch.from_numpy(img).to(dev)
        tdep = torch.from_numpy(np.ascontiguousarray(depth, dtype=np.float32)).to(dev)
        pb = unproject_batch(tdep.unsqueeze(0), timg.unsqueeze(0), density=density, invert=invert,
                             depth_scale=depth_scale, smooth=smooth, smooth_ksize=smooth_ksize, fov=fov)
        pts = pb.xyz[0].cpu().numpy()
        cols = pb.rgb[0].to(torch.float32).cpu().numpy()
        return pts, cols
    except Exception as e:
        logger.error(f"Error in point cloud generation: {str(e)}")   # app.py:248-250
        raise


def generate_gis_bounds(bbox_row) -> dict:
    """bounds dict of generate_gis_metadata (app.py:393-400) from a device bbox row."""
    b = [float(x) for x in (bbox_row.tolist() if hasattr(bbox_row, "tolist") else bbox_row)]
    return {"minX": b[0], "maxX": b[1], "minY": b[2], "maxY": b[3], "minZ": b[4], "maxZ": b[5]}


def preview_subsample(xyz, rgb, max_preview: int = 20000):
    """Preview stride subsample (app.py:496-506) on device; returns python lists."""
    torch = _torch()
    n = xyz.shape[0]
    stride = max(1, n // max_preview) if n > max_preview else 1
    cnt = (n + stride - 1) // stride
    oxyz = torch.empty((cnt, 3), dtype=torch.float32, device=xyz.device)
    orgb = torch.empty((cnt, 3), dtype=torch.float32, device=xyz.device)
    _lib.call("i2pc_gather_stride", _ptr(xyz.contiguous()), _ptr(rgb.contiguous()), n, stride,
              _ptr(oxyz), _ptr(orgb), _stream_handle())
    return oxyz.cpu().double().tolist(), orgb.cpu().double().tolist()


@dataclass
class SorResult:
    xyz: "object"     # torch.float32 [m, 3] kept points, original order (device)
    rgb: "object"     # torch.uint8 [m, 3] or None
    index: "object"   # torch.int64 [m] kept indices, ascending (Open3D's `ind`)
    bbox: "object"    # torch.float64 [6] of the kept points (NaN if none)
    avg: "object"     # torch.float64 [n] mean distance of every point to its k nearest


def remove_statistical_outlier(xyz, rgb=None, nb_neighbors: int = 20, std_ratio: float = 2.0) -> SorResult:
    """Open3D PointCloud.remove_statistical_outlier (refine_point_cloud, app.py:252-269) on the device.

    xyz: torch.float32 [n, 3] on the device; rgb: torch.uint8 [n, 3] or None.
    Raises ValueError on the parameters Open3D rejects (nb_neighbors < 1, std_ratio <= 0).
    """
    torch = _torch()
    if nb_neighbors < 1 or not std_ratio > 0:
        raise ValueError("Illegal input parameters, the number of neighbors and standard deviation ratio "
                         "must be positive.")
    if not xyz.is_cuda:
        raise _lib.I2PCError("remove_statistical_outlier expects device tensors")
    xyz = xyz.reshape(-1, 3).contiguous().to(torch.float32)
    n, dev = xyz.shape[0], xyz.device
    if rgb is not None:
        rgb = rgb.reshape(-1, 3).contiguous()
        if rgb.dtype != torch.uint8 or rgb.shape[0] != n or not rgb.is_cuda:
            raise TypeError("rgb must be a device uint8 [n, 3] tensor matching xyz")
    oxyz = torch.empty_like(xyz)
    orgb = torch.empty_like(rgb) if rgb is not None else None
    oidx = torch.empty(n, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    bbox = torch.empty(6, dtype=torch.float64, device=dev)
    avg = torch.empty(n, dtype=torch.float64, device=dev)
    lib = _lib.load()
    ws = _workspace(lib.i2pc_sor_workspace_bytes(n), dev)
    _lib.call("i2pc_sor", _ptr(xyz), _ptr(rgb), n, int(nb_neighbors), float(std_ratio), _ptr(oxyz), _ptr(orgb),
              _ptr(oidx), _ptr(cnt), _ptr(bbox), _ptr(avg), _ptr(ws), ws.numel(), _stream_handle())
    m = int(cnt.item())
    return SorResult(oxyz[:m], orgb[:m] if orgb is not None else None, oidx[:m], bbox, avg)


# ----------------------------------------------------------------- tile-parallel (C4)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_void_p)
_lib.register("i2pc_comm_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int])
_lib.register("i2pc_comm_create", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_void_p)])
_lib.register("i2pc_comm_destroy", None, [ctypes.c_void_p])
_lib.register("i2pc_unproject_band_rccl", ctypes.c_int,
              [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.c_int, ctypes.c_int, ctypes.POINTER(_lib.UnprojectParams), ctypes.c_void_p, ctypes.c_void_p,
               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p])
GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                             ctypes.c_void_p)
_lib.register("i2pc_unproject_band_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                                       ctypes.c_int])
_lib.register("i2pc_unproject_band_w", ctypes.c_int,
              [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.c_int, ctypes.c_int, ctypes.POINTER(_lib.UnprojectParams), ctypes.c_void_p, ctypes.c_void_p,
               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, EXCHANGE_FN,
               GATHER_FN, ctypes.c_void_p, ctypes.c_void_p])
_lib.register("i2pc_unproject_band", ctypes.c_int,
              [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.c_int, ctypes.c_int, ctypes.POINTER(_lib.UnprojectParams), ctypes.c_void_p, ctypes.c_void_p,
               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, EXCHANGE_FN, ctypes.c_void_p,
               ctypes.c_void_p])


class _DevView:
    """A device buffer handed over by the C side, viewed as a torch tensor (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2}


def _as_tensor(ptr: int, n: int, typestr: str):
    torch = _torch()
    return torch.as_tensor(_DevView(ptr, n, typestr), device="cuda")


def band_workspace_bytes(img_h: int, img_w: int, smooth: bool = False, nranks: int = 1) -> int:
    """Workspace of a window-selection band call (an RcclComm, or `gather=`) over `nranks` bands."""
    return int(_lib.load().i2pc_unproject_band_workspace_bytes(img_h, img_w, int(bool(smooth)), int(nranks)))


def band_rows(img_h: int, parts: int, step: int = 1) -> list:
    """Split image rows into `parts` contiguous bands [row0, row1) whose starts are multiples
    of the density step (so every band owns whole point rows), as even as that allows."""
    rows_pts = (img_h + step - 1) // step
    out = []
    for r in range(parts):
        p0 = rows_pts * r // parts
        p1 = rows_pts * (r + 1) // parts
        out.append((min(p0 * step, img_h), min(p1 * step, img_h)))
    return out


def unproject_band(depth, image_band, img_h: int, img_w: int, row0: int, row1: int, exchange=None,
                   density: str = "high", invert: bool = True, depth_scale: float = 10.0,
                   fov: Optional[float] = None, workspace=None, comm=None, out=None,
                   projection: str = "pinhole", smooth: bool = False, smooth_ksize: int = 5,
                   gather=None, nranks: Optional[int] = None):
    """This rank's band [row0, row1) of one image's unprojection (i2pc_unproject_band).

    smooth     : smooth_depth (app.py:208-214): the band's blurred field is recomputed with its
                 k/2 halo rows locally, bit-identical to the whole image's
    comm       : a distributed.RcclComm: the exchange runs on the device (RCCL all-reduce and
                 all-gather on the current stream, i2pc_unproject_band_rccl, window selection) --
                 no host callback, graph-capturable; otherwise `exchange` (host callable, below)
    gather     : with `exchange`: callable(send: int32 [words], recv: int32 [nranks, words]) that
                 all-gathers every rank's words (e.g. distributed.band_gather(group)); selects the
                 one-sweep window mode (i2pc_unproject_band_w) instead of the four histogram levels
    nranks     : the number of bands (ranks) of a `gather` run
    out        : optional (xyz, rgb, bbox, stats) device tensors to write (graph capture)

    depth      : torch.float32 [h, w] model-resolution depth of the WHOLE image (device)
    image_band : torch.uint8 [row1 - row0, img_w, C] the band's image rows (device)
    exchange   : callable(hist: int32 tensor, counters: int64 [4, B] tensor or None) that
                 all-reduces in place across the ranks (hist SUM; counters rows 0-1 SUM,
                 row 2 MIN, row 3 MAX) -- e.g. distributed.band_exchange(group)
    workspace  : optional device uint8 buffer (default: the per-device cached one)
    -> (xyz [Nb, 3] f32, rgb [Nb, 3] u8, band bbox f64 [6], stats f64 [4]) on the device.
    """
    torch = _torch()
    if density not in DENSITY_STEP:
        raise KeyError(density)
    step = DENSITY_STEP[density]
    if image_band.dim() == 2:
        image_band = image_band.unsqueeze(-1)
    if not depth.is_cuda or not image_band.is_cuda:
        raise _lib.I2PCError("unproject_band expects device tensors")
    depth = depth.contiguous().to(torch.float32)
    image_band = image_band.contiguous()
    C = image_band.shape[-1]
    if tuple(image_band.shape[:2]) != (row1 - row0, img_w):
        raise ValueError(f"image_band {tuple(image_band.shape)} does not hold rows [{row0}, {row1}) x {img_w}")
    wn = (img_w + step - 1) // step
    nb = ((row1 + step - 1) // step - row0 // step) * wn
    dev = depth.device
    if out is not None:
        xyz, rgb, bbox, stats = out
        # the kernels write nb points: a buffer sized for another band or density would overrun
        for name, t, dt, need in (("xyz", xyz, torch.float32, nb * 3), ("rgb", rgb, torch.uint8, nb * 3),
                                  ("bbox", bbox, torch.float64, 6), ("stats", stats, torch.float64, 4)):
            if (t.dtype != dt or t.device != dev or not t.is_contiguous() or t.numel() < need
                    or (name in ("xyz", "rgb") and (t.dim() != 2 or t.shape[1] != 3))):
                raise ValueError(f"out {name}: need a contiguous {dt} tensor on {dev} with >= {need} elements"
                                 + (" shaped [>= nb, 3]" if name in ("xyz", "rgb") else "")
                                 + f", got {t.dtype} {tuple(t.shape)} on {t.device}")
    else:
        xyz = torch.empty((nb, 3), dtype=torch.float32, device=dev)
        rgb = torch.empty((nb, 3), dtype=torch.uint8, device=dev)
        bbox = torch.empty(6, dtype=torch.float64, device=dev)
        stats = torch.empty(4, dtype=torch.float64, device=dev)
    lib = _lib.load()
    if comm is not None:
        ws_bytes = band_workspace_bytes(img_h, img_w, smooth, comm.nranks)
    elif gather is not None:
        if not nranks or nranks < 1:
            raise ValueError("a gather band run needs nranks (the number of bands)")
        ws_bytes = band_workspace_bytes(img_h, img_w, smooth, nranks)
    else:
        ws_bytes = lib.i2pc_unproject_workspace_bytes(1, img_h, img_w, int(bool(smooth)))
    if workspace is not None:
        if workspace.dtype != torch.uint8 or not workspace.is_cuda or workspace.numel() < ws_bytes:
            raise ValueError(f"workspace must be a device uint8 buffer of >= {ws_bytes} bytes")
        ws = workspace
    else:
        ws = _workspace(ws_bytes, dev)
    if comm is not None:
        p = _lib.UnprojectParams(step=step, invert=int(bool(invert)), depth_scale=float(depth_scale),
                                 fov_deg=float(fov) if fov else 0.0, smooth=int(bool(smooth)),
                                 smooth_ksize=int(smooth_ksize), projection=PROJECTION[projection])
        _lib.call("i2pc_unproject_band_rccl", _ptr(depth), depth.shape[-2], depth.shape[-1], _ptr(image_band), C,
                  img_h, img_w, row0, row1, ctypes.byref(p), _ptr(xyz), _ptr(rgb), _ptr(bbox), _ptr(stats),
                  _ptr(ws), ws.numel(), comm.handle, _stream_handle())
        return xyz, rgb, bbox, stats
    if exchange is None:
        raise ValueError("unproject_band needs an exchange callable or an RcclComm")
    errors = []

    def _cb(user, hist, words, counters, batch, stream):
        try:
            h = _as_tensor(hist, int(words), "<i4") if hist and words > 0 else None
            c = _as_tensor(counters, 4 * int(batch), "<i8").view(4, int(batch)) if counters else None
            exchange(h, c)
            return 0
        except Exception as e:           # surfaced after the call returns
            errors.append(e)
            return 1

    def _gcb(user, send, recv, words, stream):
        try:
            gather(_as_tensor(send, int(words), "<i4"), _as_tensor(recv, int(nranks) * int(words), "<i4")
                   .view(int(nranks), int(words)))
            return 0
        except Exception as e:
            errors.append(e)
            return 1

    cb = EXCHANGE_FN(_cb)
    gcb = GATHER_FN(_gcb) if gather is not None else None
    p = _lib.UnprojectParams(step=step, invert=int(bool(invert)), depth_scale=float(depth_scale),
                             fov_deg=float(fov) if fov else 0.0, smooth=int(bool(smooth)),
                             smooth_ksize=int(smooth_ksize), projection=PROJECTION[projection])
    try:
        if gcb is not None:
            _lib.call("i2pc_unproject_band_w", _ptr(depth), depth.shape[-2], depth.shape[-1], _ptr(image_band), C,
                      img_h, img_w, row0, row1, ctypes.byref(p), _ptr(xyz), _ptr(rgb), _ptr(bbox), _ptr(stats),
                      _ptr(ws), ws.numel(), int(nranks), cb, gcb, None, _stream_handle())
        else:
            _lib.call("i2pc_unproject_band", _ptr(depth), depth.shape[-2], depth.shape[-1], _ptr(image_band), C,
                      img_h, img_w, row0, row1, ctypes.byref(p), _ptr(xyz), _ptr(rgb), _ptr(bbox), _ptr(stats),
                      _ptr(ws), ws.numel(), cb, None, _stream_handle())
    except _lib.I2PCError:
        if errors:
            raise errors[0]
        raise
    return xyz, rgb, bbox, stats

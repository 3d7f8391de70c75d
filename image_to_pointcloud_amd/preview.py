"""Depth preview (create_depth_preview, backend/app.py:124-172) on MI355X.

The uint8 image (fill, exact p2/p98 of the model-resolution depth, clip,
normalise, invert, (d*255).astype(uint8)) and the colour-table lookup run in one
stream-ordered C-ABI call (`i2pc_depth_preview`); only the PNG encode and base64
run on the host, as in the reference.

The colour table is matplotlib's "plasma" (the data OpenCV's COLORMAP_PLASMA
samples), rounded to uint8 and stored B,G,R like cv2.applyColorMap's output.
cv2 is absent from this image, so the table and the PNG bytes are "parity
unpinned"; the uint8 image before the table is pinned bit-exact against the
reference (tests/golden/preview_cases.npz).
"""
from __future__ import annotations

import base64
import ctypes
import io
import logging

import numpy as np

from . import _lib, geometry

logger = logging.getLogger(__name__)

DEPTH_PREVIEW_MAX = 2048      # app.py:43

# 256 x (B, G, R) uint8
PLASMA_BGR = bytes.fromhex(
    "87080d8807108907138a07168c06198d061b8e061d8f062090062291062491052692052893052a94052c95052e96052f"
    "9705319705339804359904379a04389a043a9b043c9c043e9c043f9d04419e03439e03449f03469f0348a00349a1034b"
    "a1024ca2024ea20250a30251a30253a40255a40156a40158a50159a5015ba6015ca6015ea60160a70061a70063a70064"
    "a70066a80067a80069a8006aa8006ca8006ea8006fa80071a80172a80174a80175a80177a80178a8027aa8027ba8037d"
    "a8037ea80480a70481a70583a70584a60686a60787a60888a5098aa50a8ba50b8da40c8ea40d8fa30e91a30f92a21094"
    "a11195a11396a014989f15999f169a9e179c9d189d9d199e9c1aa09b1ba19a1da29a1ea3991fa59820a69721a79622a8"
    "9523aa9424ab9426ac9327ad9228ae9129b0902ab18f2bb28e2cb38d2eb48c2fb58b30b68a31b78932b88833ba8834bb"
    "8735bc8637bd8538be8439bf833ac0823bc1813cc2803dc37f3ec47e40c57d41c67c42c77b43c87a44c97a45ca7946cb"
    "7847cc7749cc764acd754bce744ccf734dd0724ed1714fd27151d37052d46f53d56e54d56d55d66c56d76b57d86a58d9"
    "6a5ada695bda685cdb675ddc665edd655fde6461de6362df6363e06264e16165e26066e25f68e35e69e45d6ae55d6be5"
    "5c6ce65b6ee75a6fe75970e85871e95772e95774ea5675eb5576eb5477ec5379ed527aed517bee517cef507eef4f7ff0"
    "4e80f04d81f14c83f14b84f24b85f34a87f34988f44889f4478bf5468cf5458df6448ff64490f74391f74293f74194f8"
    "4095f83f97f93e98f93e9af93d9bfa3c9cfa3b9efa3a9ffb39a1fb38a2fb38a3fc37a5fc36a6fc35a8fc34a9fc33abfd"
    "33acfd32aefd31affd30b1fd2fb2fd2fb4fd2eb5fd2db7fe2cb8fe2cbafe2bbbfe2abdfe2abefe29c0fe29c2fd28c3fd"
    "27c5fd27c6fd27c8fd26cafd26cbfd25cdfc25cefc25d0fc25d2fc24d3fb24d5fb24d7fb24d8fa24dafa24dcf925ddf9"
    "25dff825e1f825e2f725e4f726e6f626e8f626e9f527ebf527edf427eef327f0f327f2f226f4f125f5f124f7f021f9f0"
)

_lib.register("i2pc_depth_preview", ctypes.c_int,
              [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p])

_LUT = {}


def _lut(device, table: bytes = PLASMA_BGR):
    import torch
    key = (device.index, table)
    if key not in _LUT:
        _LUT[key] = torch.frombuffer(bytearray(table), dtype=torch.uint8).to(device)
    return _LUT[key]


def depth_preview_batch(depth, invert: bool = True, out=None, stats=None, table: bytes = PLASMA_BGR):
    """depth: float32 device tensor [B, h, w] (model resolution) -> uint8 BGR [B, h, w, 3] on the device."""
    import torch
    if depth.dim() == 2:
        depth = depth.unsqueeze(0)
    if depth.dtype != torch.float32 or not depth.is_cuda:
        raise _lib.I2PCError("depth_preview_batch expects a float32 device tensor")
    depth = depth.contiguous()
    B, h, w = depth.shape
    if out is None:
        out = torch.empty((B, h, w, 3), dtype=torch.uint8, device=depth.device)
    lib = _lib.load()
    nbytes = lib.i2pc_unproject_workspace_bytes(B, h, w, 0)
    ws = geometry._workspace(nbytes, depth.device)
    _lib.call("i2pc_depth_preview", depth.data_ptr(), B, h, w, int(bool(invert)), _lut(depth.device, table).data_ptr(),
              out.data_ptr(), None if stats is None else stats.data_ptr(), ws.data_ptr(), ws.numel(),
              torch.cuda.current_stream().cuda_stream)
    return out


def encode_png_data_url(bgr: np.ndarray) -> str:
    """uint8 BGR [h, w, 3] -> "data:image/png;base64,..." (cv2.imencode('.png') + base64, app.py:164-167)."""
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(bgr[:, :, ::-1])).save(buf, format="PNG")
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode("utf-8")


def preview_size(h: int, w: int, max_dim: int = DEPTH_PREVIEW_MAX):
    """(out_h, out_w) of the preview: unchanged up to max_dim, else the reference's
    (int(round(dw * s)), int(round(dh * s))) with s = max_dim / max(dh, dw) (app.py:155-160)."""
    dmax = max(h, w)
    if dmax <= max_dim:
        return h, w
    s = max_dim / float(dmax)
    return int(round(h * s)), int(round(w * s))


def colored_preview(depth, invert: bool = True):
    """Device preview image as the reference encodes it: float32 depth [h, w] -> uint8 BGR
    [h', w', 3], the colour-mapped image INTER_AREA-downscaled when larger than 2048 px."""
    t = depth_preview_batch(depth, invert)[0]
    oh, ow = preview_size(t.shape[0], t.shape[1])
    if (oh, ow) != tuple(t.shape[:2]):
        from .preprocess import resize_area
        t = resize_area(t, ow, oh)                    # cv2.resize(..., INTER_AREA), app.py:158-160
    return t


def create_depth_preview(depth, invert: bool = True):
    """Drop-in for app.py:124: numpy (or device) depth -> PNG data URL, or None on failure."""
    import torch
    try:
        dev = geometry.require_device()
        t = depth if isinstance(depth, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(depth, np.float32))
        t = t.to(device=dev, dtype=torch.float32)
        img = colored_preview(t, invert).cpu().numpy()
        return encode_png_data_url(img)
    except Exception as e:        # the reference logs and returns None (app.py:169-171)
        logger.error(f"Failed to create depth preview: {e}")
        return None

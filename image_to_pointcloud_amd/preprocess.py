"""GPU network-input pipeline (app.py:103 + :109) with Pillow-exact resampling.

`Preprocessor(in_h, in_w, spec)` owns a device plan (coefficient tables) for one
input size; calling it on a uint8 BGR batch already in HBM returns either
pixel_values (float32 NCHW, bit-identical to DPTImageProcessorPil) or the bf16
patch rows the patch-embedding GEMM consumes.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

from . import _lib

_lib.register("i2pc_preprocess_plan_create", ctypes.c_int,
              [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
               ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)])
_lib.register("i2pc_preprocess_plan_destroy", None, [ctypes.c_void_p])
_lib.register("i2pc_preprocess", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_void_p, ctypes.c_void_p])


@dataclass(frozen=True)
class ProcessorSpec:
    """The DPTImageProcessor settings of a checkpoint (recalled hub configs, not in the container)."""
    size: tuple = (384, 384)
    mean: tuple = (0.5, 0.5, 0.5)
    std: tuple = (0.5, 0.5, 0.5)
    keep_aspect_ratio: bool = False
    multiple: int = 1


DPT_LARGE_PROCESSOR = ProcessorSpec()                                  # Intel/dpt-large, Intel/dpt-hybrid-midas
DEPTH_ANYTHING_PROCESSOR = ProcessorSpec(size=(518, 518), mean=(0.485, 0.456, 0.406),
                                         std=(0.229, 0.224, 0.225), keep_aspect_ratio=True, multiple=14)


def output_size(in_h: int, in_w: int, spec: ProcessorSpec):
    """get_resize_output_image_size (transformers image_processing_pil_dpt.py:70-106)."""
    def constrain(val, mult):
        x = round(val / mult) * mult
        if x < 0:
            x = math.ceil(val / mult) * mult
        return x
    oh, ow = spec.size
    sh, sw = oh / in_h, ow / in_w
    if spec.keep_aspect_ratio:
        if abs(1 - sw) < abs(1 - sh):
            sh = sw
        else:
            sw = sh
    return constrain(sh * in_h, spec.multiple), constrain(sw * in_w, spec.multiple)


def patch_pitch(patch: int) -> int:
    """Row pitch of the bf16 patch rows: 3*p*p rounded up to the GEMM K granule (64)."""
    return (3 * patch * patch + 63) // 64 * 64


class Preprocessor:
    def __init__(self, in_h: int, in_w: int, spec: ProcessorSpec = DPT_LARGE_PROCESSOR, patch: int = 0):
        self.in_h, self.in_w = in_h, in_w
        self.out_h, self.out_w = output_size(in_h, in_w, spec)
        self.patch = patch
        self.patch_pitch = patch_pitch(patch)
        lib = _lib.load()
        mean = (ctypes.c_float * 3)(*spec.mean)
        std = (ctypes.c_float * 3)(*spec.std)
        h = ctypes.c_void_p()
        _lib.call("i2pc_preprocess_plan_create", in_h, in_w, self.out_h, self.out_w, mean, std, patch,
                  ctypes.byref(h))
        self._h = h
        self._destroy = lib.i2pc_preprocess_plan_destroy

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._destroy(h)
            self._h = None

    def __call__(self, bgr, layout: str = "nchw", out=None):
        """bgr: torch.uint8 [B, in_h, in_w, 3] on the device."""
        import torch
        if bgr.dim() == 3:
            bgr = bgr.unsqueeze(0)
        B, H, W, C = bgr.shape
        if (H, W, C) != (self.in_h, self.in_w, 3) or bgr.dtype != torch.uint8 or not bgr.is_cuda:
            raise ValueError(f"expected uint8 device tensor [B,{self.in_h},{self.in_w},3], got {tuple(bgr.shape)}")
        bgr = bgr.contiguous()
        if layout == "nchw":
            if out is None:
                out = torch.empty((B, 3, self.out_h, self.out_w), dtype=torch.float32, device=bgr.device)
            code = 0
        elif layout == "patches":
            p = self.patch
            if out is None:
                out = torch.zeros((B * (self.out_h // p) * (self.out_w // p), self.patch_pitch), dtype=torch.bfloat16,
                                  device=bgr.device)
            if out.shape[-1] != self.patch_pitch or not out.is_contiguous():
                raise ValueError(f"patch rows need a contiguous [rows, {self.patch_pitch}] buffer")
            code = 1
        else:
            raise ValueError(layout)
        _lib.call("i2pc_preprocess", self._h, bgr.data_ptr(), B, code, out.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
        return out


_lib.register("i2pc_resize_area", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p])


def reference_downscale_size(h: int, w: int, max_dim: int = 3072):
    """app.py:437-443: (new_w, new_h) when max(h, w) > max_dim, else None."""
    m = max(h, w)
    if m <= max_dim:
        return None
    scale = max_dim / float(m)
    return int(round(w * scale)), int(round(h * scale))


def resize_area(images, out_w: int, out_h: int, out=None):
    """cv2.resize(img, (out_w, out_h), interpolation=cv2.INTER_AREA) for uint8 downscaling on the
    device (i2pc_resize_area).  images: torch.uint8 [H, W, C] or [B, H, W, C] on the device."""
    import torch
    x = images if images.dim() == 4 else images.unsqueeze(0)
    if x.dtype != torch.uint8 or not x.is_cuda:
        raise TypeError("resize_area expects a device uint8 tensor")
    x = x.contiguous()
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty((B, out_h, out_w, C), dtype=torch.uint8, device=x.device)
    _lib.call("i2pc_resize_area", x.data_ptr(), B, H, W, C, out.data_ptr(), out_h, out_w,
              torch.cuda.current_stream().cuda_stream)
    return out if images.dim() == 4 else out[0]

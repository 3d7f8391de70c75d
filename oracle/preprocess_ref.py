"""CPU restatement of the depth network's input pipeline (TEST INFRASTRUCTURE ONLY).

Reference call chain: backend/app.py:103 `cv2.cvtColor(BGR2RGB)` -> PIL image ->
app.py:109 `processor(images=pil_image)` = transformers DPTImageProcessorPil
(transformers 5.15.0, .../dpt/image_processing_pil_dpt.py:192-267):
  1. resize with Pillow (12.2) `Image.resize(size, BICUBIC, reducing_gap=None)`:
     separable, horizontal then vertical, 8-bit fixed point (PRECISION_BITS 22),
     bicubic a = -0.5, support scaled by the downscale factor (antialias),
     uint8 intermediate -- restated from Pillow's published libImaging/Resample.c;
  2. rescale: float32(float64(u8) * (1/255))         (image_transforms.py:89-122);
  3. normalize: (x - mean) / std in float32           (image_transforms.py:384-440).
Output size: get_resize_output_image_size (image_processing_pil_dpt.py:70-106).
Pinned bit-exact against Pillow + DPTImageProcessorPil in tests/test_preprocess.py.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def bicubic_filter(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size: int, out_size: int, support_base: float = 2.0):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc: (xmin[out], count[out], kk int32[out, ksize])."""
    in0, in1 = 0.0, float(in_size)
    scale = filterscale = (in1 - in0) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = support_base * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.float64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)        # C (int) cast truncates toward zero
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        for x in range(xmax):
            w = bicubic_filter((x + xmin - center + 0.5) * ss)
            kk[xx, x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                kk[xx, x] /= ww
        bounds[xx] = (xmin, xmax)
    fixed = np.where(kk < 0, np.trunc(-0.5 + kk * (1 << PRECISION_BITS)),
                     np.trunc(0.5 + kk * (1 << PRECISION_BITS))).astype(np.int64)
    return bounds, fixed


def _clip8(ss):
    v = ss >> PRECISION_BITS
    return np.clip(v, 0, 255).astype(np.uint8)


def pil_resize_bicubic(rgb: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """Image.fromarray(rgb).resize((out_w, out_h), BICUBIC) for uint8 HxWx3."""
    img = np.asarray(rgb, dtype=np.uint8)
    in_h, in_w = img.shape[:2]
    if (in_w, in_h) == (out_w, out_h):
        return img.copy()
    out = img.astype(np.int64)
    if out_w != in_w:
        b, k = precompute_coeffs(in_w, out_w)
        tmp = np.empty((in_h, out_w, 3), dtype=np.int64)
        for xx in range(out_w):
            xmin, cnt = b[xx]
            ss = (1 << (PRECISION_BITS - 1)) + np.einsum("hkc,k->hc", out[:, xmin:xmin + cnt, :], k[xx, :cnt])
            tmp[:, xx, :] = _clip8(ss)
        out = tmp
    if out_h != in_h:
        b, k = precompute_coeffs(in_h, out_h)
        tmp = np.empty((out_h, out.shape[1], 3), dtype=np.int64)
        for yy in range(out_h):
            ymin, cnt = b[yy]
            ss = (1 << (PRECISION_BITS - 1)) + np.einsum("kwc,k->wc", out[ymin:ymin + cnt], k[yy, :cnt])
            tmp[yy] = _clip8(ss)
        out = tmp
    return out.astype(np.uint8)


def output_size(in_h: int, in_w: int, size, keep_aspect_ratio: bool, multiple: int):
    """get_resize_output_image_size (image_processing_pil_dpt.py:70-106)."""
    def constrain(val, mult, min_val=0, max_val=None):
        x = round(val / mult) * mult
        if max_val is not None and x > max_val:
            x = math.floor(val / mult) * mult
        if x < min_val:
            x = math.ceil(val / mult) * mult
        return x
    oh, ow = size
    sh, sw = oh / in_h, ow / in_w
    if keep_aspect_ratio:
        if abs(1 - sw) < abs(1 - sh):
            sh = sw
        else:
            sw = sh
    return constrain(sh * in_h, multiple), constrain(sw * in_w, multiple)


def dpt_preprocess(bgr: np.ndarray, size=(384, 384), mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5),
                   keep_aspect_ratio=False, multiple=1) -> np.ndarray:
    """BGR uint8 HxWx3 -> float32 [3, H', W'] exactly as app.py:103,109 produce pixel_values[0]."""
    rgb = np.ascontiguousarray(bgr[:, :, ::-1])
    oh, ow = output_size(rgb.shape[0], rgb.shape[1], size, keep_aspect_ratio, multiple)
    r = pil_resize_bicubic(rgb, ow, oh)
    x = (r.astype(np.float64) * (1 / 255)).astype(np.float32)
    m = np.array(mean, dtype=np.float32)
    s = np.array(std, dtype=np.float32)
    x = (x - m) / s
    return np.ascontiguousarray(x.transpose(2, 0, 1))

"""CPU restatement of cv2.resize(..., interpolation=cv2.INTER_AREA) for uint8 downscaling.
TEST INFRASTRUCTURE ONLY.

backend/app.py:436-445 downscales inputs above 3072 px with INTER_AREA.  OpenCV is not
installed here, so this restates its published algorithm (imgproc/src/resize.cpp:
computeResizeAreaTab, ResizeArea_Invoker, resizeAreaFast_) -- parity against cv2 itself
is unpinned.  Float32 arithmetic in OpenCV's order; cvRound = round half to even.
"""
from __future__ import annotations

import numpy as np


def _tab(dsize: int, ssize: int, scale: float):
    """Per destination index: list of (source index, float32 weight) in OpenCV's order."""
    out = []
    for d in range(dsize):
        f1 = d * scale
        f2 = f1 + scale
        cw = min(scale, ssize - f1)
        s1, s2 = int(np.ceil(f1)), int(np.floor(f2))
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        e = []
        if s1 - f1 > 1e-3:
            e.append((s1 - 1, np.float32((s1 - f1) / cw)))
        for sx in range(s1, s2):
            e.append((sx, np.float32(1.0 / cw)))
        if f2 - s2 > 1e-3:
            e.append((s2, np.float32(min(min(f2 - s2, 1.0), cw) / cw)))
        out.append(e)
    return out


def resize_area(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    src = img if img.ndim == 3 else img[:, :, None]
    h, w, c = src.shape
    sx = 1.0 / (out_w / w)
    sy = 1.0 / (out_h / h)
    ix, iy = int(round(sx)), int(round(sy))
    eps = np.finfo(np.float64).eps
    if abs(sx - ix) < eps and abs(sy - iy) < eps:
        s = src[: out_h * iy, : out_w * ix].astype(np.int64).reshape(out_h, iy, out_w, ix, c).sum(axis=(1, 3))
        if ix == 2 and iy == 2:
            out = (s + 2) >> 2
        else:
            out = np.rint((s.astype(np.float32) * np.float32(1.0 / (ix * iy))).astype(np.float32))
        res = np.clip(out, 0, 255).astype(np.uint8)
    else:
        xt = _tab(out_w, w, sx)
        yt = _tab(out_h, h, sy)
        nx = max(len(e) for e in xt)
        xi = np.zeros((out_w, nx), np.int64)
        xa = np.zeros((out_w, nx), np.float32)
        for d, e in enumerate(xt):
            for k, (s_, a) in enumerate(e):
                xi[d, k], xa[d, k] = s_, a
        f = src.astype(np.float32)
        res = np.empty((out_h, out_w, c), np.uint8)
        for dy, e in enumerate(yt):
            acc = None
            for j, (sy_, beta) in enumerate(e):
                row = f[sy_]
                buf = np.zeros((out_w, c), np.float32)
                for k in range(nx):
                    term = row[xi[:, k]] * xa[:, k][:, None]
                    live = (xa[:, k] != 0)[:, None]
                    buf = np.where(live, buf + term, buf).astype(np.float32)
                t = (beta * buf).astype(np.float32)
                acc = t if acc is None else (acc + t).astype(np.float32)
            res[dy] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    return res if img.ndim == 3 else res[:, :, 0]


def downscale_like_reference(image: np.ndarray, max_dim: int = 3072):
    """The size rule of app.py:437-443 -> (new_w, new_h), or None when no resize happens."""
    ih, iw = image.shape[:2]
    m = max(ih, iw)
    if m <= max_dim:
        return None
    scale = max_dim / float(m)
    return int(round(iw * scale)), int(round(ih * scale))

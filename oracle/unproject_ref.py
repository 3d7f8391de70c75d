"""CPU restatement of the reference's depth -> point-cloud arithmetic.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the product path never
imports this module.

Every function cites the reference line it restates.  The numeric types follow
what the reference computes under numpy 2.x (the container has numpy 2.2.6,
`backend/requirements.txt:9` pins only `numpy>=1.24.0`):

* `np.percentile(d, [2, 98])` (app.py:197) on a float32 array: q = [2,98] /
  float32(100) -> float64; virtual index v = (n-1)*q (float64); a = s[floor v],
  b = s[floor v + 1] (float32); diff = float32(b - a); result (float64) =
  a + diff*t if t < 0.5 else b - diff*(1-t)
  (numpy/lib/_function_base_impl.py:4257,106-109,4736-4769,4615-4660).
* In the normal branch p2/p98 are np.float64 scalars, so clip/normalize/invert
  (app.py:200-206) run in float64.  In the min/max fallback branch (app.py:199)
  they are Python floats (NEP 50 "weak" scalars) and the same expressions run
  in float32.  In the constant branch d is float32 zeros.
* The per-point loop (app.py:231-244) is Python double arithmetic; the result
  is rounded once to float32 by `np.array(points, dtype=np.float32)` (app.py:246).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

DENSITY_STEP = {"low": 4, "medium": 2, "high": 1}  # app.py:226


# ----------------------------------------------------------------------------
# numpy semantics the reference depends on
# ----------------------------------------------------------------------------

def percentile_2_98(d: np.ndarray) -> tuple[float, float]:
    """np.percentile(d, [2, 98]) for a float32 array, linear method (app.py:197).

    Restated from numpy 2.2 `_quantile` / `_lerp`: the two order statistics at
    floor(v) and floor(v)+1 are interpolated in float64 with the t >= 0.5
    branch of `_lerp`.
    """
    flat = np.asarray(d, dtype=np.float32).ravel()
    n = flat.size
    out = []
    idx = []
    plan = []
    for qpct in (2, 98):
        q = float(qpct) / 100.0               # int / float32(100) promotes to float64
        v = (n - 1) * q                       # linear: get_virtual_index = (n-1)*q
        if v >= n - 1:                        # _get_indexes: above bounds -> last
            i0 = i1 = n - 1
        elif v < 0:
            i0 = i1 = 0
        else:
            i0 = int(math.floor(v))
            i1 = i0 + 1
        t = v - math.floor(v)
        plan.append((i0, i1, t))
        idx += [i0, i1]
    part = np.partition(flat, sorted(set(idx)))
    for i0, i1, t in plan:
        a = np.float32(part[i0])
        b = np.float32(part[i1])
        diff = np.float32(b - a)
        if t >= 0.5:
            r = float(b) - float(diff) * (1.0 - t)
        else:
            r = float(a) + float(diff) * t
        out.append(r)
    return out[0], out[1]


def nanmedian_f32(d: np.ndarray) -> np.float32:
    """np.nanmedian(d) for a float32 array (app.py:195).

    NaNs are dropped (infinities are kept); the median of m values is the
    float32 mean of the middle one/two order statistics: f32(f32(a+b)/2).
    An all-NaN array returns its last element (NaN).
    """
    flat = np.asarray(d, dtype=np.float32).ravel()
    keep = flat[~np.isnan(flat)]
    m = keep.size
    if m == 0:
        return np.float32(flat[-1])
    h = m // 2
    if m % 2:
        return np.float32(np.partition(keep, h)[h])
    part = np.partition(keep, [h - 1, h])
    s = np.float32(np.float32(part[h - 1]) + np.float32(part[h]))
    return np.float32(s / np.float32(2))


def resize_linear_cv2(depth: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """cv2.resize(depth, (W, H), interpolation=cv2.INTER_LINEAR) on float32 (app.py:188).

    Restated from OpenCV's resize.cpp geometry (half-pixel centres, coordinates
    computed in double then cast to float, clamp to the first/last sample,
    horizontal pass then vertical pass, separate multiply and add in float32).
    PARITY UNPINNED against cv2 itself (OpenCV is not installed here); pinned
    against torch bilinear align_corners=False within fp32 rounding.
    """
    src = np.asarray(depth, dtype=np.float32)
    in_h, in_w = src.shape
    if (in_h, in_w) == (out_h, out_w):
        return src.copy()
    x0, x1, ax0, ax1 = _linear_taps(in_w, out_w)
    y0, y1, by0, by1 = _linear_taps(in_h, out_h)
    right = x0 >= in_w - 1          # HResizeLinear: dx >= xmax copies S[sx] (one tap)
    with np.errstate(invalid="ignore", over="ignore"):
        hor = src[:, x0] * ax0[None, :] + src[:, x1] * ax1[None, :]          # float32
        hor[:, right] = src[:, x0[right]]
        out = hor[y0, :] * by0[:, None] + hor[y1, :] * by1[:, None]          # float32, both taps
    return out.astype(np.float32)


def _linear_taps(in_size: int, out_size: int):
    scale = 1.0 / (out_size / in_size)                 # scale_x = 1./inv_scale_x (double)
    dx = np.arange(out_size, dtype=np.float64)
    fx = ((dx + 0.5) * scale - 0.5).astype(np.float32)  # (float)((dx+0.5)*scale_x - 0.5)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    low = sx < 0
    fx[low] = 0.0
    sx[low] = 0
    high = sx >= in_size - 1
    fx[high] = 0.0
    sx[high] = in_size - 1
    s1 = np.minimum(sx + 1, in_size - 1)
    a0 = (np.float32(1.0) - fx).astype(np.float32)
    return sx, s1, a0, fx


def gaussian_kernel(k: int) -> np.ndarray:
    """cv2.getGaussianKernel(k, 0) (OpenCV's getGaussianKernelBitExact, restated from the published
    source): the fixed small-kernel tables for k <= 7, else sigma = 0.15 k + 0.35 (the documented
    0.3 ((k - 1) 0.5 - 1) + 0.8), taps exp(-x^2 / (2 sigma^2)) normalised to sum 1 via one reciprocal.
    PARITY UNPINNED (no OpenCV here; OpenCV evaluates exp in soft-float, libm here)."""
    small = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
             7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}
    if k in small:
        return np.array(small[k], dtype=np.float64)
    sigma = 0.15 * k + 0.35
    scale2x = -0.125 / (sigma * sigma)
    h = (k - 1) // 2
    v = [math.exp(float(x * x) * scale2x) for x in range(1 - k, 0, 2)]
    s = 0.0
    for t in v:
        s += t
    mul = 1.0 / (s * 2.0 + 1.0)
    half = [t * mul for t in v]
    return np.array(half + [mul] + half[::-1], dtype=np.float64)


def _reflect101(i: np.ndarray, n: int) -> np.ndarray:
    """cv2 borderInterpolate(BORDER_REFLECT_101), repeated for kernels wider than the axis."""
    if n == 1:
        return np.zeros_like(i)
    i = i.copy()
    while True:
        bad = (i < 0) | (i >= n)
        if not bad.any():
            return i
        i = np.where(i < 0, -i, np.where(i >= n, 2 * (n - 1) - i, i))


def gaussian_blur(d: np.ndarray, k: int) -> np.ndarray:
    """cv2.GaussianBlur(d, (k, k), 0) as called at app.py:212: separable, rows then columns,
    BORDER_REFLECT_101, taps in the array's dtype, accumulated in tap order.
    PARITY UNPINNED (no OpenCV here): summation order follows the tap order."""
    a = np.asarray(d)
    kt = gaussian_kernel(k).astype(a.dtype)
    h, w = a.shape
    r = k // 2
    cols = np.arange(w)
    tmp = np.zeros_like(a)
    for t in range(k):
        tmp = tmp + a[:, _reflect101(cols + t - r, w)] * kt[t]
    rows = np.arange(h)
    out = np.zeros_like(a)
    for t in range(k):
        out = out + tmp[_reflect101(rows + t - r, h), :] * kt[t]
    return out


def gaussian_blur_5(d: np.ndarray) -> np.ndarray:
    """The default call (smooth_ksize 5 -> k = 5): OpenCV's fixed [1,4,6,4,1]/16 kernel."""
    return gaussian_blur(d, 5)


# ----------------------------------------------------------------------------
# depth_to_point_cloud (app.py:174-250)
# ----------------------------------------------------------------------------

def normalize_depth(depth_full: np.ndarray, invert: bool):
    """app.py:191-206: sanitize, percentile clip/normalize, invert.

    Returns (d, stats) where d is float64 (normal branch) or float32 (fallback
    branches) and stats = dict(p2, p98, branch, median).
    """
    d = np.asarray(depth_full).astype(np.float32)                      # :191
    med = None
    finite_mask = np.isfinite(d)                                        # :193
    if not np.all(finite_mask):
        med = nanmedian_f32(d)                                          # :195
        d = np.where(finite_mask, d, med).astype(np.float32)           # :196
    p2, p98 = percentile_2_98(d)                                        # :197
    branch = 0
    if p98 <= p2:                                                       # :198
        p2, p98 = float(d.min()), float(d.max())                        # :199 python floats
        branch = 1
    if p98 > p2:                                                        # :200
        if branch == 0:
            dd = np.clip(d.astype(np.float64), p2, p98)                 # :201 float64
            dd = (dd - p2) / (p98 - p2 + 1e-6)                          # :202 float64
        else:
            lo, hi = np.float32(p2), np.float32(p98)                    # weak python floats -> f32
            dd = np.clip(d, lo, hi).astype(np.float32)
            den = np.float32(p98 - p2 + 1e-6)
            dd = ((dd - lo).astype(np.float32) / den).astype(np.float32)
    else:
        dd = np.zeros_like(d)                                           # :204 float32
        branch = 2
    if invert:
        dd = 1.0 - dd                                                   # :206 keeps dtype
        dd = dd.astype(dd.dtype)
    return dd, {"p2": p2, "p98": p98, "branch": branch, "median": med}


def depth_preview_u8(depth: np.ndarray, invert: bool = True) -> np.ndarray:
    """create_depth_preview (app.py:124-150) up to the colour map: the uint8 image
    (d * 255.0).astype(np.uint8) of the model-resolution depth normalised exactly
    as app.py:191-206 does (the two blocks are the same code)."""
    d, _ = normalize_depth(depth, invert)
    return (d * 255.0).astype(np.uint8)                                   # :146


def intrinsics(w: int, h: int, fov: Optional[float]):
    """app.py:219-223.  (The REST route drops `fov`, so the reference always takes
    the 1.2*max(w,h) branch -- SURVEY D5.)"""
    cx, cy = w / 2.0, h / 2.0
    if fov and fov > 0:
        f = (w / 2.0) / np.tan(np.deg2rad(fov) / 2.0)
    else:
        f = max(w, h) * 1.2
    return cx, cy, float(f)


def depth_to_point_cloud(image: np.ndarray, depth: np.ndarray, density: str = "medium",
                         invert: bool = True, depth_scale: float = 10.0,
                         smooth: bool = False, smooth_ksize: int = 5,
                         fov: Optional[float] = None, loop: bool = True):
    """Restatement of depth_to_point_cloud (app.py:174-250).

    loop=True runs the reference's per-point Python loop (app.py:231-244), the
    faithful single-threaded CPU baseline.  loop=False evaluates the same IEEE
    double expressions vectorized (bit-identical: numpy does not contract
    a*b+c into an FMA).
    """
    img_h, img_w = image.shape[:2]
    if depth.shape[:2] != (img_h, img_w):
        depth = resize_linear_cv2(depth, img_w, img_h)                  # :187-188
    d, _ = normalize_depth(depth, invert)
    if smooth:                                                          # :209-214
        k = max(3, int(smooth_ksize) // 2 * 2 + 1)                      # :211
        d = gaussian_blur(d, k)                                         # :212
    h, w = img_h, img_w
    cx, cy, f = intrinsics(w, h, fov)
    step = DENSITY_STEP[density]
    color_ok = image.ndim == 3 and image.shape[2] >= 3
    if loop:
        points, colors = [], []
        for v in range(0, h, step):                                     # :231
            for u in range(0, w, step):                                 # :232
                z = float(d[v, u]) * float(depth_scale)                 # :233
                x = (u - cx) * (z if z != 0.0 else 1e-6) / f            # :234
                y = (v - cy) * (z if z != 0.0 else 1e-6) / f            # :235
                points.append([x, y, z])
                if color_ok:                                            # :240-244
                    b, g, r = image[v, u][:3]
                    colors.append([int(r), int(g), int(b)])
                else:
                    colors.append([128, 128, 128])
        return np.array(points, dtype=np.float32), np.array(colors, dtype=np.float32)
    vs = np.arange(0, h, step)
    us = np.arange(0, w, step)
    dv = d[np.ix_(vs, us)].astype(np.float64)
    z = dv * float(depth_scale)
    zz = np.where(z != 0.0, z, 1e-6)
    x = ((us[None, :].astype(np.float64) - cx) * zz) / f
    y = ((vs[:, None].astype(np.float64) - cy) * zz) / f
    pts = np.stack([x.ravel(), y.ravel(), z.ravel()], axis=1).astype(np.float32)
    if color_ok:
        px = image[np.ix_(vs, us)][..., :3].reshape(-1, 3)
        cols = px[:, ::-1].astype(np.float32)
    else:
        cols = np.full((pts.shape[0], 3), 128, dtype=np.float32)
    return pts, cols


def depth_to_point_cloud_equirect(image: np.ndarray, depth: np.ndarray, density: str = "medium",
                                  invert: bool = True, depth_scale: float = 10.0):
    """Equirectangular variant (C4 panoramas; NOT in the reference -- parity unpinned beyond
    this restatement).  Resize / normalisation exactly as depth_to_point_cloud (app.py:186-206);
    the normalised depth times depth_scale is the range r along the ray of longitude
    lon = (u + 0.5) 2pi / W - pi and latitude lat = pi/2 - (v + 0.5) pi / H:
    x = (r cos lat) sin lon, y = -(r sin lat), z = (r cos lat) cos lon (float64, then float32),
    the operation order i2pc_unproject evaluates with projection = 1."""
    img_h, img_w = image.shape[:2]
    if depth.shape[:2] != (img_h, img_w):
        depth = resize_linear_cv2(depth, img_w, img_h)
    d, _ = normalize_depth(depth, invert)
    step = DENSITY_STEP[density]
    vs = np.arange(0, img_h, step)
    us = np.arange(0, img_w, step)
    lon = (us.astype(np.float64) + 0.5) * (2.0 * np.pi / img_w) - np.pi
    lat = np.pi / 2.0 - (vs.astype(np.float64) + 0.5) * (np.pi / img_h)
    r = d[np.ix_(vs, us)].astype(np.float64) * float(depth_scale)
    rh = r * np.cos(lat)[:, None]
    x = rh * np.sin(lon)[None, :]
    y = -(r * np.sin(lat)[:, None])
    z = rh * np.cos(lon)[None, :]
    pts = np.stack([x.ravel(), y.ravel(), z.ravel()], axis=1).astype(np.float32)
    if image.ndim == 3 and image.shape[2] >= 3:
        cols = image[np.ix_(vs, us)][..., :3].reshape(-1, 3)[:, ::-1].astype(np.float32)
    else:
        cols = np.full((pts.shape[0], 3), 128, dtype=np.float32)
    return pts, cols


def gis_bounds(points: np.ndarray) -> dict:
    """generate_gis_metadata bounds (app.py:393-400)."""
    return {
        "minX": float(points[:, 0].min()), "maxX": float(points[:, 0].max()),
        "minY": float(points[:, 1].min()), "maxY": float(points[:, 1].max()),
        "minZ": float(points[:, 2].min()), "maxZ": float(points[:, 2].max()),
    }


def preview(points: np.ndarray, colors: Optional[np.ndarray], max_preview: int = 20000):
    """Preview subsample (app.py:496-506)."""
    if len(points) > max_preview:
        stride = max(1, len(points) // max_preview)
        pprev = points[::stride]
        cprev = colors[::stride] if colors is not None and len(colors) else np.zeros_like(pprev)
    else:
        pprev = points
        cprev = colors if colors is not None and len(colors) else np.zeros_like(points)
    return pprev.astype(float).tolist(), cprev.astype(float).tolist()


def point_count(h: int, w: int, density: str) -> int:
    s = DENSITY_STEP[density]
    return ((h + s - 1) // s) * ((w + s - 1) // s)

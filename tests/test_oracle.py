"""Pin the CPU oracle against the reference's own outputs (golden fixtures)."""
import hashlib

import numpy as np
import pytest

from oracle import unproject_ref as ref


def _bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


@pytest.mark.parametrize("loop", [True, False])
def test_oracle_matches_reference_fixtures(unproject_cases, loop):
    for c in unproject_cases:
        pts, cols = ref.depth_to_point_cloud(c["image"], c["depth"], density=c["density"],
                                             invert=c["invert"], depth_scale=c["scale"], loop=loop)
        assert _bits_equal(pts, c["points"]), c["name"]
        assert _bits_equal(cols, c["colors"]), c["name"]
        b = ref.gis_bounds(pts)
        got = np.array([b[k] for k in ("minX", "maxX", "minY", "maxY", "minZ", "maxZ")])
        assert _bits_equal(got, c["bounds"]), c["name"]
        assert len(pts) == ref.point_count(c["h"], c["w"], c["density"])


def test_percentile_restatement_matches_numpy():
    rng = np.random.Generator(np.random.PCG64(11))
    for n in (1, 2, 3, 50, 147_456, 268_324):
        d = rng.normal(size=n).astype(np.float32)
        if n > 100:
            d[:n // 10] = d[0]          # ties
        p2, p98 = ref.percentile_2_98(d)
        e2, e98 = np.percentile(d, [2, 98])
        assert (p2, p98) == (float(e2), float(e98)), n


def test_nanmedian_restatement_matches_numpy():
    rng = np.random.Generator(np.random.PCG64(12))
    for n in (1, 2, 7, 8, 1001):
        d = rng.normal(size=n).astype(np.float32)
        d[rng.choice(n, max(0, n // 5), replace=False)] = np.nan
        if n > 5:
            d[0] = np.inf
        got = ref.nanmedian_f32(d)
        exp = np.nanmedian(d)
        assert np.float32(exp).tobytes() == np.float32(got).tobytes(), n


def test_pipeline_preview_and_bounds(pipeline_case):
    s = pipeline_case["summary"]
    pts, cols = ref.depth_to_point_cloud(pipeline_case["image"], pipeline_case["depth"],
                                         density=s["gisData"]["pointDensity"], loop=False)
    assert len(pts) == s["pointCloud"]["points"]
    assert ref.gis_bounds(pts) == s["gisData"]["bounds"]
    pp, pc = ref.preview(pts, cols)
    assert len(pp) == s["preview_len"]
    assert hashlib.sha256(np.asarray(pp, np.float64).tobytes()).hexdigest() == s["preview_points_sha256"]
    assert hashlib.sha256(np.asarray(pc, np.float64).tobytes()).hexdigest() == s["preview_colors_sha256"]


def test_resize_linear_matches_torch_bilinear():
    torch = pytest.importorskip("torch")
    rng = np.random.Generator(np.random.PCG64(13))
    for (h, w, H, W) in ((384, 384, 1024, 1024), (37, 53, 100, 90), (518, 686, 768, 1024)):
        d = rng.random((h, w), dtype=np.float32)
        got = ref.resize_linear_cv2(d, W, H)
        t = torch.nn.functional.interpolate(torch.from_numpy(d)[None, None], size=(H, W),
                                            mode="bilinear", align_corners=False)[0, 0].numpy()
        assert np.max(np.abs(got - t)) < 2e-4   # torch rounds the source coordinate in fp32, cv2 in fp64


def test_depth_preview_u8_matches_reference_fixtures():
    """The uint8 image create_depth_preview (app.py:124-150) hands to cv2.applyColorMap,
    recorded from the reference itself (tests/golden/gen_golden.py, section 9)."""
    import json
    import os
    import numpy as np
    from oracle import unproject_ref as ref
    here = os.path.join(os.path.dirname(__file__), "golden")
    meta = json.load(open(os.path.join(here, "preview_cases.json")))
    z = np.load(os.path.join(here, "preview_cases.npz"))
    assert len(meta) == 10
    for m in meta:
        got = ref.depth_preview_u8(z[m["name"] + "__depth"], m["invert"])
        exp = z[m["name"] + "__u8"]
        assert got.dtype == exp.dtype and np.array_equal(got, exp), m["name"]


def test_gaussian_kernel_tables_and_sampled():
    """oracle.gaussian_kernel: OpenCV's fixed tables for k <= 7, and the sampled kernels sum to 1,
    are symmetric and peak in the middle (cv2 absent: parity unpinned beyond these properties)."""
    from oracle import unproject_ref as r
    assert np.array_equal(r.gaussian_kernel(5), np.array([1, 4, 6, 4, 1]) / 16.0)
    assert np.array_equal(r.gaussian_kernel(3), np.array([0.25, 0.5, 0.25]))
    for k in (9, 11, 15, 31):
        t = r.gaussian_kernel(k)
        assert len(t) == k and abs(t.sum() - 1.0) < 1e-12
        assert np.array_equal(t, t[::-1]) and t.argmax() == k // 2
    # sigma 0.15 k + 0.35 (OpenCV's documented 0.3 ((k - 1) 0.5 - 1) + 0.8)
    t = r.gaussian_kernel(9)
    s = 0.15 * 9 + 0.35
    x = np.arange(9) - 4
    g = np.exp(-x * x / (2 * s * s))
    assert np.allclose(t, g / g.sum(), rtol=1e-14, atol=0)


def test_blur_matches_direct_convolution():
    from oracle import unproject_ref as r
    rng = np.random.default_rng(2)
    d = rng.random((13, 17))
    for k in (3, 9):
        got = r.gaussian_blur(d, k)
        kt = r.gaussian_kernel(k)
        # dense reference: reflect-101 padded separable convolution
        p = np.pad(d, k // 2, mode="reflect")
        tmp = sum(p[:, t:t + 17] * kt[t] for t in range(k))
        exp = sum(tmp[t:t + 13, :] * kt[t] for t in range(k))
        assert np.allclose(got, exp, rtol=1e-13, atol=1e-15)

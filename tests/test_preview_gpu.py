"""GPU depth preview (create_depth_preview, app.py:124-172).

Bar: the uint8 image before the colour table is bit-exact with the one the
reference hands to cv2.applyColorMap (tests/golden/preview_cases.npz, recorded
from the reference); the colour lookup is checked against the table on the host.
"""
import json
import os

import numpy as np
import pytest

from oracle import unproject_ref as ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(__file__), "golden")
IDENTITY = bytes(np.repeat(np.arange(256, dtype=np.uint8), 3))


def test_preview_u8_bit_exact_vs_reference():
    from image_to_pointcloud_amd import preview
    meta = json.load(open(os.path.join(HERE, "preview_cases.json")))
    z = np.load(os.path.join(HERE, "preview_cases.npz"))
    for m in meta:
        d = torch.from_numpy(z[m["name"] + "__depth"]).cuda()
        got = preview.depth_preview_batch(d, m["invert"], table=IDENTITY)[0, ..., 0].cpu().numpy()
        assert np.array_equal(got, z[m["name"] + "__u8"]), m["name"]


def test_preview_batched_and_colour_table():
    from image_to_pointcloud_amd import preview
    rng = np.random.Generator(np.random.PCG64(3))
    d = rng.random((3, 518, 686), dtype=np.float32) * 4.0
    d[1] = 2.0                                   # constant map in the middle of the batch
    d[2, 10, 10] = np.nan
    out = preview.depth_preview_batch(torch.from_numpy(d).cuda(), True).cpu().numpy()
    lut = np.frombuffer(preview.PLASMA_BGR, np.uint8).reshape(256, 3)
    for i in range(3):
        assert np.array_equal(out[i], lut[ref.depth_preview_u8(d[i], True)]), i


def test_create_depth_preview_data_url():
    import base64, io
    from PIL import Image
    from image_to_pointcloud_amd import preview
    d = np.linspace(0, 1, 64 * 48, dtype=np.float32).reshape(48, 64)
    url = preview.create_depth_preview(d, invert=True)
    assert url.startswith("data:image/png;base64,")
    img = np.array(Image.open(io.BytesIO(base64.b64decode(url.split(",", 1)[1]))))
    lut = np.frombuffer(preview.PLASMA_BGR, np.uint8).reshape(256, 3)
    assert np.array_equal(img[:, :, ::-1], lut[ref.depth_preview_u8(d, True)])


def test_preview_above_2048_is_area_downscaled():
    """Depth maps wider than DEPTH_PREVIEW_MAX: the colour-mapped preview is INTER_AREA-resized to
    (round(dw * s), round(dh * s)), s = 2048 / max(dh, dw) (app.py:155-160); checked against the
    colour table + the INTER_AREA restatement (oracle/area_ref.py, cv2 itself unpinned)."""
    from oracle import area_ref
    from image_to_pointcloud_amd import preview
    rng = np.random.Generator(np.random.PCG64(5))
    h, w = 1036, 2600
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    d = (2.0 + np.sin(u / 50.0) * np.cos(v / 30.0) + rng.normal(0, 0.05, (h, w))).astype(np.float32)
    oh, ow = preview.preview_size(h, w)
    assert (oh, ow) == (int(round(h * 2048 / w)), 2048)
    got = preview.colored_preview(torch.from_numpy(d).cuda(), True).cpu().numpy()
    lut = np.frombuffer(preview.PLASMA_BGR, np.uint8).reshape(256, 3)
    exp = area_ref.resize_area(lut[ref.depth_preview_u8(d, True)], ow, oh)
    assert got.shape == (oh, ow, 3) and np.array_equal(got, exp)
    assert preview.create_depth_preview(d, invert=True).startswith("data:image/png;base64,")

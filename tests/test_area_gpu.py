"""GPU INTER_AREA downscale (i2pc_resize_area, the >3072 px path of app.py:436-445) against
the CPU restatement oracle/area_ref.py, bit-exact.  OpenCV is absent, so parity with
cv2 itself is unpinned; the integer-scale case is also checked against a plain box mean."""
import numpy as np
import pytest

from oracle import area_ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _img(h, w, c, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, (h, w, c), dtype=np.uint8)


@pytest.mark.parametrize("h,w,c,oh,ow", [(700, 523, 3, 525, 392), (4096, 3000, 3, 3072, 2250), (333, 517, 1, 100, 77),
                                         (600, 800, 3, 300, 400), (900, 600, 3, 300, 200), (64, 64, 4, 63, 64),
                                         (10, 10, 3, 1, 1)])
def test_resize_area_matches_oracle(h, w, c, oh, ow):
    from image_to_pointcloud_amd import preprocess
    img = _img(h, w, c, h + w)
    got = preprocess.resize_area(torch.from_numpy(img).cuda(), ow, oh).cpu().numpy()
    exp = area_ref.resize_area(img, ow, oh)
    assert got.shape == exp.shape and np.array_equal(got, exp), np.argwhere(got != exp)[:5]
    if h % oh == 0 and w % ow == 0 and (h // oh, w // ow) != (2, 2):
        box = img.reshape(oh, h // oh, ow, w // ow, c).mean(axis=(1, 3))
        assert np.abs(got.astype(np.float64) - box).max() <= 0.5 + 1e-9


def test_reference_size_rule():
    from image_to_pointcloud_amd import preprocess
    assert preprocess.reference_downscale_size(3072, 100) is None
    assert preprocess.reference_downscale_size(4096, 3000) == (2250, 3072)
    assert preprocess.reference_downscale_size(4000, 8001) == area_ref.downscale_like_reference(np.zeros((4000, 8001)))
    with pytest.raises(Exception):
        preprocess.resize_area(torch.zeros((4, 4, 3), dtype=torch.uint8, device="cuda"), 8, 8)

"""CPU checks of the INTER_AREA restatement (oracle/area_ref.py; cv2 absent: parity unpinned)."""
import numpy as np

from oracle import area_ref


def test_cell_weights_partition_each_output_pixel():
    for ssize, dsize in ((4096, 3072), (523, 392), (7, 3), (1000, 999)):
        scale = 1.0 / (dsize / ssize)
        for e in area_ref._tab(dsize, ssize, scale):
            assert abs(sum(float(a) for _, a in e) - 1.0) < 1e-5
            idx = [s for s, _ in e]
            assert idx == list(range(idx[0], idx[0] + len(idx))) and 0 <= idx[0] and idx[-1] < ssize


def test_constant_image_stays_constant_and_box_mean():
    img = np.full((90, 120, 3), 77, np.uint8)
    assert (area_ref.resize_area(img, 50, 40) == 77).all()
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (60, 90, 3), dtype=np.uint8)
    got = area_ref.resize_area(img, 30, 20)          # 3 x 3 boxes
    box = img.reshape(20, 3, 30, 3, 3).mean(axis=(1, 3))
    assert np.abs(got - box).max() <= 0.5 + 1e-9
    got2 = area_ref.resize_area(img, 45, 30)         # 2 x 2: (sum + 2) >> 2
    s = img.astype(np.int64).reshape(30, 2, 45, 2, 3).sum(axis=(1, 3))
    assert np.array_equal(got2, ((s + 2) >> 2).astype(np.uint8))


def test_reference_size_rule():
    assert area_ref.downscale_like_reference(np.zeros((3072, 10))) is None
    assert area_ref.downscale_like_reference(np.zeros((4096, 3000))) == (2250, 3072)

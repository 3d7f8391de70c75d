"""Preprocessing (app.py:103,109): oracle vs Pillow/transformers (CPU) and HIP kernel vs both (GPU)."""
import numpy as np
import pytest

from oracle import preprocess_ref as pre

PIL = pytest.importorskip("PIL.Image")

SHAPES = [(64, 80, 48, 40), (37, 53, 24, 24), (100, 60, 100, 60), (30, 30, 61, 45)]


def _img(h, w, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("h,w,oh,ow", SHAPES)
def test_pil_bicubic_restatement_bit_exact(h, w, oh, ow):
    img = _img(h, w, h * w)
    got = pre.pil_resize_bicubic(img, ow, oh)
    exp = np.asarray(PIL.fromarray(img).resize((ow, oh), resample=PIL.BICUBIC, reducing_gap=None))
    assert np.array_equal(got, exp)


def test_dpt_processor_restatement_bit_exact():
    tr = pytest.importorskip("transformers")
    from transformers.models.dpt.image_processing_pil_dpt import DPTImageProcessorPil
    proc = DPTImageProcessorPil()          # DPT-Large defaults: 384x384, mean = std = 0.5
    for (h, w) in ((96, 120), (384, 384), (200, 150)):
        bgr = _img(h, w, 7 + h)
        exp = proc(images=PIL.fromarray(bgr[:, :, ::-1].copy()), return_tensors="np")["pixel_values"][0]
        got = pre.dpt_preprocess(bgr)
        assert got.dtype == np.float32 and np.array_equal(got, exp)
    # Depth-Anything-V2 processor settings (hub config recalled: 518, keep aspect, multiple of 14, ImageNet)
    proc = DPTImageProcessorPil(size={"height": 518, "width": 518}, keep_aspect_ratio=True, ensure_multiple_of=14,
                                image_mean=[0.485, 0.456, 0.406], image_std=[0.229, 0.224, 0.225])
    bgr = _img(120, 160, 3)
    exp = proc(images=PIL.fromarray(bgr[:, :, ::-1].copy()), return_tensors="np")["pixel_values"][0]
    got = pre.dpt_preprocess(bgr, size=(518, 518), mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                             keep_aspect_ratio=True, multiple=14)
    assert np.array_equal(got, exp)

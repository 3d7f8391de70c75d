"""GPU preprocessing (k_preprocess: Pillow bicubic + rescale + normalise) bit-exact with the
CPU restatement (itself pinned to Pillow / DPTImageProcessorPil, tests/test_preprocess.py) at
the bench's size, the Depth-Anything keep-aspect size, wide keep-aspect panoramas and inputs wider
than one LDS row stage."""
import numpy as np
import pytest

from oracle import preprocess_ref as pre

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h,w,size,keep", [(1024, 1024, (384, 384), False), (768, 1024, (518, 518), True),
                                           (301, 997, (384, 384), False), (2048, 1024, (518, 518), True),
                                           (300, 4000, (384, 384), False),
                                           # wide keep-aspect outputs (phone panoramas after the REST 3072-px
                                           # downscale) split into column tiles: 518x2296 and 518x2652
                                           (691, 3072, (518, 518), True), (600, 3072, (518, 518), True),
                                           # input rows at and beyond one LDS stage (8192 px = 24 KB)
                                           (40, 8192, (384, 384), False), (36, 9000, (384, 384), False)])
def test_preprocess_bit_exact(h, w, size, keep):
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec, output_size
    spec = ProcessorSpec(size=size, keep_aspect_ratio=keep, multiple=14 if keep else 1)
    rng = np.random.Generator(np.random.PCG64(h * w))
    imgs = rng.integers(0, 256, (2, h, w, 3), dtype=np.uint8)
    oh, ow = output_size(h, w, spec)
    patch = 14 if keep else 16
    prep = Preprocessor(h, w, spec, patch=patch if (oh % patch == 0 and ow % patch == 0) else 0)
    t = torch.from_numpy(imgs).cuda()
    pix = prep(t, layout="nchw").cpu().numpy()
    exp = np.stack([pre.dpt_preprocess(im, size=spec.size, keep_aspect_ratio=keep, multiple=spec.multiple)
                    for im in imgs])
    assert pix.shape == exp.shape and np.array_equal(pix, exp)

"""Depth network parity: the bf16 HIP DPT against transformers' fp32 DPTForDepthEstimation.

Same seeded weights (transformers key layout), same preprocessed input.
Tolerance (bf16 operands / fp32 accumulation vs an fp32 network):
relative L2 error of the predicted depth <= 2e-2 and max |err| <= 6e-2 * max |ref|.
The preprocessing itself is checked bit-exact against DPTImageProcessorPil.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
transformers = pytest.importorskip("transformers")
pytestmark = pytest.mark.gpu


def _hf_model(spec, sd, dev):
    from transformers import DPTConfig, DPTForDepthEstimation
    cfg = DPTConfig(**spec.hf_config_kwargs())
    m = DPTForDepthEstimation(cfg)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert not [k for k in missing if "pooler" not in k], missing
    return m.to(dev).eval()


def _images(B, h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    # smooth-ish content so the depth map is not white noise
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    out = []
    for i in range(B):
        base = 127 + 100 * np.sin(u / (9.0 + i)) * np.cos(v / (13.0 + i))
        img = np.clip(base[..., None] + rng.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8)
        out.append(img)
    return np.stack(out)


def test_state_dict_layout_matches_transformers():
    from transformers import DPTConfig, DPTForDepthEstimation
    from image_to_pointcloud_amd.dpt import DPT_TINY, state_dict_keys
    m = DPTForDepthEstimation(DPTConfig(**DPT_TINY.hf_config_kwargs()))
    hf = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ours = state_dict_keys(DPT_TINY)
    assert ours == hf


@pytest.mark.parametrize("which,B,hw", [("tiny", 3, (128, 128)), ("tiny", 2, (200, 150)), ("large", 2, (384, 384)),
                                        ("large", 2, (1024, 1024))])
def test_dpt_forward_matches_transformers_fp32(which, B, hw):
    from image_to_pointcloud_amd.dpt import DPT_LARGE, DPT_TINY, DPTDepthModel, synthetic_state_dict
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    from oracle import preprocess_ref as pre
    spec = DPT_LARGE if which == "large" else DPT_TINY
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, seed=0)
    ours = DPTDepthModel(spec, sd, dev)
    ref = _hf_model(spec, sd, dev)
    pspec = ProcessorSpec(size=(spec.image, spec.image))
    imgs = _images(B, hw[0], hw[1], 7)
    prep = Preprocessor(hw[0], hw[1], pspec, patch=spec.patch)
    timgs = torch.from_numpy(imgs).to(dev)
    pix = prep(timgs, layout="nchw")
    exp_pix = np.stack([pre.dpt_preprocess(im, size=pspec.size) for im in imgs])
    assert np.array_equal(pix.cpu().numpy(), exp_pix), "preprocess not bit-exact"
    patches = prep(timgs, layout="patches")
    depth = ours(patches, B)
    torch.cuda.synchronize()
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
    assert depth.shape == exp.shape
    err = (depth - exp)
    rel = (err.norm() / exp.norm()).item()
    mx = (err.abs().max() / exp.abs().max()).item()
    assert exp.abs().max() > 0 and exp.std() > 1e-3 * exp.abs().max(), "degenerate reference depth"
    assert rel <= 2e-2 and mx <= 6e-2, f"rel L2 {rel:.3e} max {mx:.3e}"

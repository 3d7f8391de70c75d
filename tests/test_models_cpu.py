"""CPU checks of the network definitions: the state-dict layouts match transformers'
own model classes key-for-key, and the algorithmic FLOP counts match SURVEY §8d."""
import pytest

torch = pytest.importorskip("torch")
transformers = pytest.importorskip("transformers")


@pytest.mark.parametrize("which", ["tiny", "small"])
def test_depth_anything_state_dict_layout(which):
    from transformers import DepthAnythingConfig, DepthAnythingForDepthEstimation
    from image_to_pointcloud_amd.depth_anything import DA_TINY, DA_V2_SMALL, state_dict_keys
    spec = DA_V2_SMALL if which == "small" else DA_TINY
    m = DepthAnythingForDepthEstimation(DepthAnythingConfig(**spec.hf_config_kwargs()))
    hf = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert state_dict_keys(spec) == hf


def test_dpt_state_dict_layout():
    from transformers import DPTConfig, DPTForDepthEstimation
    from image_to_pointcloud_amd.dpt import DPT_TINY, state_dict_keys
    m = DPTForDepthEstimation(DPTConfig(**DPT_TINY.hf_config_kwargs()))
    assert state_dict_keys(DPT_TINY) == {k: tuple(v.shape) for k, v in m.state_dict().items()}


def test_flop_counts_match_survey():
    from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
    from image_to_pointcloud_amd.dpt import DPT_LARGE
    # DA-small @518 ~ 80.7 + 34.6 = 115 GFLOP; DPT-Large @384 ~ 483.7 + 32.7 = 516 GFLOP
    assert abs(DA_V2_SMALL.flops_per_image() / 1e9 - 115.3) < 0.03 * 115.3
    assert abs(DPT_LARGE.flops_per_image() / 1e9 - 516.4) < 0.03 * 516.4


def test_depth_anything_sizes():
    from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
    assert DA_V2_SMALL.sizes(37, 37) == [(148, 148), (74, 74), (37, 37), (19, 19)]
    assert DA_V2_SMALL.sizes(37, 49) == [(148, 196), (74, 98), (37, 49), (19, 25)]


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_dpt_hybrid_state_dict_layout(which):
    """Every tensor of DPTForDepthEstimation(is_hybrid=True) (BiT-R50 stem + ViT-B/16), same names and shapes."""
    from transformers import DPTConfig, DPTForDepthEstimation
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID, DPT_HYBRID_TINY, state_dict_keys
    spec = DPT_HYBRID if which == "full" else DPT_HYBRID_TINY
    m = DPTForDepthEstimation(DPTConfig(**spec.hf_config_kwargs()))
    assert {k: tuple(v.shape) for k, v in m.state_dict().items()} == state_dict_keys(spec)


def test_dpt_hybrid_flops_match_flop_counter():
    """HybridSpec.flops_per_image (conv + linear part) against torch's FlopCounter on the
    transformers model (attention is added analytically, as for DPT-Large)."""
    import torch
    from torch.utils.flop_counter import FlopCounterMode
    from transformers import DPTConfig, DPTForDepthEstimation
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID_TINY as spec
    m = DPTForDepthEstimation(DPTConfig(**spec.hf_config_kwargs())).eval()
    x = torch.zeros(1, 3, spec.image, spec.image)
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        m(pixel_values=x)
    T = spec.grid ** 2 + 1
    attn = spec.layers * 4.0 * T * T * spec.hidden
    counted = fc.get_total_flops()
    # the fusion 1x1 projections run here BEFORE the 2x upsample (they commute): 4x fewer FLOPs
    g, F = spec.grid, spec.fusion
    moved = sum(3 * 2.0 * s * s * F * F for s in (4 * g, 2 * g, g, (g + 1) // 2))
    # FlopCounter counts SDPA on CPU as 0 or as bmm depending on the backend: accept either
    ours = spec.flops_per_image() + moved
    assert abs(counted - ours) <= 0.01 * ours or abs(counted + attn - ours) <= 0.01 * ours, (counted, ours)

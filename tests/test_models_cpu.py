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

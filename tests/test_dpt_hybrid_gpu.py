"""DPT-Hybrid (BiT-R50 + ViT-B/16, BASELINE configs[4]) against transformers' fp32
DPTForDepthEstimation(is_hybrid=True) on the same seeded weights and the same preprocessed input.

Tolerances (stated per dtype), achieved values printed and logged:
  BiT stem alone (bf16)        : relative L2 <= 1e-2 per stage map
  network bf16                 : relative L2 of the depth <= 1.5e-2, max <= 4e-2 * max|ref|
  network fp8 (MX e4m3, E8M0)  : relative L2 <= 6e-2, max <= 2e-1 * max|ref| (3-bit mantissa
                                 operands: ~2^-5 relative rounding per element)
End to end (C5): fp8 depth -> unprojection is bit-exact with the oracle on the device depth and
the coloured binary PLY holds every point.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
transformers = pytest.importorskip("transformers")
pytestmark = pytest.mark.gpu


def _hf(spec, sd, dev):
    from transformers import DPTConfig, DPTForDepthEstimation
    m = DPTForDepthEstimation(DPTConfig(**spec.hf_config_kwargs()))
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert not [k for k in missing if "pooler" not in k], missing
    return m.to(dev).eval()


def _images(B, h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    out = []
    for i in range(B):
        base = 127 + 100 * np.sin(u / (9.0 + i)) * np.cos(v / (13.0 + i))
        out.append(np.clip(base[..., None] + rng.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8))
    return np.stack(out)


def _report(case, **vals):
    from test_dpt_gpu import _report as rep
    rep(case, **vals)


def test_bit_stem_matches_transformers():
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID, DPTHybridModel, synthetic_state_dict
    spec, B = DPT_HYBRID, 2
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, 0)
    ours = DPTHybridModel(spec, sd, dev, dtype="bf16")
    ref = _hf(spec, sd, dev)
    g = torch.Generator(device="cpu").manual_seed(3)
    pix = torch.randn(B, 3, 384, 384, generator=g).to(dev)
    feats = ours._bit(pix, B)
    torch.cuda.synchronize()
    with torch.no_grad():
        exp = ref.dpt.embeddings.backbone(pix).feature_maps
    for i, (a, e) in enumerate(zip(feats, exp)):
        e = e.permute(0, 2, 3, 1).float()
        assert a.shape == e.shape, (a.shape, e.shape)
        rel = ((a.float() - e).norm() / e.norm()).item()
        _report(f"bit stage{i + 1} {tuple(e.shape)}", rel_l2=rel)
        assert rel <= 1e-2, (i, rel)


@pytest.mark.parametrize("which,dtype,B,hw", [("tiny", "bf16", 2, (128, 128)), ("tiny", "fp8", 2, (160, 120)),
                                              ("full", "bf16", 2, (384, 384)), ("full", "fp8", 2, (384, 384)),
                                              ("full", "fp8", 2, (1024, 1024))])
def test_dpt_hybrid_matches_transformers_fp32(which, dtype, B, hw):
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID, DPT_HYBRID_TINY, DPTHybridModel, synthetic_state_dict
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    spec = DPT_HYBRID if which == "full" else DPT_HYBRID_TINY
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, 0)
    ours = DPTHybridModel(spec, sd, dev, dtype=dtype)
    ref = _hf(spec, sd, dev)
    imgs = _images(B, hw[0], hw[1], 7)
    prep = Preprocessor(hw[0], hw[1], ProcessorSpec(size=(spec.image, spec.image)))
    pix = prep(torch.from_numpy(imgs).to(dev), layout="nchw")
    depth = ours(pix, B)
    torch.cuda.synchronize()
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
    assert depth.shape == exp.shape
    err = depth - exp
    rel = (err.norm() / exp.norm()).item()
    mx = (err.abs().max() / exp.abs().max()).item()
    assert exp.abs().max() > 0 and exp.std() > 1e-3 * exp.abs().max(), "degenerate reference depth"
    _report(f"dpt-hybrid-{which} {dtype} B={B} {hw[0]}x{hw[1]}", rel_l2=rel, max_rel=mx)
    bound = (1.5e-2, 4e-2) if dtype == "bf16" else (6e-2, 2e-1)
    assert rel <= bound[0] and mx <= bound[1], f"rel L2 {rel:.3e} max {mx:.3e}"


def test_c5_pipeline_fp8_to_coloured_ply(tmp_path):
    """C5 end to end on 2 x 1024^2: preprocess -> DPT-Hybrid fp8 -> unprojection + RGB gather
    (bit-exact vs the oracle on the device depth) -> coloured binary PLY of every point."""
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    from image_to_pointcloud_amd import writers
    from oracle import unproject_ref as oref
    dev = torch.device("cuda")
    imgs = _images(2, 1024, 1024, 5)
    pipe = PointCloudPipeline(2, 1024, 1024, spec=DPT_HYBRID, density="high", device=dev, dtype="fp8")
    pb = pipe.run(torch.from_numpy(imgs).to(dev))
    torch.cuda.synchronize()
    depth = pipe.depth.cpu().numpy()
    assert depth.shape == (2, 384, 384) and np.isfinite(depth).all()
    for i in range(2):
        ep, ec = oref.depth_to_point_cloud(imgs[i], depth[i], density="high", loop=False)
        assert pb.xyz[i].cpu().numpy().tobytes() == ep.tobytes()
        assert pb.rgb[i].cpu().numpy().astype(np.float32).tobytes() == ec.tobytes()
    path = str(tmp_path / "c5.ply")
    writers.write_ply(path, pb.xyz[0], pb.rgb[0])
    data = open(path, "rb").read()
    head = data[: data.index(b"end_header\n") + len(b"end_header\n")].decode()
    assert "element vertex 1048576" in head and "property uchar red" in head
    assert len(data) - len(head) == 1048576 * (3 * 8 + 3)        # double xyz + uchar rgb (Open3D layout)

"""DPT-Hybrid (BiT-R50 + ViT-B/16, BASELINE configs[4]) against transformers' fp32
DPTForDepthEstimation(is_hybrid=True) on the same seeded weights and the same preprocessed input.

Tolerances (stated per dtype), achieved values printed and logged.  Each case
also measures a control -- transformers' OWN forward in bf16 against its fp32 forward -- which
is how much any bf16 implementation of these weights must move:
  BiT stem alone (bf16)        : relative L2 per stage map <= max(1e-2, 1.5 x control)
  network bf16                 : relative L2 of the depth <= max(1.5e-2, 1.5 x control),
                                 max <= 4e-2 * max|ref|
  network fp8 (MX e4m3, E8M0)  : relative L2 <= max(5e-2, 1.5 x fp8 control), max <= 3e-1 *
                                 max|ref|.  The fp8 control is transformers' fp32 forward with the
                                 SAME MX quantisation (e4m3 RNE, smallest power-of-two scale per 32
                                 k) applied to both operands of the same GEMMs (_mx_control): how
                                 far any MX fp8 implementation of these GEMMs must move.  Every fp8
                                 GEMM rounds both operands to a 3-bit mantissa (~2.6 % rms relative
                                 per element), and on these random weights the errors of ~60 GEMMs
                                 in sequence add up to several per cent.
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


# transformers modules of each quantisation point of dpt_hybrid.FP8_POINTS (modeling_dpt.py names)
_POINT_MODULES = {
    "qkv": r"dpt\.encoder\.layer\.\d+\.attention\.attention\.(query|key|value)$",
    "o": r"dpt\.encoder\.layer\.\d+\.attention\.output\.dense$",
    "fc1": r"dpt\.encoder\.layer\.\d+\.intermediate\.dense$",
    "fc2": r"dpt\.encoder\.layer\.\d+\.output\.dense$",
    "readout": r"neck\.reassemble_stage\.(readout_projects\.\d+\.0|layers\.\d+\.(projection|resize))$",
    "neck": r"neck\.convs\.\d+$",
    "fusion": r"neck\.fusion_stage\.layers\.\d+\.residual_layer\d\.convolution\d$",
    "head": r"head\.head\.0$",
}


def _mx_qdq(x, dim, upto=None):
    """MX fp8 quantise-dequantise (csrc/mx.h): blocks of 32 along `dim` (only its first `upto`
    entries), scale = the smallest power of two 2^e with max|block| / 2^e <= 448, e4m3fn
    round-to-nearest-even."""
    xt = x.movedim(dim, -1)
    K = xt.shape[-1] if upto is None else upto
    assert K % 32 == 0, K
    head = xt[..., :K].float()
    xb = head.reshape(*head.shape[:-1], K // 32, 32)
    am = xb.abs().amax(-1, keepdim=True)
    m, E = torch.frexp(am)
    e = (E - 9 + (m > 0.875).to(E.dtype)).clamp(-127, 127)
    e = torch.where(am == 0, torch.full_like(e, -127), e)
    sc = torch.exp2(e.to(torch.float32))
    q = ((xb / sc).to(torch.float8_e4m3fn).float() * sc).reshape(head.shape).to(x.dtype)
    out = torch.cat([q, xt[..., K:]], -1) if K < xt.shape[-1] else q
    return out.movedim(-1, dim)


def _mx_control(ref, pix, exp, fp8_points, hidden):
    """relative L2 of transformers' fp32 depth with MX fp8 operands at `fp8_points` against `exp`."""
    import copy
    import re
    m = copy.deepcopy(ref)
    pats = [re.compile(_POINT_MODULES[p]) for p in fp8_points]
    hooks = []
    for name, mod in m.named_modules():
        if not any(p.search(name) for p in pats) or not isinstance(mod, (torch.nn.Linear, torch.nn.Conv2d)):
            continue
        # the readout linear's CLS half stays bf16 in dpt_hybrid (split GEMM): quantise the token half
        upto = hidden if "readout_projects" in name else None
        with torch.no_grad():
            mod.weight.copy_(_mx_qdq(mod.weight, 1, upto))
        hooks.append(mod.register_forward_pre_hook(
            lambda _m, args, upto=upto: (_mx_qdq(args[0], args[0].dim() - 1 if args[0].dim() != 4 else 1, upto),)
            + tuple(args[1:])))
    # deterministic MIOpen algorithms: the control's spread between runs of the same mix came from the
    # conv algorithm choice, and the bound below is relative to it
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
        d = m(pixel_values=pix).predicted_depth.float()
    for h in hooks:
        h.remove()
    del m
    return ((d - exp).norm() / exp.norm()).item()


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
    import copy
    with torch.no_grad():
        exp = ref.dpt.embeddings.backbone(pix).feature_maps
        ctl = copy.deepcopy(ref).to(torch.bfloat16).dpt.embeddings.backbone(pix.to(torch.bfloat16)).feature_maps
    for i, (a, e, c) in enumerate(zip(feats, exp, ctl)):
        control = ((c.float() - e).norm() / e.norm()).item()
        e = e.permute(0, 2, 3, 1).float()
        assert a.shape == e.shape, (a.shape, e.shape)
        rel = ((a.float() - e).norm() / e.norm()).item()
        _report(f"bit stage{i + 1} {tuple(e.shape)}", rel_l2=rel, torch_bf16_control=control)
        assert rel <= max(1e-2, 1.5 * control), (i, rel, control)


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
    import copy
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
        ctl = copy.deepcopy(ref).to(torch.bfloat16)(pixel_values=pix.to(torch.bfloat16)).predicted_depth.float()
    control = ((ctl - exp).norm() / exp.norm()).item()
    assert depth.shape == exp.shape
    err = depth - exp
    rel = (err.norm() / exp.norm()).item()
    mx = (err.abs().max() / exp.abs().max()).item()
    assert exp.abs().max() > 0 and exp.std() > 1e-3 * exp.abs().max(), "degenerate reference depth"
    if dtype == "bf16":
        _report(f"dpt-hybrid-{which} {dtype} B={B} {hw[0]}x{hw[1]}", rel_l2=rel, max_rel=mx, torch_bf16_control=control)
        bound = (max(1.5e-2, 1.5 * control), 4e-2)
    else:
        from image_to_pointcloud_amd.dpt_hybrid import FP8_POINTS
        pts = [p for p in FP8_POINTS if ours._f8(p)]
        fctl = _mx_control(ref, pix, exp, pts, spec.hidden)
        _report(f"dpt-hybrid-{which} {dtype} B={B} {hw[0]}x{hw[1]}", rel_l2=rel, max_rel=mx, torch_bf16_control=control,
                mx_fp8_control=fctl)
        bound = (max(5e-2, 1.5 * fctl), 3e-1)
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


def test_c5_batch64_pipeline_fp8_to_coloured_ply(tmp_path):
    """C5 at its configured batch (BASELINE configs[4]: 64 x 1024^2, DPT-Hybrid fp8): the ViT GEMMs
    run at M = 36,928 with multi-round persistent schedules and tail splits that B = 2 never reaches.
    * depth finite and non-degenerate for every image;
    * images 0, 31 and 63 of the batch against transformers' fp32 forward of the same three images
      on the same weights: relative L2 <= max(5e-2, 1.5 x the MX-fp8 control), max <= 3e-1 x max|ref|
      (the bound of the B = 2 test, test_dpt_hybrid_matches_transformers_fp32);
    * the same three images as a batch of 3 through the same model give the same depth (batch
      invariance, VERDICT r05 item 7: the GroupNorm statistics once tiled each image by batch * hw,
      and the fp8 roundings amplified the different partial sums to 3-6 % rel L2; every kernel now
      sums an image's values in an order fixed by that image alone -- bound 1e-3, measured 0);
    * the unprojection of images 0, 31 and 63 bit-exact vs the oracle on the device depth;
    * one coloured binary PLY holding all 67,108,864 points, spot-checked record by record."""
    import os
    from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID, FP8_POINTS, synthetic_state_dict
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    from image_to_pointcloud_amd import writers
    from oracle import unproject_ref as oref
    dev = torch.device("cuda")
    B, S = 64, 1024
    rng = np.random.Generator(np.random.PCG64(64))
    imgs = rng.integers(0, 256, (B, S, S, 3), dtype=np.uint8)
    v, u = np.meshgrid(np.arange(S), np.arange(S), indexing="ij")
    for i in (0, 31, 63):       # structured images where the checks look (uniform noise elsewhere)
        base = 127 + 100 * np.sin(u / (9.0 + i)) * np.cos(v / (13.0 + i))
        imgs[i] = np.clip(base[..., None] + rng.normal(0, 20, (S, S, 3)), 0, 255).astype(np.uint8)
    timgs = torch.from_numpy(imgs).to(dev)
    pipe = PointCloudPipeline(B, S, S, spec=DPT_HYBRID, density="high", device=dev, dtype="fp8")
    pb = pipe.run(timgs)
    torch.cuda.synchronize()
    depth = pipe.depth.cpu().numpy()
    assert depth.shape == (B, 384, 384) and np.isfinite(depth).all()
    per_std = depth.reshape(B, -1).std(axis=1)
    assert (per_std > 1e-3 * np.abs(depth).max()).all(), "degenerate depth in some image"
    assert pb.xyz.shape == (B, S * S, 3) and pb.rgb.shape == (B, S * S, 3)
    picks = [0, 31, 63]
    sub = timgs[picks].contiguous()
    small = PointCloudPipeline(3, S, S, spec=DPT_HYBRID, density="high", device=dev, model=pipe.model, dtype="fp8")
    small.infer_depth(sub)
    torch.cuda.synchronize()
    d3 = small.depth.cpu().numpy()
    ref = _hf(DPT_HYBRID, synthetic_state_dict(DPT_HYBRID, 0), dev)
    pix = Preprocessor(S, S, ProcessorSpec(size=(384, 384)))(sub, layout="nchw")
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
    fctl = _mx_control(ref, pix, exp, [p for p in FP8_POINTS if pipe.model._f8(p)], DPT_HYBRID.hidden)
    bound = max(5e-2, 1.5 * fctl)
    e = exp.cpu().numpy()
    for j, i in enumerate(picks):
        rel = float(np.linalg.norm(depth[i] - e[j]) / np.linalg.norm(e[j]))
        mx = float(np.abs(depth[i] - e[j]).max() / np.abs(e[j]).max())
        rel3 = float(np.linalg.norm(d3[j] - e[j]) / np.linalg.norm(e[j]))
        self_rel = float(np.linalg.norm(depth[i] - d3[j]) / np.linalg.norm(d3[j]))
        _report(f"c5 batch64 image {i} vs transformers fp32", rel_l2=rel, max_rel=mx, mx_fp8_control=fctl,
                batch3_rel_l2=rel3, batch64_vs_batch3_rel_l2=self_rel)
        assert rel <= bound and mx <= 3e-1, (i, rel, mx, bound)
        assert rel3 <= bound, (i, rel3, bound)
        assert self_rel <= 1e-3, (i, self_rel)     # batch invariance
    del ref
    for i in picks:
        ep, ec = oref.depth_to_point_cloud(imgs[i], depth[i], density="high", loop=False)
        assert pb.xyz[i].cpu().numpy().tobytes() == ep.tobytes(), i
        assert pb.rgb[i].cpu().numpy().astype(np.float32).tobytes() == ec.tobytes(), i
    path = str(tmp_path / "c5_b64.ply")
    writers.write_ply(path, pb.xyz, pb.rgb)
    n = B * S * S
    with open(path, "rb") as fh:
        head = fh.read(512)
    head = head[: head.index(b"end_header\n") + len(b"end_header\n")]
    assert f"element vertex {n}".encode() in head and b"property uchar red" in head
    assert os.path.getsize(path) - len(head) == n * (3 * 8 + 3)   # double xyz + uchar rgb (Open3D layout)
    rec = np.memmap(path, dtype=np.dtype([("xyz", "<f8", 3), ("rgb", "u1", 3)]), mode="r", offset=len(head))
    for i in picks:
        for p in (0, 12345, S * S - 1):
            r = rec[i * S * S + p]
            assert np.array_equal(r["xyz"], pb.xyz[i, p].cpu().numpy().astype(np.float64)), (i, p)
            assert np.array_equal(r["rgb"], pb.rgb[i, p].cpu().numpy()), (i, p)
    del rec
    os.remove(path)


def test_fp8_quantisation_point_ablation():
    """Which MX fp8 quantisation point costs the accuracy: the fp8 network
    with ONE group of GEMMs back in bf16 at a time (dpt_hybrid.FP8_POINTS), relative L2 of the depth
    against transformers fp32 on 384^2 and 1024^2 inputs, beside the MX fp8 control of the same mix
    (transformers fp32 with MX operands at the same points, _mx_control).  Prints the table
     and checks every mix, the default (DEFAULT_BF16_POINTS) included, against
    max(5e-2, 1.5 x its control) at both sizes."""
    from image_to_pointcloud_amd.dpt_hybrid import (DEFAULT_BF16_POINTS, DPT_HYBRID, FP8_POINTS, DPTHybridModel,
                                                    synthetic_state_dict)
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    spec, B = DPT_HYBRID, 2
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, 0)
    ref = _hf(spec, sd, dev)
    cases = []
    for hw in ((384, 384), (1024, 1024)):
        imgs = _images(B, hw[0], hw[1], 7)
        prep = Preprocessor(hw[0], hw[1], ProcessorSpec(size=(spec.image, spec.image)))
        pix = prep(torch.from_numpy(imgs).to(dev), layout="nchw")
        with torch.no_grad():
            exp = ref(pixel_values=pix).predicted_depth.float()
        cases.append((hw, pix, exp))
    configs = ([("all fp8", ()), ("default", tuple(DEFAULT_BF16_POINTS))] + [(f"{p} bf16", (p,)) for p in FP8_POINTS]
               + [("qkv+fc2 bf16", ("qkv", "fc2")), ("qkv+fc1+fc2 bf16", ("qkv", "fc1", "fc2")),
                  ("qkv+fc2+neck bf16", ("qkv", "fc2", "neck"))])
    table, ctl = {}, {}
    for name, pts in configs:
        model = DPTHybridModel(spec, sd, dev, dtype="fp8", bf16_points=pts)
        f8pts = [p for p in FP8_POINTS if model._f8(p)]
        errs, ctls = [], []
        for hw, pix, exp in cases:
            depth = model(pix, B)
            torch.cuda.synchronize()
            errs.append(((depth - exp).norm() / exp.norm()).item())
            ctls.append(_mx_control(ref, pix, exp, f8pts, spec.hidden))
        table[name], ctl[name] = errs, ctls
        _report(f"dpt-hybrid fp8 ablation: {name}", rel_l2_384=errs[0], rel_l2_1024=errs[1],
                mx_fp8_control_384=ctls[0], mx_fp8_control_1024=ctls[1])
        del model
        torch.cuda.empty_cache()
    # every mix within the MX fp8 control's noise; the default mix also within 5e-2 or 1.5x its control
    for name in table:
        for e, c in zip(table[name], ctl[name]):
            assert e <= max(5e-2, 1.5 * c), (name, e, c)

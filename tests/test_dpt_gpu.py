"""Depth network parity: the bf16 HIP DPT against transformers' fp32 DPTForDepthEstimation.

Same seeded weights (transformers key layout), same preprocessed input.
Tolerance (bf16 operands / fp32 accumulation vs an fp32 network): relative L2
error of the predicted depth <= max(1e-2, 1.5 x control) and max |err| <= 4e-2 * max |ref|, where
the control is transformers' OWN bf16 forward of the same weights against its fp32 forward (what
plain bf16 arithmetic moves this network; measured r02 without it: rel L2 0.97e-2 at 384^2 and
1.12e-2 at 1024^2 input).
Every case prints the error it reached.  The preprocessing itself is checked bit-exact against
DPTImageProcessorPil.

End to end (`test_end_to_end_points_vs_fp32_reference`): transformers-fp32 depth -> oracle
unprojection against HIP bf16 depth -> HIP unprojection.  The north star's 1e-4 relative XYZ
bound holds for the unprojection given identical depth (bit-exact, test_unproject_gpu.py); with a
bf16 network in front it cannot hold point for point (D9), so this test splits the points into
clip / far / interior classes, reports each class's error, and bounds the interior class.
"""
import json
import os
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
    import copy
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
        # control: transformers' OWN forward in bf16 on the same weights -- how far plain bf16
        # arithmetic moves this network from its fp32 forward
        ctl = copy.deepcopy(ref).to(torch.bfloat16)(pixel_values=pix.to(torch.bfloat16)).predicted_depth.float()
    control = ((ctl - exp).norm() / exp.norm()).item()
    assert depth.shape == exp.shape
    err = (depth - exp)
    rel = (err.norm() / exp.norm()).item()
    mx = (err.abs().max() / exp.abs().max()).item()
    assert exp.abs().max() > 0 and exp.std() > 1e-3 * exp.abs().max(), "degenerate reference depth"
    _report(f"dpt-{which} B={B} {hw[0]}x{hw[1]}", rel_l2=rel, max_rel=mx, torch_bf16_control=control)
    # SURVEY 8c's 1e-2, or 1.5x what torch's own bf16 forward of these weights reaches
    bound = max(1e-2, 1.5 * control)
    assert rel <= bound and mx <= 4e-2, f"rel L2 {rel:.3e} max {mx:.3e} (torch bf16 control {control:.3e})"


def _report(case, **vals):
    """Print the achieved error (pytest -rP shows it) and append it to $I2PC_PARITY_LOG if set."""
    line = {"case": case, **{k: float(v) for k, v in vals.items()}}
    print("parity", json.dumps(line))
    path = os.environ.get("I2PC_PARITY_LOG")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps(line) + "\n")


def test_end_to_end_points_vs_fp32_reference():
    """bf16 HIP depth -> HIP points vs transformers-fp32 depth -> oracle points (DPT-Large, 2 x 384^2),
    the point error split by cause (app.py:197-206 normalises the depth to
    n = (clip(depth, p2, p98) - p2) / (p98 - p2) and z = depth_scale * (1 - n)):
    * `clip`: pixels at or outside [p2, p98] in either path -- their n is pinned to 0 / 1 by one path
      and free in the other, or both are pinned to percentiles that moved;
    * `far`: interior pixels with z < 0.1 * depth_scale (n > 0.9, near the p98 clip) -- relative XYZ
      error is |dn| / (1 - n), so a small absolute error is a large relative one there;
    * `interior`: the rest -- the bulk of the cloud.
    Per class the p50 / p99 of the relative XYZ error and of the absolute error in units of
    depth_scale are reported.  The north star's 1e-4 relative XYZ holds for the unprojection given
    identical depth (bit-exact, test_unproject_gpu.py); behind a bf16 network it is the
    network's depth error that moves the points: the interior class is bounded through the
    absolute error |dz| / depth_scale (the normalised-depth error itself), the relative error of the
    other two classes is reported, not bounded (it divides by z -> 0 or by a clip decision)."""
    from image_to_pointcloud_amd import geometry
    from image_to_pointcloud_amd.dpt import DPT_LARGE, DPTDepthModel, synthetic_state_dict
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    from oracle import unproject_ref as oref
    spec, B, hw = DPT_LARGE, 2, (384, 384)
    scale = 10.0
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, seed=0)
    ours = DPTDepthModel(spec, sd, dev)
    ref = _hf_model(spec, sd, dev)
    imgs = _images(B, hw[0], hw[1], 11)
    prep = Preprocessor(hw[0], hw[1], ProcessorSpec(size=(spec.image, spec.image)), patch=spec.patch)
    timgs = torch.from_numpy(imgs).to(dev)
    with torch.no_grad():
        exp_depth = ref(pixel_values=prep(timgs, layout="nchw")).predicted_depth.float().cpu().numpy()
    depth = ours(prep(timgs, layout="patches"), B)
    pb = geometry.unproject_batch(depth, timgs, density="high", depth_scale=scale)
    torch.cuda.synchronize()
    got_depth = depth.cpu().numpy()
    stats = pb.stats.cpu().numpy()
    acc = {c: {"rel": [], "abs": []} for c in ("clip", "far", "interior")}
    fracs = []
    for i in range(B):
        ep, ec = oref.depth_to_point_cloud(imgs[i], exp_depth[i], density="high", depth_scale=scale, loop=False)
        got = pb.xyz[i].cpu().numpy().astype(np.float64)
        assert np.array_equal(pb.rgb[i].cpu().numpy().astype(np.float32), ec)   # integer outputs: exact
        _, est = oref.normalize_depth(exp_depth[i], True)
        dg, de = got_depth[i].astype(np.float32).ravel(), exp_depth[i].astype(np.float32).ravel()
        clip = ((dg <= stats[i, 0]) | (dg >= stats[i, 1]) | (de <= est["p2"]) | (de >= est["p98"]))
        far = ~clip & (np.minimum(np.abs(got[:, 2]), np.abs(ep[:, 2])) < 0.1 * scale)
        inner = ~clip & ~far
        den = np.maximum(np.abs(ep).max(axis=1), scale * 1e-5)                  # floor: depth_scale * 1e-5
        err = np.abs(got - ep).max(axis=1)
        rel, ab = err / den, err / scale
        fracs.append(float((rel <= 1e-4).mean()))
        for c, msk in (("clip", clip), ("far", far), ("interior", inner)):
            acc[c]["rel"].append(rel[msk])
            acc[c]["abs"].append(ab[msk])
    out = {"frac_within_1e4": float(np.mean(fracs))}
    n_all = sum(len(np.concatenate(v["rel"])) for v in acc.values())
    for c, v in acc.items():
        r, a = np.concatenate(v["rel"]), np.concatenate(v["abs"])
        out[f"{c}_share"] = len(r) / n_all
        if len(r):
            out.update({f"{c}_rel_p50": float(np.median(r)), f"{c}_rel_p99": float(np.quantile(r, 0.99)),
                        f"{c}_abs_p50": float(np.median(a)), f"{c}_abs_p99": float(np.quantile(a, 0.99))})
    _report("e2e dpt-large 2x384^2 high: bf16 network + HIP unproject vs fp32 network + oracle", **out)
    # the bulk of the cloud: the normalised-depth error the bf16 network leaves (its depth is within
    # ~1-2 % rel L2 of fp32, test_dpt_forward_matches_transformers_fp32; p98 - p2 spans a fraction of
    # the depth, so the normalised error is a few times that)
    # (measured r06: interior 93 % of the points, |dz| / depth_scale p50 0.44 % / p99 1.7 %, relative
    # p50 0.87 % / p99 6.1 %; far 2.8 % of the points, relative p99 147 %; clip 4.1 %, relative p99 ~24
    # -- z pinned at 0 by one path's p98 clip)
    assert out["interior_share"] >= 0.8, out
    assert out["interior_abs_p50"] <= 1e-2 and out["interior_abs_p99"] <= 5e-2, out
    assert out["interior_rel_p50"] <= 2e-2, out


def test_captured_pipeline_survives_workspace_regrow():
    """A captured pipeline owns its unprojection workspace: a later, larger one-off call that
    regrows the shared per-device scratch must not change what replay() writes."""
    from image_to_pointcloud_amd import geometry
    from image_to_pointcloud_amd.dpt import DPT_TINY
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    from oracle import unproject_ref as oref
    dev = torch.device("cuda")
    imgs = _images(2, 96, 80, 3)
    timgs = torch.from_numpy(imgs).to(dev)
    pipe = PointCloudPipeline(2, 96, 80, spec=DPT_TINY, density="high", device=dev)
    pipe.capture(timgs)
    big_b, big = 64, 256
    need = geometry.workspace_bytes(big_b, big, big)
    held = geometry._WS.get(dev.index if dev.index is not None else torch.cuda.current_device())
    assert held is None or held.numel() < need, "the one-off call below must force a regrow"
    bd = torch.rand((big_b, 32, 32), device=dev)
    bi = torch.randint(0, 256, (big_b, big, big, 3), dtype=torch.uint8, device=dev)
    geometry.unproject_batch(bd, bi, density="high")          # regrows (and frees) the shared scratch
    torch.cuda.synchronize()
    torch.empty(need * 4, dtype=torch.uint8, device=dev).fill_(0xA5)   # recycle the freed block
    out = pipe.replay()
    torch.cuda.synchronize()
    depth = pipe.depth.cpu().numpy()
    for i in range(2):
        ep, ec = oref.depth_to_point_cloud(imgs[i], depth[i], density="high", loop=False)
        assert out.xyz[i].cpu().numpy().tobytes() == ep.tobytes()
        assert out.rgb[i].cpu().numpy().astype(np.float32).tobytes() == ec.tobytes()


def test_c3_dpt_large_512_batch():
    """C3's per-GPU shard (32 x 512^2 through preprocess -> DPT-Large bf16 -> unprojection,
    density high): depth finite and non-degenerate; the unprojection of the device depth of
    images 0, 17 and 31 bit-exact with the oracle (points and colours)."""
    from image_to_pointcloud_amd.dpt import DPT_LARGE
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    from oracle import unproject_ref as oref
    dev = torch.device("cuda")
    B = 32
    imgs = _images(B, 512, 512, 13)
    pipe = PointCloudPipeline(B, 512, 512, spec=DPT_LARGE, density="high", device=dev)
    pb = pipe.run(torch.from_numpy(imgs).to(dev))
    torch.cuda.synchronize()
    depth = pipe.depth.cpu().numpy()
    assert depth.shape == (B, 384, 384) and np.isfinite(depth).all() and depth.std() > 0
    assert pb.xyz.shape == (B, 512 * 512, 3)
    for i in (0, 17, 31):
        ep, ec = oref.depth_to_point_cloud(imgs[i], depth[i], density="high", loop=False)
        assert pb.xyz[i].cpu().numpy().tobytes() == ep.tobytes(), i
        assert pb.rgb[i].cpu().numpy().astype(np.float32).tobytes() == ec.tobytes(), i


def test_c2_benchmarked_graph_32x1024():
    """The headline workload exactly as bench.py times it (BASELINE configs[1]):
    PointCloudPipeline(32, 1024, 1024, DPT_LARGE, seed 0) on bench._images, captured into one HIP
    graph and replayed (bench.py main()).  Reference per-image path: backend/app.py:460-476.
    * two replays are bit-identical to each other and to an eager run() of the same pipeline
      (xyz, rgb, bbox, stats and the model-resolution depth);
    * the depth is finite and non-degenerate for every image;
    * images 0, 15 and 31 unproject bit-exact vs oracle.unproject_ref on the device depth
      (points, colours, bounds);
    * no image took the exact selection from scratch (SelState.level != 16: the bench's fast path)."""
    import bench
    from image_to_pointcloud_amd.dpt import DPT_LARGE
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    from oracle import unproject_ref as oref
    dev = torch.device("cuda")
    B, S = 32, 1024
    pipe = PointCloudPipeline(B, S, S, spec=DPT_LARGE, density="high", device=dev, seed=0)
    images = bench._images(B, S, 0, dev)
    out = pipe.capture(images)

    def snap():
        return [t.clone() for t in (out.xyz, out.rgb, out.bbox, out.stats, pipe.depth)]

    def bits(t):      # bit identity (stats[:, 3] is NaN for a map without non-finite pixels)
        return t.view({8: torch.int64, 4: torch.int32, 1: torch.uint8}[t.element_size()])

    pipe.replay()
    torch.cuda.synchronize()
    r1 = snap()
    pipe.replay()
    torch.cuda.synchronize()
    r2 = snap()
    names = ("xyz", "rgb", "bbox", "stats", "depth")
    for n, a, b in zip(names, r1, r2):
        assert torch.equal(bits(a), bits(b)), f"replay 1 vs replay 2 differ in {n}"
    st = pipe._ws[:624 * B].view(torch.int32).view(B, 156)[:, 85].cpu()
    assert int((st == 16).sum()) == 0, f"selection from scratch on images {torch.nonzero(st == 16).flatten().tolist()}"
    eo = pipe.run(images)
    torch.cuda.synchronize()
    for n, a, b in zip(names, r1, (eo.xyz, eo.rgb, eo.bbox, eo.stats, pipe.depth)):
        assert torch.equal(bits(a), bits(b)), f"replay vs eager run() differ in {n}"
    depth = r1[4].cpu().numpy()
    assert depth.shape == (B, 384, 384) and np.isfinite(depth).all()
    per_std = depth.reshape(B, -1).std(axis=1)
    assert (per_std > 1e-3 * np.abs(depth).max()).all(), "degenerate depth in some image"
    imgs = images.cpu().numpy()
    bbox = r1[2].cpu().numpy()
    for i in (0, 15, 31):
        ep, ec = oref.depth_to_point_cloud(imgs[i], depth[i], density="high", loop=False)
        assert r1[0][i].cpu().numpy().tobytes() == ep.tobytes(), i
        assert r1[1][i].cpu().numpy().astype(np.float32).tobytes() == ec.tobytes(), i
        eb = oref.gis_bounds(ep)                                  # app.py:393-400
        exp = np.array([eb["minX"], eb["maxX"], eb["minY"], eb["maxY"], eb["minZ"], eb["maxZ"]], np.float64)
        assert np.array_equal(bbox[i], exp), (i, bbox[i], exp)
    _report("c2 benchmarked graph 32x1024^2", replays_identical=1, eager_identical=1,
            selection_from_scratch=int((st == 16).sum()))


def test_dpt_any_grid_pos_interpolation_and_fusion_resize():
    """DPT on an odd patch grid (112 x 112 network input -> 7 x 7 patches against the checkpoint's
    8 x 8): the position table is interpolated (DPTViTEmbeddings._resize_pos_embed) and the
    fusion stage resizes the residual feature to the fused map (4 -> 8 vs 7,
    modeling_dpt.py:696-699).  (transformers' ViT-DPT reshapes tokens to a square grid, so a
    non-square grid, which this module also runs, has no reference to compare with.)"""
    from image_to_pointcloud_amd.dpt import DPT_TINY, DPTDepthModel, synthetic_state_dict
    from image_to_pointcloud_amd.preprocess import Preprocessor, ProcessorSpec
    spec, B = DPT_TINY, 2
    dev = torch.device("cuda")
    sd = synthetic_state_dict(spec, seed=0)
    ours = DPTDepthModel(spec, sd, dev)
    ref = _hf_model(spec, sd, dev)
    imgs = _images(B, 100, 150, 9)
    prep = Preprocessor(100, 150, ProcessorSpec(size=(112, 112)), patch=16)
    timgs = torch.from_numpy(imgs).to(dev)
    pix = prep(timgs, layout="nchw")
    depth = ours(prep(timgs, layout="patches"), B, 7, 7)
    torch.cuda.synchronize()
    with torch.no_grad():
        exp = ref(pixel_values=pix).predicted_depth.float()
    assert depth.shape == exp.shape, (depth.shape, exp.shape)
    rel = ((depth - exp).norm() / exp.norm()).item()
    _report("dpt-tiny 7x7 grid", rel_l2=rel)
    assert rel <= 1e-2, rel

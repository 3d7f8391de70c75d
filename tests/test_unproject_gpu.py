"""GPU parity of the HIP unprojection against the reference fixtures and the oracle.

Bar: bit-exact xyz (float32), colours, bounds and percentile stats -- the
kernels evaluate the reference's arithmetic in the same IEEE order.
"""
import numpy as np
import pytest

from oracle import unproject_ref as ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _geom():
    from image_to_pointcloud_amd import geometry
    return geometry


def _same_bits(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def _first_diff(a, b):
    idx = np.argwhere(a != b)
    if len(idx) == 0:
        return "shape/dtype"
    i = tuple(idx[0])
    return f"first diff at {i}: got {a[i]!r} expected {b[i]!r} ({len(idx)} diffs)"


def test_golden_cases_bit_exact(unproject_cases):
    g = _geom()
    for c in unproject_cases:
        pts, cols = g.depth_to_point_cloud(c["image"], c["depth"], density=c["density"],
                                           invert=c["invert"], depth_scale=c["scale"])
        assert _same_bits(pts, c["points"]), (c["name"], _first_diff(pts, c["points"]))
        assert _same_bits(cols, c["colors"]), c["name"]


def test_golden_bounds_from_device_bbox(unproject_cases):
    g = _geom()
    for c in unproject_cases:
        dev = torch.device("cuda")
        pb = g.unproject_batch(torch.from_numpy(c["depth"]).to(dev)[None], torch.from_numpy(c["image"]).to(dev)[None],
                               density=c["density"], invert=c["invert"], depth_scale=c["scale"])
        got = pb.bbox[0].cpu().numpy()
        assert _same_bits(got, c["bounds"]), (c["name"], got, c["bounds"])


def _smooth_depth(h, w, seed, noise=0.05):
    rng = np.random.Generator(np.random.PCG64(seed))
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    base = 0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w) * np.cos(4 * np.pi * v / h))
    return np.maximum(base + rng.normal(0.0, noise, size=(h, w)), 0.0).astype(np.float32)


def _rgb(h, w, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("shape", [(384, 384, 1024, 1024), (37, 53, 100, 90), (518, 686, 768, 1024), (96, 96, 95, 97)])
@pytest.mark.parametrize("density", ["high", "medium", "low"])
def test_resized_depth_matches_oracle(shape, density):
    h, w, H, W = shape
    g = _geom()
    dep = _smooth_depth(h, w, 21)
    img = _rgb(H, W, 22)
    pts, cols = g.depth_to_point_cloud(img, dep, density=density)
    ep, ec = ref.depth_to_point_cloud(img, dep, density=density, loop=False)
    assert _same_bits(pts, ep), _first_diff(pts, ep)
    assert _same_bits(cols, ec)


def test_batched_mixed_branches_match_per_image_oracle():
    g = _geom()
    B, h, w, H, W = 8, 48, 40, 96, 80
    deps = np.stack([_smooth_depth(h, w, 100 + i) for i in range(B)])
    deps[1] = 3.0                                  # constant branch
    deps[2] = 1.0; deps[2, 0, :5] = 4.0            # min/max float32 branch
    deps[3, 5, 5] = np.nan; deps[3, 7, 9] = np.inf  # nanmedian fill
    deps[4, :, :] = np.nan                          # all-NaN
    imgs = np.stack([_rgb(H, W, 200 + i) for i in range(B)])
    dev = torch.device("cuda")
    for density in ("high", "medium"):
        for invert in (True, False):
            pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev),
                                   density=density, invert=invert, depth_scale=12.5)
            xyz = pb.xyz.cpu().numpy()
            rgb = pb.rgb.cpu().numpy()
            for i in range(B):
                with np.errstate(all="ignore"):
                    ep, ec = ref.depth_to_point_cloud(imgs[i], deps[i], density=density, invert=invert,
                                                      depth_scale=12.5, loop=False)
                assert _same_bits(xyz[i], ep), (i, density, invert, _first_diff(xyz[i], ep))
                assert _same_bits(rgb[i].astype(np.float32), ec)


def test_full_width_mixed_branches_match_oracle():
    """Resized depth, widths a multiple of 64 (the fast kernel's full-wave layout): every
    normalisation branch, both inversions, points, colours and bbox bit-exact."""
    g = _geom()
    B, h, w, H, W = 6, 24, 40, 64, 128
    deps = np.stack([_smooth_depth(h, w, 300 + i) for i in range(B)])
    deps[1] = 3.0                                   # constant branch
    deps[2] = 1.0; deps[2, 0, :5] = 4.0             # min/max float32 branch
    deps[3, 5, 5] = np.nan; deps[3, 7, 9] = np.inf  # nanmedian fill
    deps[4, :, :] = np.nan                          # all-NaN
    imgs = np.stack([_rgb(H, W, 400 + i) for i in range(B)])
    dev = torch.device("cuda")
    for invert in (True, False):
        pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev),
                               density="high", invert=invert, depth_scale=7.5)
        xyz = pb.xyz.cpu().numpy()
        rgb = pb.rgb.cpu().numpy()
        bbox = pb.bbox.cpu().numpy()
        for i in range(B):
            with np.errstate(all="ignore"):
                ep, ec = ref.depth_to_point_cloud(imgs[i], deps[i], density="high", invert=invert,
                                                  depth_scale=7.5, loop=False)
            assert _same_bits(xyz[i], ep), (i, invert, _first_diff(xyz[i], ep))
            assert _same_bits(rgb[i].astype(np.float32), ec), (i, invert)
            exp_bb = np.array([ep[:, 0].min(), ep[:, 0].max(), ep[:, 1].min(), ep[:, 1].max(),
                               ep[:, 2].min(), ep[:, 2].max()], np.float64)
            assert np.array_equal(bbox[i], exp_bb), (i, invert)


def test_percentile_stats_match_numpy():
    g = _geom()
    dev = torch.device("cuda")
    for (h, w) in ((1024, 1024), (384, 384), (1, 1), (1, 7), (3, 2)):
        d = _smooth_depth(h, w, 31) if h * w > 10 else np.random.default_rng(0).random((h, w), dtype=np.float32)
        img = _rgb(h, w, 32)
        pb = g.unproject_batch(torch.from_numpy(d).to(dev)[None], torch.from_numpy(img).to(dev)[None], density="high")
        st = pb.stats[0].cpu().numpy()
        p2, p98 = ref.percentile_2_98(d)
        if p98 > p2:
            assert st[0] == p2 and st[1] == p98, ((h, w), st, p2, p98)


def test_full_size_high_density_properties():
    """1024^2 x batch 4 from 384^2 depth: bit-exact vs oracle on image 0, shape/size invariants on all."""
    g = _geom()
    dev = torch.device("cuda")
    B = 4
    deps = np.stack([_smooth_depth(384, 384, 40 + i) for i in range(B)])
    imgs = np.stack([_rgb(1024, 1024, 50 + i) for i in range(B)])
    pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev), density="high")
    xyz = pb.xyz.cpu().numpy()
    assert xyz.shape == (B, 1024 * 1024, 3)
    ep, ec = ref.depth_to_point_cloud(imgs[0], deps[0], density="high", loop=False)
    assert _same_bits(xyz[0], ep)
    assert _same_bits(pb.rgb[0].cpu().numpy().astype(np.float32), ec)
    bb = pb.bbox.cpu().numpy()
    for i in range(B):
        x = xyz[i]
        exp = np.array([x[:, 0].min(), x[:, 0].max(), x[:, 1].min(), x[:, 1].max(), x[:, 2].min(), x[:, 2].max()],
                       dtype=np.float64)
        assert _same_bits(bb[i], exp)
        # invert=True, scale 10: z in [0, 10] and the p98-clipped pixels give z = 10*1e-6/(R+1e-6)
        assert x[:, 2].min() >= 0.0 and x[:, 2].max() <= 10.0


@pytest.mark.parametrize("ksize,shape", [(5, (60, 50)), (1, (60, 50)), (3, (41, 37)), (7, (60, 50)),
                                         (9, (60, 50)), (14, (33, 70)), (31, (12, 9))])
def test_smooth_path_matches_oracle_blur(ksize, shape):
    """GaussianBlur for every kernel app.py:211 can form (k = max(3, ksize // 2 * 2 + 1)): the
    small-kernel tables (3, 5, 7), sampled Gaussians (9, 15), and a kernel wider than the image
    (31 on 12 x 9: repeated BORDER_REFLECT_101)."""
    g = _geom()
    h, w = shape
    dep = _smooth_depth(h, w, 61)
    img = _rgb(h, w, 62)
    pts, _ = g.depth_to_point_cloud(img, dep, density="medium", smooth=True, smooth_ksize=ksize)
    ep, _ = ref.depth_to_point_cloud(img, dep, density="medium", smooth=True, smooth_ksize=ksize, loop=False)
    assert _same_bits(pts, ep), _first_diff(pts, ep)


def test_preview_subsample_matches_reference(pipeline_case):
    import hashlib
    g = _geom()
    s = pipeline_case["summary"]
    dev = torch.device("cuda")
    pb = g.unproject_batch(torch.from_numpy(pipeline_case["depth"]).to(dev)[None],
                           torch.from_numpy(pipeline_case["image"]).to(dev)[None], density="high")
    pp, pc = g.preview_subsample(pb.xyz[0], pb.rgb[0])
    assert len(pp) == s["preview_len"]
    assert hashlib.sha256(np.asarray(pp, np.float64).tobytes()).hexdigest() == s["preview_points_sha256"]
    assert hashlib.sha256(np.asarray(pc, np.float64).tobytes()).hexdigest() == s["preview_colors_sha256"]
    assert g.generate_gis_bounds(pb.bbox[0].cpu()) == s["gisData"]["bounds"]


def test_bad_arguments_raise():
    g = _geom()
    from image_to_pointcloud_amd._lib import I2PCError
    with pytest.raises(KeyError):
        g.depth_to_point_cloud(_rgb(8, 8, 1), _smooth_depth(8, 8, 1), density="ultra")
    with pytest.raises(I2PCError):
        g.depth_to_point_cloud(_rgb(8, 8, 1), _smooth_depth(8, 8, 1), smooth=True, smooth_ksize=99)


@pytest.mark.parametrize("window", [False, True])
@pytest.mark.parametrize("density,parts", [("high", 1), ("high", 3), ("medium", 2), ("low", 4)])
def test_band_unproject_matches_whole_image(density, parts, window):
    """C4 tile-parallel mode: `parts` ranks (threads on their own streams here, with an
    in-process all-reduce as the exchange) each unproject a row band of one image; the
    concatenated bands are bit-identical to the whole-image unprojection, every rank gets
    the same p2/p98 / nanmedian stats, and the min/max of the band bboxes is the bbox."""
    dep = _smooth_depth(48, 64, 51)
    dep[3, 4] = np.nan                      # exercises the nanmedian pass as well
    _band_check(dep, _rgb(301, 410, 52), parts, density, window=window)


@pytest.mark.parametrize("ksize,parts,shape,density", [(5, 3, (48, 64, 301, 410), "high"),
                                                      (9, 4, (60, 50, 120, 100), "medium"),
                                                      (31, 5, (12, 9, 40, 30), "high"),     # halo wider than a band
                                                      (15, 8, (96, 128, 64, 128), "low")])
def test_band_smoothing_matches_whole_image_and_oracle(ksize, parts, shape, density):
    window = parts % 2 == 1                 # both selection modes
    """smooth_depth in C4's band mode (app.py:208-214): each band recomputes its normalised
    field plus the blur's k/2 halo rows (reflect-101 at the image edges, repeated for a kernel
    wider than the image), so the smoothed bands concatenate bit-identically to the whole
    image's smoothed points, which are bit-exact with the oracle's GaussianBlur."""
    h, w, H, W = shape
    dep = _smooth_depth(h, w, 111)
    dep[2, 3] = np.nan
    img = _rgb(H, W, 112)
    whole = _band_check(dep, img, parts, density, depth_scale=10.0, smooth=True, smooth_ksize=ksize, window=window)
    ep, ec = ref.depth_to_point_cloud(img, dep, density=density, depth_scale=10.0, smooth=True,
                                      smooth_ksize=ksize, loop=False)
    assert _same_bits(whole.xyz[0].cpu().numpy(), ep), _first_diff(whole.xyz[0].cpu().numpy(), ep)


def test_c4_panorama_full_size_bands_and_oracle():
    """C4 at its real size: an 8192 x 4096 panorama with 518 x 1036 model-resolution depth
    (the DA processor's keep-aspect output for it), density high (33,554,432 points).  The
    whole-image unprojection is bit-exact with the vectorised oracle, and the 8-band split
    (8 'ranks') concatenates bit-identically to it."""
    dep = _smooth_depth(518, 1036, 71)
    img = _rgb(4096, 8192, 72)
    whole = _band_check(dep, img, 8, "high", depth_scale=10.0)
    _band_check(dep, img, 8, "high", depth_scale=10.0, window=True)
    ep, ec = ref.depth_to_point_cloud(img, dep, density="high", depth_scale=10.0, loop=False)
    assert _same_bits(whole.xyz[0].cpu().numpy(), ep), _first_diff(whole.xyz[0].cpu().numpy(), ep)
    assert _same_bits(whole.rgb[0].cpu().numpy().astype(np.float32), ec)


def _band_check(dep, img, parts, density, depth_scale=12.0, projection="pinhole", smooth=False, smooth_ksize=5,
                window=False, scratch=False):
    """`parts` ranks (threads on their own streams, an in-process all-reduce / all-gather as the
    exchange) each unproject a row band; checks the bands against the whole image.  window:
    the one-sweep window mode (i2pc_unproject_band_w) instead of the histogram levels."""
    import threading
    g = _geom()
    dev = torch.device("cuda")
    H, W = img.shape[:2]
    tdep = torch.from_numpy(dep).to(dev)
    timg = torch.from_numpy(img).to(dev)
    whole = g.unproject_batch(tdep[None], timg[None], density=density, depth_scale=depth_scale,
                              projection=projection, smooth=smooth, smooth_ksize=smooth_ksize)
    torch.cuda.synchronize()
    step = g.DENSITY_STEP[density]
    bands = g.band_rows(H, parts, step)
    results, slots, errs = [None] * parts, [None] * parts, []
    bar = threading.Barrier(parts)
    nbytes = (g.band_workspace_bytes(H, W, smooth, parts) if window
              else g._lib.load().i2pc_unproject_workspace_bytes(1, H, W, int(smooth)))
    gslots = [None] * parts

    def gather_for(i):
        def ga(send, recv):
            torch.cuda.current_stream().synchronize()
            gslots[i] = send.clone()
            bar.wait()
            for r in range(parts):
                recv[parts - 1 - r].copy_(gslots[r])     # (any fixed rank order works)
            torch.cuda.current_stream().synchronize()
            bar.wait()
        return ga

    def exchange_for(i):
        def ex(hist, cnt):
            torch.cuda.current_stream().synchronize()
            slots[i] = (None if hist is None else hist.clone(), None if cnt is None else cnt.clone())
            bar.wait()
            if hist is not None:
                hist.copy_(torch.stack([s[0] for s in slots]).sum(0).to(torch.int32))
            if cnt is not None:
                c = torch.stack([s[1] for s in slots])
                cnt[:2] = c[:, :2].sum(0)
                cnt[2] = c[:, 2].min(0).values
                cnt[3] = c[:, 3].max(0).values
            torch.cuda.current_stream().synchronize()
            bar.wait()
        return ex

    def run(i):
        try:
            if scratch:                     # (thread-local knob: every rank selects from scratch)
                from image_to_pointcloud_amd import ops
                ops.set_tuning("sel_scratch", 1)
            with torch.cuda.stream(torch.cuda.Stream()):
                r0, r1 = bands[i]
                ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                results[i] = g.unproject_band(tdep, timg[r0:r1], H, W, r0, r1, exchange_for(i), density=density,
                                              depth_scale=depth_scale, workspace=ws, projection=projection,
                                              smooth=smooth, smooth_ksize=smooth_ksize,
                                              gather=gather_for(i) if window else None,
                                              nranks=parts if window else None)
                torch.cuda.current_stream().synchronize()
        except Exception as e:   # pragma: no cover - reported below
            errs.append(e)
            bar.abort()

    ts = [threading.Thread(target=run, args=(i,)) for i in range(parts)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs
    xyz = torch.cat([r[0] for r in results]).cpu().numpy()
    rgb = torch.cat([r[1] for r in results]).cpu().numpy()
    assert _same_bits(xyz, whole.xyz[0].cpu().numpy()), _first_diff(xyz, whole.xyz[0].cpu().numpy())
    assert _same_bits(rgb, whole.rgb[0].cpu().numpy())
    for r in results:
        assert _same_bits(r[3].cpu().numpy(), whole.stats[0].cpu().numpy())
    bb = torch.stack([r[2] for r in results]).cpu().numpy()
    glob = np.empty(6)
    glob[0::2] = bb[:, 0::2].min(0)
    glob[1::2] = bb[:, 1::2].max(0)
    assert _same_bits(glob, whole.bbox[0].cpu().numpy())
    return whole


@pytest.mark.parametrize("zero_frac,shape", [(0.03, (384, 384, 1024, 1024)), (0.03, (96, 128, 600, 800)),
                                              (0.5, (384, 384, 1024, 1024)), (0.9, (64, 64, 300, 300))])
def test_selection_with_a_spike_of_equal_values(zero_frac, shape):
    """Depth maps whose p2 (or p98) rank falls inside a block of exactly equal values -- a ReLU
    network's zero floor: the target's level-0 bin holds more keys than a candidate list, so the
    histogram levels must resolve it.  Whole-image and 3-band results bit-exact with the oracle."""
    h, w, H, W = shape
    dep = _smooth_depth(h, w, 101)
    rng = np.random.Generator(np.random.PCG64(102))
    blocks = 0
    while (dep == 0).mean() < zero_frac:       # square zero blocks -> exact zeros after the resize
        y, x = rng.integers(0, h - 7), rng.integers(0, w - 7)
        dep[y:y + 8, x:x + 8] = 0.0
        blocks += 1
    img = _rgb(H, W, 103)
    whole = _band_check(dep, img, 3, "high", depth_scale=10.0)
    _band_check(dep, img, 3, "high", depth_scale=10.0, window=True)   # spikes through the window exchange
    ep, ec = ref.depth_to_point_cloud(img, dep, density="high", depth_scale=10.0, loop=False)
    assert _same_bits(whole.xyz[0].cpu().numpy(), ep), _first_diff(whole.xyz[0].cpu().numpy(), ep)


def test_relu_floor_at_p2_stays_on_the_window_path():
    """Image 5 of the C2 bench batch (DPT-Large, seeded weights; 3 % exact zeros of the head's ReLU
    floor at model resolution, tests/golden/c2_relu_floor_depth.npz): the p2 rank falls on the zero
    floor, whose level-0 bin was just under the window budget, so it stayed in the window and the
    window's candidate list overflowed -- the image went to the selection from scratch on every call
    (r05, +0.64 ms per C2 step).  k_window now splits the bin off as a spike: the selection must
    resolve without the fallback (SelState.level != 16) and the points stay bit-exact vs the oracle."""
    import os
    from image_to_pointcloud_amd import geometry as G
    dep = np.load(os.path.join(os.path.dirname(__file__), "golden", "c2_relu_floor_depth.npz"))["depth"]
    dev = torch.device("cuda")
    img = _rgb(1024, 1024, 105)
    ws = torch.zeros(G.workspace_bytes(1, 1024, 1024, False), dtype=torch.uint8, device=dev)
    pb = G.unproject_batch(torch.from_numpy(dep).to(dev)[None], torch.from_numpy(img).to(dev)[None], density="high",
                           workspace=ws)
    torch.cuda.synchronize()
    state = ws[:624].cpu().numpy().view(np.uint32)
    level = int(state[344 // 4 - 1])      # SelState.level: the uint32 before p2 (offset 344)
    assert level != 16, "the ReLU-floor map went to the selection from scratch"
    ep, ec = ref.depth_to_point_cloud(img, dep, density="high", loop=False)
    assert _same_bits(pb.xyz[0].cpu().numpy(), ep), _first_diff(pb.xyz[0].cpu().numpy(), ep)
    assert _same_bits(pb.rgb[0].cpu().numpy().astype(np.float32), ec)


@pytest.mark.parametrize("density", ["high", "low"])
def test_equirect_projection_matches_oracle_and_bands(density):
    """Equirectangular mode (C4 panoramas; not in the reference, so parity is against the
    oracle's restatement only): selection / normalisation / colours bit-exact as in the pinhole
    mode, xyz within 2 float32 ulps of the float64 oracle (device sin/cos vs libm's), and the
    4-band split bit-identical to the whole image."""
    dep = _smooth_depth(64, 128, 91)
    img = _rgb(512, 1024, 92)
    whole = _band_check(dep, img, 4, density, depth_scale=10.0, projection="equirect", window=density == "high")
    ep, ec = ref.depth_to_point_cloud_equirect(img, dep, density=density, depth_scale=10.0)
    got = whole.xyz[0].cpu().numpy()
    assert got.shape == ep.shape
    ulp = np.spacing(np.maximum(np.abs(ep), np.float32(1e-30)).astype(np.float32))
    assert np.all(np.abs(got - ep) <= 2 * ulp), float(np.max(np.abs(got - ep) / ulp))
    assert _same_bits(whole.rgb[0].cpu().numpy().astype(np.float32), ec)
    pin = _geom().unproject_batch(torch.from_numpy(dep).cuda()[None], torch.from_numpy(img).cuda()[None],
                                  density=density, depth_scale=10.0)
    assert _same_bits(whole.stats[0].cpu().numpy(), pin.stats[0].cpu().numpy())
    # radius = depth: |xyz| equals the pinhole z (the normalised depth times the scale)
    r = np.linalg.norm(got.astype(np.float64), axis=1)
    np.testing.assert_allclose(r, pin.xyz[0, :, 2].cpu().numpy().astype(np.float64), rtol=1e-6, atol=1e-6)
    print("parity", {"case": f"equirect {density}", "bit_exact_frac": float(np.mean(got == ep))})


def test_band_rccl_exchange_single_rank_and_graph_capture():
    """C4 with the device-side exchange: a one-rank RCCL communicator (i2pc_comm_create) drives
    i2pc_unproject_band_rccl over the whole image -- bit-identical to i2pc_unproject -- and the
    same call captured into a HIP graph replays to the same bytes (no host callback inside)."""
    from image_to_pointcloud_amd.distributed import RcclComm
    g = _geom()
    dev = torch.device("cuda")
    dep = _smooth_depth(96, 128, 81)
    img = _rgb(600, 800, 82)
    tdep, timg = torch.from_numpy(dep).to(dev), torch.from_numpy(img).to(dev)
    whole = g.unproject_batch(tdep[None], timg[None], density="high")
    comm = RcclComm(nranks=1, rank=0)
    ws = torch.empty(g.band_workspace_bytes(600, 800, False, 1), dtype=torch.uint8, device=dev)
    xyz, rgb, bbox, stats = g.unproject_band(tdep, timg, 600, 800, 0, 600, comm=comm, workspace=ws)
    torch.cuda.synchronize()
    assert _same_bits(xyz.cpu().numpy(), whole.xyz[0].cpu().numpy())
    assert _same_bits(stats.cpu().numpy(), whole.stats[0].cpu().numpy())
    out = (torch.zeros_like(xyz), torch.zeros_like(rgb), torch.zeros_like(bbox), torch.zeros_like(stats))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.unproject_band(tdep, timg, 600, 800, 0, 600, comm=comm, workspace=ws, out=out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g.unproject_band(tdep, timg, 600, 800, 0, 600, comm=comm, workspace=ws, out=out)
    for t in out:
        t.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert _same_bits(out[0].cpu().numpy(), whole.xyz[0].cpu().numpy())
    assert _same_bits(out[1].cpu().numpy(), whole.rgb[0].cpu().numpy())
    comm.close()


@pytest.mark.parametrize("shape,density", [((60, 90, 120, 720), "high"),        # 180 threads/row -> tpr 192, one idle wave
                                           ((50, 257, 40, 2056), "high"),       # 3 column tiles, the last 8 points
                                           ((64, 80, 300, 1200), "medium"),     # step 2: 600 points/row, tpr 192
                                           ((40, 40, 77, 1040), "low"),         # step 4: 260 points/row, tpr 128
                                           ((96, 128, 200, 256), "high")])      # 64 threads/row, 4 rows per pass
@pytest.mark.parametrize("rpt", [8, 3, 1])
def test_row_kernel_layouts_match_fast_kernel_and_oracle(shape, density, rpt):
    """k_unproject_rows over its thread layouts (threads per row 64/128/192/256, idle waves,
    partial column tiles, steps 1/2/4, 1-8 rows per thread) against k_unproject_fast
    (i2pc_set_tuning('unp_rows', 0)) bit for bit, and the oracle; NaN fill and invert on."""
    from image_to_pointcloud_amd import ops
    h, w, H, W = shape
    g = _geom()
    dev = torch.device("cuda")
    B = 3
    deps = np.stack([_smooth_depth(h, w, 40 + i) for i in range(B)])
    deps[1, 3, 4] = np.nan
    imgs = np.stack([_rgb(H, W, 50 + i) for i in range(B)])
    outs = []
    try:
        for rows in (1, 0):
            ops.set_tuning("unp_rows", rows)
            ops.set_tuning("unp_rpt", rpt)
            pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev), density=density,
                                   invert=True, depth_scale=7.5)
            outs.append((pb.xyz.cpu().numpy(), pb.rgb.cpu().numpy(), pb.bbox.cpu().numpy()))
    finally:
        ops.set_tuning("unp_rows", 1)
        ops.set_tuning("unp_rpt", 8)
    for a, b in zip(outs[0], outs[1]):
        assert _same_bits(a, b), _first_diff(a, b)
    for i in (0, 1):
        with np.errstate(all="ignore"):
            ep, ec = ref.depth_to_point_cloud(imgs[i], deps[i], density=density, invert=True, depth_scale=7.5,
                                              loop=False)
        assert _same_bits(outs[0][0][i], ep), (i, _first_diff(outs[0][0][i], ep))
        assert _same_bits(outs[0][1][i].astype(np.float32), ec)


def test_row_kernel_equirect_matches_fast_kernel():
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    dep = torch.from_numpy(_smooth_depth(64, 128, 7)[None]).to(dev)
    img = torch.from_numpy(_rgb(256, 1100, 8)[None]).to(dev)
    outs = []
    try:
        for rows in (1, 0):
            ops.set_tuning("unp_rows", rows)
            pb = g.unproject_batch(dep, img, density="high", projection="equirect")
            outs.append(pb.xyz.cpu().numpy())
    finally:
        ops.set_tuning("unp_rows", 1)
    assert _same_bits(outs[0], outs[1]), _first_diff(outs[0], outs[1])


def _sel_cases():
    """Maps that stress the window-only selection (k_sweep_w / k_resolve_w): spikes of equal
    values at either percentile (zero floor / saturated maximum, just inside and just outside the
    rank), quantised values, NaN / Inf, constant and tiny maps."""
    rng = np.random.Generator(np.random.PCG64(7))
    base = _smooth_depth(96, 128, 61)
    out = {"smooth": base}
    for frac in (0.015, 0.0199, 0.0201, 0.025, 0.3):          # zero floor around the p2 rank
        d = base.copy()
        d.ravel()[rng.permutation(d.size)[:int(frac * d.size)]] = 0.0
        out[f"zero_{frac}"] = d
    for frac in (0.019, 0.0205, 0.05):                          # saturated maximum around p98
        d = base.copy()
        d.ravel()[rng.permutation(d.size)[:int(frac * d.size)]] = np.float32(base.max())
        out[f"sat_{frac}"] = d
    # a spike window next to the nanmedian fill's third window (k_sweep_w's per-wave spike and
    # below-window counts share one LDS row: r03 laid window 0's spike count over below[2])
    for k in ("zero_0.025", "zero_0.3", "sat_0.05"):
        d = out[k].copy(); d[7, 8] = np.nan; d[50, 90] = np.nan
        out[k + "_nan"] = d
    out["quantised"] = (np.round(base * 16) / 16).astype(np.float32)
    out["two_valued"] = np.where(rng.random(base.shape) < 0.5, 1.0, 2.0).astype(np.float32)
    d = base.copy(); d[3, 4] = np.nan; d[10, 11] = np.inf; d[20, 0] = -np.inf
    out["nan_inf"] = d
    d = base.copy(); d.ravel()[rng.permutation(d.size)[:d.size * 2 // 5]] = np.nan
    out["nan_40pct"] = d
    # sparse non-finite pixels (a few % of the resized map): the unread twin of each percentile
    # pair lies k ranks outside every window and is skipped by rank (fill_targets)
    d = base.copy(); idx = rng.permutation(d.size)[:d.size // 200]
    d.ravel()[idx[0::3]] = np.nan; d.ravel()[idx[1::3]] = np.inf; d.ravel()[idx[2::3]] = -np.inf
    out["sparse_nonfinite"] = d
    # +-inf in the last model column and row: cv2's single-tap border copies them unblended, so the
    # resized map holds +-inf there, not the NaN an inf * 0 weight would make
    d = base.copy(); d[5:40, -1] = np.inf; d[-1, 7:30] = -np.inf
    out["inf_border"] = d
    out["constant"] = np.full_like(base, 2.5)
    # p2 == p98 with a wider range: the min / max branch (app.py:198-199) from a range-only pass
    d = np.full_like(base, 1.0)
    d.ravel()[rng.permutation(d.size)[:d.size // 100]] = rng.uniform(0.5, 3.0, d.size // 100).astype(np.float32)
    out["near_constant"] = d
    d = d.copy(); d[4, 9] = np.nan
    out["near_constant_nan"] = d
    out["all_nan"] = np.full_like(base, np.nan)
    # the nanmedian's middle pair near FLT_MAX: np.mean of them in float32 overflows to +inf, so the
    # ranks above the median no longer read max(F(r - k), med) -- the window paths must not drop
    # F(r) there (fill_targets / finish_targets)
    d = base.copy(); idx = rng.permutation(d.size)
    d.ravel()[idx[:d.size * 9 // 10]] = np.float32(3.0e38); d.ravel()[idx[-3:]] = np.nan
    out["huge_median_nan"] = d
    return out


@pytest.mark.parametrize("size", [(300, 400), (96, 128)])
def test_window_selection_matches_histogram_levels_and_oracle(size):
    """The batch path's window-only selection against the histogram levels (i2pc_set_tuning
    'sel_windows' 0) and the oracle, bit for bit, on maps built to make windows miss."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    H, W = size
    cases = _sel_cases()
    names = list(cases)
    deps = np.stack([cases[k] for k in names])
    imgs = np.stack([_rgb(H, W, 70 + i) for i in range(len(names))])
    outs = []
    try:
        for win in (1, 0):
            ops.set_tuning("sel_windows", win)
            pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev), density="high",
                                   invert=True, depth_scale=10.0)
            outs.append((pb.xyz.cpu().numpy(), pb.stats.cpu().numpy()))
    finally:
        ops.set_tuning("sel_windows", 1)
    for i, k in enumerate(names):
        assert _same_bits(outs[0][1][i], outs[1][1][i]), (k, outs[0][1][i], outs[1][1][i])
        assert _same_bits(outs[0][0][i], outs[1][0][i]), (k, _first_diff(outs[0][0][i], outs[1][0][i]))
        with np.errstate(all="ignore"):
            ep, _ = ref.depth_to_point_cloud(imgs[i], deps[i], density="high", invert=True, depth_scale=10.0,
                                             loop=False)
        assert _same_bits(outs[0][0][i], ep), (k, _first_diff(outs[0][0][i], ep))


def test_selection_from_scratch_matches_windows_and_oracle():
    """The selection from scratch (the fallback of a missed window: k_sel_slow's level 0 and the
    k_scratch radix levels, grid-wide; knob sel_scratch forces it) gives the window path's bits on
    every stress map, NaN / Inf fills, constant and all-NaN maps included, and the oracle's."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    H, W = 300, 400
    cases = _sel_cases()
    names = list(cases)
    deps = np.stack([cases[k] for k in names])
    imgs = np.stack([_rgb(H, W, 170 + i) for i in range(len(names))])
    outs = []
    try:
        for scr in (0, 1):
            ops.set_tuning("sel_scratch", scr)
            pb = g.unproject_batch(torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev), density="high",
                                   invert=True, depth_scale=10.0)
            outs.append((pb.xyz.cpu().numpy(), pb.stats.cpu().numpy()))
    finally:
        ops.set_tuning("sel_scratch", 0)
    for i, k in enumerate(names):
        assert _same_bits(outs[0][1][i], outs[1][1][i]), (k, outs[0][1][i], outs[1][1][i])
        assert _same_bits(outs[0][0][i], outs[1][0][i]), (k, _first_diff(outs[0][0][i], outs[1][0][i]))
        with np.errstate(all="ignore"):
            ep, _ = ref.depth_to_point_cloud(imgs[i], deps[i], density="high", invert=True, depth_scale=10.0,
                                             loop=False)
        assert _same_bits(outs[1][0][i], ep), (k, _first_diff(outs[1][0][i], ep))


@pytest.mark.parametrize("parts", [1, 3])
def test_band_selection_from_scratch(parts):
    """C4 band mode with every rank forced to the selection from scratch (each rank selects the whole
    image; no exchange): bands still concatenate bit-identically to the whole image."""
    dep = _smooth_depth(48, 64, 151)
    dep[3, 4] = np.nan
    _band_check(dep, _rgb(301, 410, 152), parts, "high", window=True, scratch=True)


def test_panorama_selection_from_scratch_time():
    """One 8192 x 4096 panorama forced to the selection from scratch (~95 ms when one
    workgroup did it): bit-identical to the window path, and well under 3 ms per call."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    dep = torch.from_numpy(_smooth_depth(518, 1036, 171)).to(dev)[None]
    img = torch.from_numpy(_rgb(4096, 8192, 172)).to(dev)[None]
    ws = torch.empty(g.workspace_bytes(1, 4096, 8192), dtype=torch.uint8, device=dev)
    ref_out = g.unproject_batch(dep, img, density="high", workspace=ws)
    ref_xyz, ref_stats = ref_out.xyz.cpu().numpy(), ref_out.stats.cpu().numpy()
    try:
        ops.set_tuning("sel_scratch", 1)
        got = g.unproject_batch(dep, img, density="high", workspace=ws)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.unproject_batch(dep, img, density="high", workspace=ws, out=got)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
    finally:
        ops.set_tuning("sel_scratch", 0)
    print(f"parity {{\"test\": \"panorama_scratch\", \"ms_per_call\": {ms:.3f}}}")
    assert _same_bits(got.xyz.cpu().numpy(), ref_xyz)
    assert _same_bits(got.stats.cpu().numpy(), ref_stats)
    assert ms < 3.0, ms


@pytest.mark.parametrize("parts", [1, 2, 3, 4])
def test_forked_selection_parts_bit_identical(parts):
    """i2pc_unproject's selection chain as 1-4 sub-batches on forked side streams (knob sel_parts),
    joined before one unprojection launch: bit-identical to one chain and to the oracle, and the
    same under HIP graph capture (the fork is captured through its events)."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    B, h, w, H, W = 17, 48, 64, 96, 128
    deps = np.stack([_smooth_depth(h, w, 500 + i) for i in range(B)])
    deps[5, 2, 3] = np.nan
    imgs = np.stack([_rgb(H, W, 600 + i) for i in range(B)])
    tdep, timg = torch.from_numpy(deps).to(dev), torch.from_numpy(imgs).to(dev)
    ws = torch.empty(g.workspace_bytes(B, H, W), dtype=torch.uint8, device=dev)
    try:
        ops.set_tuning("sel_parts", 1)
        one = g.unproject_batch(tdep, timg, density="high", workspace=ws)
        torch.cuda.synchronize()
        ref_xyz, ref_stats = one.xyz.cpu().numpy(), one.stats.cpu().numpy()
        ops.set_tuning("sel_parts", parts)
        got = g.unproject_batch(tdep, timg, density="high", workspace=ws)
        torch.cuda.synchronize()
        assert _same_bits(got.xyz.cpu().numpy(), ref_xyz)
        assert _same_bits(got.stats.cpu().numpy(), ref_stats)
        out = g.PointBatch(torch.zeros_like(got.xyz), torch.zeros_like(got.rgb), torch.zeros_like(got.bbox),
                           torch.zeros_like(got.stats))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g.unproject_batch(tdep, timg, density="high", workspace=ws, out=out)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g.unproject_batch(tdep, timg, density="high", workspace=ws, out=out)
        out.xyz.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert _same_bits(out.xyz.cpu().numpy(), ref_xyz)
    finally:
        ops.set_tuning("sel_parts", 0)
    for i in (0, 5, 16):
        ep, _ = ref.depth_to_point_cloud(imgs[i], deps[i], density="high", loop=False)
        assert _same_bits(ref_xyz[i], ep), i


@pytest.mark.parametrize("size", [(300, 400), (96, 128)])
def test_single_image_local_band_chain_matches_resolve_and_oracle(size):
    """A single image's windows resolved through the band kernels with a local exchange (knob
    sel_lband 1; automatic from 4 M pixels) against k_resolve_w (sel_lband 0) and the oracle, bit for
    bit, on the maps built to make windows miss (spikes, NaN / Inf, constant, all-NaN)."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    H, W = size
    cases = _sel_cases()
    try:
        for i, (k, dep) in enumerate(cases.items()):
            img = _rgb(H, W, 90 + i)
            td, ti = torch.from_numpy(dep[None]).to(dev), torch.from_numpy(img[None]).to(dev)
            outs = []
            for lb in (1, 0):
                ops.set_tuning("sel_lband", lb)
                pb = g.unproject_batch(td, ti, density="high", invert=True, depth_scale=10.0)
                outs.append((pb.xyz.cpu().numpy()[0], pb.stats.cpu().numpy()[0]))
            assert _same_bits(outs[0][1], outs[1][1]), (k, outs[0][1], outs[1][1])
            assert _same_bits(outs[0][0], outs[1][0]), (k, _first_diff(outs[0][0], outs[1][0]))
            with np.errstate(all="ignore"):
                ep, _ = ref.depth_to_point_cloud(img, dep, density="high", invert=True, depth_scale=10.0, loop=False)
            assert _same_bits(outs[0][0], ep), (k, _first_diff(outs[0][0], ep))
    finally:
        ops.set_tuning("sel_lband", -1)


def test_single_large_image_local_band_chain_bit_identical():
    """A 2048 x 4096 image (above the automatic threshold) with a NaN patch: the local band chain,
    k_resolve_w and numpy's percentiles agree."""
    from image_to_pointcloud_amd import ops
    g = _geom()
    dev = torch.device("cuda")
    H, W, h, w = 2048, 4096, 518, 1036
    dep = _smooth_depth(h, w, 77)
    dep[100:120, 200:260] = np.nan
    img = _rgb(H, W, 78)
    td, ti = torch.from_numpy(dep[None]).to(dev), torch.from_numpy(img[None]).to(dev)
    outs = []
    try:
        for lb in (-1, 0):
            ops.set_tuning("sel_lband", lb)
            pb = g.unproject_batch(td, ti, density="high")
            outs.append((pb.xyz.cpu().numpy()[0], pb.stats.cpu().numpy()[0]))
    finally:
        ops.set_tuning("sel_lband", -1)
    assert _same_bits(outs[0][1], outs[1][1]), (outs[0][1], outs[1][1])
    assert _same_bits(outs[0][0], outs[1][0]), _first_diff(outs[0][0], outs[1][0])

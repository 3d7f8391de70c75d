"""The persistent 256-column GEMM engines (single-stage k_gemm_p, ping-pong k_gemm_8p) against the
tile kernel (bit-exact) and torch fp32; split-K against the unsplit tile kernel and torch fp32.

Both engines accumulate the same MFMA sequence and apply the epilogue in the same
fp32 order (bias, activation, residual, second residual, bf16 rounding), so their
outputs must be identical bit for bit.  Shapes cover several tiles per workgroup
(more tiles than CUs: the cross-tile prefetch and counted epilogue waits), a
partial last M-tile, K = 64 (one K-step per tile), and every epilogue the engine
implements.  torch tolerance: relative Frobenius error <= 8e-3.
"""
import ctypes
import math

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
F = torch.nn.functional


def _ops():
    from image_to_pointcloud_amd import ops
    return ops


def _bf(x):
    return x.to(torch.bfloat16)


def _both(fn):
    """(persistent engine forced, tile kernel) outputs; the ping-pong engine (k_gemm_8p, forced
    wherever it applies) and the automatic choice must equal both."""
    ops = _ops()
    outs = []
    try:
        for mode in (1, 2, 4):
            ops.set_gemm_engine(mode)
            outs.append(fn().clone())
    finally:
        ops.set_gemm_engine(0)
    try:   # split-K (automatic modes) adds partial sums in another order: compared below
        ops.set_tuning("gemm_splitk", 0)
        auto = fn().clone()
    finally:
        ops.set_tuning("gemm_splitk", 1)
    split = fn()
    torch.cuda.synchronize()
    assert torch.equal(auto, outs[0]), "automatic engine choice differs from the tile kernel"
    assert _fro(split, outs[0]) <= 2e-3, f"split-K vs unsplit: {_fro(split, outs[0])}"
    assert torch.equal(outs[2], outs[0]), \
        f"ping-pong engine differs from the tile kernel: {(outs[2].float() - outs[0].float()).abs().max().item()}"
    return outs[1], outs[0]


def _fro(got, ref):
    got, ref = got.float(), ref.float()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,N,K,act", [(8200, 2048, 1024, None), (18464, 3072, 64, "gelu"), (9000, 1024, 192, None), (4100, 4096, 512, "gelu"),
                                       (300, 256, 512, None), (257, 512, 128, "relu"), (20000, 384, 512, "gelu"),
                                       (18464, 4096, 1024, "gelu"), (43840, 1536, 384, "gelu")])
def test_linear_plain_engines_bitexact(M, N, K, act):
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = _bf(torch.randn(M, K, generator=g)).to(dev)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    got, ref = _both(lambda: ops.linear(x, w, bias=b, act=act, out=out))
    try:
        ops.set_gemm_engine(2)
        lab = ops.gemm_kernel_label(_desc_of(ops, x, w, b, out))
        assert "k_gemm_p" in lab, "persistent engine not selected"
        ops.set_gemm_engine(4)
        lab = ops.gemm_kernel_label(_desc_of(ops, x, w, b, out))
        assert ("k_gemm_8p" in lab) == (K >= 128 and N % 256 == 0), lab
    finally:
        ops.set_gemm_engine(0)
    assert torch.equal(got, ref), f"engines differ: {(got.float() - ref.float()).abs().max().item()}"
    y = x.float() @ w.float().T + b
    y = F.gelu(y) if act == "gelu" else F.relu(y) if act == "relu" else y
    assert _fro(got, y) <= 8e-3


def _desc_of(ops, x, w, b, out):
    d = ops.GemmDesc()
    d.a, d.lda, d.m, d.n, d.k = x.data_ptr(), x.stride(0), x.shape[0], w.shape[0], w.shape[1]
    d.w, d.ldw = w.data_ptr(), w.stride(0)
    d.bias = b.data_ptr()
    d.c, d.ldc = out.data_ptr(), out.stride(0)
    return d


@pytest.mark.parametrize("M,N,K", [(8200, 1024, 1024), (18464, 1024, 4096), (1000, 256, 192)])
def test_linear_residual_f32_engines_bitexact(M, N, K):
    """Transformer residual: out = x + (h @ W^T + b), fp32 stream updated in place."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(M * 3 + K)
    h = _bf(torch.randn(M, K, generator=g)).to(dev)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    x0 = torch.randn(M, N, generator=g).to(dev)

    def run():
        x = x0.clone()
        ops.linear(h, w, bias=b, res=x, out=x)
        return x
    got, ref = _both(run)
    assert torch.equal(got, ref)
    assert _fro(got, x0 + h.float() @ w.float().T + b) <= 8e-3


def _pack_conv(w):
    return _bf(w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)).contiguous()


@pytest.mark.parametrize("B,H,W,C,Co,stride", [(20, 64, 64, 256, 256, 1), (4, 48, 48, 512, 256, 2),
                                                (3, 37, 29, 256, 256, 1), (8, 96, 96, 256, 128, 1)])
def test_conv_engines_bitexact(B, H, W, C, Co, stride):
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(B + H + C)
    x = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
    w = (torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev)
    b = torch.randn(Co, generator=g).to(dev)
    wp = _pack_conv(w)
    got, ref = _both(lambda: ops.conv2d(x, wp, bias=b, stride=stride))
    assert torch.equal(got, ref)
    r = F.conv2d(x.float().permute(0, 3, 1, 2), _bf(w).float(), b, stride=stride, padding=1).permute(0, 2, 3, 1)
    assert _fro(got, r) <= 8e-3


def test_conv_residual_units_engines_bitexact():
    """Pre-activation residual unit: ReLU-in conv + ReLU, then conv + bias + res + res2 (and res only)."""
    ops = _ops()
    dev = torch.device("cuda")
    B, H, W, C = 20, 48, 48, 256
    g = torch.Generator(device="cpu").manual_seed(11)
    x = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
    hid = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
    w1 = _pack_conv(torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev)
    w2 = _pack_conv(torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev)
    b1 = (torch.randn(C, generator=g) * 0.1).to(dev)
    b2 = (torch.randn(C, generator=g) * 0.1).to(dev)
    y1, r1 = _both(lambda: ops.conv2d(x, w1, bias=b1, relu_in=True, act="relu"))
    assert torch.equal(y1, r1)
    y2, r2 = _both(lambda: ops.conv2d(y1, w2, bias=b2, res=x, res2=hid))
    assert torch.equal(y2, r2)
    y3, r3 = _both(lambda: ops.conv2d(y1, w2, bias=b2, res=x))
    assert torch.equal(y3, r3)


@pytest.mark.parametrize("s,C", [(4, 256), (2, 512)])
def test_conv_transpose_engines_bitexact(s, C):
    ops = _ops()
    dev = torch.device("cuda")
    B, H, W = 16, 24, 24
    g = torch.Generator(device="cpu").manual_seed(s + C)
    x = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
    w = (torch.randn(C, C, s, s, generator=g) / math.sqrt(C)).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    wp = _bf(w.permute(2, 3, 1, 0).reshape(s * s * C, C)).contiguous()
    bt = b.repeat(s * s).contiguous()
    got, ref = _both(lambda: ops.conv_transpose(x, wp, bt, s))
    assert torch.equal(got, ref)
    r = F.conv_transpose2d(x.float().permute(0, 3, 1, 2), _bf(w).float(), b, stride=s).permute(0, 2, 3, 1)
    assert _fro(got, r) <= 8e-3


def _label_of_conv(ops, x, w, k, stride, relu_in):
    B, H, W, C = x.shape
    OH, OW = (H + 2 - k) // stride + 1, (W + 2 - k) // stride + 1
    d = ops.GemmDesc()
    d.a, d.m, d.n, d.k = x.data_ptr(), B * OH * OW, w.shape[0], w.shape[1]
    d.conv, d.conv_batch, d.conv_h, d.conv_w, d.conv_c = 1, B, H, W, C
    d.conv_oh, d.conv_ow, d.conv_k, d.conv_stride, d.conv_pad, d.conv_relu_in = OH, OW, k, stride, 1, int(relu_in)
    d.w, d.ldw = w.data_ptr(), w.stride(0)
    d.c, d.ldc = x.data_ptr(), w.shape[0]
    return ops.gemm_kernel_label(d), ops._lib.load().i2pc_gemm_workspace_bytes(ctypes.byref(d))


@pytest.mark.parametrize("B,H,C,Co,stride,mode", [(32, 12, 1024, 256, 1, "plain"), (32, 24, 1024, 256, 1, "plain"),
                                                  (32, 24, 1024, 1024, 2, "plain"), (32, 12, 512, 256, 1, "relu"),
                                                  (32, 12, 512, 256, 1, "res2"), (7, 24, 512, 128, 1, "plain")])
def test_conv_split_k(B, H, C, Co, stride, mode):
    """Few-tile long-K convs of the DPT neck (12x12 / 24x24 maps, K = 9 * Cin) run split-K: the
    label says so, the workspace size is what the plan needs, results are deterministic, within
    2e-3 (relative Frobenius) of the unsplit tile kernel and 8e-3 of torch fp32."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(B + H + C + Co)
    x = _bf(torch.randn(B, H, H, C, generator=g)).to(dev)
    w = (torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev)
    b = (torch.randn(Co, generator=g) * 0.1).to(dev)
    wp = _pack_conv(w)
    OH = (H - 1) // stride + 1
    r1 = _bf(torch.randn(B, OH, OH, Co, generator=g)).to(dev)
    r2 = _bf(torch.randn(B, OH, OH, Co, generator=g)).to(dev)
    relu_in = mode == "relu"
    kw = dict(bias=b, stride=stride, relu_in=relu_in, act="relu" if relu_in else None)
    if mode == "res2":
        kw.update(res=r1, res2=r2)
    lab, nb = _label_of_conv(ops, x, wp, 3, stride, relu_in)
    assert "split-K" in lab and nb > 0, lab
    got = ops.conv2d(x, wp, **kw).clone()
    again = ops.conv2d(x, wp, **kw)
    assert torch.equal(got, again), "split-K is not deterministic"
    try:
        ops.set_tuning("gemm_splitk", 0)
        assert "split-K" not in _label_of_conv(ops, x, wp, 3, stride, relu_in)[0]
        unsplit = ops.conv2d(x, wp, **kw).clone()
    finally:
        ops.set_tuning("gemm_splitk", 1)
    e_unsplit = _fro(got, unsplit)
    xin = F.relu(x.float()) if relu_in else x.float()
    r = F.conv2d(xin.permute(0, 3, 1, 2), _bf(w).float(), b, stride=stride, padding=1).permute(0, 2, 3, 1)
    if relu_in:
        r = F.relu(r)
    if mode == "res2":
        r = r + r1.float() + r2.float()
    e_ref = _fro(got, r)
    print(f"split-K {lab}: vs unsplit {e_unsplit:.2e}, vs torch fp32 {e_ref:.2e}")
    assert e_unsplit <= 2e-3 and e_ref <= 8e-3


@pytest.mark.parametrize("M,N,K,act", [(300, 256, 4096, "gelu"), (32, 1024, 1024, None)])
def test_linear_split_k(M, N, K, act):
    """A dense few-tile long-K GEMM splits (16 slices here); K = 1024 (the CLS readout) does not."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(M + K)
    x = _bf(torch.randn(M, K, generator=g)).to(dev)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    lab = ops.gemm_kernel_label(_desc_of(ops, x, w, b, out))
    assert ("split-K" in lab) == (K >= 4096), lab
    got = ops.linear(x, w, bias=b, act=act, out=out).clone()
    try:
        ops.set_tuning("gemm_splitk", 0)
        unsplit = ops.linear(x, w, bias=b, act=act, out=out).clone()
    finally:
        ops.set_tuning("gemm_splitk", 1)
    y = x.float() @ w.float().T + b
    y = F.gelu(y) if act == "gelu" else y
    assert _fro(got, unsplit) <= 2e-3 and _fro(got, y) <= 8e-3


@pytest.mark.parametrize("M,N,K,res", [(43840, 384, 1536, True), (43840, 384, 384, True), (5000, 384, 640, False)])
def test_tile_384x192_bitexact(M, N, K, res):
    """Depth-Anything-V2-Small's N = 384 GEMMs (FC2, attention-out: fp32 residual) on one round of
    384 x 192 tiles: bit-identical to the 128 x 128 tiles they replace, within 8e-3 of torch fp32."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    h = _bf(torch.randn(M, K, generator=g)).to(dev)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    x0 = torch.randn(M, N, generator=g).to(dev)

    def run():
        if res:
            x = x0.clone()
            ops.linear(h, w, bias=b, res=x, out=x)
            return x
        return ops.linear(h, w, bias=b, act="gelu").clone()
    d = _desc_of(ops, h, w, b, x0)
    lab = ops.gemm_kernel_label(d)
    assert lab.startswith("k_gemm<384, 192") == (M >= 40000), lab
    got = run()
    try:
        ops.set_tuning("gemm_tile192", 0)
        assert not ops.gemm_kernel_label(d).startswith("k_gemm<384, 192")
        ref = run()
    finally:
        ops.set_tuning("gemm_tile192", 1)
    assert torch.equal(got, ref)
    y = h.float() @ w.float().T + b
    y = x0 + y if res else F.gelu(y)
    assert _fro(got, y) <= 8e-3


@pytest.mark.parametrize("lnf", [False, True])
@pytest.mark.parametrize("M,N", [(18464, 4096), (6500, 4096)])
def test_tail160_bitexact(M, N, lnf):
    """A persistent GEMM whose last partial round runs as 160 x 256 tiles (knob gemm_tail160; DPT-Large
    FC1: 4 rounds of 256^2 + 13 x 16 tiles of 160 rows) computes every output exactly as the
    un-split launch: plain GELU epilogue and the LayerNorm-fold consumer (EPI_LNF)."""
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(M + N + lnf)
    K = 1024
    x = ((torch.rand(M, K, generator=g) * 2 - 1)).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    kw = {}
    if lnf:
        kw = dict(ln_rows=torch.stack([torch.rand(M, generator=g) + 0.5, torch.randn(M, generator=g)], 1).to(dev),
                  col_sum=torch.randn(N, generator=g).to(dev))
    outs = []
    try:
        for on in (1, 0):
            ops.set_tuning("gemm_tail160", on)
            outs.append(ops.linear(x, w, bias=b, act="gelu", **kw))
            torch.cuda.synchronize()
    finally:
        ops.set_tuning("gemm_tail160", 1)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


@pytest.mark.parametrize("M,N,K,act,res", [(18464, 3072, 1024, None, False), (18464, 4096, 1024, "gelu", False),
                                           (18464, 1024, 1024, None, True), (18464, 1024, 4096, None, True),
                                           (43840, 384, 1536, None, True), (6000, 2048, 640, None, False)])
def test_stagger_bitexact(M, N, K, act, res):
    """gemm_stagger (waves 4-7 issue the next K-stage half-way through the step) changes only when the
    LDS-DMA loads are issued, never what is multiplied: outputs are bit-identical with it off, on the
    persistent engine (QKV / FC1 shapes), the 320 x 256 and 384 x 192 tile kernels (O / FC2 shapes)."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = _bf(torch.randn(M, K, generator=g)).to(dev)
    w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    x0 = torch.randn(M, N, generator=g).to(dev)
    outs = []
    try:
        for on in (1, 0):
            ops.set_tuning("gemm_stagger", on)
            if res:
                y = x0.clone()
                ops.linear(x, w, bias=b, res=y, out=y)
            else:
                y = ops.linear(x, w, bias=b, act=act)
            torch.cuda.synchronize()
            outs.append(y)
    finally:
        ops.set_tuning("gemm_stagger", 1)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,H,W,Co", [(32, 148, 148, 64), (3, 37, 29, 64), (2, 19, 19, 128), (4, 296, 296, 64),
                                      (1, 5, 70, 64)])
def test_conv3_halo_bitexact(B, H, W, Co):
    """The 64-channel 3x3 convs of Depth-Anything-V2-Small's fusion / head on k_conv3_halo (one input
    halo per 16 x 16 output pixels in LDS; knob conv_halo) equal the implicit-GEMM tile kernel bit for
    bit -- same K order (tap-major, two 32-k sub-steps) -- for the unit's three epilogues (ReLU-in +
    bias + ReLU; bias + res + res2; bias + res), image sizes that leave partial tiles and several
    N-tiles; and torch fp32 within 8e-3."""
    ops = _ops()
    dev = torch.device("cuda")
    C = 64
    g = torch.Generator(device="cpu").manual_seed(B * 7 + H + Co)
    x = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
    res = _bf(torch.randn(B, H, W, Co, generator=g)).to(dev)
    res2 = _bf(torch.randn(B, H, W, Co, generator=g)).to(dev)
    w = (torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev)
    b = (torch.randn(Co, generator=g) * 0.1).to(dev)
    wp = _pack_conv(w)
    cases = [dict(relu_in=True, act="relu"), dict(res=res, res2=res2), dict(res=res)]
    d = ops.GemmDesc()
    d.a = d.w = d.c = 16
    d.m, d.n, d.k, d.lda, d.ldw, d.ldc = B * H * W, Co, 9 * C, C, 9 * C, Co
    d.conv, d.conv_batch, d.conv_h, d.conv_w, d.conv_c = 1, B, H, W, C
    d.conv_oh, d.conv_ow, d.conv_k, d.conv_stride, d.conv_pad = H, W, 3, 1, 1
    assert ops.gemm_kernel_label(d).startswith("k_conv3_halo<"), ops.gemm_kernel_label(d)
    for kw in cases:
        outs = []
        try:
            for on in (3, 0):
                ops.set_tuning("conv_halo", on)
                outs.append(ops.conv2d(x, wp, bias=b, **kw).clone())
        finally:
            ops.set_tuning("conv_halo", 3)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), (kw.keys(), (outs[0].float() - outs[1].float()).abs().max().item())
        xin = F.relu(x.float()) if kw.get("relu_in") else x.float()
        r = F.conv2d(xin.permute(0, 3, 1, 2), _bf(w).float(), b, padding=1).permute(0, 2, 3, 1)
        if kw.get("act") == "relu":
            r = F.relu(r)
        if "res" in kw:
            r = r + res.float()
        if "res2" in kw:
            r = r + res2.float()
        assert _fro(outs[0], r) <= 8e-3


@pytest.mark.parametrize("case", ["linear", "linear_384", "conv", "halo", "splitk", "f32res"])
def test_simple_epilogue_bitexact(case):
    """The tile / halo-conv kernels' compiled-down epilogues (gemm_simple_epi 1: bias, activation, a bf16
    residual, bf16 out) write the bytes of the generic epilogue (gemm_simple_epi 0) for every combination
    they take (a second bf16 residual included), and the fp32 one (split-K's partial sums; bias + an fp32
    residual stream in place, DPT-Hybrid's bf16 FC2)."""
    ops = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(len(case))
    calls = []
    if case == "f32res":
        M, N, K = 3000, 768, 1024
        a = _bf(torch.randn(M, K, generator=g)).to(dev)
        w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
        b = (torch.randn(N, generator=g) * 0.1).to(dev)
        x0 = torch.randn(M, N, generator=g).to(dev)

        def inplace():
            x = x0.clone()
            return ops.linear(a, w, bias=b, res=x, out=x)
        calls.append(inplace)
    elif case == "splitk":
        M, N, K = 300, 256, 4096
        a = _bf(torch.randn(M, K, generator=g)).to(dev)
        w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
        b = (torch.randn(N, generator=g) * 0.1).to(dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        assert "split-K" in ops.gemm_kernel_label(_desc_of(ops, a, w, b, out))
        for act in (None, "gelu"):
            calls.append(lambda act=act: ops.linear(a, w, bias=b, act=act))
    elif case in ("linear", "linear_384"):
        M, N, K = (2000, 1024, 512) if case == "linear" else (43840, 384, 384)
        a = _bf(torch.randn(M, K, generator=g)).to(dev)
        w = _bf(torch.randn(N, K, generator=g) / math.sqrt(K)).to(dev)
        b = (torch.randn(N, generator=g) * 0.1).to(dev)
        r = _bf(torch.randn(M, N, generator=g)).to(dev)
        for act in (None, "relu", "gelu"):
            for res in (None, r):
                calls.append(lambda act=act, res=res: ops.linear(a, w, bias=b, act=act, res=res))
    else:
        B, H, W, C, Co = (4, 48, 40, 256, 256) if case == "conv" else (3, 37, 29, 64, 64)
        x = _bf(torch.randn(B, H, W, C, generator=g)).to(dev)
        res = _bf(torch.randn(B, H, W, Co, generator=g)).to(dev)
        res2 = _bf(torch.randn(B, H, W, Co, generator=g)).to(dev)
        wp = _pack_conv((torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(dev))
        b = (torch.randn(Co, generator=g) * 0.1).to(dev)
        for kw in (dict(relu_in=True, act="relu"), dict(res=res), dict(res=res, res2=res2), dict()):
            calls.append(lambda kw=kw: ops.conv2d(x, wp, bias=b, **kw))
    try:
        if case not in ("halo", "splitk", "f32res"):
            ops.set_gemm_engine(1)          # the tile kernel
        for fn in calls:
            outs = []
            for on in (1, 0):
                ops.set_tuning("gemm_simple_epi", on)
                outs.append(fn().clone())
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1])
    finally:
        ops.set_tuning("gemm_simple_epi", 1)
        ops.set_gemm_engine(0)

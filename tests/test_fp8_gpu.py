"""MX fp8 path (DPT-Hybrid fp8, BASELINE configs[4]) against torch on the same quantised operands.

* Producers (i2pc_quant_fp8, i2pc_layernorm_fp8): bit-exact with the torch restatement of the
  block rule (ops.quantize_mx: E8M0 scale = smallest 2^e with max|v| / 2^e <= 448, e4m3fn RNE).
* i2pc_gemm_fp8 (v_mfma_scale_f32_16x16x128_f8f6f4): against an fp32 torch GEMM / conv of the
  DEQUANTISED operands -- the only difference is fp32 summation order, so the bound is
  |err| <= 1e-4 * max|ref| (+ for fp8 outputs: one e4m3 rounding, compared after dequantisation
  with the e4m3 half-ulp 2^-4 relative bound).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda")


def _bits_equal(a, b, x=None):
    if torch.equal(a.data, b.data) and torch.equal(a.scale, b.scale):
        return True
    ns = int((a.scale != b.scale).sum())
    bad = (a.data != b.data).nonzero()
    msg = [f"scale mismatches {ns}/{a.scale.numel()}, data mismatches {bad.shape[0]}/{a.data.numel()}"]
    for r, c in bad[:8].tolist():
        e = int(b.scale[r, c // 32]) - 127
        v = float(x[r, c]) * 2.0 ** -e if x is not None else float("nan")
        msg.append(f"  [{r},{c}] scaled {v!r} got 0x{int(a.data[r, c]):02x} ref 0x{int(b.data[r, c]):02x} "
                   f"scale got {int(a.scale[r, c // 32])} ref {int(b.scale[r, c // 32])}")
    raise AssertionError("\n".join(msg))


def test_e4m3_conversion_table(dev):
    """Every e4m3fn value, the midpoints between neighbours (ties to even) and points just off
    them: the device conversion (v_cvt_pk_fp8_f32 via quant_fp8 at scale 2^0) against torch."""
    from image_to_pointcloud_amd import ops
    codes = torch.arange(0, 0x7f, dtype=torch.uint8)             # +0 .. 448 (0x7f is NaN)
    vals = codes.view(torch.float8_e4m3fn).float()
    mids = (vals[:-1] + vals[1:]) / 2
    probe = torch.cat([vals, mids, mids * (1 + 2 ** -20), mids * (1 - 2 ** -20), -vals, -mids])
    probe = probe.view(-1, 1).repeat(1, 2).view(-1)             # [v, v]: every value twice
    probe = torch.cat([probe, torch.zeros((-probe.numel()) % 128)])
    rows = probe.numel() // 128
    x = probe.view(rows, 128).clone()
    x[:, ::32] = 448.0                                         # pin every block's scale to 2^0
    got = ops.quant_fp8(x.to(dev))
    ref = ops.quantize_mx(x.to(dev))
    assert _bits_equal(got, ref, x)


@pytest.mark.parametrize("dtype,relu", [(torch.bfloat16, False), (torch.float32, False), (torch.bfloat16, True)])
def test_quant_rows_bit_exact(dev, dtype, relu):
    from image_to_pointcloud_amd import ops
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.randn(300, 768, generator=g) * torch.logspace(-3, 3, 768)).to(dtype).to(dev)
    x[7, :32] = 0                      # an all-zero block
    got = ops.quant_fp8(x, relu=relu)
    ref = ops.quantize_mx(torch.relu(x.float()) if relu else x.float())
    assert _bits_equal(got, ref, torch.relu(x.float()) if relu else x.float())


def test_quant_row_remap_skips_cls(dev):
    from image_to_pointcloud_amd import ops
    B, T, D = 3, 17, 256
    x = torch.randn(B * T, D, device=dev)
    got = ops.quant_fp8(x, rows=B * (T - 1), a_map=(T - 1, T, 1))
    ref = ops.quantize_mx(x.view(B, T, D)[:, 1:].reshape(-1, D))
    assert _bits_equal(got, ref)


@pytest.mark.parametrize("dim", [768, 1024])
def test_layernorm_fp8(dev, dim):
    from image_to_pointcloud_amd import ops
    g = torch.Generator(device="cpu").manual_seed(dim)
    x = (torch.randn(1000, dim, generator=g) * 3 + 0.5).to(dev)
    gm = (1 + 0.1 * torch.randn(dim, generator=g)).to(dev)
    bt = (0.1 * torch.randn(dim, generator=g)).to(dev)
    got = ops.layernorm_fp8(x, gm, bt, 1e-12)
    ref = ops.quantize_mx(torch.nn.functional.layer_norm(x, (dim,), gm, bt, 1e-12))
    # fp32 LN rounding may move a value across an e4m3 rounding boundary (rare +-1 codes) or move a
    # block's maximum across a power of two (rare scale steps; that block's codes then all differ,
    # so they are compared only where the scales agree)
    same = got.scale == ref.scale
    assert same.float().mean() > 1 - 1e-3
    def order(codes):                  # e4m3 sign-magnitude codes -> monotone integers (+0 == -0)
        c = codes.to(torch.int16)
        return torch.where(c >= 128, 128 - c, c)
    diff = (order(got.data) - order(ref.data)).abs()
    diff = diff * same.repeat_interleave(32, dim=1)[:, :dim]
    assert (diff > 1).sum() == 0 and (diff > 0).float().mean() < 1e-3


def _ref_linear(x, w, bias=None, act=None, rbias=None, g=1, table=None, trows=1):
    y = x.dequantize() @ w.dequantize().t()
    if bias is not None:
        y = y + bias
    if rbias is not None:
        y = y + rbias.repeat_interleave(g, dim=0)[: y.shape[0]]
    if table is not None:
        y = y + table.repeat(y.shape[0] // trows + 1, 1)[: y.shape[0]]
    if act == "gelu":
        y = torch.nn.functional.gelu(y)
    elif act == "relu":
        y = torch.relu(y)
    return y


def _close(got, ref, tol=1e-4):
    err = (got.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= tol * scale, f"max err {err:.3e} vs {tol:.0e} * {scale:.3e}"


@pytest.mark.parametrize("M,N,K", [(577 * 3, 2304, 768), (4097, 768, 3072), (300, 256, 128)])
def test_linear_fp8_bf16_out(dev, M, N, K):
    from image_to_pointcloud_amd import ops
    x = ops.quantize_mx(torch.randn(M, K, device=dev))
    w = ops.quantize_mx(torch.randn(N, K, device=dev) / K ** 0.5)
    b = torch.randn(N, device=dev)
    got = ops.linear_fp8(x, w, bias=b)
    _close(got, _ref_linear(x, w, b), 1e-2)       # bf16 output rounding
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    res = torch.randn(M, N, device=dev)
    out.copy_(res)
    got = ops.linear_fp8(x, w, bias=b, res=out)  # fp32 residual stream in place
    _close(got, _ref_linear(x, w, b) + res)


def test_linear_fp8_gelu_fp8_out_rowbias_table(dev):
    from image_to_pointcloud_amd import ops
    B, T, N, K = 4, 576, 768, 768
    M = B * T
    x = ops.quantize_mx(torch.randn(M, K, device=dev))
    w = ops.quantize_mx(torch.randn(N, K, device=dev) / K ** 0.5)
    b = 0.1 * torch.randn(N, device=dev)
    rb = torch.randn(B, N, device=dev)
    got = ops.linear_fp8(x, w, bias=b, act="gelu", row_bias=rb, row_bias_group=T, out_fp8=True)
    ref = _ref_linear(x, w, b, "gelu", rbias=rb, g=T)
    deq = got.dequantize()
    # one e4m3 rounding of the output (half ulp = 2^-4 of the value's binade) + block scale
    assert ((deq - ref).abs() <= ref.abs() * 2.0 ** -4 + 2.0 ** -9 * ref.abs().max()).all()
    tb = torch.randn(T, N, device=dev)
    got = ops.linear_fp8(x, w, bias=b, table=tb, table_rows=T)
    _close(got, _ref_linear(x, w, b, table=tb, trows=T), 1e-2)


def _conv_ref(x, w, Co, k, stride, pad, bias=None, relu_in=False):
    xd = x.dequantize().permute(0, 3, 1, 2)
    if relu_in:
        xd = torch.relu(xd)
    C = xd.shape[1]
    wd = w.dequantize().view(Co, k, k, C).permute(0, 3, 1, 2)
    y = torch.nn.functional.conv2d(xd, wd, bias=bias, stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,H,W,C,Co,k,stride", [(2, 24, 24, 256, 256, 3, 1), (3, 13, 17, 768, 768, 3, 2),
                                                  (2, 48, 40, 256, 128, 3, 1), (2, 12, 12, 1024, 256, 1, 1)])
def test_conv_fp8(dev, B, H, W, C, Co, k, stride):
    from image_to_pointcloud_amd import ops
    pad = k // 2
    x = ops.quantize_mx(torch.randn(B, H, W, C, device=dev))
    w = ops.quantize_mx(torch.randn(Co, k * k * C, device=dev) / (k * k * C) ** 0.5)
    b = torch.randn(Co, device=dev)
    got = ops.conv2d_fp8(x, w, bias=b, k=k, stride=stride, pad=pad)
    _close(got, _conv_ref(x, w, Co, k, stride, pad, b), 1e-2)


def test_conv_fp8_residual_unit(dev):
    """Pre-activation residual unit on fp8: conv1(relu(x)) + ReLU -> fp8 (Q8 epilogue) ->
    conv2 + bias + x + hidden (bf16 residuals)."""
    from image_to_pointcloud_amd import ops
    B, H, W, C = 2, 24, 20, 256
    xb = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    hid = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    x = ops.quant_fp8(xb)
    w1 = ops.quantize_mx(torch.randn(C, 9 * C, device=dev) / (9 * C) ** 0.5)
    w2 = ops.quantize_mx(torch.randn(C, 9 * C, device=dev) / (9 * C) ** 0.5)
    b1, b2 = 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev)
    t = ops.conv2d_fp8(x, w1, bias=b1, relu_in=True, act="relu", out_fp8=True)
    ref_t = torch.relu(_conv_ref(x, w1, C, 3, 1, 1, b1, relu_in=True))
    assert ((t.dequantize() - ref_t).abs() <= ref_t.abs() * 2.0 ** -4 + 2.0 ** -9 * ref_t.abs().max()).all()
    h = ops.conv2d_fp8(t, w2, bias=b2, res=xb, res2=hid)
    ref = _conv_ref(t, w2, C, 3, 1, 1, b2) + xb.float() + hid.float()
    _close(h, ref, 1e-2)


@pytest.mark.parametrize("B,H,W,C,add", [(2, 96, 96, 256, False), (3, 13, 7, 128, True), (1, 5, 9, 384, False)])
def test_upsample2x_fp8_bit_exact(dev, B, H, W, C, add):
    """i2pc_upsample2x_fp8 (the DPT-Hybrid head's operand straight from the last fusion upsample) equals
    quant_fp8 of the bf16 upsample2x output byte for byte (data and scales)."""
    from image_to_pointcloud_amd import ops
    g = torch.Generator(device="cpu").manual_seed(H * W + C)
    x = (torch.randn(B, H, W, C, generator=g) * torch.logspace(-2, 2, C)).to(torch.bfloat16).to(dev)
    a = torch.randn(B, 2 * H, 2 * W, C, generator=g).to(torch.bfloat16).to(dev) if add else None
    x[0, 0, 0, :32] = 0
    got = ops.upsample2x(x, add=a, out_fp8=True)
    ref = ops.quant_fp8(ops.upsample2x(x, add=a))
    torch.cuda.synchronize()
    assert got.data.shape == ref.data.shape
    assert _bits_equal(ops.Fp8(got.data.view(-1, C), got.scale.view(-1, C // 32)),
                       ops.Fp8(ref.data.view(-1, C), ref.scale.view(-1, C // 32)))

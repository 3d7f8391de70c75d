"""BiT stem kernels of DPT-Hybrid (csrc/bit.hip) against torch on the same bf16 inputs:
GroupNorm (+ shortcut, ReLU), the SAME-padded 3x3/2 max pool, the 7x7/2 stem im2col (through
the conv it feeds).  Bounds: bf16 output rounding (2^-8 relative) plus fp32 statistics."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
F = torch.nn.functional


def _nchw(x):
    return x.permute(0, 3, 1, 2).float()


@pytest.mark.parametrize("B,H,W,C", [(2, 96, 96, 64), (3, 48, 48, 512), (2, 24, 24, 1024), (2, 13, 29, 256),
                                     (1, 192, 192, 64)])
def test_group_norm_modes(B, H, W, C):
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(C + H)
    x = (torch.randn(B, H, W, C, generator=g) * 3 + 1).to(torch.bfloat16).to(dev)
    r = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    gm, bt = (1 + 0.1 * torch.randn(C, generator=g)).to(dev), (0.1 * torch.randn(C, generator=g)).to(dev)
    rg, rb = (1 + 0.1 * torch.randn(C, generator=g)).to(dev), (0.1 * torch.randn(C, generator=g)).to(dev)
    ref_x = F.group_norm(_nchw(x), 32, gm, bt, 1e-5)
    ref_r = F.group_norm(_nchw(r), 32, rg, rb, 1e-5)
    for shortcut, relu, exp in [(None, True, torch.relu(ref_x)), (r, True, torch.relu(ref_x + _nchw(r))),
                                ((r, rg, rb), True, torch.relu(ref_x + ref_r)), (None, False, ref_x)]:
        got = _nchw(ops.group_norm(x, gm, bt, relu=relu, shortcut=shortcut))
        err = (got - exp).abs().max().item()
        assert err <= 2e-2 * exp.abs().max().item(), (shortcut is None, relu, err)


@pytest.mark.parametrize("C", [64, 256, 1024])
def test_group_norm_large_offset(C):
    """Activations whose mean is ~200x their spread (BiT after a residual can drift there): the
    statistics come from shifted sums merged by Chan's formula, so the variance does not cancel
    away as E[x^2] - mean^2 in fp32 would.  The reference is fp64 group_norm of the
    same bf16 values."""
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(C)
    B, H, W = 2, 48, 40
    x = (torch.randn(B, H, W, C, generator=g) * 0.05 + 10.0).to(torch.bfloat16).to(dev)
    gm, bt = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    ref = F.group_norm(_nchw(x).double(), 32, gm.double(), bt.double(), 1e-5)
    got = _nchw(ops.group_norm(x, gm, bt, relu=False)).double()
    err = (got - ref).abs().max().item()
    # bf16 output of unit-variance values: ~4e-3 relative; a cancelled variance would be off by O(1)
    assert err <= 3e-2, err
    print("parity", {"case": f"groupnorm offset C={C}", "max_abs_err": err})


@pytest.mark.parametrize("H,W", [(192, 192), (97, 64), (5, 6)])
def test_maxpool_same_padding(H, W):
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    x = torch.relu(torch.randn(2, H, W, 64, device=dev)).to(torch.bfloat16)
    oh, pt = ops.same_pad(H, 3, 2)
    ow, pl = ops.same_pad(W, 3, 2)
    th, tw = max((oh - 1) * 2 + 3 - H, 0), max((ow - 1) * 2 + 3 - W, 0)
    ref = F.max_pool2d(F.pad(_nchw(x), [pl, tw - pl, pt, th - pt], value=0.0), 3, 2)
    got = _nchw(ops.maxpool3s2(x))
    assert torch.equal(got, ref)


def test_stem_conv_same_padding():
    """im2col rows x standardised 7x7 weights == conv2d on the DynamicPad2d-padded input."""
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    pix = torch.randn(2, 3, 384, 384, generator=g).to(dev)
    w = torch.randn(64, 3, 7, 7, generator=g).to(dev) / 12
    cols, (oh, ow) = ops.stem_im2col(pix, k_pitch=192)
    wp = torch.zeros(64, 192, device=dev)
    wp[:, :147] = w.permute(0, 2, 3, 1).reshape(64, 147)
    got = ops.linear(cols, wp.to(torch.bfloat16)).view(2, oh, ow, 64)
    ref = F.conv2d(F.pad(pix, [2, 3, 2, 3]), w, stride=2)
    assert (oh, ow) == (192, 192)
    err = (_nchw(got) - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("B,H,W,ks,kp", [(2, 384, 384, 7, 152), (1, 37, 45, 7, 152), (3, 130, 257, 7, 192),
                                         (1, 20, 20, 3, 32)])
def test_stem_im2col_exact(B, H, W, ks, kp):
    """im2col rows bit-exact against torch unfold of the SAME-padded input (k = (ky*ks + kx)*3 + c,
    zero beyond ks*ks*3), covering partial 64-pixel output segments."""
    from image_to_pointcloud_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(H * W + ks)
    pix = torch.randn(B, 3, H, W, generator=g).to(dev)
    cols, (oh, ow) = ops.stem_im2col(pix, ksize=ks, k_pitch=kp)
    _, pt = ops.same_pad(H, ks, 2)
    _, pl = ops.same_pad(W, ks, 2)
    ph = max((oh - 1) * 2 + ks - H - pt, 0)
    pw = max((ow - 1) * 2 + ks - W - pl, 0)
    xp = F.pad(pix, [pl, pw, pt, ph])
    u = F.unfold(xp, ks, stride=2)[..., : oh * ow]                   # [B, 3*ks*ks, L], (c, ky, kx)
    u = u.view(B, 3, ks * ks, oh * ow).permute(0, 3, 2, 1).reshape(B * oh * ow, ks * ks * 3)
    ref = torch.zeros(B * oh * ow, kp, device=dev)
    ref[:, : ks * ks * 3] = u
    assert torch.equal(cols, ref.to(torch.bfloat16))

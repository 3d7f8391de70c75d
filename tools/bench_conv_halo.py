"""k_conv3_halo variants (knob conv_halo 1-4) against the implicit GEMM (conv_halo=0) on Depth-Anything-
V2-Small's 64-channel 3x3 conv shapes (batch 32): median event time per call, bit-equality to the GEMM."""
import math, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
shapes = [(32, 148, 148, False, True), (32, 148, 148, True, False), (32, 296, 296, False, False), (32, 74, 74, False, True)]
variants = [int(v) for v in os.environ.get("HALO_VARIANTS", "0,1,2,3,4").split(",")]


def timeit(fn, iters=20):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


for B, H, W, relu, res in shapes:
    x = torch.randn(B, H, W, 64, generator=g).to(torch.bfloat16).to(dev)
    r = torch.randn(B, H, W, 64, generator=g).to(torch.bfloat16).to(dev) if res else None
    w = (torch.randn(64, 9 * 64, generator=g) / 24).to(torch.bfloat16).to(dev)
    b = torch.randn(64, generator=g).to(dev)
    kw = dict(relu_in=True, act="relu") if relu else dict(res=r)
    outs, times = {}, {v: [] for v in variants}
    for rnd in range(3):
        for v in variants:
            ops.set_tuning("conv_halo", v)
            out = torch.empty(B, H, W, 64, dtype=torch.bfloat16, device=dev)
            times[v].append(timeit(lambda: ops.conv2d(x, w, bias=b, out=out, **kw)))
            outs[v] = out
    ops.set_tuning("conv_halo", 3)
    fl = 2.0 * B * H * W * 64 * 576
    line = " | ".join(f"v{v} {statistics.median(times[v]) * 1e6:7.1f} us {fl / statistics.median(times[v]) / 1e12:5.0f} TF"
                      f"{'' if torch.equal(outs[v], outs[variants[0]]) else ' DIFF'}" for v in variants)
    print(f"B{B} {H}x{W} relu={relu} res={res}: {line}", flush=True)

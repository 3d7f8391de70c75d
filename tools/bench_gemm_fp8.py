"""fp8 (MX, scaled MFMA) vs bf16 GEMM / conv timing on the DPT-Hybrid shapes (batch 64, 384^2).
   python tools/bench_gemm_fp8.py"""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")


def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


g = torch.Generator(device="cpu").manual_seed(0)
B = int(os.environ.get("B", "64"))
M = B * 577
for name, m, n, k, q8 in [("qkv", M, 2304, 768, False), ("o", M, 768, 768, False), ("fc1", M, 3072, 768, True),
                          ("fc2", M, 768, 3072, False)]:
    xf = (torch.rand(m, k, generator=g) * 2 - 1).to(dev)
    wf = ((torch.rand(n, k, generator=g) * 2 - 1) / math.sqrt(k)).to(dev)
    b = torch.randn(n, generator=g).to(dev)
    x8, w8 = ops.quantize_mx(xf), ops.quantize_mx(wf)
    xb, wb = xf.to(torch.bfloat16), wf.to(torch.bfloat16)
    outb = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    out8 = ops.empty_fp8((m, n), dev) if q8 else torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    tb = timeit(lambda: ops.linear(xb, wb, bias=b, out=outb))
    t8 = timeit(lambda: ops.linear_fp8(x8, w8, bias=b, out=out8, out_fp8=q8))
    f = 2 * m * n * k
    print(f"{name:4s} M={m} N={n} K={k}: bf16 {tb*1e6:8.1f} us {f/tb/1e12:7.1f} TF | fp8 {t8*1e6:8.1f} us {f/t8/1e12:7.1f} TF"
          f"{' (fp8 out)' if q8 else ''}  x{tb/t8:.2f}")
for (H, C, Co) in [(12, 256, 256), (24, 256, 256), (48, 256, 256), (96, 256, 256), (192, 256, 128), (24, 768, 256)]:
    xf = (torch.rand(B, H, H, C, generator=g) * 2 - 1).to(dev)
    wf = ((torch.rand(Co, 9 * C, generator=g) * 2 - 1) / math.sqrt(9 * C)).to(dev)
    x8, w8 = ops.quantize_mx(xf), ops.quantize_mx(wf)
    xb, wb = xf.to(torch.bfloat16), wf.to(torch.bfloat16)
    tb = timeit(lambda: ops.conv2d(xb, wb), iters=10)
    t8 = timeit(lambda: ops.conv2d_fp8(x8, w8), iters=10)
    f = 2 * B * H * H * Co * 9 * C
    print(f"conv {B}x{H}x{H}x{C}->{Co}: bf16 {tb*1e6:8.1f} us {f/tb/1e12:7.1f} TF | fp8 {t8*1e6:8.1f} us {f/t8/1e12:7.1f} TF  x{tb/t8:.2f}")

"""A/B of GEMM engine modes on the DPT-Large (batch 32) linear shapes, interleaved rounds in one
process (cdna_hip_programming.md rule 24): mode 0 = automatic (single-stage persistent k_gemm_p
where a persistent engine runs), mode 3 = the same plan with the ping-pong k_gemm_8p there.
Random operands; prints the median / min per mode and the bit-equality of the two outputs."""
import math, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")
M = 32 * 577
shapes = [("qkv", M, 3072, 1024, None), ("fc1", M, 4096, 1024, "gelu"), ("o", M, 1024, 1024, None),
          ("fc2", M, 1024, 4096, None), ("big", 8192, 8192, 4096, None)]
if os.environ.get("AB_SHAPES") == "hybrid":        # DPT-Hybrid (C5, batch 64) bf16 linears
    MH = 64 * 577
    shapes = [("hqkv", MH, 2304, 768, None), ("hfc2", MH, 768, 3072, None), ("ho", MH, 768, 768, None),
              ("hfc1", MH, 3072, 768, "gelu")]
modes = [int(m) for m in os.environ.get("AB_MODES", "0,3").split(",")]
g = torch.Generator(device="cpu").manual_seed(0)


def timeit(fn, iters=20):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


for name, m, n, k, act in shapes:
    x = (torch.rand(m, k, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(n, k, generator=g) * 2 - 1) / math.sqrt(k)).to(torch.bfloat16).to(dev)
    b = torch.randn(n, generator=g).to(dev)
    outs = {md: torch.empty(m, n, dtype=torch.bfloat16, device=dev) for md in modes}
    times = {md: [] for md in modes}
    labels = {}
    for md in modes:
        ops.set_gemm_engine(md)
        ops.linear(x, w, bias=b, act=act, out=outs[md]); torch.cuda.synchronize()
        d = ops.GemmDesc()
        d.a, d.lda, d.m, d.n, d.k = x.data_ptr(), x.stride(0), m, n, k
        d.w, d.ldw, d.bias, d.c, d.ldc = w.data_ptr(), w.stride(0), b.data_ptr(), outs[md].data_ptr(), n
        labels[md] = ops.gemm_kernel_label(d)
    for _ in range(5):
        for md in modes:
            ops.set_gemm_engine(md)
            times[md].append(timeit(lambda: ops.linear(x, w, bias=b, act=act, out=outs[md])))
    ops.set_gemm_engine(0)
    same = all(torch.equal(outs[modes[0]], outs[md]) for md in modes)
    fl = 2 * m * n * k
    line = " | ".join(f"mode {md} {labels[md]}: med {statistics.median(times[md])*1e6:7.1f} us "
                      f"{fl/statistics.median(times[md])/1e12:6.1f} TF (min {min(times[md])*1e6:7.1f})" for md in modes)
    print(f"{name:4s} {m}x{n}x{k} act={act}: {line} | bitequal={same}", flush=True)

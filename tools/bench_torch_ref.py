"""Calibration only: the library (hipBLASLt / torch SDPA) rate on the DPT-Large shapes, to size our kernels' headroom."""
import math, sys
import torch
F = torch.nn.functional
dev = torch.device("cuda")
M = 32 * 577
def timeit(fn, iters=20):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3
for name, m, n, k in [("qkv", M, 3072, 1024), ("o", M, 1024, 1024), ("fc1", M, 4096, 1024), ("fc2", M, 1024, 4096),
                      ("sq8k", 8192, 8192, 8192)]:
    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: F.linear(x, w, b))
    print(f"hipblaslt {name:5s} {m}x{n}x{k}: {t*1e6:8.1f} us {2*m*n*k/t/1e12:7.1f} TF", flush=True)
q = torch.randn(32, 16, 577, 64, device=dev, dtype=torch.bfloat16)
t = timeit(lambda: F.scaled_dot_product_attention(q, q, q, scale=0.125))
print(f"sdpa 32x16x577x64: {t*1e6:8.1f} us {4*32*16*577*577*64/t/1e12:7.1f} TF", flush=True)

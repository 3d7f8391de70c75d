"""Cost of the tile GEMM's epilogues on the DPT-Large O-projection shape (M 18464, N 1024, K 1024,
320 x 256 tiles): bf16 out, fp32 out, fp32 out + fp32 residual in place, + the LayerNorm-fold
producer (bf16 copy + chunk partials) on the tile kernel and on the persistent engine's EPI_LNP (knob
gemm_lnp_p); and the same for FC2 (K 4096).  Interleaved rounds."""
import math, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")
M, N = 32 * 577, 1024
g = torch.Generator(device="cpu").manual_seed(0)


def timeit(fn, iters=20):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for K in (1024, 4096):
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    res = torch.randn(M, N, generator=g).to(dev)
    o16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    o32 = torch.empty(M, N, dtype=torch.float32, device=dev)
    part = torch.empty(M, N // 64, 2, dtype=torch.float32, device=dev)
    ln = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    shift = torch.zeros(M, dtype=torch.float32, device=dev)
    variants = {
        "bf16 out": lambda: ops.linear(x, w, bias=b, out=o16),
        "fp32 out": lambda: ops.linear(x, w, bias=b, out=o32, out_f32=True),
        "fp32 + res (in place)": lambda: ops.linear(x, w, bias=b, res=res, out=res),
        "fp32 + res + LN producer (tile)": lambda: (ops.set_tuning("gemm_lnp_p", 0), ops.linear(
            x, w, bias=b, res=res, out=res, ln_part=part, out_bf16=ln, ln_shift=shift)),
        "LN producer (persistent 160)": lambda: (ops.set_tuning("gemm_lnp_p", 1), ops.linear(
            x, w, bias=b, res=res, out=res, ln_part=part, out_bf16=ln, ln_shift=shift)),
        "bf16-stream producer (tile)": lambda: (ops.set_tuning("gemm_lnp_p", 0), ops.linear(
            x, w, bias=b, res=ln, res_shift=shift, out=ln, ln_part=part, ln_shift=shift)),
    }
    t = {k: [] for k in variants}
    for _ in range(5):
        for k, fn in variants.items():
            fn(); torch.cuda.synchronize()
            t[k].append(timeit(fn))
    print(f"M {M} N {N} K {K}: " + " | ".join(f"{k}: {statistics.median(v):6.1f} us" for k, v in t.items()), flush=True)

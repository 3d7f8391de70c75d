"""Quarter-engine (I2PC_GEMM_Q=1) vs tile kernel on shapes of increasing complexity; prints
where they differ (debug helper)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
for (M, N, K) in [(256, 256, 128), (256, 256, 256), (256, 256, 1024), (512, 256, 1024), (256, 512, 1024),
                  (8200, 2048, 1024), (18464, 3072, 1024)]:
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(dev)
    outs = []
    for mode in (1, 2):
        ops.set_gemm_engine(mode)
        outs.append(ops.linear(x, w).float())
    ops.set_gemm_engine(0)
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs()
    bad = (d > 0).nonzero()
    ref = (x.float() @ w.float().t())
    e1 = (outs[1] - ref).abs().max().item()
    msg = f"M={M} N={N} K={K}: mismatches {bad.shape[0]}  max|q-ref| {e1:.3e}"
    if bad.shape[0]:
        r, c = bad[:, 0], bad[:, 1]
        msg += f" rows {r.min().item()}..{r.max().item()} ({torch.unique(r // 256).tolist()[:8]} tiles) cols {c.min().item()}..{c.max().item()} "
        msg += f"row%256 uniq {torch.unique(r % 256).numel()} col%256 uniq {torch.unique(c % 256).numel()}"
        msg += f" first {bad[:4].tolist()}"
    print(msg, flush=True)

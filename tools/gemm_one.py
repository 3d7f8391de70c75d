"""Run one GEMM shape N times (for rocprofv3 counter passes)."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops
m, n, k = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (18464, 3072, 1024)))
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
x = (torch.rand(m, k, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
w = ((torch.rand(n, k, generator=g) * 2 - 1) / math.sqrt(k)).to(torch.bfloat16).to(dev)
b = torch.randn(n, generator=g).to(dev)
out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
for _ in range(20):
    ops.linear(x, w, bias=b, out=out)
torch.cuda.synchronize()

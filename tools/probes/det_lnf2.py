"""Which per-column operand of the LN-fold consumer (256 x 128 tiles, N = 1152) carries the run-to-run
difference: csum = 0, bias = 0, or rs.y = 0."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from image_to_pointcloud_amd import ops
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
M, N, K = 43840, 1152, 384
x = (torch.randn(M, K, generator=g) * 2).to(torch.bfloat16).to(dev)
w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(torch.bfloat16).to(dev)
b0 = torch.randn(N, generator=g).to(dev)
rs0 = torch.stack([torch.rand(M, generator=g) + 0.5, torch.randn(M, generator=g)], 1).to(dev).contiguous()
cs0 = torch.randn(N, generator=g).to(dev)
for name, b, cs, rs in (("all", b0, cs0, rs0), ("csum0", b0, torch.zeros_like(cs0), rs0),
                        ("bias0", torch.zeros_like(b0), cs0, rs0),
                        ("rsy0", b0, cs0, torch.stack([rs0[:, 0], torch.zeros(M, device=dev)], 1).contiguous())):
    outs = []
    for _ in range(8):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ops.linear(x, w, bias=b, ln_rows=rs, col_sum=cs, out=out)
        outs.append(out)
    torch.cuda.synchronize()
    nd = sum(0 if torch.equal(outs[0], o) else 1 for o in outs[1:])
    print(name, f"{nd}/7 differ", flush=True)

"""Geometry-stage microbenchmark: B x 384^2 depth -> 1024^2 points (density high).
Usage: bench_unproject.py [B] [density] [H W h w] (image H x W from an h x w depth map);
DEPTH=const|nan01 for SURVEY 8d's constant-depth and 0.1 %-NaN variants, NAN1=1 for one NaN."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import geometry
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dens = sys.argv[2] if len(sys.argv) > 2 else "high"
h = w = 384; H = W = 1024
if len(sys.argv) > 6:
    H, W, h, w = (int(x) for x in sys.argv[3:7])
v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
rng = np.random.default_rng(0)
dep = np.stack([(0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w + i) * np.cos(4 * np.pi * v / h)) + rng.normal(0, 0.05, (h, w))).astype(np.float32) for i in range(B)])
if os.environ.get("NAN1"):            # one NaN model pixel per map (the C4 tool's synthetic panorama)
    dep[:, 7, 11] = np.nan
kind = os.environ.get("DEPTH", "smooth")   # SURVEY 8d's microbenchmark variants
if kind == "const":
    dep[:] = 2.5
elif kind == "nan01":                    # 0.1 % of the model pixels NaN
    for i in range(B):
        dep[i].ravel()[rng.permutation(h * w)[:(h * w) // 1000]] = np.nan
img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
d = torch.from_numpy(dep).to(dev)
out = geometry.unproject_batch(d, img, density=dens)
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    geometry.unproject_batch(d, img, density=dens, out=out)
e1.record(); torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 20 * 1e-3
N = out.xyz.shape[1]
byts = B * (4.0 * h * w + 18.0 * N)
print(f"B={B} {dens}: {t*1e6:.1f} us/call, {B*N/t/1e6:.0f} Mpts/s, algorithmic {byts/t/1e9:.0f} GB/s ({byts/t/8e12*100:.1f}% of 8 TB/s)")

# cold caches: a 1 GiB write between calls evicts the L2s and the 256 MiB Infinity Cache, as the
# network does between two unprojections inside the pipeline step
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
ts = []
for _ in range(10):
    flush.zero_()
    a = torch.cuda.Event(enable_timing=True); c = torch.cuda.Event(enable_timing=True)
    a.record()
    geometry.unproject_batch(d, img, density=dens, out=out)
    c.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(c) * 1e-3)
t = sorted(ts)[len(ts) // 2]
print(f"B={B} {dens} cold: {t*1e6:.1f} us/call (median of 10), {B*N/t/1e6:.0f} Mpts/s, algorithmic {byts/t/1e9:.0f} GB/s")

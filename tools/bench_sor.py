"""Statistical outlier removal microbenchmark: a 1024^2 high-density cloud (1,048,576 points)
unprojected from a 384^2 depth map, nb_neighbors 20, std_ratio 2.0 (refine_point_cloud defaults)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from image_to_pointcloud_amd import geometry as g

dev = torch.device("cuda")
rng = np.random.Generator(np.random.PCG64(1))
h = w = 384
v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
d = (0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w) * np.cos(4 * np.pi * v / h))
     + rng.normal(0, 0.05, (h, w))).astype(np.float32)
for size, dens in ((1024, "high"), (1024, "medium"), (2048, "high")):
    img = torch.from_numpy(rng.integers(0, 256, (size, size, 3), dtype=np.uint8)).to(dev)
    pb = g.unproject_batch(torch.from_numpy(d).to(dev)[None], img[None], density=dens)
    xyz, rgb = pb.xyz[0], pb.rgb[0]
    r = g.remove_statistical_outlier(xyz, rgb)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        r = g.remove_statistical_outlier(xyz, rgb)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 5 * 1e-3
    n = xyz.shape[0]
    print(f"sor {size}^2 {dens}: n={n} kept={r.index.numel()} {t*1e3:8.2f} ms/cloud  {n/t/1e6:8.1f} Mpts/s")

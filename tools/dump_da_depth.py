"""Dump the Depth-Anything-V2-Small depth of the synthetic C4 panorama (seeded weights), as
tools/c4_panorama.py --network computes it, to gpurun_out/da_pano_depth.npy (selection diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
from image_to_pointcloud_amd.pipeline import PointCloudPipeline

H, W = 4096, 8192
dev = torch.device("cuda", 0)
full = np.empty((H, W, 3), np.uint8)
for y in range(H):
    full[y] = np.random.Generator(np.random.PCG64(1000 + y)).integers(0, 256, (W, 3), dtype=np.uint8)
net = PointCloudPipeline(1, H, W, spec=DA_V2_SMALL, density="high", device=dev)
d = net.infer_depth(torch.from_numpy(full).to(dev)[None])[0].cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/da_pano_depth.npy", d)
print(d.shape, d.dtype, float(d.min()), float(d.max()), float((d == 0).mean()), len(np.unique(d)))

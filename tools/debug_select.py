"""Selection-state dump after one geometry call (bench_unproject inputs): per image the
level-0 windows, candidate counts and the targets' key intervals (SelState words)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import geometry
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
h = w = 384; H = W = 1024
v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
rng = np.random.default_rng(0)
dep = np.stack([(0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w + i) * np.cos(4 * np.pi * v / h)) + rng.normal(0, 0.05, (h, w))).astype(np.float32) for i in range(B)])
img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
d = torch.from_numpy(dep).to(dev)
ws = torch.zeros(geometry.workspace_bytes(B, H, W), dtype=torch.uint8, device=dev)
geometry.unproject_batch(d, img, density="high", workspace=ws)
torch.cuda.synchronize()
st = ws[: B * 320].view(torch.int32).cpu().numpy().view(np.uint32).reshape(B, 80)
for b in range(B):
    r = st[b]
    print(f"b{b} phase={r[0]} rlo={r[6]:#x} rhi={r[7]:#x} nwin={r[10]} wbin={list(r[12:16])} ccount={list(r[48:52])} "
          f"tlo={[hex(x) for x in r[20:24]]} thi={[hex(x) for x in r[24:28]]} nslot={r[9]} smode={list(r[44:48])}")

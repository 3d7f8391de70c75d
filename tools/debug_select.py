"""Selection-state dump after one geometry call: per image the level-0 windows, candidate
counts and the targets' key intervals (SelState words; layout of csrc/unproject.hip).
    python tools/debug_select.py [B] [--nan] [--band] [--net]   (--net: DPT-Large depth of random images)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import geometry
from image_to_pointcloud_amd.distributed import RcclComm
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4
band = "--band" in sys.argv
h, w = (518, 1036) if band else (384, 384)
H, W = (1024, 2048) if band else (1024, 1024)
B = 1 if band else B
v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
rng = np.random.default_rng(0)
dep = np.stack([(0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w + i) * np.cos(4 * np.pi * v / h)) + rng.normal(0, 0.05, (h, w))).astype(np.float32) for i in range(B)])
if "--nan" in sys.argv:
    dep[:, 7, 11] = np.nan
img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
d = torch.from_numpy(dep).to(dev)
if "--net" in sys.argv:
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    import bench
    img = bench._images(B, H, 0, dev)          # the bench's images (PCG64 seeds 1000 + i)
    pipe = PointCloudPipeline(B, H, W, device=dev)
    d = pipe.infer_depth(img).clone()
    torch.cuda.synchronize()
    if os.environ.get("DBG_SAVE"):
        np.save(os.environ["DBG_SAVE"], d[[int(x) for x in os.environ.get("DBG_IDX", "6").split(",")]].cpu().numpy())
    x = d[0].flatten().double().cpu().numpy()
    q = np.percentile(x, [0, 1, 2, 5, 25, 50, 75, 95, 98, 99, 100])
    print("depth[0] percentiles 0/1/2/5/25/50/75/95/98/99/100:", np.array2string(q, precision=5))
    hist, _ = np.histogram(x, bins=2048, range=(x.min(), x.max()))
    print("model map: max L0-bin share", hist.max() / x.size, "bins holding 50%:", int(np.searchsorted(np.cumsum(np.sort(hist)[::-1]), x.size / 2)) + 1)
ws = torch.zeros(geometry.workspace_bytes(B, H, W), dtype=torch.uint8, device=dev)
if band:
    comm = RcclComm(nranks=1, rank=0)
    geometry.unproject_band(d[0], img[0], H, W, 0, H, comm=comm, workspace=ws)
else:
    geometry.unproject_batch(d, img, density="high", workspace=ws)
torch.cuda.synchronize()
W32 = 108
st = ws[: B * W32 * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(B, W32)
for b in range(B):
    r = st[b]
    if "--net" in sys.argv and r[9] == 0 and all(x == 0xffffffff for x in r[50:54]) and B > 4:
        print(f"b{b} ok phase={r[0]} level={r[85]} wbin={list(map(int, r[12:16]))} ccount={list(map(int, r[76:78]))}")
        continue
    print(f"b{b} phase={r[0]} level={r[85]} n={r[1]} nan={r[2]} nonfin={r[3]} ntgt={r[8]} nslot={r[9]} nwin={r[10]} fill={r[11]} "
          f"wbin={list(map(int, r[12:18]))} ninf={int(r[18])},{int(r[19])} ccount={list(map(int, r[76:80]))}")
    print("   tlo", [hex(x) for x in r[30:40]])
    print("   thi", [hex(x) for x in r[40:50]])
    print("   tslot", list(map(int, r[50:60])), "rank", list(map(int, r[20:30])))

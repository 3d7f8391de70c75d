"""Per-call census of the network step: every GEMM / conv launch with its shape, kernel instance,
HIP-event time and rate, plus the non-GEMM launches by label, sorted by time (one eager step after
warm-up).  Used to pick which shapes to work on.

    python tools/gemm_census.py [--model dpt-large] [--size 1024] [--batch 32] [--top 40]
"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="dpt-large")
ap.add_argument("--dtype", default=None)
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()

from image_to_pointcloud_amd import ops
from image_to_pointcloud_amd.pipeline import PointCloudPipeline
import bench

_label = ops.gemm_kernel_label
ops.gemm_kernel_label = lambda d: f"{_label(d)} | m{d.m} n{d.n} k{d.k}"

spec = bench._spec(a.model)
dtype = a.dtype or ("fp8" if a.model == "dpt-hybrid" else "bf16")
dev = torch.device("cuda")
pipe = PointCloudPipeline(a.batch, a.size, a.size, spec=spec, density="high", device=dev, seed=0, dtype=dtype)
images = bench._images(a.batch, a.size, 0, dev)
for _ in range(3):
    pipe.pre(images, layout=pipe.layout, out=pipe._patches)
    pipe.model(pipe._patches, pipe.batch)
torch.cuda.synchronize()
ops.profile = []
pipe.pre(images, layout=pipe.layout, out=pipe._patches)
pipe.model(pipe._patches, pipe.batch)
torch.cuda.synchronize()
recs, ops.profile = ops.profile, None
per = {}
for label, flops, nbytes, e0, e1 in recs:
    d = per.setdefault(label, [0, 0.0, 0.0, 0.0])
    d[0] += 1
    d[1] += e0.elapsed_time(e1) * 1e-3
    d[2] += flops
    d[3] += nbytes
total = sum(v[1] for v in per.values())
print(f"network launches {sum(v[0] for v in per.values())}, {total * 1e3:.3f} ms (event-timed, eager)")
for label, (n, t, f, b) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
    rate = f"{f / t / 1e12:7.1f} TF/s" if f else f"{b / t / 1e9:7.0f} GB/s"
    print(f"{t * 1e3:7.3f} ms {100 * t / total:5.1f}%  x{n:<3d} {t / n * 1e6:8.1f} us  {rate}  {label}")

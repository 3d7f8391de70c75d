"""Run-to-run determinism of the DA-v2 pipeline: hashes of depth / xyz / bbox over three runs in this
process (first differing tensor reported)."""
import hashlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from image_to_pointcloud_amd.pipeline import PointCloudPipeline
import bench
dev = torch.device("cuda")
model = sys.argv[1] if len(sys.argv) > 1 else "depth-anything-v2"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pipe = PointCloudPipeline(B, 1024, 1024, spec=bench._spec(model), density="high", device=dev, seed=0)
images = bench._images(B, 1024, 0, dev)
hs = lambda t: hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]
ref = None
for it in range(3):
    out = pipe.run(images)
    torch.cuda.synchronize()
    d = pipe.depth.clone()
    h = (hs(d), hs(out.xyz), hs(out.bbox))
    print(model, it, h, flush=True)
    if ref is None:
        ref = d
    elif not torch.equal(ref, d):
        diff = (ref.float() - d.float()).abs()
        print("  depth differs: max", diff.max().item(), "count", int((diff > 0).sum()), flush=True)

"""Selection diagnostics: the per-image SelState (unproject.hip) after an i2pc_unproject call of one
depth map (.npy, model resolution) at a given image size, and after a one-rank window band call."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from image_to_pointcloud_amd import geometry as G
from image_to_pointcloud_amd.distributed import RcclComm

u4 = np.uint32
SEL = np.dtype([("phase", u4), ("n", u4), ("nan_count", u4), ("nonfinite_count", u4), ("kmin", u4), ("kmax", u4),
                ("rlo", u4), ("rhi", u4), ("ntgt", u4), ("nslot", u4), ("nwin", u4), ("fill", u4), ("wbin", u4, 6),
                ("ninf_neg", u4), ("ninf_pos", u4), ("rank", u4, 10), ("tlo", u4, 10), ("thi", u4, 10),
                ("tslot", u4, 10), ("slo", u4, 4), ("shi", u4, 4), ("smult", u4, 4), ("smode", u4, 4),
                ("ccount", u4, 4), ("med_ranks", u4), ("has_med", u4), ("med", np.float32), ("mode", np.int32),
                ("err", u4), ("level", u4), ("p2", np.float64), ("p98", np.float64), ("den64", np.float64),
                ("lo32", np.float32), ("hi32", np.float32), ("den32", np.float32), ("pad2", np.float32),
                ("bbox_key", u4, 6), ("pad3", u4, 2), ("rden64", np.float64), ("pad4", np.float64),
                ("wspike", u4, 3), ("wbelow", u4, 3), ("wcntF", u4, 3), ("wminF", u4, 3), ("wmaxF", u4, 3),
                ("wcntL", u4, 3), ("wminL", u4, 3), ("wmaxL", u4, 3), ("wvlo", np.float32, 3),
                ("wvhi", np.float32, 3), ("wvF", np.float32, 3), ("wvL", np.float32, 3), ("twin", u4, 10),
                ("pad5", u4, 2)])   # alignas(16): sizeof(SelState) == 624 (unproject.hip static_assert)
assert SEL.itemsize == 624


def show(tag, ws):
    s = np.frombuffer(ws[:SEL.itemsize].cpu().numpy().tobytes(), dtype=SEL)[0]
    print(tag, {k: (s[k].tolist() if hasattr(s[k], "tolist") else s[k]) for k in SEL.names
                if k not in ("pad2", "pad3", "pad4", "slo", "shi", "smult", "smode", "bbox_key")})


ap = argparse.ArgumentParser()
ap.add_argument("depth")
ap.add_argument("--height", type=int, default=4096)
ap.add_argument("--width", type=int, default=8192)
a = ap.parse_args()
dev = torch.device("cuda", 0)
d = torch.from_numpy(np.load(a.depth).astype(np.float32)).to(dev)
img = torch.zeros((a.height, a.width, 3), dtype=torch.uint8, device=dev)
ws = torch.zeros(G.band_workspace_bytes(a.height, a.width, False, 1), dtype=torch.uint8, device=dev)
pb = G.unproject_batch(d[None], img[None], density="high", workspace=ws)
torch.cuda.synchronize()
print("batch stats", pb.stats[0].tolist())
show("batch", ws)
comm = RcclComm(nranks=1, rank=0)
r = G.unproject_band(d, img, a.height, a.width, 0, a.height, comm=comm, workspace=ws)
torch.cuda.synchronize()
print("band stats", r[3].tolist())
show("band", ws)
comm.close()

"""Diagnostic: per-block s_memtime phases of the 128x128 GEMM (needs I2PC_LIB=.../libi2pc_stamps.so)."""
import ctypes, math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import ops, _lib
m, n, k = (int(v) for v in sys.argv[1:4])
bm = int(sys.argv[4]) if len(sys.argv) > 4 else 128
dev = torch.device("cuda")
x = (torch.rand(m, k) * 2 - 1).to(torch.bfloat16).to(dev)
w = ((torch.rand(n, k) * 2 - 1) / math.sqrt(k)).to(torch.bfloat16).to(dev)
out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
for _ in range(5): ops.linear(x, w, out=out)
torch.cuda.synchronize()
ops.linear(x, w, out=out); torch.cuda.synchronize()
lib = _lib.load()
nb = ((m + bm - 1) // bm) * (n // bm)
buf = (ctypes.c_ulonglong * (nb * 8))()
lib.i2pc_debug_stamps(buf, nb * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
t0 = a[:, 0].min()
pro = a[:, 1] - a[:, 0]; loop = a[:, 2] - a[:, 1]; epi = a[:, 3] - a[:, 2]
print(f"blocks {nb}: prologue med {np.median(pro):.0f} cyc, loop med {np.median(loop):.0f} (per K-step {np.median(loop)/(k//64):.0f}), epilogue med {np.median(epi):.0f}")
print(f"epi phase1 med {np.median(a[:,4]-a[:,2]):.0f} phase2 med {np.median(a[:,3]-a[:,4]):.0f}")
print(f"span {a[:,3].max()-t0} cyc; start spread: first wave of starts median {np.median(a[:512,0]-t0):.0f}")
order = np.argsort(a[:, 0])
print("first 8 blocks start/loop/epi:", [(int(a[i,0]-t0), int(loop[i]), int(epi[i])) for i in order[:8]])

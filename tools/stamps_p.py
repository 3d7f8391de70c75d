"""Diagnostic: per-tile s_memtime phases of the persistent GEMM engine (I2PC_LIB=.../libi2pc_stamps.so).

usage: I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so python tools/stamps_p.py M N K [gelu|lnp]
(lnp: the LayerNorm-fold producer with the fp32 residual in place, EPI_LNP)"""
import ctypes, math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import ops, _lib
m, n, k = (int(v) for v in sys.argv[1:4])
act = sys.argv[4] if len(sys.argv) > 4 else None
lnp = act == "lnp"
if lnp:
    act = None
dev = torch.device("cuda")
x = (torch.rand(m, k) * 2 - 1).to(torch.bfloat16).to(dev)
w = ((torch.rand(n, k) * 2 - 1) / math.sqrt(k)).to(torch.bfloat16).to(dev)
b = torch.randn(n).to(dev)
out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
kw = {}
if lnp:
    out = torch.randn(m, n, device=dev)
    kw = dict(res=out, ln_part=torch.empty(m, n // 64, 2, device=dev),
              out_bf16=torch.empty(m, n, dtype=torch.bfloat16, device=dev), ln_shift=torch.zeros(m, device=dev))
for _ in range(10): ops.linear(x, w, bias=b, act=act, out=out, **kw)
torch.cuda.synchronize()
lib = _lib.load()
lib.i2pc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = 256
buf = (ctypes.c_ulonglong * (nb * 64))()
ctypes.memset(buf, 0, ctypes.sizeof(buf))
lib.i2pc_debug_stamps(buf, nb * 64)   # zero the device copy? (it reads); run once more then read
ops.linear(x, w, bias=b, act=act, out=out, **kw); torch.cuda.synchronize()
lib.i2pc_debug_stamps(buf, nb * 64)
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8, 8).astype(np.int64)
print(f"{m}x{n}x{k} act={act} lnp={lnp}")
t0 = a[:, 0, 0][a[:, 0, 0] > 0].min()
for ti in range(8):
    v = a[:, ti, :]
    ok = (v[:, 0] > 0) & (v[:, 3] >= v[:, 0])
    if not ok.any():
        continue
    v = v[ok]
    print(f"tile#{ti}: blocks {ok.sum():3d}  start(med) {np.median(v[:,0]-t0):8.0f}  wait0 {np.median(v[:,1]-v[:,0]):6.0f}  "
          f"kloop {np.median(v[:,2]-v[:,1]):7.0f} (/step {np.median(v[:,2]-v[:,1])/(k//64):5.0f}, waits/step {np.median(v[:,4])/(k//64):5.0f})  epi {np.median(v[:,3]-v[:,2]):6.0f}  "
          f"end(max) {np.max(v[:,3]-t0):8.0f}")

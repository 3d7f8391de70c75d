"""Diagnostic: per-block s_memtime phases of the tile GEMM kernel k_gemm (I2PC_LIB=.../libi2pc_stamps.so).

usage: I2PC_LIB=image_to_pointcloud_amd/libi2pc_stamps.so python tools/stamps_tile.py M N K BM BN [bf16|lnp|lnpbf]
(lnp: fp32 residual in place + the LayerNorm-fold producer, the DPT-Large O / FC2 epilogue)
Prints the per-block start / first-stage wait / K-loop / epilogue phase 1 / phase 2 medians and the
distribution of block end times (cycles of s_memtime, the shader clock)."""
import ctypes, math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from image_to_pointcloud_amd import ops, _lib
m, n, k, bm, bn = (int(v) for v in sys.argv[1:6])
mode = sys.argv[6] if len(sys.argv) > 6 else "bf16"
dev = torch.device("cuda")
x = (torch.rand(m, k) * 2 - 1).to(torch.bfloat16).to(dev)
w = ((torch.rand(n, k) * 2 - 1) / math.sqrt(k)).to(torch.bfloat16).to(dev)
b = torch.randn(n).to(dev)
if mode == "lnp":
    out = torch.randn(m, n, device=dev)
    kw = dict(res=out, ln_part=torch.empty(m, n // 64, 2, device=dev),
              out_bf16=torch.empty(m, n, dtype=torch.bfloat16, device=dev), ln_shift=torch.zeros(m, device=dev))
elif mode == "lnpbf":   # the bf16 residual stream: res = out (bf16, in place) + res_shift, bf16 shifted output
    out = torch.randn(m, n, device=dev).to(torch.bfloat16)
    C = 64 if n % 256 == 0 else 32   # the networks' LayerNorm chunk (DA-v2's 384 columns: 32)
    kw = dict(res=out, res_shift=torch.zeros(m, device=dev), ln_part=torch.empty(m, n // C, 2, device=dev),
              ln_shift=torch.zeros(m, device=dev), ln_chunk=C)
else:
    out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    kw = {}
call = lambda: ops.linear(x, w, bias=b, out=out, **kw)
for _ in range(20):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    call()
e1.record()
torch.cuda.synchronize()
print(f"{m}x{n}x{k} {bm}x{bn} {mode}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call (event-timed, 20 calls)")
call()
torch.cuda.synchronize()
lib = _lib.load()
nb = ((m + bm - 1) // bm) * (n // bn)
buf = (ctypes.c_ulonglong * (nb * 8))()
lib.i2pc_debug_stamps(buf, nb * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
t0 = a[:, 0].min()
st = a[:, 0] - t0
pro = a[:, 1] - a[:, 0]
loop = a[:, 2] - a[:, 1]
p1 = a[:, 4] - a[:, 2]
p2 = a[:, 3] - a[:, 4]
end = a[:, 3] - t0
q = lambda v: "/".join(f"{np.percentile(v, p):.0f}" for p in (5, 50, 95))
print(f"blocks {nb} (cycles, p5/p50/p95): start {q(st)}  first stage {q(pro)}  K-loop {q(loop)} "
      f"(per K-step {np.median(loop) / (k // 64):.0f})  epi phase1 {q(p1)}  phase2 {q(p2)}  end {q(end)}  span {end.max()}")
if (a[:, 5] > 0).all():
    print(f"  RQ path: pass-0 phase 2 + pass-1 phase 1 {q(a[:, 6] - a[:, 4])}  pass-1 residual wait {q(a[:, 5] - a[:, 6])}  "
          f"last pass start -> end {q(a[:, 3] - a[:, 7])}")

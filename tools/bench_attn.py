"""Attention microbenchmark on the DPT-Large / DA-small shapes (I2PC_ATTN_OLD=1 selects the previous kernel)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops
SHAPES = [(32, 577, 16), (32, 1370, 6), (8, 1370, 6)]
if os.environ.get("ATTN_SHAPE"): SHAPES = [SHAPES[int(os.environ["ATTN_SHAPE"])]]
Q2 = os.environ.get("ATTN_Q2", "1") == "1"
for B, T, H in SHAPES:
    qkv = torch.randn(B * T, 3 * H * 64, device="cuda") * 1.5
    if Q2:   # the Q block in the exp2 domain, as a QKV GEMM with ops.fold_q_scale weights writes it
        qkv[:, :H * 64] *= 0.125 * ops.LOG2E
    qkv = qkv.to(torch.bfloat16)
    out = torch.empty(B * T, H * 64, dtype=torch.bfloat16, device="cuda")
    ops.attention(qkv, B, T, H, 0.125, out=out, q_log2=Q2); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): ops.attention(qkv, B, T, H, 0.125, out=out, q_log2=Q2)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"q2={int(Q2)} old={os.environ.get('I2PC_ATTN_OLD', '0')} occ={os.environ.get('I2PC_ATTN_OCC', '-')} B={B} T={T} H={H}: {t*1e6:8.1f} us {4*B*H*T*T*64/t/1e12:6.1f} TF")

"""Accuracy of i2pc_attention_q2 against fp64 softmax attention on the same bf16 inputs (Q in the exp2
domain, as the networks feed it); the library comes from I2PC_LIB when set (variant builds)."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops
dev = torch.device("cuda")
for (B, T, H) in [(32, 577, 16), (8, 1370, 6)]:
    for sd in (1.0, 3.0, 6.0):
        g = torch.Generator(device="cpu").manual_seed(int(sd * 10) + T)
        D = H * 64
        q = torch.randn(B, T, H, 64, generator=g) * math.sqrt(sd / 8.0) * 1.4426950408889634
        k = torch.randn(B, T, H, 64, generator=g) * math.sqrt(sd * 8.0) / 8.0
        v = torch.randn(B, T, H, 64, generator=g)
        qkv = torch.cat([q.reshape(B, T, D), k.reshape(B, T, D), v.reshape(B, T, D)], -1).to(torch.bfloat16).to(dev)
        out = torch.empty(B * T, D, dtype=torch.bfloat16, device=dev)
        ops.attention(qkv.view(B * T, 3 * D), B, T, H, 1.0, out=out, q_log2=True)
        torch.cuda.synchronize()
        x = qkv.double().view(B, T, 3, H, 64)
        Q, K, V = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
        s = (Q @ K.transpose(-1, -2)) * math.log(2.0)
        ref = (torch.softmax(s, -1) @ V).transpose(1, 2).reshape(B * T, D)
        got = out.double()
        rel = ((got - ref).norm() / ref.norm()).item()
        mx = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"B={B} T={T} H={H} score_sd~{sd}: rel_l2 {rel:.3e} max_rel {mx:.3e}", flush=True)

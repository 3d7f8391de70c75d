"""attn_rb variants of the q2 kernel (r06: also the since-removed software-pipelined k_attention_sp) on the C2 / DA-v2 / C3 attention shapes, in one
process, interleaved: median event time per call and the largest output difference."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd import ops

dev = torch.device("cuda")


def timeit(fn, iters=20):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


for T, H, B in ((577, 16, 32), (1370, 6, 32), (577, 16, 64), (1370, 6, 62)):
    g = torch.Generator(device="cpu").manual_seed(T)
    qkv = torch.randn(B * T, 3, H, 64, generator=g) * 1.2
    qkv[:, 0] *= 0.125 * 1.4426950408889634
    qkv = qkv.reshape(B * T, 3 * H * 64).to(torch.bfloat16).to(dev)
    V = [int(v) for v in os.environ.get('RB_VARIANTS', '0,1').split(',')]
    times = {v: [] for v in V}
    outs = {}
    for rnd in range(5):
        for sp in V:
            ops.set_tuning("attn_rb", sp)
            out = torch.empty(B * T, H * 64, dtype=torch.bfloat16, device=dev)
            times[sp].append(timeit(lambda: ops.attention(qkv, B, T, H, 0.125, out=out, q_log2=True)))
            outs[sp] = out
    ops.set_tuning("attn_rb", 1)
    fl = 4.0 * B * H * T * T * 64
    t0 = statistics.median(times[V[0]])
    line = " | ".join(f"rb{v} {statistics.median(times[v]) * 1e6:7.1f} us {fl / statistics.median(times[v]) / 1e12:5.0f} TF "
                      f"x{t0 / statistics.median(times[v]):5.3f} {'=' if torch.equal(outs[v], outs[V[0]]) else '~%.2g' % (outs[v].float() - outs[V[0]].float()).abs().max().item()}"
                      for v in V)
    print(f"T{T} H{H} B{B}: {line}", flush=True)

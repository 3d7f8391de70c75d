"""k_head_upconv on the networks' head shapes: time per call (HIP events on the launch stream,
median of interleaved repetitions) and the MFMA rate of its 3x3 conv.

  python tools/bench_head.py [C2 C5 DA]   # C2 (DPT-Large B=32), C5 (DPT-Hybrid B=64), DA-v2 (B=32)
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from image_to_pointcloud_amd import ops  # noqa: E402

SHAPES = {  # name: (B, h, w, C pitch, channels used, H, W)
    "C2 dpt-large": (32, 192, 192, 128, 128, 384, 384),
    "C5 dpt-hybrid": (64, 192, 192, 128, 128, 384, 384),
    "DA-v2 small": (32, 296, 296, 64, 32, 518, 518),
}


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    cases = []
    only = sys.argv[1:]
    for name, (B, h, w, C, cin, H, W) in SHAPES.items():
        if only and not any(o in name for o in only):
            continue
        x = torch.randn(B, h, w, C, generator=g).to(torch.bfloat16).to(dev)
        w2 = (torch.randn(32, 9 * C, generator=g) / (9 * cin) ** 0.5).to(torch.bfloat16).to(dev)
        b2 = (torch.randn(32, generator=g) * 0.1).to(dev)
        w4 = (torch.randn(32, generator=g) / 32 ** 0.5).to(dev)
        out = torch.empty(B, H, W, device=dev)
        cases.append((name, (x, H, W, w2, b2, w4, 0.05, out, cin), 2.0 * B * H * W * 32 * 9 * cin))
    times = {c[0]: [] for c in cases}
    for rep in range(7):
        for name, a, _ in cases:
            x, H, W, w2, b2, w4, b4, out, cin = a
            for _ in range(2):
                ops.head_upconv(x, H, W, w2, b2, w4, b4, out=out, cin=cin)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                ops.head_upconv(x, H, W, w2, b2, w4, b4, out=out, cin=cin)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / 5)
    for name, _, flops in cases:
        us = statistics.median(times[name])
        print(f"{name:14s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  ({flops / 1e9:.1f} GFLOP)", flush=True)


if __name__ == "__main__":
    main()

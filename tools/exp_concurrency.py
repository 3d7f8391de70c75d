"""Does a HIP graph run two independent half-batch network branches concurrently?
One DPT-Large forward on B images (one stream) vs two model instances on B/2 images each,
captured on two forked streams into one graph.  Prints ms per B images for both."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_to_pointcloud_amd.dpt import DPT_LARGE, DPTDepthModel, synthetic_state_dict
from image_to_pointcloud_amd.preprocess import patch_pitch
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
gh = gw = DPT_LARGE.image // DPT_LARGE.patch
sd = synthetic_state_dict(DPT_LARGE, 0)
ma, mb = DPTDepthModel(DPT_LARGE, sd, dev), DPTDepthModel(DPT_LARGE, sd, dev)
pp = patch_pitch(DPT_LARGE.patch)
x = torch.randn(B * gh * gw, pp, device=dev).to(torch.bfloat16)
xa, xb = x[: B // 2 * gh * gw], x[B // 2 * gh * gw:]


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(); fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def one():
    ma(x, B, gh, gw)


s2 = torch.cuda.Stream()


def two():
    cur = torch.cuda.current_stream()
    s2.wait_stream(cur)
    ma(xa, B // 2, gh, gw)
    with torch.cuda.stream(s2):
        mb(xb, B // 2, gh, gw)
    cur.wait_stream(s2)


def two_seq():
    ma(xa, B // 2, gh, gw)
    mb(xb, B // 2, gh, gw)


g1, g2, g3 = capture(one), capture(two), capture(two_seq)
print(f"B={B}: one stream {timed(g1.replay):.3f} ms; two half-batches on two streams {timed(g2.replay):.3f} ms; "
      f"two half-batches on one stream {timed(g3.replay):.3f} ms")

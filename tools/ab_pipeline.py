"""In-process A/B of kernel-selection knobs on the bench pipeline (one device, one process, interleaved
rounds: cdna_hip_programming.md rule 24).  Each variant re-captures the HIP graph with its knobs and
times `steps` replays; prints per-variant median / min ms per step over the rounds.

    python tools/ab_pipeline.py [--model dpt-large] [--size 1024] [--batch 32] \
        --variant base: --variant notail:gemm_tail=0 --variant p:engine=3
"""
import argparse, os, statistics, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="dpt-large")
ap.add_argument("--dtype", default=None)
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--variant", action="append", default=[], help="name:knob=v,knob=v (engine=<mode> for the GEMM engine)")
a = ap.parse_args()

from image_to_pointcloud_amd import ops
from image_to_pointcloud_amd.pipeline import PointCloudPipeline
import bench

spec = bench._spec(a.model)
dtype = a.dtype or ("fp8" if a.model == "dpt-hybrid" else "bf16")
dev = torch.device("cuda")
pipe = PointCloudPipeline(a.batch, a.size, a.size, spec=spec, density="high", device=dev, seed=0, dtype=dtype)
images = bench._images(a.batch, a.size, 0, dev)
variants = []
for v in a.variant or ["base:"]:
    name, _, kv = v.partition(":")
    knobs = dict((k, int(x)) for k, x in (p.split("=") for p in kv.split(",") if p))
    variants.append((name, knobs))
defaults = {"gemm_tail": 1, "gemm_bn128": 1, "gemm_splitk": 1, "gemm_split_tile": 0, "gemm_tile192": 1, "gemm_lnp_p": 0, "gemm_lnp_stream": 0, "conv_halo": 3, "gelu_tanh": 1, "gemm_resq": 2, "gemm_simple_epi": 1, "gemm_tail160": 1, "gemm_stagger": 1, "unp_rows": 1, "unp_nt": 1, "unp_rpt": 8, "attn_lazy": 1, "attn_scalar": 1, "attn_rb": 1, "ln_f2": 1, "resize_rows": 1, "engine": 0}


def apply(knobs):
    for k, dv in defaults.items():
        val = knobs.get(k, dv)
        if k == "engine":
            ops.set_gemm_engine(val)
        else:
            ops.set_tuning(k, val)


times = {n: [] for n, _ in variants}
outs = {}
for r in range(a.rounds):
    for name, knobs in variants:
        apply(knobs)
        pipe.capture(images)
        for _ in range(3):
            pipe.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            pipe.replay()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) / a.steps * 1e3)
        if r == 0:
            outs[name] = pipe._out.xyz[:2].clone()
apply({})
base = variants[0][0]
for name, _ in variants:
    med = statistics.median(times[name])
    same = torch.equal(outs[name], outs[base])
    pts = a.batch * pipe.points_per_image
    print(f"{name:12s} med {med:7.3f} ms/step  min {min(times[name]):7.3f}  {pts / med / 1e3:8.1f} Mpts/s  "
          f"vs {base}: {statistics.median(times[base]) / med:6.3f}x  xyz bit-equal: {same}", flush=True)

"""C4: tile-parallel unprojection of one 8192 x 4096 panorama across the ranks of one node.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P tools/c4_panorama.py [--height 4096 --width 8192 --steps 10]

Each rank holds the model-resolution depth (518 x 1036, the Depth-Anything processor's
keep-aspect size for 2:1; synthetic smooth field + a NaN) and ONLY its band of
the image rows; the band call runs the exact global p2/p98 through three histogram
all-reduces per selection pass, then unprojects its band.  With one GPU per rank the
exchange is device-side (i2pc_unproject_band_rccl on an RCCL communicator of libi2pc.so,
and --graph captures each rank's whole band call into a HIP graph); when ranks share a GPU
it falls back to the host-callback exchange over gloo (correctness runs only).  Rank 0 prints one JSON line (points/s over the job, max
over ranks), and --check compares every band bit-for-bit with the whole-image unprojection.

--network runs the depth network too, on a STREAM of panoramas: a step takes one panorama per
rank, and rank k preprocesses panorama k to the Depth-Anything-V2-Small input (518 x 1036,
keep-aspect /14) and runs the network (seeded random weights) -- all ranks at once -- then
for each panorama its owner broadcasts the 518 x 1036 depth over RCCL and every rank
unprojects its band of it (ms_per_image = a step / its N panoramas: network / N + broadcast +
band call).  --projection equirect back-projects the panorama on the sphere (i2pc.h; the
reference only has the pinhole model); --smooth applies smooth_depth (the band's blurred field
with its halo rows, recomputed locally); --levels takes the four histogram levels with a host
exchange instead of the one-sweep window selection.  --gather then all-gathers every band's points
onto every rank (the whole panorama's point cloud, row-major), timed apart as
gather_ms; with --check the assembled cloud must equal the whole-image unprojection bit for bit.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import torch.distributed as dist

from image_to_pointcloud_amd import distributed as D
from image_to_pointcloud_amd import geometry as G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--width", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--density", default="high")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--graph", action="store_true", help="replay each rank's band call as a HIP graph (RCCL mode)")
    ap.add_argument("--network", action="store_true", help="depth from Depth-Anything-V2-Small on rank 0, broadcast")
    ap.add_argument("--projection", default="pinhole", choices=["pinhole", "equirect"])
    ap.add_argument("--smooth", action="store_true", help="smooth_depth (GaussianBlur, --ksize)")
    ap.add_argument("--ksize", type=int, default=5)
    ap.add_argument("--levels", action="store_true", help="histogram-level selection, host-callback exchange")
    ap.add_argument("--gather", action="store_true",
                    help="then all-gather every band's points onto every rank (SURVEY 8e step 3), timed apart")
    a = ap.parse_args()
    rank, local, world = D.world()
    ngpu = torch.cuda.device_count()
    backend = "nccl" if world <= ngpu else "gloo"
    dev = torch.device("cuda", local % ngpu)
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    H, W = a.height, a.width
    h, w = 518, 1036
    rng = np.random.Generator(np.random.PCG64(1))
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    dep = (0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w) * np.cos(4 * np.pi * v / h))
           + rng.normal(0, 0.05, (h, w))).astype(np.float32)
    dep[7, 11] = np.nan
    tdep = torch.from_numpy(dep).to(dev)
    step = G.DENSITY_STEP[a.density]
    r0, r1 = G.band_rows(H, world, step)[rank]
    # this rank's image rows only (row y of the synthetic panorama is seeded 1000 + y)
    band = np.empty((r1 - r0, W, 3), np.uint8)
    for y in range(r0, r1):
        band[y - r0] = np.random.Generator(np.random.PCG64(1000 + y)).integers(0, 256, (W, 3), dtype=np.uint8)
    timg = torch.from_numpy(band).to(dev)
    nets = world if a.network else 1        # panoramas per step
    if a.network:
        from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
        from image_to_pointcloud_amd.pipeline import PointCloudPipeline
        full = np.empty((H, W, 3), np.uint8)    # this rank's panorama of the step (same content on every rank)
        for y in range(H):
            full[y] = np.random.Generator(np.random.PCG64(1000 + y)).integers(0, 256, (W, 3), dtype=np.uint8)
        tfull = torch.from_numpy(full).to(dev)[None]
        net = PointCloudPipeline(1, H, W, spec=DA_V2_SMALL, density=a.density, device=dev)
        h, w = net.pre.out_h, net.pre.out_w
        del full
        own = torch.empty((h, w), dtype=torch.float32, device=dev)
        deps = [torch.empty((h, w), dtype=torch.float32, device=dev) for _ in range(world)]

        def infer():
            own.copy_(net.infer_depth(tfull)[0])        # every rank: its own panorama's depth
            for k in range(world):                      # then panorama k's depth from its owner
                if world > 1:
                    if k == rank:
                        deps[k].copy_(own)
                    if backend == "nccl":
                        dist.broadcast(deps[k], k)
                    else:                               # gloo: through host memory
                        hk = deps[k].cpu()
                        dist.broadcast(hk, k)
                        deps[k].copy_(hk)
                else:
                    deps[k].copy_(own)
        infer()
        tdep = deps[0]
    if a.levels:
        comm = None
    else:
        comm = D.RcclComm() if world > 1 and backend == "nccl" else (D.RcclComm(nranks=1, rank=0) if world == 1 else None)
    ex = D.band_exchange() if comm is None else None
    gather = D.band_gather() if comm is None and not a.levels else None
    nbytes = (G.band_workspace_bytes(H, W, a.smooth, world) if comm is not None or gather is not None
              else G.workspace_bytes(1, H, W, a.smooth))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    res = None

    def band_call(d=None):
        return G.unproject_band(tdep if d is None else d, timg, H, W, r0, r1, ex, density=a.density, comm=comm,
                                workspace=ws, out=res, projection=a.projection, smooth=a.smooth,
                                smooth_ksize=a.ksize, gather=gather, nranks=world if gather else None)

    def run():
        if a.network:
            infer()
            for k in range(world):
                r = band_call(deps[k])
            return r
        return band_call()
    for _ in range(max(1, a.warmup)):
        res = run()
    torch.cuda.synchronize()
    step_fn = run
    if a.graph and comm is not None:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            band_call()
        if a.network:
            graphs = []
            for k in range(world):
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk):
                    band_call(deps[k])
                graphs.append(gk)
            step_fn = lambda: (infer(), [gk.replay() for gk in graphs])   # noqa: E731
        else:
            step_fn = graph.replay
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step_fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = D.max_over_ranks(time.perf_counter() - t0, dev) if world > 1 else time.perf_counter() - t0
    bbox = D.reduce_bbox(res[2]) if world > 1 else res[2]
    gathered, gather_ms = None, None
    if a.gather:
        nmax = max(D.band_point_counts(H, W, world, step))
        pad = (res[0].new_zeros((nmax, 3)), res[1].new_zeros((nmax, 3)))
        gathered = D.gather_band_points(res[0], res[1], H, W, step, pad=pad)   # (warm-up)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            gathered = D.gather_band_points(res[0], res[1], H, W, step, pad=pad)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        g_el = D.max_over_ranks(time.perf_counter() - t1, dev) if world > 1 else time.perf_counter() - t1
        gather_ms = round(g_el / a.steps * 1e3, 3)
    ok = None
    if a.check:
        full = np.empty((H, W, 3), np.uint8)
        for y in range(H):
            full[y] = np.random.Generator(np.random.PCG64(1000 + y)).integers(0, 256, (W, 3), dtype=np.uint8)
        if a.network:
            tdep = deps[world - 1]      # the last band call of the step unprojected the last panorama
        whole = G.unproject_batch(tdep[None], torch.from_numpy(full).to(dev)[None], density=a.density,
                                  projection=a.projection, smooth=a.smooth, smooth_ksize=a.ksize)
        wn = (W + step - 1) // step
        p0 = (r0 // step) * wn
        ok = bool(torch.equal(whole.xyz[0][p0:p0 + res[0].shape[0]], res[0])
                  and torch.equal(whole.rgb[0][p0:p0 + res[1].shape[0]], res[1])
                  and torch.equal(whole.stats[0].view(torch.int64), res[3].view(torch.int64))   # NaN-aware
                  and torch.equal(whole.bbox[0], bbox))
        if gathered is not None:        # the assembled panorama equals the whole-image call
            ok = ok and bool(torch.equal(whole.xyz[0], gathered[0]) and torch.equal(whole.rgb[0], gathered[1]))
        if world > 1:
            t = torch.tensor([int(ok)], device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = bool(t.item())
    n = ((H + step - 1) // step) * ((W + step - 1) // step)
    if rank == 0:
        print(json.dumps({"metric": "Mpoints/sec tile-parallel unprojection of one panorama (C4)",
                          "value": round(n * nets * a.steps / el / 1e6, 1), "unit": "Mpoints/s", "n_ranks": world,
                          "backend": backend if world > 1 else None,
                          "exchange": ("RCCL on device (i2pc_unproject_band_rccl: counters all-reduce + window "
                                       "candidates all-gather)" if comm is not None else
                                       "host callback (" + ("histogram levels" if a.levels else "window selection") + ")"),
                          "hip_graph": bool(a.graph and comm is not None),
                          "ms_per_image": round(el / (a.steps * nets) * 1e3, 3), "panoramas_per_step": nets,
                          "smooth": a.smooth,
                          "image": [H, W], "depth": [h, w], "density": a.density, "points": n,
                          "depth_source": "depth-anything-v2-small (seeded weights): panorama k on rank k, "
                                          "RCCL broadcast from its owner"
                          if a.network else "synthetic smooth field + NaN",
                          "projection": a.projection,
                          "points_gathered": None if gathered is None else int(gathered[0].shape[0]),
                          "gather_ms": gather_ms,
                          "bit_exact_vs_whole_image": ok, "stats": res[3].tolist(), "bbox": bbox.tolist()}))
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

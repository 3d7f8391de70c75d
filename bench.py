#!/usr/bin/env python3
"""Mpoints/sec end-to-end (depth + unproject) on synthetic 1024x1024 RGB batches.

BASELINE.json metric / configs[1]: DPT-Large bf16, batch 32 x 1024^2, one
MI355X per rank.  A step = preprocess + DPT-Large forward + depth resize +
exact p2/p98 + normalise + unproject (density "high", 1,048,576 points/image)
+ RGB gather + bbox, for the rank's batch, inputs already resident in HBM,
replayed as one HIP graph.  Ranks shard images (weak scaling, no data-path
collective: each rank owns its images' point buffers).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line.  Besides the contract fields it carries
  roofline      -- the dominant kernel (by time in one eager, event-timed step):
                   achieved = algorithmic FLOPs / average launch duration
                   (HIP events on the launch stream), peak = 2.5 PF bf16 dense;
  roofline_unproject -- the geometry stage against HBM (8 TB/s), algorithmic
                   bytes 4*h'*w' + 18*N per image;
  cpu_baseline  -- the reference CPU path restated (oracle/: Pillow-exact
                   preprocessing, transformers fp32 DPT-Large forward on all
                   host threads, the reference's per-point Python loop) on ONE
                   1024^2 image, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (AMD's 5 PF headline is 2:1 sparse)
FP8_PEAK_TFLOPS = 5000.0       # dense MX fp8 (v_mfma_scale_f32_*_f8f6f4, 2x bf16 per clock)


def _peak(label: str) -> float:
    """Dense MFMA peak of the dtype a kernel computes in (fp8 engine labels: k_gemm_f8<...>)."""
    return FP8_PEAK_TFLOPS if label.startswith("k_gemm_f8") else BF16_PEAK_TFLOPS


class ByteAccountingError(RuntimeError):
    """A kernel label's algorithmic bytes / measured time exceed the HBM peak: its byte formula
    (ops.py `_Timed`) charges more than 'every operand read once, every output written once'."""


def check_byte_accounting(kernels: dict, peak_gbs: float = HBM_PEAK_GBS) -> dict:
    """Raise ByteAccountingError naming every kernel whose algorithmic rate is above the HBM peak
    (k_resize once charged four input taps per output and read 13 TB/s)."""
    over = {k: v["gbs"] for k, v in kernels.items() if v.get("gbs") and v["gbs"] > peak_gbs}
    if over:
        raise ByteAccountingError(f"algorithmic GB/s above the {peak_gbs:.0f} GB/s HBM peak: {over}")
    return {"ok": True, "max_gbs": max([v["gbs"] for v in kernels.values() if v.get("gbs")] or [0.0]),
            "peak_gbs": peak_gbs}


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without a torch.distributed.run environment, N > 1 "
                         "starts torch.distributed.run with N ranks as a child process and relays its output")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend at N > 1: nccl (= RCCL over xGMI, one GPU per rank) or gloo "
                         "(ranks may share a GPU: rank r uses device r %% device_count; the point gather is "
                         "staged through host memory)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--density", default="high", choices=["low", "medium", "high"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-profile", action="store_true")
    ap.add_argument("--no-all-gather", action="store_true",
                    help="world > 1: skip the C3 all-gather of every rank's point buffers (RCCL over xGMI), "
                         "which by default runs inside every step, overlapped with the next step's compute")
    ap.add_argument("--no-medium", action="store_true",
                    help="N = 1, density high: skip the density-medium sub-record (the reference's default "
                         "density, a second pipeline on the same model, timed after the headline steps)")
    ap.add_argument("--strict-accounting", action="store_true",
                    help="raise ByteAccountingError when a kernel's algorithmic GB/s exceeds the HBM peak "
                         "(default: report it in the line's byte_accounting field)")
    ap.add_argument("--model", default="dpt-large", choices=["dpt-large", "dpt-hybrid", "depth-anything-v2"])
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp8"],
                    help="network arithmetic (fp8 = MX e4m3 on the scaled MFMA; DPT-Hybrid only). "
                         "Default: fp8 for dpt-hybrid (BASELINE configs[4]), bf16 otherwise")
    a = ap.parse_args()
    if a.dtype is None:
        a.dtype = "fp8" if a.model == "dpt-hybrid" else "bf16"
    return a


def _spec(name):
    if name == "depth-anything-v2":
        from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
        return DA_V2_SMALL
    if name == "dpt-hybrid":
        from image_to_pointcloud_amd.dpt_hybrid import DPT_HYBRID
        return DPT_HYBRID
    from image_to_pointcloud_amd.dpt import DPT_LARGE
    return DPT_LARGE


def _images(batch, size, rank, device):
    import numpy as np
    import torch
    out = torch.empty((batch, size, size, 3), dtype=torch.uint8, device=device)
    for i in range(batch):
        rng = np.random.Generator(np.random.PCG64(1000 + rank * batch + i))   # image i seeded 1000+i
        out[i] = torch.from_numpy(rng.integers(0, 256, (size, size, 3), dtype=np.uint8)).to(device)
    return out


def _kernel_profile(pipe, images, reps=5):
    """Eager steps with HIP events around every network launch + the geometry stage; the
    geometry stage and the unprojection kernel inside it are the medians over `reps` steps
    (each right after the network, as in the timed loop), the network launches the last step's."""
    import torch
    from image_to_pointcloud_amd import _lib, geometry, ops
    stream = torch.cuda.current_stream()
    lib = _lib.load()
    geo, unp = [], []
    for _ in range(reps):
        ops.profile = []
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        pipe.pre(images, layout=pipe.layout, out=pipe._patches)
        depth = pipe.model(pipe._patches, pipe.batch)
        lib.i2pc_profile_enable(1)
        e0.record(stream)
        geometry.unproject_batch(depth, images, density=pipe.density, invert=pipe.invert,
                                 depth_scale=pipe.depth_scale, out=pipe._out, workspace=pipe._ws)
        e1.record(stream)
        torch.cuda.synchronize()
        unp.append(lib.i2pc_profile_unproject_ms())
        lib.i2pc_profile_enable(0)
        geo.append(e0.elapsed_time(e1))
    unp_ms = sorted(unp)[len(unp) // 2]
    recs = ops.profile
    ops.profile = None
    per = {}
    for label, flops, nbytes, a, b in recs:
        t = a.elapsed_time(b) * 1e-3
        d = per.setdefault(label, {"n": 0, "t": 0.0, "flops": 0.0, "bytes": 0.0})
        d["n"] += 1
        d["t"] += t
        d["flops"] += flops
        d["bytes"] += nbytes
    geo_t = sorted(geo)[len(geo) // 2] * 1e-3
    return per, geo_t, (unp_ms * 1e-3 if unp_ms > 0 else None)


def _density_record(a, spec, pipe, images, device, density):
    """The same workload at another density step on the same model (s = 2, the reference's
    default `medium`, app.py:52,226, beside the headline s = 1): a second captured pipeline, `a.warmup`
    untimed and `a.steps` timed replays, then the geometry stage / unprojection kernel by HIP events."""
    import torch
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    B, S = a.batch, a.size
    p = PointCloudPipeline(B, S, S, spec=spec, density=density, device=device, model=pipe.model, dtype=a.dtype)
    if a.no_graph:
        step = lambda: p.run(images)       # noqa: E731
    else:
        p.capture(images)
        step = p.replay
    for _ in range(max(a.warmup, 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rec = {"density": density, "points_per_image": p.points_per_image,
           "value": round(B * p.points_per_image * a.steps / el / 1e6, 2), "unit": "Mpoints/s",
           "ms_per_step": round(el / a.steps * 1e3, 3), "steps": a.steps}
    if not a.no_kernel_profile:
        _, geo_t, unp_t = _kernel_profile(p, images)
        geo_bytes = B * (4.0 * p.pre.out_h * p.pre.out_w + 18.0 * p.points_per_image)
        rec["unproject_stage"] = {"ms": round(geo_t * 1e3, 3), "achieved_gbs": round(geo_bytes / geo_t / 1e9, 1),
                                  "frac": round(geo_bytes / geo_t / 1e9 / HBM_PEAK_GBS, 4),
                                  "bytes_per_step": geo_bytes}
        if unp_t:
            rec["unproject_kernel"] = {"us": round(unp_t * 1e6, 1), "achieved_gbs": round(geo_bytes / unp_t / 1e9, 1),
                                       "frac": round(geo_bytes / unp_t / 1e9 / HBM_PEAK_GBS, 4)}
    del p
    return rec


def kernels_sha16() -> str:
    """Hash of the device-code sources (csrc/*.hip and the headers they include): what a PMC traffic
    table depends on.  The host-only C++ (ABI glue, executor, writers) does not change a kernel's bytes."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "image_to_pointcloud_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))):
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def _pmc_traffic(tag: str):
    """HBM bytes per launch by kernel label from the newest profiles/r*_<tag>_pmc_traffic.json
    (tools/gpu.sh profile: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench,
    gfx950 FETCH_SIZE x2 correction of MI355X_MICROARCH.md) -> (table, source, stale), or
    ({}, None, None).  stale: the table was collected on other kernel sources than this run's
    (kernels_sha16), or predates the recorded hash."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_pmc_traffic.json")))
    if not files:
        return {}, None, None
    with open(files[-1]) as fh:
        d = json.load(fh)
    return d.get("kernels", {}), os.path.relpath(files[-1], ROOT), d.get("kernels_sha16") != kernels_sha16()


def _traffic(table, src, *names, calls_per_step=None):
    """PMC HBM bytes per CALL of a kernel label: every dispatch of the call in one step summed / the
    calls per step.  A persistent GEMM call may be a main launch plus a tail launch of another row
    tile (k_gemm_p<256, ...> + k_gemm_p<160, ...>): all row-tile variants of the label count.  The
    per-dispatch average when the table predates per-step sums or the call count is unknown."""
    import re
    for n in names:
        m = re.match(r"(k_gemm_p|k_gemm_f8)<\d+, (.*)>$", n)
        keys = ([k for k in table if re.match(re.escape(m[1]) + r"<\d+, " + re.escape(m[2]) + ">$", k)]
                if m else [n] if n in table else [])
        if not keys:
            continue
        if calls_per_step and all("hbm_bytes_per_step" in table[k] for k in keys):
            tot = sum(table[k]["hbm_bytes_per_step"] for k in keys)
            return round(tot / calls_per_step), f"{src}: {' + '.join(sorted(keys))} (per call)"
        return table[keys[0]]["hbm_bytes_per_launch"], f"{src}: {keys[0]} (per dispatch)"
    return None, None


def _clock_probe(device, iters=16384):
    """Shader clock (GHz) the chip holds under a dense bf16 MFMA loop right now: median over one
    workgroup per CU of s_memtime ticks / s_memrealtime (100 MHz) ticks (i2pc_clock_probe)."""
    import torch
    from image_to_pointcloud_amd import _lib
    props = torch.cuda.get_device_properties(device)
    wg = int(props.multi_processor_count)
    out = torch.zeros(2 * wg, dtype=torch.int64, device=device)
    _lib.call("i2pc_clock_probe", wg, iters, out.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
    v = out.view(wg, 2).double().cpu()
    ghz = sorted((v[:, 0] / v[:, 1] * 0.1).tolist())
    return ghz[len(ghz) // 2]


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_baseline(spec, size, density, images=3):
    """Reference CPU path (restated) on `images` images of the bench's size (seeds 1000+i, the
    bench's first images), density high: a bounded sample of ~10 s of CPU work."""
    import numpy as np
    import torch

    from oracle import preprocess_ref, unproject_ref
    from image_to_pointcloud_amd.pipeline import default_processor

    threads = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    threads = min(threads, int(cap)) if cap else threads
    torch.set_num_threads(threads)
    if spec.family == "depth-anything":
        from transformers import DepthAnythingConfig as Cfg, DepthAnythingForDepthEstimation as Net
        from image_to_pointcloud_amd.depth_anything import synthetic_state_dict
    elif spec.family == "dpt-hybrid":
        from transformers import DPTConfig as Cfg, DPTForDepthEstimation as Net
        from image_to_pointcloud_amd.dpt_hybrid import synthetic_state_dict
    else:
        from transformers import DPTConfig as Cfg, DPTForDepthEstimation as Net
        from image_to_pointcloud_amd.dpt import synthetic_state_dict
    model = Net(Cfg(**spec.hf_config_kwargs()))
    model.load_state_dict(synthetic_state_dict(spec, 0), strict=False)
    model.eval()
    _log(f"CPU baseline: transformers {spec.name} built, {threads} threads")
    proc = default_processor(spec)
    psize = proc.size if spec.family == "depth-anything" else (spec.image, spec.image)
    t_net = t_geo = 0.0
    n = 0
    for i in range(images):
        rng = np.random.Generator(np.random.PCG64(1000 + i))
        img = rng.integers(0, 256, (size, size, 3), dtype=np.uint8)
        t0 = time.perf_counter()
        pix = preprocess_ref.dpt_preprocess(img, size=psize, mean=proc.mean, std=proc.std,      # app.py:103,109
                                            keep_aspect_ratio=proc.keep_aspect_ratio, multiple=proc.multiple)
        with torch.no_grad():                                           # app.py:111-116
            depth = model(pixel_values=torch.from_numpy(pix)[None]).predicted_depth[0].numpy().astype(np.float32)
        t1 = time.perf_counter()
        pts, _ = unproject_ref.depth_to_point_cloud(img, depth, density=density, loop=True)  # app.py:174-250
        unproject_ref.gis_bounds(pts)
        t2 = time.perf_counter()
        t_net += t1 - t0
        t_geo += t2 - t1
        n += len(pts)
        _log(f"CPU baseline: image {i} network {t1 - t0:.2f} s, per-point loop {t2 - t1:.2f} s")
    return {"value": n / (t_net + t_geo) / 1e6, "unit": "Mpoints/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
            "sample": f"{images} images {size}x{size}, density {density} ({n} points): Pillow-exact preprocessing + "
                      f"transformers fp32 {spec.name} forward on {threads} threads"
                      + (f" (capped by OMP_NUM_THREADS={cap}, the job's CPU share, of {os.cpu_count()} host threads)"
                         if cap and threads < (os.cpu_count() or 1) else "")
                      + f" ({t_net:.2f} s) + the reference "
                      f"per-point Python loop, single-threaded ({t_geo:.2f} s)",
            "seconds": t_net + t_geo}


def _launch_ranks(a) -> int:
    """`--gpus N > 1` without a torch.distributed.run environment: start N ranks as a CHILD
    torch.distributed.run (this process has not touched the GPU: no exec after HIP init) and
    return its exit code; rank 0's JSON line reaches our stdout unchanged."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def _multi_gpu_diag(a, pipe, images, og, own_s, world, device):
    """N > 1: why the whole-job number is what it is, per rank.
    step_ms -- this rank's own timed-loop time per step (the job's value uses the max over ranks);
    compute_ms -- the same rank running its step alone, no gather, timed right after the loop;
    gather_wait_ms -- per step, how long the compute stream waited for the overlapped all-gather
    (OverlappedGather.gather_wait_ms; host-staged gloo: the whole synchronous staging)."""
    import torch
    import torch.distributed as dist
    wait_ms = og.gather_wait_ms() / a.steps if og is not None else 0.0
    run = og.runs[0] if og is not None else ((lambda: pipe.run(images)) if a.no_graph else pipe.replay)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    comp_ms = (time.perf_counter() - t0) / a.steps * 1e3
    mine = torch.tensor([own_s / a.steps * 1e3, comp_ms, wait_ms], dtype=torch.float64)
    backend = dist.get_backend()
    if backend != "gloo":
        mine = mine.to(device)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    per = [{"rank": r, "step_ms": round(float(v[0]), 3), "compute_ms": round(float(v[1]), 3),
            "gather_wait_ms": round(float(v[2]), 3)} for r, v in enumerate(allv)]
    return {"world": world, "backend": backend,
            "rccl_world_size": dist.get_world_size() if backend == "nccl" else None,
            "rccl_max_channels": int(os.environ["NCCL_MAX_NCHANNELS"]) if backend == "nccl" else None,
            "all_gather": og is not None,
            "gathered_bytes_per_step_per_rank": og.recv_bytes_per_step if og is not None else 0,
            "sent_bytes_per_step_per_rank": og.send_bytes_per_step if og is not None else 0,
            "per_rank": per}


def _log(msg: str) -> None:
    """Progress on stderr (a GPU run that writes nothing for minutes looks hung to its supervisor)."""
    print(f"bench: {msg}", file=sys.stderr, flush=True)


def main():
    a = _args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(_launch_ranks(a))
    if env_world is not None and int(env_world) != a.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {a.gpus}", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    from image_to_pointcloud_amd import distributed as D
    rank, local, world = D.world()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        ndev = torch.cuda.device_count()
        if a.backend == "nccl":
            if local >= ndev:
                print(f"bench.py: rank {rank} needs GPU {local}, {ndev} visible (nccl needs one GPU per rank; "
                      f"--backend gloo lets ranks share one)", file=sys.stderr)
                sys.exit(2)
            torch.cuda.set_device(local)
            D.cap_rccl_channels()               # bound RCCL's CU share before the communicator exists
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(ndev, 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    spec = _spec(a.model)

    B, S = a.batch, a.size
    _log(f"rank {rank}/{world}: building {spec.name} {a.dtype} pipeline, batch {B} x {S}^2")
    pipe = PointCloudPipeline(B, S, S, spec=spec, density=a.density, device=device, seed=0, dtype=a.dtype)
    images = _images(B, S, rank, device)
    gather = world > 1 and not a.no_all_gather
    finish = lambda: None                   # noqa: E731
    if gather:
        # C3: two point-buffer sets (a second pipeline sharing the model), gather k under step k+1
        pipe2 = PointCloudPipeline(B, S, S, spec=spec, density=a.density, device=device, model=pipe.model,
                                   dtype=a.dtype)
        if a.no_graph:
            runs = [lambda: pipe.run(images), lambda: pipe2.run(images)]
        else:
            pipe.capture(images)
            pipe2.capture(images)
            runs = [pipe.replay, pipe2.replay]
        og = D.OverlappedGather(runs, world, B, pipe.points_per_image, device, timing=True)
        step, finish = og.step, og.finish
    elif a.no_graph:
        step = lambda: pipe.run(images)     # noqa: E731
        step()
    else:
        pipe.capture(images)
        step = pipe.replay
    _log("captured; warming up")
    for _ in range(a.warmup):
        step()
    finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if gather:
        og.reset_stats()
    # the shader clock this box holds under dense MFMA load, right before and right after the timed
    # steps (outside the timed region), so the line's fractions can be read at the run's own clock
    clk0 = _clock_probe(device) if rank == 0 else None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    finish()                                # the last step's gather is part of the job
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    own = time.perf_counter() - t0
    clk1 = _clock_probe(device) if rank == 0 else None
    clock = None
    if rank == 0:
        clock = {"before": round(clk0, 4), "after": round(clk1, 4), "ghz": round((clk0 + clk1) / 2, 4),
                 "method": "i2pc_clock_probe: one workgroup per CU, 4 x 16384 dense bf16 32x32x16 MFMAs on random "
                           "operands, median over CUs of s_memtime / s_memrealtime ticks x 0.1 GHz; run right "
                           "before and right after the timed steps"}
    elapsed = D.max_over_ranks(own, device)
    multi = _multi_gpu_diag(a, pipe, images, og if gather else None, own, world, device) if world > 1 else None
    points_step = world * B * pipe.points_per_image
    value = points_step * a.steps / elapsed / 1e6
    ms = elapsed / a.steps * 1e3

    roofline = roof_geo = rooflines = None
    kernels = accounting = None
    _log(f"timed {a.steps} steps: {ms:.3f} ms per step")
    if rank == 0 and not a.no_kernel_profile:
        _log("kernel profile (eager, HIP events)")
        per, geo_t, unp_t = _kernel_profile(pipe, images)
        pmc, pmc_src, pmc_stale = _pmc_traffic(f"{spec.name}-{a.dtype}" + ("" if S == 1024 else f"-{S}")
                                               + ("" if a.density == "high" else f"-{a.density}"))
        dom = max(per.items(), key=lambda kv: kv[1]["t"])
        name, d = dom
        # the bound of a kernel: whichever of its algorithmic FLOPs (at the dtype's dense MFMA peak)
        # and algorithmic HBM bytes (at 8 TB/s) takes longer
        t_mfma = d["flops"] / (_peak(name) * 1e12) if d["flops"] else 0.0
        t_hbm = d["bytes"] / (HBM_PEAK_GBS * 1e9)
        if d["flops"] > 0 and t_mfma >= t_hbm:
            ach = d["flops"] / d["n"] / (d["t"] / d["n"]) / 1e12
            pk = _peak(name)
            roofline = {"kernel": name, "bound": "mfma", "achieved": round(ach, 2), "peak": pk,
                        "unit": "TFLOP/s", "frac": round(ach / pk, 4), "traffic": None,
                        "launches": d["n"], "avg_us": round(d["t"] / d["n"] * 1e6, 2),
                        "flops_per_launch": d["flops"] / d["n"],
                        "share_of_step": round(d["t"] / (ms * 1e-3), 3)}
            roofline["traffic"], roofline["traffic_source"] = _traffic(pmc, pmc_src, name, calls_per_step=d["n"])
            roofline["algorithmic_bytes_per_launch"] = round(d["bytes"] / d["n"])
            if roofline["traffic"]:
                roofline["traffic_over_algorithmic"] = round(roofline["traffic"] / (d["bytes"] / d["n"]), 3)
            # beside frac, not instead of it: the peak scaled to the clock this run's probe measured
            roofline["clock_ghz_run"] = clock["ghz"]
            roofline["frac_at_run_clock"] = round(ach / (pk * clock["ghz"] / 2.4), 4)
            if name.startswith("k_gemm_p"):
                roofline["note"] = ("avg_us and traffic are per i2pc_gemm call: the persistent launch plus its tail "
                                    "launches (a 256x128 round-quantisation tail, or rows past the last full round on "
                                    "smaller row tiles); rocprofv3 lists them as k_gemm_p<256, ...> and "
                                    "k_gemm_p<160, ...>, and traffic sums every one of them")
        else:
            ach = d["bytes"] / (d["t"]) / 1e9
            roofline = {"kernel": name, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                        "launches": d["n"], "avg_us": round(d["t"] / d["n"] * 1e6, 2),
                        "bytes_per_launch": d["bytes"] / d["n"], "share_of_step": round(d["t"] / (ms * 1e-3), 3)}
            if d["flops"]:
                roofline["tflops"] = round(d["flops"] / d["t"] / 1e12, 1)
            roofline["traffic"], roofline["traffic_source"] = _traffic(pmc, pmc_src, name, calls_per_step=d["n"])
            if roofline["traffic"]:
                roofline["traffic_over_algorithmic"] = round(roofline["traffic"] / (d["bytes"] / d["n"]), 3)
        if roofline.get("traffic"):
            roofline["traffic_stale"] = pmc_stale     # the PMC table came from another libi2pc.so build
        geo_bytes = B * (4.0 * pipe.pre.out_h * pipe.pre.out_w + 18.0 * pipe.points_per_image)
        roof_geo = {"kernel": "i2pc_unproject (select + unproject + bbox launches)", "bound": "hbm",
                    "achieved": round(geo_bytes / geo_t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(geo_bytes / geo_t / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                    "ms": round(geo_t * 1e3, 3), "bytes_per_step": geo_bytes}
        # images whose percentiles the last call took from the selection from scratch (the exact
        # fallback, ~0.2-0.6 ms; SelState.level == 16 in the pipeline's workspace, unproject.hip)
        try:
            st = pipe._ws[:624 * B].view(torch.int32).view(B, 156).cpu()
            roof_geo["selection_from_scratch"] = int((st[:, 85] == 16).sum())
        except Exception:   # (diagnostic only)
            pass
        rooflines = {"unproject_stage": roof_geo}
        if unp_t:
            a_unp = geo_bytes / unp_t / 1e9
            rooflines["unproject_kernel"] = {
                "kernel": "k_unproject_rows (back-projection + RGB gather + bbox)", "bound": "hbm",
                "achieved": round(a_unp, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(a_unp / HBM_PEAK_GBS, 4), "traffic": None, "us": round(unp_t * 1e6, 1),
                "bytes_per_launch": geo_bytes, "bytes_per_point": 18.0,
                "note": "algorithmic bytes 4*h'*w' + 18*N per image (SURVEY 8d), one launch per batch"}
            step = {"high": 1, "medium": 2, "low": 4}[pipe.density]
            t, src = _traffic(pmc, pmc_src, f"k_unproject_rows<{step}>", f"k_unproject_fast<{step}>",
                              calls_per_step=1)
            rooflines["unproject_kernel"].update(traffic=t, traffic_source=src)
            if t:
                rooflines["unproject_kernel"]["traffic_over_algorithmic"] = round(t / geo_bytes, 3)
        net_t = sum(v["t"] for v in per.values())
        net_f = sum(v["flops"] for v in per.values())
        # mixed-precision networks: the peak is the FLOP-weighted harmonic mean of the kernels'
        # dtype peaks (time at peak = sum flops_k / peak_k)
        t_peak = sum(v["flops"] / (_peak(k) * 1e12) for k, v in per.items())
        mix_peak = net_f / t_peak / 1e12 if t_peak > 0 else BF16_PEAK_TFLOPS
        rooflines["dpt_blocks"] = {"kernel": "all network launches (GEMM/conv/attention/LN/resize/head)",
                                   "bound": "mfma", "achieved": round(net_f / net_t / 1e12, 1),
                                   "peak": round(mix_peak, 1), "unit": "TFLOP/s",
                                   "frac": round(t_peak / net_t, 4), "traffic": None,
                                   "frac_at_run_clock": round(t_peak / net_t * 2.4 / clock["ghz"], 4),
                                   "ms": round(net_t * 1e3, 3),
                                   "fp8_flop_share": round(sum(v["flops"] for k, v in per.items()
                                                               if k.startswith("k_gemm_f8")) / max(net_f, 1.0), 4),
                                   # attainment against each kernel's own bound (MFMA or HBM, whichever is slower)
                                   "roofline_frac": round(sum(max(v["flops"] / (_peak(k) * 1e12),
                                                                  v["bytes"] / (HBM_PEAK_GBS * 1e9))
                                                              for k, v in per.items()) / net_t, 4)}
        kernels = {k: {"launches": v["n"], "ms": round(v["t"] * 1e3, 3),
                       "tflops": round(v["flops"] / v["t"] / 1e12, 1) if v["flops"] else None,
                       "gbs": round(v["bytes"] / v["t"] / 1e9, 1) if v["bytes"] else None}
                   for k, v in sorted(per.items(), key=lambda kv: -kv[1]["t"])}
        try:
            accounting = check_byte_accounting(kernels)
        except ByteAccountingError as e:
            if a.strict_accounting:
                raise
            _log(f"ByteAccountingError: {e}")
            accounting = {"ok": False, "error": f"ByteAccountingError: {e}"}

    medium = None
    if rank == 0 and world == 1 and a.density == "high" and not a.no_medium:
        _log("density medium (the reference's default, app.py:52,226) on the same model")
        medium = _density_record(a, spec, pipe, images, device, "medium")

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        _log("CPU baseline (restated reference path)")
        try:
            cpu = _cpu_baseline(spec, S, a.density)
        except Exception as e:   # the GPU figure stands on its own; say why the baseline is missing
            cpu = {"value": None, "unit": "Mpoints/s", "cores": os.cpu_count(), "kind": "port",
                   "sample": f"failed: {type(e).__name__}: {e}"}

    if rank == 0:
        flops_img = (spec.flops_per_image(pipe.gh, pipe.gw) if spec.family == "depth-anything"
                     else spec.flops_per_image())
        out = {
            "metric": "Mpoints/sec end-to-end (depth+unproject), 1024² batch",
            "value": round(value, 2), "unit": "Mpoints/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": a.dtype, "data": f"synthetic (uint8 RGB uniform, PCG64 seeds 1000+i; seeded random {spec.name} weights)",
            "config": {"workload": f"{spec.name} {a.dtype} depth + unproject, batch {B} x {S}x{S} per GPU, density {a.density}"
                                   + ((", RCCL all-gather of every rank's points overlapped with the next step"
                                       if a.backend == "nccl" else
                                       ", gloo all-gather of every rank's points (host-staged, synchronous)")
                                      if gather else ""),
                       "model": spec.name, "network_input": [pipe.pre.out_h, pipe.pre.out_w], "global_batch": B * world,
                       "image": [S, S], "points_per_image": pipe.points_per_image, "parallelism": f"dp{world}",
                       "backend": a.backend if world > 1 else None,
                       "hip_graph": not a.no_graph},
            "network_tflops": round(flops_img * B * world / (elapsed / a.steps) / 1e12, 1),
            "roofline": roofline,
            "clock": clock,
            "rooflines": rooflines,
            "cpu_baseline": cpu,
            "multi_gpu": multi,
            "density_medium": medium,
            "byte_accounting": accounting,
            "kernels": kernels,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

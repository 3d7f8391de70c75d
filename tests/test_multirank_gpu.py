"""The multi-rank device path on ONE GPU (C3 layout rehearsal): two ranks share the card over a
gloo process group, each runs its graph-captured pipelines on its own images, and the
OverlappedGather all-gathers every rank's point buffers (per-image independence,
backend/app.py:197-223).  The 8-GPU RCCL run is the driver's; this checks the same code path
end to end on the device, and that `bench.py --gpus N` really starts N ranks."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import bench
        from image_to_pointcloud_amd import distributed as D, geometry
        from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
        from image_to_pointcloud_amd.pipeline import PointCloudPipeline
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        B, S = 2, 256
        pipe = PointCloudPipeline(B, S, S, spec=DA_V2_SMALL, density="medium", device=dev, seed=0)
        pipe2 = PointCloudPipeline(B, S, S, spec=DA_V2_SMALL, density="medium", device=dev, model=pipe.model)
        images = bench._images(B, S, rank, dev)
        pipe.capture(images)
        pipe2.capture(images)
        last = {}

        def run(k, fn):
            def r():
                last[k] = fn()
                return last[k]
            return r
        og = D.OverlappedGather([run(0, pipe.replay), run(1, pipe2.replay)], ws, B, pipe.points_per_image, dev)
        for _ in range(3):
            slot = og.step()
        og.finish()
        gx, gr = og.gathered(slot)
        # the point buffers this rank's step handed to the gather (not rewritten since: the other
        # pipeline ran in between).  Not a second eager forward: with two processes on the card the
        # network is not guaranteed bit-identical run to run (the two-process
        # nondeterminism); graph replay against eager in one process: test_dpt_gpu.py
        mine = last[slot]
        torch.cuda.synchronize()
        q.put((rank, gx.cpu().numpy(), gr.cpu().numpy(), mine.xyz.cpu().numpy(), mine.rgb.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.two_process
def test_overlapped_gather_two_ranks_on_device_bit_identical():
    import torch.multiprocessing as mp
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=240) for _ in range(ws)), key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    B = out[0][3].shape[0]
    for rank, gx, gr, _, _ in out:
        assert gx.shape[0] == ws * B
        for src, _, _, mx, mr in out:      # rank src's images sit at [src*B, (src+1)*B)
            assert gx[src * B:(src + 1) * B].tobytes() == mx.tobytes(), (rank, src)
            assert gr[src * B:(src + 1) * B].tobytes() == mr.tobytes(), (rank, src)
    assert out[0][3].tobytes() != out[1][3].tobytes()     # the ranks really had different images


def _nccl_worker(port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from image_to_pointcloud_amd import distributed as D, geometry
    from image_to_pointcloud_amd.depth_anything import DA_V2_SMALL
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    import bench
    cap = D.cap_rccl_channels()                 # as bench.py does before init_process_group("nccl")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        B, S = 2, 256
        pipe = PointCloudPipeline(B, S, S, spec=DA_V2_SMALL, density="medium", device=dev, seed=0)
        pipe2 = PointCloudPipeline(B, S, S, spec=DA_V2_SMALL, density="medium", device=dev, model=pipe.model)
        images = bench._images(B, S, 0, dev)
        pipe.capture(images)
        pipe2.capture(images)
        og = D.OverlappedGather([pipe.replay, pipe2.replay], 1, B, pipe.points_per_image, dev, timing=True)
        assert dist.get_backend() == "nccl" and not og.host_staged      # the async RCCL branch
        slots = [og.step() for _ in range(3)]
        og.finish()
        wait_ms = og.gather_wait_ms()
        pending = len(og._events)
        gx, gr = og.gathered(slots[-1])
        gx0, gr0 = og.gathered(slots[-2])
        pipe.infer_depth(images)
        mine = geometry.unproject_batch(pipe.depth, images, density="medium")
        torch.cuda.synchronize()
        q.put((gx.cpu().numpy(), gr.cpu().numpy(), gx0.cpu().numpy(), gr0.cpu().numpy(),
               mine.xyz.cpu().numpy(), mine.rgb.cpu().numpy(), wait_ms, pending, cap,
               os.environ.get("NCCL_MAX_NCHANNELS")))
    finally:
        dist.destroy_process_group()


def test_overlapped_gather_rccl_world1_async_branch():
    """The RCCL data path of OverlappedGather (the async all_gather_into_tensor works and the
    compute stream's event-timed waits on them) on a world-size-1 nccl group on cuda:0, with the
    channel cap bench.py sets: three steps over the two graph-captured slots; both slots' gathered
    buffers equal the rank's own points (an eager unprojection of the same depth), and the
    gather-wait figure is finite with no event pair left pending after it is read."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    try:
        gx, gr, gx0, gr0, mx, mr, wait_ms, pending, cap, env_cap = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert gx.tobytes() == mx.tobytes() and gr.tobytes() == mr.tobytes()
    assert gx0.tobytes() == mx.tobytes() and gr0.tobytes() == mr.tobytes()
    assert np.isfinite(wait_ms) and wait_ms >= 0.0 and pending == 0
    assert cap == int(env_cap) > 0


def test_bench_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` (no launcher env) starts torch.distributed.run with two ranks as a
    child process and prints rank 0's line with n_gpus 2 and the all-gather in the workload."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--batch", "2",
           "--size", "512", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-kernel-profile"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 4
    assert "all-gather" in rec["config"]["workload"]
    assert rec["value"] > 0
    # the per-rank diagnostics of the multi-GPU line
    mg = rec["multi_gpu"]
    assert mg["world"] == 2 and mg["backend"] == "gloo" and mg["rccl_world_size"] is None and mg["all_gather"]
    pts = 512 * 512
    assert mg["gathered_bytes_per_step_per_rank"] == 1 * 2 * pts * 15
    assert mg["sent_bytes_per_step_per_rank"] == 2 * pts * 15
    assert [r["rank"] for r in mg["per_rank"]] == [0, 1]
    for r in mg["per_rank"]:
        assert r["step_ms"] > 0 and r["compute_ms"] > 0 and r["gather_wait_ms"] > 0   # gloo stages synchronously
        assert r["gather_wait_ms"] < r["step_ms"]
    # a launcher world that disagrees with --gpus is an error, not a silent 1-GPU number
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("extra", [[], ["--smooth", "--ksize", "9"], ["--levels"], ["--gather", "--density", "medium"]])
def test_c4_two_ranks_window_bands_bit_exact(extra):
    """C4 with two real ranks (gloo, sharing cuda:0, host-staged exchange): each rank unprojects its
    band of a 600 x 1000 panorama with the window selection across bands (or the histogram levels),
    optionally smoothed; --check compares every band with the whole-image unprojection."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "c4_panorama.py"),
           "--height", "600", "--width", "1000", "--steps", "2", "--warmup", "1", "--check"] + extra
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_ranks"] == 2 and rec["bit_exact_vs_whole_image"] is True, rec
    if "--gather" in extra:     # the whole 600 x 1000 panorama at step 2, assembled on every rank
        assert rec["points_gathered"] == 300 * 500, rec
    assert ("histogram levels" in rec["exchange"]) == ("--levels" in extra)

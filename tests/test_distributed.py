"""Multi-rank layout on CPU (gloo, world_size 2): batch sharding, the optional
point all-gather and the max-over-ranks clock that bench.py uses."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from image_to_pointcloud_amd import distributed as D  # noqa: E402


def test_shard_covers_batch_contiguously():
    for gb in (1, 7, 32, 256):
        for ws in (1, 2, 3, 8):
            parts = [D.shard(gb, ws, r) for r in range(ws)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(gb))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1
    with pytest.raises(ValueError):
        D.shard(8, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        B, N = 3, 5
        mine = D.shard(B * ws, ws, rank)
        idx = torch.tensor(list(mine), dtype=torch.float32)
        xyz = idx[:, None, None].expand(B, N, 3).contiguous() + torch.arange(N, dtype=torch.float32)[None, :, None]
        rgb = (idx[:, None, None].expand(B, N, 3) % 256).to(torch.uint8).contiguous()
        gx, gr = D.gather_points(xyz, rgb)
        t = D.max_over_ranks(1.0 + rank)
        q.put((rank, gx.numpy().copy(), gr.numpy().copy(), t))
    finally:
        dist.destroy_process_group()


def test_gather_points_image_major_and_max_clock():
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, gx, gr, t in out:
        assert gx.shape == (6, 5, 3) and gr.shape == (6, 5, 3)
        for img in range(6):                      # image-major: rank 0's images, then rank 1's
            assert (gx[img, :, 0] == img + torch.arange(5).numpy()).all()
            assert (gr[img] == img).all()
        assert t == 2.0


def test_band_rows_partition():
    from image_to_pointcloud_amd.geometry import band_rows
    for h in (1, 7, 100, 4096, 4097):
        for parts in (1, 2, 3, 8):
            for step in (1, 2, 4):
                bands = band_rows(h, parts, step)
                assert len(bands) == parts and bands[0][0] == 0 and bands[-1][1] == h
                for (a0, a1), (b0, b1) in zip(bands, bands[1:]):
                    assert a1 == b0
                for r0, r1 in bands:
                    assert r0 % step == 0 and (r1 % step == 0 or r1 == h) and r0 <= r1


def _band_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        ex = D.band_exchange()
        hist = torch.arange(8, dtype=torch.int32) * (rank + 1)
        cnt = torch.tensor([[rank + 1], [10 * rank], [100 - rank], [7 + rank]], dtype=torch.int64)
        ex(hist, cnt)
        # the window mode: a counters-only exchange (no histogram) and the candidate all-gather
        wcnt = torch.tensor([[rank + 1] * 8, [2] * 8, [50 - rank] * 8, [rank] * 8], dtype=torch.int64)
        ex(None, wcnt)
        send = torch.arange(6, dtype=torch.int32) + 100 * rank
        recv = torch.zeros((ws, 6), dtype=torch.int32)
        D.band_gather()(send, recv)
        bb = torch.tensor([rank, rank + 5.0, -rank, 2.0, 0.5 * rank, 1.0 + rank], dtype=torch.float64)
        q.put((rank, hist.numpy().copy(), cnt.numpy().copy(), D.reduce_bbox(bb).numpy().copy(),
               wcnt.numpy().copy(), recv.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_band_exchange_protocol():
    """The C4 exchange i2pc_unproject_band calls between selection sweeps: histogram SUM,
    level-0 counts SUM, key MIN / MAX; the window mode's counters-only exchange and candidate
    all-gather (i2pc_unproject_band_w); and the band bbox min / max."""
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, hist, cnt, bb, wcnt, recv in out:
        assert wcnt.tolist() == [[3] * 8, [4] * 8, [49] * 8, [1] * 8]
        assert recv.tolist() == [list(range(6)), [100 + i for i in range(6)]]
        assert hist.tolist() == [3 * i for i in range(8)]
        assert cnt[:, 0].tolist() == [3, 10, 99, 8]
        assert bb.tolist() == [0.0, 6.0, -1.0, 2.0, 0.0, 2.0]


def _overlap_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from image_to_pointcloud_amd.geometry import PointBatch
        B, N = 2, 4
        bufs = [PointBatch(torch.zeros(B, N, 3), torch.zeros(B, N, 3, dtype=torch.uint8), None, None) for _ in range(2)]
        state = {"k": 0}

        def make(slot):
            def run():
                k = state["k"]                      # step k writes (rank, k)-coded values into its slot
                bufs[slot].xyz.fill_(1000 * rank + k)
                bufs[slot].rgb.fill_((10 * rank + k) % 256)
                state["k"] += 1
                return bufs[slot]
            return run

        og = D.OverlappedGather([make(0), make(1)], ws, B, N, "cpu")
        seen = []
        for k in range(5):
            slot = og.step()
            if k >= 1:                              # step k-1's gather (other slot); gathered() waits for it
                gx, gr = og.gathered(slot ^ 1)
                seen.append((k - 1, gx[:, 0, 0].tolist(), gr[:, 0, 0].tolist()))
        og.finish()
        gx, gr = og.gathered(4 & 1)
        seen.append((4, gx[:, 0, 0].tolist(), gr[:, 0, 0].tolist()))
        # bench.py's multi-GPU diagnostics: bytes per step and the measured wait (host clock on CPU)
        assert og.recv_bytes_per_step == (ws - 1) * B * N * 15 and og.send_bytes_per_step == B * N * 15
        assert og.world == ws and og.gather_wait_ms() >= 0.0
        og.reset_stats()
        assert og.gather_wait_ms() == 0.0
        q.put((rank, seen))
    finally:
        dist.destroy_process_group()


def test_overlapped_gather_double_buffers():
    """C3: gather k (async) overlaps step k+1; each step's gathered buffer holds exactly that
    step's points from every rank, image-major, although the next step already overwrote
    the other slot."""
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_overlap_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seen in out:
        assert [k for k, _, _ in seen] == [0, 1, 2, 3, 4]
        for k, xs, rs in seen:
            assert xs == [float(k), float(k), 1000.0 + k, 1000.0 + k]
            assert rs == [k, k, 10 + k, 10 + k]


def _band_points_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from image_to_pointcloud_amd.geometry import band_rows
        out = []
        for H, W, step in ((10, 7, 1), (11, 6, 2), (9, 5, 4)):
            wn = (W + step - 1) // step
            n = ((H + step - 1) // step) * wn
            full = torch.arange(n * 3, dtype=torch.float32).view(n, 3)
            r0, r1 = band_rows(H, ws, step)[rank]
            p0, p1 = (r0 // step) * wn, ((r1 + step - 1) // step) * wn
            xyz, rgb = full[p0:p1].clone(), (full[p0:p1] % 256).to(torch.uint8)
            gx, gr = D.gather_band_points(xyz, rgb, H, W, step)
            out.append((gx.numpy().copy(), gr.numpy().copy(), full.numpy().copy()))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_gather_band_points_assembles_the_image():
    """C4's point all-gather: unequal bands (odd heights, density steps 1/2/4)
    padded, gathered and trimmed back into the whole image's row-major points on every rank."""
    ws, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_band_points_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        for gx, gr, full in out:
            assert (gx == full).all() and (gr == (full % 256).astype("uint8")).all()


def test_cap_rccl_channels_sets_default_and_keeps_user_value(monkeypatch):
    """bench.py bounds RCCL's CU share before init_process_group("nccl"): NCCL_MAX_NCHANNELS is set
    to the default cap unless the environment already names one."""
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    assert D.cap_rccl_channels() == D.RCCL_MAX_CHANNELS
    assert os.environ["NCCL_MAX_NCHANNELS"] == str(D.RCCL_MAX_CHANNELS)
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "4")
    assert D.cap_rccl_channels() == 4

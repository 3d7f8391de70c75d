"""Multi-GPU layout of the path: one process per GPU, images sharded by batch.

Every image is independent (percentiles, intrinsics and bbox are per image,
backend/app.py:197-223), so ranks own contiguous slices of the global batch and
compute without any data-path collective (weak scaling).  The north star's C3
configuration additionally gathers every rank's fixed-size point buffers onto
every rank (`gather_points`, one RCCL all-gather per tensor over xGMI;
`OverlappedGather` runs it under the next step's compute); the result is
image-major, i.e. exactly the concatenation of the per-image reference outputs
(SURVEY §8e).
"""
from __future__ import annotations

import os

# RCCL's copy kernels run one workgroup per channel on the same CUs as the network.  C3's all-gather
# needs ~3.5 GB received per rank per ~21 ms step (≈170 GB/s) at 8 ranks; 16 channels (16 of 256 CUs,
# 6 %) carry several hundred GB/s over the 7 xGMI links, so the cap bounds RCCL's share of the chip
# without exposing the gather.  Read by RCCL when the communicator is created.
RCCL_MAX_CHANNELS = 16


def cap_rccl_channels(n: int = None) -> int:
    """Bound the channels (= CUs) RCCL's collectives may take: sets NCCL_MAX_NCHANNELS unless the
    environment already does.  Call before the process group / communicator is created.  Returns
    the cap in force."""
    os.environ.setdefault("NCCL_MAX_NCHANNELS", str(int(n or RCCL_MAX_CHANNELS)))
    return int(os.environ["NCCL_MAX_NCHANNELS"])


def world():
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard(global_batch: int, world_size: int, rank: int) -> range:
    """Contiguous slice of the global image indices owned by `rank` (sizes differ by at most one)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world {world_size}")
    base, extra = divmod(global_batch, world_size)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_points(xyz, rgb, group=None, out_xyz=None, out_rgb=None):
    """All-gather [B, N, 3] point buffers from every rank -> [world*B, N, 3] (rank-major = image-major).

    Requires equal B on every rank (the bench's weak-scaling layout)."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    if out_xyz is None:
        out_xyz = torch.empty((ws * xyz.shape[0],) + tuple(xyz.shape[1:]), dtype=xyz.dtype, device=xyz.device)
    if out_rgb is None:
        out_rgb = torch.empty((ws * rgb.shape[0],) + tuple(rgb.shape[1:]), dtype=rgb.dtype, device=rgb.device)
    dist.all_gather_into_tensor(out_xyz, xyz.contiguous(), group=group)
    dist.all_gather_into_tensor(out_rgb, rgb.contiguous(), group=group)
    return out_xyz, out_rgb


class OverlappedGather:
    """The C3 layout: every step's point buffers all-gathered onto every rank, gather k
    overlapped with compute k + 1.

    `runs` are two step callables that write into two different point-buffer sets (slot 0 / 1,
    e.g. two graph-captured PointCloudPipelines sharing one model) and return them as a
    PointBatch.  step() computes into slot k % 2 on the current stream, then launches the two
    RCCL all-gathers of that slot asynchronously (torch.distributed async_op: the collective
    waits for the compute on its own stream, the current stream goes on with step k + 1).
    Before a slot is overwritten, the current stream waits for the gather that read it.

    With a gloo process group and device buffers (ranks sharing one GPU, the 1-GPU rehearsal
    of the multi-rank path) the gather is staged through host memory and runs synchronously:
    gloo moves host tensors; the results are the same bytes.

    timing=True records an event pair around every wait of the compute stream on a gather
    (gather_wait_ms; bench.py at N > 1).  Completed pairs are folded into a running total, so a
    long-running loop keeps at most the pairs still in flight."""

    def __init__(self, runs, world: int, batch: int, points: int, device, group=None, timing: bool = False):
        import torch
        import torch.distributed as dist
        if len(runs) != 2:
            raise ValueError("OverlappedGather needs two step callables (double-buffered point sets)")
        self.runs, self.group, self.timing = runs, group, timing
        self.world = dist.get_world_size(group)
        self.gx = [torch.empty((world * batch, points, 3), dtype=torch.float32, device=device) for _ in range(2)]
        self.gr = [torch.empty((world * batch, points, 3), dtype=torch.uint8, device=device) for _ in range(2)]
        self.host_staged = self.gx[0].is_cuda and dist.get_backend(group) == "gloo"
        self.works = [None, None]
        self.k = 0
        # diagnostics (bench.py at N > 1): bytes a rank receives per step (xyz f32 + rgb u8 of every
        # other rank's images), and the time its compute stream waited for gathers
        self.recv_bytes_per_step = (world - 1) * batch * points * 15
        self.send_bytes_per_step = batch * points * 15
        self.reset_stats()

    def reset_stats(self):
        """Start a new gather-wait measurement (gather_wait_ms)."""
        self._wait_s = 0.0         # host-side waits (host-staged gloo, CPU tensors) + folded event pairs
        self._events = []          # (before, after) CUDA events around the compute stream's waits

    def gather_wait_ms(self) -> float:
        """Milliseconds the compute stream (or, host-staged, the host) spent waiting for gathers since
        reset_stats(): for an async RCCL gather the gap between an event recorded before the stream's
        wait on the collective and one recorded after it (0 when the gather finished under the next
        step's compute).  Device waits are only measured with timing=True."""
        if self._events:
            self._events[-1][1].synchronize()
            self._fold()
        return self._wait_s * 1e3

    def _fold(self):
        """Add the completed (before, after) pairs to the running total and drop them."""
        while self._events and self._events[0][1].query():
            a, b = self._events.pop(0)
            self._wait_s += a.elapsed_time(b) * 1e-3

    def step(self):
        import torch.distributed as dist
        slot = self.k & 1
        self._wait(slot)                      # the gather that read this slot's buffers is done
        out = self.runs[slot]()
        if self.host_staged:
            import time
            import torch
            torch.cuda.current_stream().synchronize()     # the compute is not part of the wait
            t0 = time.perf_counter()
            for dst, src in ((self.gx[slot], out.xyz), (self.gr[slot], out.rgb)):
                host = dst.new_empty(dst.shape, device="cpu")
                dist.all_gather_into_tensor(host, src.cpu(), group=self.group)
                dst.copy_(host)
            self._wait_s += time.perf_counter() - t0
        else:
            self.works[slot] = (
                dist.all_gather_into_tensor(self.gx[slot], out.xyz, group=self.group, async_op=True),
                dist.all_gather_into_tensor(self.gr[slot], out.rgb, group=self.group, async_op=True))
        self.k += 1
        return slot

    def _wait(self, slot):
        w = self.works[slot]
        if w is not None:
            if self.gx[0].is_cuda:
                if not self.timing:
                    for x in w:
                        x.wait()
                else:
                    import torch
                    before, after = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    before.record()
                    for x in w:
                        x.wait()
                    after.record()
                    self._fold()
                    self._events.append((before, after))
            else:
                import time
                t0 = time.perf_counter()
                for x in w:
                    x.wait()
                self._wait_s += time.perf_counter() - t0
            self.works[slot] = None

    def finish(self):
        """Make the current stream wait for every outstanding gather."""
        self._wait(0)
        self._wait(1)

    def gathered(self, slot):
        """The gathered (xyz, rgb) of the last step that wrote `slot`, [world*B, N, 3] image-major;
        the current stream first waits for that slot's gather."""
        self._wait(slot)
        return self.gx[slot], self.gr[slot]


def max_over_ranks(seconds: float, device=None) -> float:
    """The slowest rank's elapsed time (the bench's whole-job clock)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    if dist.get_backend() == "gloo":
        device = None                           # gloo reduces host tensors
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def band_exchange(group=None):
    """The all-reduce i2pc_unproject_band needs between selection sweeps (C4 tile-parallel
    mode): histogram words and level-0 counts summed, key range min / max, over RCCL."""
    import torch.distributed as dist

    def _exchange(hist, counters):
        if not dist.is_initialized():       # one rank: the sums / min / max are its own values
            return
        host = dist.get_backend(group) == "gloo"    # gloo: reduce host copies (ranks may share a GPU)
        if hist is not None:                # (None: the window mode's counters-only exchange)
            h = hist.cpu() if host else hist
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            if host:
                hist.copy_(h)
        if counters is not None:
            c = counters.cpu() if host else counters
            sums, kmin, kmax = c[:2].contiguous(), c[2].contiguous(), c[3].contiguous()
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(kmin, op=dist.ReduceOp.MIN, group=group)
            dist.all_reduce(kmax, op=dist.ReduceOp.MAX, group=group)
            counters[:2].copy_(sums)
            counters[2].copy_(kmin)
            counters[3].copy_(kmax)
    return _exchange


def band_gather(group=None):
    """The all-gather of the window-selection band mode (i2pc_unproject_band_w): every rank's
    candidate words into recv [nranks, words]."""
    import torch
    import torch.distributed as dist

    def _gather(send, recv):
        if not dist.is_initialized():
            recv[0].copy_(send)
            return
        if dist.get_backend(group) == "gloo":
            r = torch.empty(recv.shape, dtype=recv.dtype)
            dist.all_gather(list(r.unbind(0)), send.cpu(), group=group)
            recv.copy_(r)
        else:
            dist.all_gather(list(recv.unbind(0)), send, group=group)
    return _gather


def band_point_counts(img_h: int, img_w: int, world_size: int, step: int = 1) -> list:
    """Points of every rank's band (geometry.band_rows) of an img_h x img_w image at density step."""
    from . import geometry
    wn = (img_w + step - 1) // step
    return [((r1 + step - 1) // step - r0 // step) * wn for r0, r1 in geometry.band_rows(img_h, world_size, step)]


def gather_band_points(xyz, rgb, img_h: int, img_w: int, step: int = 1, group=None, pad=None):
    """C4's last step: every rank's band points [Nb, 3] -> the whole image's points on
    every rank, row-major as the single-GPU unprojection writes them.  The bands hold different
    point counts (the last band can be shorter), so each is padded to the largest one for one RCCL
    all-gather per tensor (gloo: staged through host memory) and the pads are dropped.
    pad: optional (xyz, rgb) send buffers of the largest band's size, reused across calls."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return xyz, rgb
    world = dist.get_world_size(group)
    counts = band_point_counts(img_h, img_w, world, step)
    rank = dist.get_rank(group)
    if xyz.shape[0] != counts[rank] or rgb.shape[0] != counts[rank]:
        raise ValueError(f"band of rank {rank} holds {xyz.shape[0]} points, the split gives {counts[rank]}")
    nmax = max(counts)
    px, pr = pad if pad is not None else (xyz.new_zeros((nmax, 3)), rgb.new_zeros((nmax, 3)))
    px[:counts[rank]].copy_(xyz)
    pr[:counts[rank]].copy_(rgb)
    host = dist.get_backend(group) == "gloo"
    outs = []
    for t in (px, pr):
        if host:
            g = torch.empty((world * nmax, 3), dtype=t.dtype)
            dist.all_gather_into_tensor(g, t.cpu(), group=group)
            g = g.to(t.device)
        else:
            g = t.new_empty((world * nmax, 3))
            dist.all_gather_into_tensor(g, t, group=group)
        outs.append(torch.cat([g[k * nmax:k * nmax + counts[k]] for k in range(world)]))
    return outs[0], outs[1]


def reduce_bbox(bbox, group=None):
    """Global bounds from per-band bboxes [6] (min x, max x, min y, max y, min z, max z)."""
    import torch.distributed as dist
    host = dist.get_backend(group) == "gloo"
    b = bbox.cpu() if host else bbox
    mins, maxs = b[0::2].contiguous(), b[1::2].contiguous()
    dist.all_reduce(mins, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(maxs, op=dist.ReduceOp.MAX, group=group)
    out = bbox.clone()
    out[0::2] = mins
    out[1::2] = maxs
    return out


class RcclComm:
    """An RCCL communicator owned by libi2pc.so (i2pc_comm_create) for the device-side band
    exchange of the tile-parallel panorama mode (geometry.unproject_band(comm=...)).

    Rank 0 draws the 128-byte unique id and torch.distributed ships it to the others (any
    backend: it is a host object), or pass `unique_id` yourself (world 1 needs no process group).
    The current HIP device must be this rank's GPU."""

    def __init__(self, group=None, nranks=None, rank=None, unique_id: bytes = None):
        import ctypes
        from . import _lib, geometry  # noqa: F401  (geometry registers the i2pc_comm_* signatures)
        lib = _lib.load()
        self._lib = lib
        if nranks is None:
            import torch.distributed as dist
            nranks, rank = dist.get_world_size(group), dist.get_rank(group)
            if unique_id is None:
                obj = [self.unique_id() if rank == 0 else None]
                # src is a GLOBAL rank: the group's rank 0 (not global rank 0 for a subgroup)
                src = dist.get_global_rank(group, 0) if group is not None else 0
                dist.broadcast_object_list(obj, src=src, group=group)
                unique_id = obj[0]
        elif unique_id is None:
            if nranks != 1:
                raise ValueError("nranks > 1 needs the unique id rank 0 drew (or a process group)")
            unique_id = self.unique_id()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
        _lib.call("i2pc_comm_create", buf, int(nranks), int(rank or 0), ctypes.byref(h))
        self.handle, self.nranks, self.rank = h, nranks, rank or 0

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib, geometry  # noqa: F401
        buf = ctypes.create_string_buffer(128)
        _lib.call("i2pc_comm_unique_id", buf, 128)
        return buf.raw

    def close(self):
        """Destroy the communicator (explicitly, or by leaving a `with` block: never from a
        finaliser, which may run after HIP has shut down)."""
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._lib.i2pc_comm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

"""Two-process (or N-process) run-to-run nondeterminism: which op first differs.  N processes share the
GPU; each wraps every ops.* entry point, records stream-ordered clones of its tensor inputs and its
output (no host synchronisation), runs R eager forwards of DA-v2-Small (B=2, 256^2) and reports, per
run that differs from run 1, the first op whose output differs and whether that op's inputs matched."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

NAMES = ["linear", "conv2d", "conv_transpose", "layernorm", "attention", "upsample2x", "resize_bilinear", "head_upconv",
         "cls_pos", "f32_to_bf16", "ln_rowstats", "ln_apply", "head_out", "gemm"]


def worker(rank, q, reps):
    import bench
    from image_to_pointcloud_amd import ops
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rec = []

    def snap(t):
        if isinstance(t, tuple):
            t = t[0]
        return t.detach().clone() if torch.is_tensor(t) else None

    def wrap(name, fn):
        def w(*a, **k):
            ins = [snap(x) for x in list(a) + list(k.values()) if torch.is_tensor(x)]
            out = fn(*a, **k)
            rec.append((name, snap(out if out is not None else k.get("out")), ins))
            return out
        return w
    for n in NAMES:
        if hasattr(ops, n):
            setattr(ops, n, wrap(n, getattr(ops, n)))
    B, S = 2, 256
    pipe = PointCloudPipeline(B, S, S, spec=bench._spec("depth-anything-v2"), density="medium", device=dev, seed=0)
    images = bench._images(B, S, rank, dev)
    runs = []
    for _ in range(reps):
        rec.clear()
        pipe.infer_depth(images)
        runs.append(list(rec))
    torch.cuda.synchronize()
    lines = []
    base = runs[1]
    for j in range(2, reps):
        for i, ((n1, a, ia), (n2, b, ib)) in enumerate(zip(base, runs[j])):
            if a is None or b is None or a.shape != b.shape or torch.equal(a, b):
                continue
            din = [x for x in range(min(len(ia), len(ib))) if ia[x] is not None and ib[x] is not None
                   and ia[x].shape == ib[x].shape and not torch.equal(ia[x], ib[x])]
            d = (a.float() != b.float())
            nz = torch.nonzero(d.reshape(-1)).flatten()
            lines.append(f"proc {rank} run {j}: first diff op #{i} {n1} shape {tuple(a.shape)} {a.dtype} "
                         f"count {int(d.sum())} inputs differing {din} first flat idx {nz[:6].tolist()}")
            break
    q.put((rank, lines or [f"proc {rank}: all runs identical"]))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    n, reps = int(sys.argv[1]), int(sys.argv[2])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, q, reps)) for r in range(n)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=300) for _ in range(n)), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for _, ls in out:
        for l in ls:
            print(l, flush=True)

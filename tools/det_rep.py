"""Diagnostic: N processes on one GPU each run the network forward R times (eager, no sync between
runs except the final compare) and count how many runs differ from their first."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, q, model, reps, graph):
    import bench
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, S = 2, 256
    pipe = PointCloudPipeline(B, S, S, spec=bench._spec(model), density="medium", device=dev, seed=0)
    images = bench._images(B, S, rank, dev)
    if graph:
        pipe.capture(images)
    outs, hss, rss = [], [], []
    for _ in range(reps):
        if graph:
            pipe.replay()
        else:
            pipe.infer_depth(images)
        outs.append(pipe.depth.clone())
        bufs = next(iter(pipe.model._bufs.values()))
        hss.append([h.clone() for h in bufs["hs"]])
        rss.append(bufs["rs"].clone())
    torch.cuda.synchronize()
    bad = sum(0 if torch.equal(o, outs[1]) else 1 for o in outs[1:])
    badh = [sum(0 if torch.equal(h[k], hss[1][k]) else 1 for h in hss[1:]) for k in range(len(hss[0]))]
    badr = sum(0 if torch.equal(r, rss[1]) else 1 for r in rss[1:])
    q.put((rank, f"proc {rank} graph={graph}: {bad} of {reps - 1} runs differ from run 1; hs differ {badh}; last rs {badr}"))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    n, reps, graph = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    model = sys.argv[4] if len(sys.argv) > 4 else "depth-anything-v2"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, q, model, reps, graph)) for r in range(n)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=280) for _ in range(n)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for _, m in out:
        print(m)

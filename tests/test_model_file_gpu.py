"""The native network executor (i2pc_model_create / i2pc_depth_forward, csrc/model.cpp) against the
Python pipeline's depth stage (PointCloudPipeline.infer_depth: the same kernels driven from
depth_anything.py), bit for bit: the process_with_depth_anything drop-in (backend/app.py:99-122)
with no Python in the forward.  Depth-Anything-V2-Small (the reference's model, app.py:78-82) and a
short member of the family; square and non-square inputs (interpolated position table)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _spec(name):
    from image_to_pointcloud_amd.depth_anything import DA_TINY, DA_V2_SMALL
    return {"tiny": DA_TINY, "small": DA_V2_SMALL}[name]


def _imgs(B, H, W, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)).cuda()


@pytest.mark.parametrize("name,B,H,W", [("tiny", 2, 100, 150), ("small", 2, 256, 256), ("small", 3, 300, 200)])
def test_native_executor_matches_python_bit_for_bit(tmp_path, name, B, H, W):
    from image_to_pointcloud_amd.model_file import NativeDepthModel, export_depth_anything
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    dev = torch.device("cuda")
    pipe = PointCloudPipeline(B, H, W, spec=_spec(name), density="medium", device=dev, seed=0)
    imgs = _imgs(B, H, W, 11 + B)
    want = pipe.infer_depth(imgs).clone()
    path = export_depth_anything(pipe.model, str(tmp_path / f"{name}.i2pcnet"), H, W)
    with NativeDepthModel(path, B, H, W) as nm:
        assert (nm.depth_h, nm.depth_w) == tuple(want.shape[1:])
        got = nm(imgs)
        again = nm(imgs)
        torch.cuda.synchronize()
    assert torch.isfinite(want).all() and want.std() > 0
    assert torch.equal(got, want)
    assert torch.equal(again, want)


def test_native_executor_graph_replay_and_errors(tmp_path):
    """The forward is launch-only: captured into a HIP graph and replayed on new images it gives the
    eager result; a model made for another input size is refused (I2PCError)."""
    from image_to_pointcloud_amd import _lib
    from image_to_pointcloud_amd.model_file import NativeDepthModel, export_depth_anything
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    dev = torch.device("cuda")
    B, H, W = 2, 140, 196
    pipe = PointCloudPipeline(B, H, W, spec=_spec("tiny"), density="medium", device=dev, seed=0)
    path = export_depth_anything(pipe.model, str(tmp_path / "t.i2pcnet"), H, W)
    with pytest.raises(_lib.I2PCError, match="made for"):
        NativeDepthModel(path, B, H + 14, W)
    with NativeDepthModel(path, B, H, W) as nm:
        static = _imgs(B, H, W, 1)
        out = torch.empty((B, nm.depth_h, nm.depth_w), dtype=torch.float32, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            nm(static, out=out)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            nm(static, out=out)
        new = _imgs(B, H, W, 2)
        static.copy_(new)
        g.replay()
        torch.cuda.synchronize()
        want = pipe.infer_depth(new).clone()
        torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_plain_c_program_runs_the_depth_stage(tmp_path):
    """examples/depth_forward.c -- a C program linking libi2pc.so and the HIP runtime, no Python --
    runs the exported network on raw BGR images and writes the raw depth: bit-identical to the
    Python pipeline's depth of the same images."""
    import os
    import subprocess
    from image_to_pointcloud_amd.model_file import export_depth_anything
    from image_to_pointcloud_amd.pipeline import PointCloudPipeline
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "depth_forward")
    assert os.path.exists(exe), "examples/depth_forward not built (python -m image_to_pointcloud_amd.build)"
    B, H, W = 2, 256, 320
    pipe = PointCloudPipeline(B, H, W, spec=_spec("small"), density="medium", device=torch.device("cuda"), seed=0)
    imgs = _imgs(B, H, W, 21)
    want = pipe.infer_depth(imgs).cpu().numpy()
    net = export_depth_anything(pipe.model, str(tmp_path / "s.i2pcnet"), H, W)
    src, dst = tmp_path / "images.u8", tmp_path / "depth.f32"
    imgs.cpu().numpy().tofile(src)
    r = subprocess.run([exe, net, str(B), str(H), str(W), str(src), str(dst)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.fromfile(dst, dtype=np.float32).reshape(want.shape)
    assert got.tobytes() == want.tobytes()

"""Artefact writers (save_point_cloud, app.py:310-389) -- host code, runs on CPU.

XYZ is pinned byte-for-byte: the reference's own save_xyz output for the golden
pipeline case (sha256 recorded by tests/golden/gen_golden.py).  PLY (Open3D) and
LAS (laspy) are restated layouts ("parity unpinned": neither library is in the
image); they are checked by parsing the files back.
"""
import hashlib
import os
import struct

import numpy as np
import pytest

from image_to_pointcloud_amd import _lib

pytestmark = pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libi2pc.so not built")


def _points(pipeline_case):
    from oracle import unproject_ref as ref
    return ref.depth_to_point_cloud(pipeline_case["image"], pipeline_case["depth"], density="high", loop=False)


def test_xyz_bytes_match_reference(tmp_path, pipeline_case):
    from image_to_pointcloud_amd import writers
    pts, cols = _points(pipeline_case)
    for threads in (1, 5):
        p = str(tmp_path / f"a{threads}.xyz")
        writers.write_xyz(p, pts, cols, threads=threads)
        data = open(p, "rb").read()
        assert hashlib.sha256(data).hexdigest() == pipeline_case["summary"]["xyz_sha256"]
    # uint8 colours give the same bytes as the reference's float32 colours
    p = str(tmp_path / "u8.xyz")
    writers.write_xyz(p, pts, cols.astype(np.uint8))
    assert hashlib.sha256(open(p, "rb").read()).hexdigest() == pipeline_case["summary"]["xyz_sha256"]


def test_ply_layout(tmp_path, pipeline_case):
    from image_to_pointcloud_amd import writers
    pts, cols = _points(pipeline_case)
    p = str(tmp_path / "a.ply")
    writers.write_ply(p, pts, cols)
    data = open(p, "rb").read()
    head, body = data.split(b"end_header\n", 1)
    lines = head.decode().splitlines()
    assert lines[:2] == ["ply", "format binary_little_endian 1.0"]
    assert f"element vertex {len(pts)}" in lines
    assert [l for l in lines if l.startswith("property")] == [
        "property double x", "property double y", "property double z",
        "property uchar red", "property uchar green", "property uchar blue"]
    rec = np.frombuffer(body, dtype=np.dtype([("xyz", "<f8", 3), ("rgb", "u1", 3)]))
    assert len(rec) == len(pts)
    assert np.array_equal(rec["xyz"], pts.astype(np.float64))
    # Open3D: float32(c / 255) -> double * 255 -> truncating uchar
    exp = np.minimum(255.0, (cols / np.float32(255.0)).astype(np.float32).astype(np.float64) * 255.0).astype(np.uint8)
    assert np.array_equal(rec["rgb"], exp)


def test_las_layout(tmp_path, pipeline_case):
    from image_to_pointcloud_amd import writers
    pts, cols = _points(pipeline_case)
    p = str(tmp_path / "a.las")
    writers.write_las(p, pts, cols)
    data = open(p, "rb").read()
    assert data[:4] == b"LASF" and data[24:26] == bytes([1, 2])
    hsize, = struct.unpack_from("<H", data, 94)
    off, nvlr, fmt, rlen, npts = struct.unpack_from("<IIBHI", data, 96)
    assert (hsize, off, nvlr, fmt, rlen, npts) == (227, 227, 0, 2, 26, len(pts))
    scale = struct.unpack_from("<3d", data, 131)
    offset = struct.unpack_from("<3d", data, 155)
    assert scale == (0.01, 0.01, 0.01)
    assert offset == tuple(float(pts[:, c].min()) for c in range(3))            # app.py:354
    rec = np.frombuffer(data[227:], dtype=np.dtype([("X", "<i4", 3), ("i", "<u2"), ("b", "u1"), ("c", "u1"),
                                                    ("a", "i1"), ("u", "u1"), ("s", "<u2"), ("rgb", "<u2", 3)]))
    assert len(rec) == len(pts)
    exp = np.round((pts.astype(np.float64) - np.array(offset)) / 0.01).astype(np.int32)
    assert np.array_equal(rec["X"], exp)
    assert np.array_equal(rec["rgb"], cols.astype(np.uint16) * 256)


def test_save_point_cloud_dropin(tmp_path, monkeypatch, pipeline_case):
    from image_to_pointcloud_amd import writers
    pts, cols = _points(pipeline_case)
    monkeypatch.chdir(tmp_path)
    assert writers.save_point_cloud(pts, cols, "xyz", "job") == "outputs/job.xyz"
    assert writers.save_point_cloud(pts, cols, "LAS", "job") == "outputs/job.las"
    assert writers.save_point_cloud(pts, cols, "laz", "job2") == "outputs/job2.las"
    assert writers.save_point_cloud(pts, cols, "ply", "job") == "outputs/job.ply"
    with pytest.raises(ValueError):
        writers.save_point_cloud(pts, cols, "obj", "job")
    with pytest.raises(ValueError):
        writers.write_las(str(tmp_path / "e.las"), np.zeros((0, 3), np.float32), None)


def test_ply_batched_buffers_keep_colours(tmp_path):
    """Batched [B, N, 3] point and colour buffers (the pipeline's layout) write one cloud of B * N
    coloured points in image-major order: the colours are flattened before the count check."""
    from image_to_pointcloud_amd import writers
    rng = np.random.Generator(np.random.PCG64(5))
    xyz = rng.normal(size=(3, 7, 3)).astype(np.float32)
    rgb = rng.integers(0, 256, (3, 7, 3), dtype=np.uint8)
    path = str(tmp_path / "b.ply")
    writers.write_ply(path, xyz, rgb)
    data = open(path, "rb").read()
    head = data[: data.index(b"end_header\n") + len(b"end_header\n")]
    assert b"element vertex 21" in head and b"property uchar red" in head
    rec = np.frombuffer(data[len(head):], dtype=np.dtype([("xyz", "<f8", 3), ("rgb", "u1", 3)]))
    assert np.array_equal(rec["xyz"], xyz.reshape(-1, 3).astype(np.float64))
    assert np.array_equal(rec["rgb"], rgb.reshape(-1, 3))

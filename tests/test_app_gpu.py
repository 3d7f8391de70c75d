"""End-to-end drop-in parity of the REST job (process_image_pipeline, app.py:419-565)
against the reference's own output for the golden pipeline case
(tests/golden/pipeline_case.json): same status fields, pointCloud, gisData
(bounds from the device bbox), preview sha256 and the downloaded XYZ bytes.

The network is replaced by the fixture's depth map on both sides (the reference
case was recorded the same way: no offline weights), so everything after the
depth network runs the HIP path and must match bit-for-bit.
"""
import hashlib
import io

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytest.importorskip("fastapi")
pytestmark = pytest.mark.gpu


def test_rest_job_matches_reference(pipeline_case, monkeypatch, tmp_path):
    from fastapi.testclient import TestClient
    from PIL import Image
    from image_to_pointcloud_amd import app_api, server
    monkeypatch.chdir(tmp_path)
    depth = torch.from_numpy(pipeline_case["depth"]).cuda()
    monkeypatch.setattr(app_api, "load_model", lambda name: {"type": "depth"})
    monkeypatch.setattr(app_api, "_depth_device", lambda img, mi: depth)
    # the fixture was recorded with Open3D absent: the reference's refine_point_cloud raised
    # inside its try and returned the cloud unrefined (app.py:267-269)
    monkeypatch.setattr(app_api, "REFINE_POINT_CLOUD", False)
    buf = io.BytesIO()
    Image.fromarray(pipeline_case["image"][:, :, ::-1]).save(buf, format="PNG")     # lossless: decodes to the same BGR
    c = TestClient(server.app)
    r = c.post("/process", files={"file": ("img.png", buf.getvalue(), "image/png")},
               params={"point_density": "high", "output_format": "xyz", "fov": 30.0})
    assert r.status_code == 200
    job = r.json()["job_id"]
    st = c.get(f"/status/{job}").json()
    exp = pipeline_case["summary"]
    assert st["status"] == exp["status"], st["message"]
    assert (st["progress"], st["message"]) == (exp["progress"], exp["message"])
    res = st["results"]
    assert res["pointCloud"] == {**exp["pointCloud"], "filepath": f"outputs/{job}.xyz"}
    assert res["gisData"] == exp["gisData"]
    assert res["downloadUrl"] == f"/download/{job}"
    assert res["meshPreview"] is None
    assert res["depthMap"].startswith("data:image/png;base64,")          # reference: None (no cv2 in its container)
    assert len(res["preview"]["points"]) == exp["preview_len"]
    pp = np.asarray(res["preview"]["points"], dtype=np.float64)
    pc = np.asarray(res["preview"]["colors"], dtype=np.float64)
    assert hashlib.sha256(pp.tobytes()).hexdigest() == exp["preview_points_sha256"]
    assert hashlib.sha256(pc.tobytes()).hexdigest() == exp["preview_colors_sha256"]
    dl = c.get(f"/download/{job}")
    assert dl.status_code == 200
    assert hashlib.sha256(dl.content).hexdigest() == exp["xyz_sha256"]


class _RecordingJob(dict):
    """A job record that logs every (progress, message) its pipeline publishes."""
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.log = []

    def update(self, *a, **k):
        super().update(*a, **k)
        if "progress" in k or "message" in k:
            self.log.append((self.get("progress"), self.get("message")))


def test_job_progress_sequence_matches_reference(pipeline_case, monkeypatch, tmp_path):
    """A polling frontend sees the reference's status sequence: 10 / 20 / 40 / 60 / 80 / 100 with the
    messages of app.py:423-424, 429-430, 457-458, 465-466, 492-493 and 542-544."""
    from PIL import Image
    from image_to_pointcloud_amd import app_api
    monkeypatch.chdir(tmp_path)
    depth = torch.from_numpy(pipeline_case["depth"]).cuda()
    monkeypatch.setattr(app_api, "load_model", lambda name: {"type": "depth"})
    monkeypatch.setattr(app_api, "_depth_device", lambda img, mi: depth)
    monkeypatch.setattr(app_api, "REFINE_POINT_CLOUD", False)
    buf = io.BytesIO()
    Image.fromarray(pipeline_case["image"][:, :, ::-1]).save(buf, format="PNG")
    job = _RecordingJob(status="pending", progress=0, message="Job queued")
    req = app_api.ProcessingRequest(point_density="high", output_format="xyz")
    app_api.process_image_pipeline("job0", buf.getvalue(), req, jobs={"job0": job})
    assert job["status"] == "completed", job["message"]
    assert job.log == [(10, "Loading AI model..."), (20, "Processing image..."),
                       (40, "Estimating depth with AI..."), (60, "Generating 3D point cloud..."),
                       (80, "Saving point cloud..."), (100, "Processing complete!")]


def test_load_model_and_depth_shapes():
    from image_to_pointcloud_amd import app_api
    mi = app_api.load_model("depth-anything-v2")
    assert mi["type"] == "depth" and app_api.load_model("depth-anything-v2") is mi       # cached
    rng = np.random.Generator(np.random.PCG64(0))
    for (h, w), exp in (((384, 384), (518, 518)), ((768, 1024), (518, 686))):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        d = app_api.process_with_depth_anything(img, mi)
        assert d.dtype == np.float32 and d.shape == exp and np.isfinite(d).all()
    with pytest.raises(Exception):
        app_api.load_model("no-such-model")


def test_rest_job_with_dpt_hybrid_fp8(monkeypatch, tmp_path):
    """The REST job on the C5 network: model=dpt-hybrid loads the MX fp8 DPT-Hybrid (BiT-R50 +
    ViT-B/16) and the job completes with a coloured PLY of every point."""
    from fastapi.testclient import TestClient
    from PIL import Image
    from image_to_pointcloud_amd import app_api, server
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(app_api, "REFINE_POINT_CLOUD", False)
    rng = np.random.Generator(np.random.PCG64(4))
    img = rng.integers(0, 256, (240, 320, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG")
    c = TestClient(server.app)
    r = c.post("/process", files={"file": ("img.png", buf.getvalue(), "image/png")},
               params={"model": "dpt-hybrid", "point_density": "medium", "output_format": "ply"})
    job = r.json()["job_id"]
    st = c.get(f"/status/{job}").json()
    assert st["status"] == "completed", st["message"]
    assert app_api.models_cache["dpt-hybrid"]["model"].dtype == "fp8"
    assert st["results"]["pointCloud"]["points"] == 120 * 160
    ply = c.get(f"/download/{job}").content
    assert b"element vertex 19200" in ply[:400] and b"property uchar red" in ply[:400]

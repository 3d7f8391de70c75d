"""Generate golden fixtures by running the REFERENCE itself (build container only).

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/gen_golden.py

Imports /root/reference/backend/app.py with the modules absent from this image
stubbed (cv2, trimesh, open3d, laspy; plus a python_multipart version shim that
FastAPI checks when it registers the File(...) route) -- SURVEY.md §8c.  With
`depth.shape == image.shape[:2]` and `smooth=False`, `depth_to_point_cloud`
(app.py:174-250) never touches cv2, so it runs UNMODIFIED.  The full
`process_image_pipeline` (app.py:419-565) is also run with `cv2.imdecode`
returning a prepared BGR array and `process_with_depth_anything` returning a
prepared depth map (the network has no offline weights); preview / refine fall
back through the reference's own `except` branches exactly as they would
without Open3D.

Outputs: tests/golden/unproject_cases.npz, tests/golden/pipeline_case.npz,
tests/golden/pipeline_case.json, tests/golden/routes.json, tests/golden/preview_cases.npz
(the uint8 image create_depth_preview hands to cv2.applyColorMap, recorded by the stub).  Nothing here runs on the GPU box.
"""
from __future__ import annotations

import asyncio
import hashlib
import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np

REF_APP = "/root/reference/backend/app.py"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


class _Missing(types.ModuleType):
    """A stub module whose functions raise, like a library that fails at run time."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)

        def _fail(*a, **k):
            raise RuntimeError(f"{self.__name__}.{name} is not available in the oracle container")
        return _fail


def _install_stubs(decode_queue):
    cv2 = _Missing("cv2")
    cv2.IMREAD_COLOR = 1
    cv2.COLOR_BGR2RGB = 4
    cv2.COLOR_BGR2GRAY = 6
    cv2.INTER_AREA = 3
    cv2.INTER_LINEAR = 1
    cv2.COLORMAP_PLASMA = 15

    def imdecode(buf, flags):
        return decode_queue.pop(0)
    cv2.imdecode = imdecode
    sys.modules["cv2"] = cv2
    for name in ("trimesh", "open3d", "laspy"):
        sys.modules[name] = _Missing(name)
    pm = types.ModuleType("python_multipart")
    pm.__version__ = "0.0.20"
    sys.modules.setdefault("python_multipart", pm)


def load_reference(decode_queue):
    _install_stubs(decode_queue)
    spec = importlib.util.spec_from_file_location("reference_app", REF_APP)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def smooth_depth(h, w, seed, noise=0.05):
    rng = np.random.Generator(np.random.PCG64(seed))
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    base = 0.5 + 4.5 * (0.5 + 0.5 * np.sin(6 * np.pi * u / w) * np.cos(4 * np.pi * v / h))
    d = base + rng.normal(0.0, noise, size=(h, w))
    return np.maximum(d, 0.0).astype(np.float32)


def rgb_image(h, w, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def main():
    decode_queue = []
    ref = load_reference(decode_queue)
    cases = {}
    meta = []

    def add(name, image, depth, density, invert, scale):
        pts, cols = ref.depth_to_point_cloud(image, depth, density=density, invert=invert,
                                             depth_scale=scale, smooth=False)
        req = ref.ProcessingRequest(point_density=density, invert_depth=invert, depth_scale=scale)
        gis = ref.generate_gis_metadata(pts, req)
        p2, p98 = np.percentile(depth.astype(np.float32), [2, 98]) if np.all(np.isfinite(depth)) else (np.nan, np.nan)
        cases[f"{name}__image"] = image
        cases[f"{name}__depth"] = depth
        cases[f"{name}__points"] = pts
        cases[f"{name}__colors"] = cols
        cases[f"{name}__bounds"] = np.array([gis["bounds"][k] for k in
                                             ("minX", "maxX", "minY", "maxY", "minZ", "maxZ")], dtype=np.float64)
        meta.append({"name": name, "density": density, "invert": invert, "scale": scale,
                     "h": int(image.shape[0]), "w": int(image.shape[1]), "n": int(len(pts)),
                     "p2_raw": float(p2), "p98_raw": float(p98)})

    # 1. odd, non-square sizes x every density x invert x two scales
    img = rgb_image(37, 53, 1000)
    dep = smooth_depth(37, 53, 1)
    for density in ("low", "medium", "high"):
        for invert in (True, False):
            for scale in (10.0, 15.0):
                add(f"odd_{density}_{int(invert)}_{int(scale)}", img, dep, density, invert, scale)
    # 2. 48x64 (h x w), defaults
    add("wide_medium", rgb_image(48, 64, 1001), smooth_depth(48, 64, 2), "medium", True, 10.0)
    add("tall_high", rgb_image(64, 48, 1002), smooth_depth(64, 48, 3), "high", True, 10.0)
    # 3. constant depth: p98 <= p2 and min == max -> d = 0 -> z = depth_scale
    add("const_medium", rgb_image(31, 29, 1003), np.full((31, 29), 2.5, np.float32), "medium", True, 10.0)
    add("const_noinv", rgb_image(31, 29, 1003), np.full((31, 29), 2.5, np.float32), "medium", False, 10.0)
    # 4. min/max fallback branch: >96% equal values but min < max (float32 arithmetic)
    d = np.full((40, 40), 1.0, np.float32)
    d[0, :10] = 3.0
    d[5, 3:7] = 0.25
    add("minmax_high", rgb_image(40, 40, 1004), d, "high", True, 10.0)
    add("minmax_noinv", rgb_image(40, 40, 1004), d, "high", False, 7.5)
    # 5. non-finite values -> nanmedian fill (odd and even non-NaN counts)
    d = smooth_depth(33, 47, 4)
    rng = np.random.Generator(np.random.PCG64(5))
    flat = d.reshape(-1)
    flat[rng.choice(flat.size, 20, replace=False)] = np.nan
    flat[rng.choice(flat.size, 5, replace=False)] = np.inf
    flat[rng.choice(flat.size, 3, replace=False)] = -np.inf
    add("nonfinite_high", rgb_image(33, 47, 1005), d, "high", True, 10.0)
    d2 = smooth_depth(30, 30, 6)
    d2[3, 4] = np.nan
    add("nan_even_medium", rgb_image(30, 30, 1006), d2, "medium", True, 10.0)
    # 6. invert=False gives z == 0 at pixels <= p2 (x, y use 1e-6)
    add("zero_z_high", rgb_image(36, 36, 1007), smooth_depth(36, 36, 7, noise=0.0), "high", False, 10.0)
    # 7. larger percentile case, negative and tied values
    d3 = np.round(smooth_depth(128, 96, 8) * 8.0).astype(np.float32) / 8.0 - 1.0
    add("ties_medium", rgb_image(128, 96, 1008), d3, "medium", True, 12.5)
    add("big_low", rgb_image(200, 150, 1009), smooth_depth(200, 150, 9), "low", True, 10.0)

    np.savez_compressed(os.path.join(OUT_DIR, "unproject_cases.npz"), **cases)
    with open(os.path.join(OUT_DIR, "unproject_cases.json"), "w") as fh:
        json.dump(meta, fh, indent=1)

    # 8. the full pipeline (process_image_pipeline) -> results JSON schema/values
    h, w = 220, 200
    image = rgb_image(h, w, 1010)
    depth = smooth_depth(h, w, 10)
    decode_queue.append(image)
    ref.process_with_depth_anything = lambda img, mi: depth
    ref.load_model = lambda name: {"type": "depth"}
    job = "golden-job"
    ref.processing_jobs[job] = {"status": "pending", "progress": 0, "message": "Job queued", "results": None}
    req = ref.ProcessingRequest(point_density="high", output_format="xyz")
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            asyncio.run(ref.process_image_pipeline(job, b"\x00", req))
            with open(os.path.join(td, "outputs", f"{job}.xyz"), "rb") as fh:
                xyz_bytes = fh.read()
        finally:
            os.chdir(cwd)
    st = ref.processing_jobs[job]
    assert st["status"] == "completed", st
    res = st["results"]
    prev_pts = np.asarray(res["preview"]["points"], dtype=np.float64)
    prev_cols = np.asarray(res["preview"]["colors"], dtype=np.float64)
    summary = {
        "status": st["status"], "progress": st["progress"], "message": st["message"],
        "pointCloud": res["pointCloud"], "gisData": res["gisData"],
        "downloadUrl": res["downloadUrl"], "meshPreview": res["meshPreview"],
        "depthMap": res["depthMap"],
        "preview_len": len(res["preview"]["points"]),
        "preview_points_sha256": hashlib.sha256(prev_pts.tobytes()).hexdigest(),
        "preview_colors_sha256": hashlib.sha256(prev_cols.tobytes()).hexdigest(),
        "xyz_sha256": hashlib.sha256(xyz_bytes).hexdigest(),
        "xyz_lines": xyz_bytes.count(b"\n"),
        "xyz_head": xyz_bytes[:200].decode(),
        "request_defaults": ref.ProcessingRequest().model_dump(),
        "fov_field_present": "fov" in ref.ProcessingRequest.model_fields,
    }
    np.savez_compressed(os.path.join(OUT_DIR, "pipeline_case.npz"), image=image, depth=depth)
    with open(os.path.join(OUT_DIR, "pipeline_case.json"), "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    # route surface (query vs body params)
    routes = {}
    for r in ref.app.routes:
        if getattr(r, "path", None) in ("/process", "/status/{job_id}", "/download/{job_id}", "/models", "/health"):
            dep = getattr(r, "dependant", None)
            routes[r.path] = {
                "methods": sorted(r.methods),
                "query": [p.name for p in dep.query_params] if dep else [],
                "body": [p.name for p in dep.body_params] if dep else [],
                "path": [p.name for p in dep.path_params] if dep else [],
            }
    models = asyncio.run(ref.list_available_models())
    with open(os.path.join(OUT_DIR, "routes.json"), "w") as fh:
        json.dump({"routes": routes, "models": models}, fh, indent=1, sort_keys=True)
    # 9. depth preview (create_depth_preview, app.py:124-172): record the uint8 image the reference
    #    hands to cv2.applyColorMap (cv2 is absent: the colour table and PNG bytes stay unpinned)
    seen = []
    cv2 = sys.modules["cv2"]
    cv2.applyColorMap = lambda img, cmap: (seen.append(np.array(img, copy=True)), np.zeros(img.shape + (3,), np.uint8))[1]
    cv2.imencode = lambda ext, img: (True, np.frombuffer(b"png", np.uint8))
    prev = {}
    pmeta = []
    d_nf = smooth_depth(33, 47, 4)
    d_nf.reshape(-1)[[5, 77, 300]] = [np.nan, np.inf, -np.inf]
    d_mm = np.full((40, 40), 1.0, np.float32)
    d_mm[0, :10] = 3.0
    d_mm[5, 3:7] = 0.25
    for name, d in (("smooth", smooth_depth(37, 53, 11)), ("dpt384", smooth_depth(384, 384, 12)),
                    ("const", np.full((20, 24), 2.5, np.float32)), ("minmax", d_mm), ("nonfinite", d_nf)):
        for invert in (True, False):
            seen.clear()
            url = ref.create_depth_preview(d, invert=invert)
            assert url is not None and len(seen) == 1, (name, url)
            key = f"{name}_{int(invert)}"
            prev[key + "__depth"] = d
            prev[key + "__u8"] = seen[0]
            pmeta.append({"name": key, "invert": invert})
    np.savez_compressed(os.path.join(OUT_DIR, "preview_cases.npz"), **prev)
    with open(os.path.join(OUT_DIR, "preview_cases.json"), "w") as fh:
        json.dump(pmeta, fh, indent=1)
    print("wrote", len(meta), "unprojection cases + pipeline case + routes +", len(pmeta), "preview cases")


if __name__ == "__main__":
    main()

"""REST drop-in for the reference's FastAPI app (backend/app.py:26-37, 609-747) over
the MI355X pipeline.

Same routes, query parameters (all scalar parameters of POST /process are query
parameters and `fov` is accepted and ignored, as in the reference), status
codes and JSON schema.  GPU work runs on one worker thread, off the event
loop; jobs are serialised the same way the reference's background tasks are.

The multipart upload (`file` field, app.py:612) is parsed here with the standard
library's MIME parser, so the route does not depend on python-multipart (which
this image lacks and which FastAPI's File(...) parameters require).

    python -m image_to_pointcloud_amd.server [--host 0.0.0.0] [--port 8000]
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import uuid
from pathlib import Path

from . import app_api

try:
    from fastapi import BackgroundTasks, FastAPI, HTTPException, Request
    from fastapi.middleware.cors import CORSMiddleware
    from fastapi.responses import FileResponse
except ImportError as e:          # the REST layer is optional; the kernels are not
    raise ImportError("image_to_pointcloud_amd.server needs fastapi") from e

app = FastAPI(title="Image to Point Cloud API", version="1.0.0")
app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                   allow_headers=["*"])

_gpu = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="i2pc-gpu")

MODELS = [   # app.py:705-737
    {"id": "depth-anything-v2", "name": "Depth Anything V2", "description": "Superior depth estimation + point cloud",
     "license": "Apache-2.0", "recommended": True, "supported": True, "speed": "2-3s", "quality": "High"},
    {"id": "triposr", "name": "TripoSR", "description": "Fast mesh generation (1-2 seconds)", "license": "MIT",
     "recommended": False, "supported": False, "speed": "1-2s", "quality": "Medium"},
    {"id": "instantmesh", "name": "InstantMesh", "description": "High quality 3D assets (~10 seconds)",
     "license": "Custom", "supported": False, "speed": "~10s", "quality": "Very High"},
]


async def _run_job(job_id: str, image_data: bytes, request: app_api.ProcessingRequest):
    loop = asyncio.get_running_loop()
    await loop.run_in_executor(_gpu, app_api.process_image_pipeline, job_id, image_data, request)


def _multipart_file(content_type: str, body: bytes):
    """(filename, content_type, data) of the `file` part of a multipart/form-data body, or None."""
    from email.parser import BytesParser
    from email.policy import HTTP
    if not content_type.lower().startswith("multipart/form-data"):
        return None
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + content_type.encode("latin-1") + b"\r\n\r\n" + body)
    if not msg.is_multipart():
        return None
    for part in msg.iter_parts():
        if part.get_param("name", header="content-disposition") == "file":
            return part.get_filename(), part.get_content_type(), part.get_payload(decode=True) or b""
    return None


@app.post("/process", response_model=dict)
async def process_image(request: Request, background_tasks: BackgroundTasks,
                        model: str = "depth-anything-v2", output_format: str = "las",
                        point_density: str = "medium", coordinate_system: str = "WGS84",
                        invert_depth: bool = True, depth_scale: float = 10.0, smooth_depth: bool = False,
                        fov: float = 60.0):
    """app.py:609-664 (multipart field `file`, required)."""
    part = _multipart_file(request.headers.get("content-type", ""), await request.body())
    if part is None:
        raise HTTPException(status_code=422, detail=[{"type": "missing", "loc": ["body", "file"],
                                                      "msg": "Field required", "input": None}])
    _, ctype, image_data = part
    if not (ctype or "").startswith("image/"):
        raise HTTPException(status_code=400, detail="File must be an image")
    if len(image_data) > app_api.MAX_FILE_SIZE:
        raise HTTPException(status_code=413,
                            detail=f"File size ({len(image_data)/1024/1024:.1f}MB) exceeds maximum allowed size "
                                   f"({app_api.MAX_FILE_SIZE/1024/1024:.0f}MB)")
    job_id = str(uuid.uuid4())
    app_api.processing_jobs[job_id] = {"status": "pending", "progress": 0, "message": "Job queued", "results": None}
    request = app_api.ProcessingRequest(model=model, output_format=output_format, point_density=point_density,
                                        coordinate_system=coordinate_system, invert_depth=invert_depth,
                                        depth_scale=depth_scale, smooth_depth=smooth_depth)   # fov dropped (D5)
    background_tasks.add_task(_run_job, job_id, image_data, request)
    return {"job_id": job_id, "status": "queued"}


@app.get("/status/{job_id}", response_model=app_api.ProcessingStatus)
async def get_job_status(job_id: str):
    """app.py:666-679."""
    if job_id not in app_api.processing_jobs:
        raise HTTPException(status_code=404, detail="Job not found")
    j = app_api.processing_jobs[job_id]
    return app_api.ProcessingStatus(job_id=job_id, status=j["status"], progress=j["progress"], message=j["message"],
                                    results=j["results"])


@app.get("/download/{job_id}")
async def download_result(job_id: str):
    """app.py:681-700."""
    if job_id not in app_api.processing_jobs:
        raise HTTPException(status_code=404, detail="Job not found")
    j = app_api.processing_jobs[job_id]
    if j["status"] != "completed":
        raise HTTPException(status_code=400, detail="Job not completed")
    filepath = j["results"]["pointCloud"]["filepath"]
    if not Path(filepath).exists():
        raise HTTPException(status_code=404, detail="File not found")
    return FileResponse(filepath, media_type="application/octet-stream", filename=Path(filepath).name)


@app.get("/models")
async def list_available_models():
    """app.py:702-739."""
    return {"models": MODELS}


@app.get("/health")
async def health_check():
    """app.py:741-747."""
    return {"status": "healthy", "models_loaded": list(app_api.models_cache.keys()),
            "active_jobs": len(app_api.processing_jobs), "max_file_size_mb": app_api.MAX_FILE_SIZE / (1024 * 1024)}


def main():
    import argparse
    import uvicorn
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    a = ap.parse_args()
    Path("outputs").mkdir(exist_ok=True)
    uvicorn.run(app, host=a.host, port=a.port, log_level="info")


if __name__ == "__main__":
    main()

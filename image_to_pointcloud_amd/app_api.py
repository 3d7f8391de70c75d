"""In-process drop-ins for the reference's depth branch (backend/app.py), on MI355X.

Same names, arguments, return types and error behaviour as the reference's
functions, so backend/app.py can import them in place of its own:

  ProcessingRequest                      app.py:47-56
  load_model(model_name)                 app.py:64-96   (no hub access: weights come from a
                                                         local safetensors file or are seeded)
  process_with_depth_anything(img, mi)   app.py:99-122
  create_depth_preview(depth, invert)    app.py:124-172  (preview.py)
  depth_to_point_cloud(...)              app.py:174-250  (geometry.py)
  save_point_cloud(...)                  app.py:310-331  (writers.py)
  generate_gis_metadata(points, req)     app.py:391-417
  process_image_pipeline(job, data, req) app.py:419-565  (the depth branch, one GPU pass)

  refine_point_cloud(points, colors)     app.py:252-269  (geometry.remove_statistical_outlier:
                                                         Open3D's statistical outlier removal
                                                         restated as an exact device kNN)

REFINE_POINT_CLOUD switches the refinement step of the depth job (app.py:479) off;
the golden pipeline fixture was recorded with Open3D absent, where the reference's
refine_point_cloud raises inside its try and hands the cloud back unchanged.
"""
from __future__ import annotations

import io
import logging
import os
import traceback
from typing import Any, Dict, Optional

import numpy as np
from pydantic import BaseModel

from . import geometry, preprocess, preview, writers

logger = logging.getLogger(__name__)

MAX_IMAGE_DIM = 3072                      # app.py:42
MAX_FILE_SIZE = 50 * 1024 * 1024          # app.py:44
MAX_PREVIEW = 20000                       # app.py:497
REFINE_POINT_CLOUD = True                 # app.py:479 (see the module docstring)

models_cache: Dict[str, dict] = {}
processing_jobs: Dict[str, dict] = {}


class ProcessingRequest(BaseModel):       # app.py:47-56 (no `fov` field: the route's fov is dropped)
    model: str = "depth-anything-v2"
    output_format: str = "las"
    point_density: str = "medium"
    coordinate_system: str = "WGS84"
    gps_coords: Optional[Dict[str, float]] = None
    invert_depth: bool = True
    depth_scale: float = 10.0
    smooth_depth: bool = False
    smooth_ksize: int = 5


class ProcessingStatus(BaseModel):        # app.py:58-63
    job_id: str
    status: str
    progress: int
    message: str
    results: Optional[Dict[str, Any]] = None


# model id -> (spec factory, hub name the reference would fetch, network dtype)
def _registry():
    from .depth_anything import DA_V2_SMALL
    from .dpt import DPT_LARGE
    from .dpt_hybrid import DPT_HYBRID
    return {"depth-anything-v2": (DA_V2_SMALL, "depth-anything/Depth-Anything-V2-Small-hf", "bf16"),
            "dpt-large": (DPT_LARGE, "Intel/dpt-large", "bf16"),
            "dpt-hybrid": (DPT_HYBRID, "Intel/dpt-hybrid-midas", "fp8")}


def _load_weights(model_name: str, spec):
    """Local safetensors export of the hub checkpoint ($I2PC_WEIGHTS_DIR/<model>.safetensors),
    else seeded synthetic weights (the container has no network)."""
    d = os.environ.get("I2PC_WEIGHTS_DIR")
    if d:
        path = os.path.join(d, f"{model_name}.safetensors")
        if os.path.exists(path):
            from safetensors.torch import load_file
            return load_file(path)
    logger.warning(f"No local weights for {model_name}: using seeded synthetic weights")
    return None


def load_model(model_name: str):
    """app.py:64-96: cached model dict {"processor", "model", "type": "depth"}."""
    if model_name in models_cache:
        return models_cache[model_name]
    logger.info(f"Loading model: {model_name}")
    try:
        reg = _registry()
        if model_name in reg:
            from .pipeline import default_processor, model_for
            spec, _hub, dtype = reg[model_name]
            dev = geometry.require_device()
            model = {"processor": default_processor(spec),
                     "model": model_for(spec, _load_weights(model_name, spec), dev, dtype=dtype),
                     "type": "depth", "spec": spec, "preprocessors": {}}
        elif model_name in ("triposr", "instantmesh"):
            model = {"type": model_name, "loaded": True}             # the reference's demo stubs (app.py:72-86)
        else:
            raise ValueError(f"Unsupported model: {model_name}")
        models_cache[model_name] = model
        logger.info(f"Model {model_name} loaded successfully")
        return model
    except Exception as e:
        logger.error(f"Error loading model {model_name}: {str(e)}")
        from fastapi import HTTPException
        raise HTTPException(status_code=500, detail=f"Failed to load model: {str(e)}")


def _depth_device(image_t, model_info):
    """uint8 BGR device tensor [H, W, 3] -> model-resolution depth fp32 device tensor [h', w']."""
    from .preprocess import Preprocessor, ProcessorSpec
    spec = model_info["spec"]
    H, W = int(image_t.shape[0]), int(image_t.shape[1])
    cache = model_info.setdefault("preprocessors", {})
    pre = cache.get((H, W))
    if pre is None:
        p = model_info["processor"]
        if getattr(spec, "family", "dpt") in ("dpt", "dpt-hybrid"):
            p = ProcessorSpec(size=(spec.image, spec.image), mean=p.mean, std=p.std)
        pre = cache[(H, W)] = Preprocessor(H, W, p, patch=spec.patch)
    net = model_info["model"]
    patches = pre(image_t[None], layout=getattr(net, "input_layout", "patches"))
    gh, gw = pre.out_h // spec.patch, pre.out_w // spec.patch
    return net(patches, 1, gh, gw)[0]


def process_with_depth_anything(image: np.ndarray, model_info: dict) -> np.ndarray:
    """app.py:99-122: BGR uint8 HxWx3 -> float32 depth at the network resolution."""
    import torch
    try:
        dev = geometry.require_device()
        img = np.ascontiguousarray(image)
        if img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
            raise ValueError(f"expected a uint8 BGR HxWx3 image, got {img.dtype} {img.shape}")
        depth = _depth_device(torch.from_numpy(img).to(dev), model_info)
        return depth.cpu().numpy().astype(np.float32)
    except Exception as e:
        logger.error(f"Error in depth estimation: {str(e)}")
        raise


create_depth_preview = preview.create_depth_preview
depth_to_point_cloud = geometry.depth_to_point_cloud
save_point_cloud = writers.save_point_cloud


def refine_point_cloud(points, colors, nb_neighbors: int = 20, std_ratio: float = 2.0):
    """app.py:252-269: statistical outlier removal on the device; (points[ind], colors[ind]).

    Same error behaviour as the reference (any failure is logged and the cloud comes
    back unrefined), except that a missing libi2pc.so / HIP device raises.
    """
    from . import _lib
    try:
        if points is None or len(points) == 0:
            return points, colors
        import torch
        dev = geometry.require_device()
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(points, dtype=np.float32).reshape(-1, 3))).to(dev)
        ind = geometry.remove_statistical_outlier(t, None, nb_neighbors, std_ratio).index.cpu().numpy()
        points_f = points[ind]
        colors_f = colors[ind] if colors is not None and len(colors) == len(points) else colors
        return points_f, colors_f
    except _lib.I2PCError:
        raise
    except Exception as e:
        logger.warning(f"Point cloud refinement failed: {e}")
        return points, colors


def generate_gis_metadata(points, request: ProcessingRequest, bounds: Optional[dict] = None) -> dict:
    """app.py:391-417.  `bounds` may come from the device bbox (geometry.generate_gis_bounds)."""
    if bounds is None:
        p = np.asarray(points)
        bounds = {"minX": float(p[:, 0].min()), "maxX": float(p[:, 0].max()),
                  "minY": float(p[:, 1].min()), "maxY": float(p[:, 1].max()),
                  "minZ": float(p[:, 2].min()), "maxZ": float(p[:, 2].max())}
    md = {"coordinateSystem": request.coordinate_system, "bounds": bounds, "pointCount": len(points),
          "generatedWith": request.model, "outputFormat": request.output_format,
          "pointDensity": request.point_density, "depthScale": request.depth_scale,
          "invertDepth": request.invert_depth, "smoothDepth": request.smooth_depth}
    if request.gps_coords:
        md["gpsReference"] = request.gps_coords
    return md


def decode_image(image_data: bytes) -> np.ndarray:
    """cv2.imdecode(buf, IMREAD_COLOR) (app.py:434): 8-bit BGR HxWx3 (Pillow decoder here)."""
    from PIL import Image, ImageOps
    try:
        im = Image.open(io.BytesIO(image_data))
        im = ImageOps.exif_transpose(im)              # IMREAD_COLOR applies the EXIF orientation
        rgb = np.asarray(im.convert("RGB"))
    except Exception:
        raise ValueError("Failed to decode image data")
    return np.ascontiguousarray(rgb[:, :, ::-1])


def run_depth_job(image: np.ndarray, request: ProcessingRequest, job_id: str, model_info: dict,
                  on_progress=None) -> dict:
    """The depth branch of process_image_pipeline (app.py:456-559) as one device pass:
    depth -> preview -> unprojection + bbox -> outlier removal -> preview subsample -> artefact.
    `on_progress(progress, message)` receives the reference's milestones 60 (app.py:465-466,
    after the depth preview) and 80 (app.py:492-493, after the outlier removal)."""
    import torch
    report = on_progress if on_progress is not None else (lambda progress, message: None)
    dev = geometry.require_device()
    timg = torch.from_numpy(np.ascontiguousarray(image)).to(dev)
    depth = _depth_device(timg, model_info)
    depth_url = None
    try:                                                                  # app.py:463 -> :124-172
        depth_url = preview.encode_png_data_url(preview.colored_preview(depth, request.invert_depth).cpu().numpy())
    except Exception as e:
        logger.error(f"Failed to create depth preview: {e}")
    report(60, "Generating 3D point cloud...")
    pb = geometry.unproject_batch(depth[None], timg[None], density=request.point_density,
                                  invert=request.invert_depth, depth_scale=request.depth_scale,
                                  smooth=request.smooth_depth, smooth_ksize=request.smooth_ksize)
    xyz, rgb, bbox = pb.xyz[0], pb.rgb[0], pb.bbox[0]
    if REFINE_POINT_CLOUD:                                                # app.py:479
        sr = geometry.remove_statistical_outlier(xyz, rgb)
        xyz, rgb, bbox = sr.xyz, sr.rgb, sr.bbox
    report(80, "Saving point cloud...")
    n = xyz.shape[0]
    prev_pts, prev_cols = geometry.preview_subsample(xyz, rgb, MAX_PREVIEW)
    points = xyz.cpu().numpy()
    colors = rgb.cpu().numpy()
    if request.output_format.lower() in {"mesh_ply", "mesh"}:
        raise ValueError("mesh output (Poisson reconstruction, app.py:514-516) is out of scope for this backend")
    filepath = save_point_cloud(points, colors, request.output_format, job_id)
    metadata = generate_gis_metadata(points, request, bounds=geometry.generate_gis_bounds(bbox.cpu()))
    return {"pointCloud": {"filepath": filepath, "points": int(n), "format": request.output_format.upper()},
            "gisData": metadata, "downloadUrl": f"/download/{job_id}",
            "preview": {"points": prev_pts, "colors": prev_cols},
            "meshPreview": None, "depthMap": depth_url}


def process_image_pipeline(job_id: str, image_data: bytes, request: ProcessingRequest, jobs: dict = None):
    """app.py:419-565 (synchronous; the server runs it off the event loop)."""
    jobs = processing_jobs if jobs is None else jobs
    job = jobs[job_id]
    try:
        job.update(status="processing", progress=10, message="Loading AI model...")
        model_info = load_model(request.model)
        job.update(progress=20, message="Processing image...")
        image = decode_image(image_data)
        size = preprocess.reference_downscale_size(image.shape[0], image.shape[1], MAX_IMAGE_DIM)
        if size is not None:                                # app.py:436-445 (cv2 INTER_AREA)
            import torch
            dev = geometry.require_device()
            image = preprocess.resize_area(torch.from_numpy(np.ascontiguousarray(image)).to(dev), *size).cpu().numpy()
            logger.info(f"Resized input image to {size[0]}x{size[1]} for processing")
        if model_info.get("type") != "depth":
            raise ValueError(f"model {request.model} has no depth branch in this backend")
        job.update(progress=40, message="Estimating depth with AI...")
        results = run_depth_job(image, request, job_id, model_info,
                                on_progress=lambda pr, msg: job.update(progress=pr, message=msg))
        job.update(progress=100, status="completed", message="Processing complete!", results=results)
    except Exception as e:
        logger.error(f"Error in processing pipeline: {str(e)}")
        logger.error(traceback.format_exc())
        job.update(status="error", message=f"Error: {str(e)}")

"""Batched image -> point-cloud pipeline on one MI355X (the hot path end to end).

Replaces the depth branch of process_image_pipeline (backend/app.py:456-476)
plus the bounds of generate_gis_metadata (app.py:540 -> :391-400) for a batch:

    uint8 BGR [B,H,W,3] in HBM
      -> preprocess (Pillow-exact bicubic, normalise, patchify)     app.py:103,109
      -> DPT depth network (bf16 MFMA kernels)                       app.py:111-116
      -> depth resize + exact p2/p98 + normalise + unproject + RGB
         gather + bbox                                              app.py:174-250, 391-400
      -> xyz f32 [B,N,3], rgb u8 [B,N,3], bbox f64 [B,6]

`run()` is launch-only (all buffers preallocated), so `capture()` can record the
whole step into one HIP graph and `replay()` re-issues it with no host work.
"""
from __future__ import annotations

from typing import Optional

from . import geometry
from .dpt import DPT_LARGE, DPTSpec
from .preprocess import DEPTH_ANYTHING_PROCESSOR, DPT_LARGE_PROCESSOR, Preprocessor, ProcessorSpec


def model_for(spec, state_dict=None, device=None, seed: int = 0, dtype: str = "bf16"):
    """The network of a spec's family (DPT, DPT-Hybrid or Depth-Anything); seeded synthetic
    weights when none are given.  dtype "fp8" selects the MX fp8 engine (DPT-Hybrid only)."""
    family = getattr(spec, "family", "dpt")
    if dtype not in ("bf16", "fp8") or (dtype == "fp8" and family != "dpt-hybrid"):
        raise ValueError(f"dtype {dtype!r} is not available for {family}")
    if family == "depth-anything":
        from .depth_anything import DepthAnythingModel as Model, synthetic_state_dict
    elif family == "dpt-hybrid":
        from .dpt_hybrid import DPTHybridModel, synthetic_state_dict
        sd = state_dict if state_dict is not None else synthetic_state_dict(spec, seed)
        return DPTHybridModel(spec, sd, device, dtype=dtype)
    else:
        from .dpt import DPTDepthModel as Model, synthetic_state_dict
    return Model(spec, state_dict if state_dict is not None else synthetic_state_dict(spec, seed), device)


def default_processor(spec) -> ProcessorSpec:
    return DEPTH_ANYTHING_PROCESSOR if getattr(spec, "family", "dpt") == "depth-anything" else DPT_LARGE_PROCESSOR


class PointCloudPipeline:
    def __init__(self, batch: int, height: int, width: int, spec: DPTSpec = DPT_LARGE,
                 state_dict: Optional[dict] = None, processor: Optional[ProcessorSpec] = None,
                 density: str = "high", invert: bool = True, depth_scale: float = 10.0,
                 smooth: bool = False, fov: Optional[float] = None, device=None, seed: int = 0, model=None,
                 dtype: str = "bf16"):
        import torch
        self.device = torch.device(device) if device is not None else geometry.require_device()
        self.batch, self.height, self.width = batch, height, width
        self.spec = spec
        self.density, self.invert, self.depth_scale, self.smooth, self.fov = density, invert, depth_scale, smooth, fov
        if model is None:
            model = model_for(spec, state_dict, self.device, seed, dtype)
        self.model = model
        processor = processor or default_processor(spec)
        if getattr(spec, "family", "dpt") in ("dpt", "dpt-hybrid"):
            processor = ProcessorSpec(size=(spec.image, spec.image), mean=processor.mean, std=processor.std,
                                      keep_aspect_ratio=processor.keep_aspect_ratio, multiple=processor.multiple)
        self.pre = Preprocessor(height, width, processor, patch=spec.patch)
        self.gh, self.gw = self.pre.out_h // spec.patch, self.pre.out_w // spec.patch
        step = geometry.DENSITY_STEP[density]
        self.points_per_image = geometry.point_count(height, width, step)
        # network input: bf16 patch rows (ViT patch embedding) or fp32 NCHW pixels (BiT stem)
        self.layout = getattr(model, "input_layout", "patches")
        if self.layout == "patches":
            self._patches = torch.zeros((batch * self.gh * self.gw, self.pre.patch_pitch), dtype=torch.bfloat16,
                                        device=self.device)
        else:
            self._patches = torch.zeros((batch, 3, self.pre.out_h, self.pre.out_w), dtype=torch.float32,
                                        device=self.device)
        self._out = geometry.PointBatch(
            xyz=torch.empty((batch, self.points_per_image, 3), dtype=torch.float32, device=self.device),
            rgb=torch.empty((batch, self.points_per_image, 3), dtype=torch.uint8, device=self.device),
            bbox=torch.empty((batch, 6), dtype=torch.float64, device=self.device),
            stats=torch.empty((batch, 4), dtype=torch.float64, device=self.device))
        # the pipeline owns its unprojection workspace: a captured graph bakes its address in,
        # so it must never be the shared per-device scratch that other calls may regrow
        self._ws = torch.empty(max(geometry.workspace_bytes(batch, height, width, smooth), 1),
                               dtype=torch.uint8, device=self.device)
        self._graph = None
        self._static_in = None
        self.depth = None

    def infer_depth(self, images):
        """images: uint8 [B,H,W,3] BGR on the device -> model-resolution depth fp32 [B, h', w']."""
        self.pre(images, layout=self.layout, out=self._patches)
        self.depth = self.model(self._patches, self.batch, self.gh, self.gw)
        return self.depth

    def run(self, images):
        """images: uint8 [B,H,W,3] BGR on the device -> PointBatch (device tensors, reused across calls)."""
        self.infer_depth(images)
        return geometry.unproject_batch(self.depth, images, density=self.density, invert=self.invert,
                                        depth_scale=self.depth_scale, smooth=self.smooth, fov=self.fov,
                                        out=self._out, workspace=self._ws)

    __call__ = run

    def capture(self, images):
        """Record run(images) into a HIP graph (images must stay at the same address)."""
        import torch
        self._static_in = images
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self.run(images)        # warm every allocation and workspace outside the capture
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = self.run(images)
        self._graph = g
        return out

    def replay(self):
        self._graph.replay()
        return self._out


"""Prepared-network file of the native executor (libi2pc.so: i2pc_model_create / i2pc_depth_forward).

`process_with_depth_anything` (backend/app.py:99-122) loads a transformers model and runs the
processor and the forward in Python.  The C ABI runs the same network with no Python: a host
program (C, Go over cgo, a ctypes stub in app.py -- INTEGRATION.md) passes the path of a file this
module writes from a loaded `DepthAnythingModel` -- every weight already in the layout the kernels
take (bf16 [out][in] linears, LayerNorm-folded QKV / FC1 with their column sums, LayerScale folded
into O / FC2, [Co][ky*kx*Ci] convs, ConvTranspose as [s*s*Co][Ci], channels padded to the GEMM
granules) plus the position table interpolated for the input size the file is made for.  The
executor then issues exactly the launches `DepthAnythingModel.forward` issues, in the same order with
the same descriptors, so its depth equals the Python path's bit for bit
(tests/test_model_file_gpu.py).

Format (little endian):
  b"I2PCNET1"
  int32[32]  ints   (I_* below)
  float32[16] floats (F_* below)
  ntensors x { char name[48] (NUL padded); int32 dtype (0 fp32, 1 bf16); int32 ndim;
               int64 dims[4]; int64 offset (from the data start); int64 nbytes }
  data (every tensor at a 256-byte aligned offset)
"""
from __future__ import annotations

import struct

MAGIC = b"I2PCNET1"
FAMILY_DEPTH_ANYTHING = 1
VERSION = 2   # 2: the Q rows of the QKV weights carry the softmax scale * log2(e) (ops.fold_q_scale)
# int header slots
(I_FAMILY, I_VERSION, I_IN_H, I_IN_W, I_OUT_H, I_OUT_W, I_GH, I_GW, I_PATCH, I_HIDDEN, I_LAYERS, I_HEADS, I_MLP,
 I_FUSION, I_HEAD_HIDDEN, I_H1P, I_NECK0, I_FAC0, I_OUT0, I_NTENSORS, I_PITCH, I_STRIDE0) = (
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 20, 24, 28, 29, 30)
# float header slots
F_EPS, F_B_H3, F_MEAN0, F_STD0 = 0, 1, 2, 5
NAME_LEN = 48
ENTRY = struct.Struct("<48sii4qqq")


def _fac_code(fac) -> int:
    """Reassemble factor as an int: 4, 2, 1, or -s for a stride-s 3x3 conv (factor 1/s)."""
    return int(fac) if fac >= 1 else -int(round(1 / fac))


def _tensors(model, gh: int, gw: int):
    """(name, tensor) of everything DepthAnythingModel.forward reads, in the executor's names."""
    t = [("pe.w", model.w_pe), ("pe.b", model.b_pe), ("cls", model.cls), ("pos0", model.pos0),
         ("pos.table", model.pos_table(gh, gw))]
    for i, L in enumerate(model.layers):
        for k in ("ln1_g", "ln1_b", "w_qkv", "b_qkv", "w_qkv_f", "b_qkv_f", "s_qkv", "w_o", "b_o", "w_1_f", "b_1_f",
                  "s_1", "w_2", "b_2"):
            t.append((f"L{i}.{k}", L[k]))
    t += [("ln_g", model.ln_g), ("ln_b", model.ln_b)]
    for j, st in enumerate(model.stages):
        for k in ("w_proj", "b_proj", "w_neck", "w_rs", "b_rs"):
            if k in st:
                t.append((f"S{j}.{k}", st[k]))
    for j, fl in enumerate(model.fusion):
        t += [(f"F{j}.w_proj", fl["w_proj"]), (f"F{j}.b_proj", fl["b_proj"])]
        for r, rn in (("residual_layer1", "r1"), ("residual_layer2", "r2")):
            for c, cn in (("convolution1", "c1"), ("convolution2", "c2")):
                t += [(f"F{j}.{rn}{cn}.w", fl[f"{r}.{c}.w"]), (f"F{j}.{rn}{cn}.b", fl[f"{r}.{c}.b"])]
    t += [("H.w1", model.w_h1), ("H.b1", model.b_h1), ("H.w2", model.w_h2), ("H.b2", model.b_h2), ("H.w3", model.w_h3)]
    return t


def export_depth_anything(model, path: str, in_h: int, in_w: int, processor=None) -> str:
    """Write `model` (a DepthAnythingModel) for in_h x in_w input images to `path`."""
    import torch
    from .pipeline import default_processor
    from .preprocess import output_size, patch_pitch
    spec = model.spec
    proc = processor or default_processor(spec)
    out_h, out_w = output_size(in_h, in_w, proc)
    gh, gw = out_h // spec.patch, out_w // spec.patch
    tens = _tensors(model, gh, gw)
    ints = [0] * 32
    ints[I_FAMILY], ints[I_VERSION] = FAMILY_DEPTH_ANYTHING, VERSION
    ints[I_IN_H], ints[I_IN_W], ints[I_OUT_H], ints[I_OUT_W], ints[I_GH], ints[I_GW] = in_h, in_w, out_h, out_w, gh, gw
    ints[I_PATCH], ints[I_HIDDEN], ints[I_LAYERS], ints[I_HEADS], ints[I_MLP] = (
        spec.patch, spec.hidden, spec.layers, spec.heads, spec.mlp)
    ints[I_FUSION], ints[I_HEAD_HIDDEN], ints[I_H1P] = spec.fusion, spec.head_hidden, model.h1p
    for j, st in enumerate(model.stages):
        ints[I_NECK0 + j] = st["c"]
        ints[I_FAC0 + j] = _fac_code(st["fac"])
    for j, o in enumerate(spec.out_indices):
        ints[I_OUT0 + j] = o
    ints[I_NTENSORS] = len(tens)
    ints[I_PITCH] = patch_pitch(spec.patch)
    floats = [0.0] * 16
    floats[F_EPS], floats[F_B_H3] = spec.eps, model.b_h3
    floats[F_MEAN0:F_MEAN0 + 3] = list(proc.mean)
    floats[F_STD0:F_STD0 + 3] = list(proc.std)
    entries, blobs, off = [], [], 0
    for name, x in tens:
        if len(name.encode()) >= NAME_LEN:
            raise ValueError(name)
        x = x.detach().contiguous()
        dt = {torch.float32: 0, torch.bfloat16: 1}[x.dtype]
        raw = x.view(torch.int16 if dt else torch.int32).cpu().numpy().tobytes()
        dims = list(x.shape) + [1] * (4 - x.dim())
        entries.append(ENTRY.pack(name.encode(), dt, x.dim(), *dims, off, len(raw)))
        blobs.append((off, raw))
        off = (off + len(raw) + 255) // 256 * 256
    with open(path, "wb") as fh:
        fh.write(MAGIC)
        fh.write(struct.pack("<32i", *ints))
        fh.write(struct.pack("<16f", *floats))
        fh.write(b"".join(entries))
        data = bytearray(off)
        for o, raw in blobs:
            data[o:o + len(raw)] = raw
        fh.write(bytes(data))
    return path


def read_header(path: str) -> dict:
    """The ints / floats / tensor table of a prepared-network file (host only; tests)."""
    with open(path, "rb") as fh:
        if fh.read(8) != MAGIC:
            raise ValueError(f"{path}: not an i2pc network file")
        ints = struct.unpack("<32i", fh.read(128))
        floats = struct.unpack("<16f", fh.read(64))
        tabs = {}
        for _ in range(ints[I_NTENSORS]):
            name, dt, nd, d0, d1, d2, d3, off, nb = ENTRY.unpack(fh.read(ENTRY.size))
            tabs[name.rstrip(b"\0").decode()] = dict(dtype=dt, shape=(d0, d1, d2, d3)[:nd], offset=off, nbytes=nb)
    return dict(ints=ints, floats=floats, tensors=tabs)


def _register():
    import ctypes
    from . import _lib
    P, I = ctypes.c_void_p, ctypes.c_int
    _lib.register("i2pc_model_create", I, [ctypes.c_char_p, I, I, I, ctypes.POINTER(P)])
    _lib.register("i2pc_model_destroy", I, [P])
    _lib.register("i2pc_model_io", I, [P] + [ctypes.POINTER(I)] * 5)
    _lib.register("i2pc_depth_forward", I, [P, P, P, P])
    _lib.register("i2pc_model_file_info", I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_float), ctypes.POINTER(I)])


_register()


def file_info(path: str):
    """(ints, floats, ntensors) of a prepared-network file as libi2pc.so reads it (host only)."""
    import ctypes
    from . import _lib
    ints = (ctypes.c_int32 * 32)()
    floats = (ctypes.c_float * 16)()
    n = ctypes.c_int()
    _lib.call("i2pc_model_file_info", path.encode(), ints, floats, ctypes.byref(n))
    return list(ints), list(floats), n.value


class NativeDepthModel:
    """The C executor (i2pc_model_create / i2pc_depth_forward) from Python: the ctypes binding a
    caller of the C ABI writes."""

    def __init__(self, path: str, batch: int, in_h: int, in_w: int):
        import ctypes
        from . import _lib
        h = ctypes.c_void_p()
        _lib.call("i2pc_model_create", path.encode(), int(batch), int(in_h), int(in_w), ctypes.byref(h))
        self._h, self._lib = h, _lib.load()
        v = [ctypes.c_int() for _ in range(5)]
        _lib.call("i2pc_model_io", h, *[ctypes.byref(x) for x in v])
        self.batch, self.in_h, self.in_w, self.depth_h, self.depth_w = (x.value for x in v)

    def forward(self, bgr, out=None):
        """bgr: torch.uint8 [batch, in_h, in_w, 3] on the device -> depth fp32 [batch, depth_h, depth_w]."""
        import torch
        from . import _lib
        if tuple(bgr.shape) != (self.batch, self.in_h, self.in_w, 3) or bgr.dtype != torch.uint8 or not bgr.is_cuda:
            raise ValueError(f"expected uint8 device images {(self.batch, self.in_h, self.in_w, 3)}")
        bgr = bgr.contiguous()
        if out is None:
            out = torch.empty((self.batch, self.depth_h, self.depth_w), dtype=torch.float32, device=bgr.device)
        _lib.call("i2pc_depth_forward", self._h, bgr.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out

    __call__ = forward

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.i2pc_model_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

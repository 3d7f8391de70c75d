"""Torch-tensor wrappers over the network entry points of the C ABI (include/i2pc.h).

Every function launches a hand-written gfx950 kernel from libi2pc.so on the
current stream; nothing here computes on the host, and nothing falls back to
PyTorch arithmetic.  Tensors must already live on the device.
Layouts: activations bf16 NHWC / [rows][features]; residual stream fp32.
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _lib

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_void_p = ctypes.c_void_p


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("a", c_void_p), ("lda", c_int64), ("m", c_int32), ("n", c_int32), ("k", c_int32),
        ("a_group", c_int32), ("a_group_stride", c_int32), ("a_offset", c_int32),
        ("conv", c_int32), ("conv_batch", c_int32), ("conv_h", c_int32), ("conv_w", c_int32),
        ("conv_c", c_int32), ("conv_oh", c_int32), ("conv_ow", c_int32), ("conv_k", c_int32),
        ("conv_stride", c_int32), ("conv_pad", c_int32), ("conv_relu_in", c_int32),
        ("w", c_void_p), ("ldw", c_int64),
        ("bias", c_void_p),
        ("row_bias", c_void_p), ("row_bias_group", c_int32),
        ("table", c_void_p), ("table_rows", c_int32),
        ("act", c_int32),
        ("res", c_void_p), ("res_f32", c_int32), ("ldr", c_int64),
        ("res2", c_void_p), ("ldr2", c_int64),
        ("c", c_void_p), ("c_f32", c_int32), ("ldc", c_int64),
        ("out_group", c_int32), ("out_group_stride", c_int32), ("out_offset", c_int32),
        ("convt_s", c_int32), ("convt_h", c_int32), ("convt_w", c_int32), ("convt_c", c_int32),
        ("ln_rows", c_void_p), ("col_sum", c_void_p), ("ln_part", c_void_p), ("c_bf16", c_void_p),
        ("ldc_bf16", c_int64), ("ln_shift", c_void_p), ("ln_chunk", c_int32), ("res_shift", c_void_p),
    ]


_lib.register("i2pc_gemm", ctypes.c_int, [ctypes.POINTER(GemmDesc), c_void_p])
_lib.register("i2pc_gemm_ws", ctypes.c_int, [ctypes.POINTER(GemmDesc), c_void_p, ctypes.c_size_t, c_void_p])
_lib.register("i2pc_gemm_workspace_bytes", ctypes.c_size_t, [ctypes.POINTER(GemmDesc)])
_lib.register("i2pc_gemm_kernel_name", ctypes.c_char_p, [ctypes.POINTER(GemmDesc)])
_lib.register("i2pc_gemm_set_engine", ctypes.c_int, [ctypes.c_int])
_lib.register("i2pc_set_tuning", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int])
_lib.register("i2pc_ln_rowstats", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, c_void_p,
                                                 c_void_p, c_void_p, c_void_p])
_lib.register("i2pc_ln_rowstats_w", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                                   c_void_p, c_void_p, c_void_p, c_void_p])
_lib.register("i2pc_ln_apply", ctypes.c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, ctypes.c_int,
                                              ctypes.c_int, c_void_p, c_int64, c_void_p])
_lib.register("i2pc_layernorm_stats", ctypes.c_int, [c_void_p, c_int64, c_void_p, c_void_p, ctypes.c_float,
                                                     ctypes.c_int, ctypes.c_int, c_void_p, c_int64, c_void_p, c_void_p])
_lib.register("i2pc_layernorm", ctypes.c_int, [c_void_p, c_int64, c_void_p, c_void_p, ctypes.c_float,
                                               ctypes.c_int, ctypes.c_int, c_void_p, c_int64, c_void_p])
_lib.register("i2pc_attention", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_float, c_void_p, c_void_p])
_lib.register("i2pc_attention_q2", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p])
_lib.register("i2pc_attention_q2_fp8", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                                      ctypes.c_int64, c_void_p, ctypes.c_int64, c_void_p])
_lib.register("i2pc_attention_fp8", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                                   c_void_p, c_int64, c_void_p, c_int64, c_void_p])
_lib.register("i2pc_upsample2x", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, c_void_p, c_void_p, c_void_p])
_lib.register("i2pc_upsample2x_fp8", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p])
_lib.register("i2pc_resize_bilinear", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     c_void_p, c_void_p, c_void_p])
_lib.register("i2pc_cls_pos", ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             c_void_p, c_void_p])
_lib.register("i2pc_f32_to_bf16", ctypes.c_int, [c_void_p, c_int64, c_void_p, c_void_p])
_lib.register("i2pc_head_out", ctypes.c_int, [c_void_p, c_int64, ctypes.c_int, c_void_p, ctypes.c_float,
                                              c_void_p, c_void_p])
_lib.register("i2pc_head_upconv", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                                  ctypes.c_float, c_void_p, c_void_p])

ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2}


def _torch():
    import torch
    return torch


def _p(t):
    return 0 if t is None else t.data_ptr()


def _stream():
    return _torch().cuda.current_stream().cuda_stream


def _check(t, dtype, name):
    torch = _torch()
    if t is None:
        return
    if not t.is_cuda:
        raise _lib.I2PCError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


# ---------------------------------------------------------------- launch timing
# When `profile` is a list, every wrapped launch appends (kernel label, flops,
# bytes, start event, end event) recorded on the launch stream; bench.py turns
# that into per-kernel durations and roofline fractions.
profile = None


class _Timed:
    def __init__(self, label, flops=0.0, nbytes=0.0):
        self.label, self.flops, self.nbytes = label, flops, nbytes

    def __enter__(self):
        if profile is not None:
            torch = _torch()
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record(torch.cuda.current_stream())
        return self

    def __exit__(self, *exc):
        if profile is not None:
            torch = _torch()
            self.e1.record(torch.cuda.current_stream())
            profile.append((self.label, self.flops, self.nbytes, self.e0, self.e1))
        return False


def gemm_kernel_label(desc: GemmDesc) -> str:
    """Name of the kernel instance i2pc_gemm dispatches to (asked of the C side, so it cannot drift)."""
    return _lib.load().i2pc_gemm_kernel_name(ctypes.byref(desc)).decode()


# every knob i2pc_set_tuning accepts (include/i2pc.h), checked by tests/test_abi.py
TUNING_KNOBS = ("gemm_tail", "gemm_bn128", "gemm_splitk", "gemm_split_tile", "gemm_tile192", "gemm_lnp_p", "gemm_lnp_stream", "conv_halo", "gelu_tanh", "gemm_resq", "gemm_simple_epi", "gemm_tail160",
                "gemm_stagger", "unp_rows",
                "unp_nt", "unp_rpt", "sel_windows", "sel_parts", "sel_rows", "sel_lband", "sel_scratch", "attn_lazy", "attn_scalar",
                "attn_rb", "ln_f2", "ln_apply_gs", "resize_rows")


def set_tuning(name: str, value: int) -> None:
    """Kernel-selection knob (i2pc_set_tuning) for calls made from THIS host thread (thread-local
    in libi2pc.so); the names are TUNING_KNOBS."""
    _lib.call("i2pc_set_tuning", name.encode(), int(value))


def set_gemm_engine(mode: int) -> None:
    """0 = automatic, 1 = tile kernel only, 2 = persistent engine wherever its epilogue applies,
    3 = automatic with the ping-pong engine, 4 = ping-pong engine wherever it applies."""
    _lib.call("i2pc_gemm_set_engine", int(mode))


def gemm_bytes(d: GemmDesc, esz: float = 2.0, c_esz: float = None) -> float:
    """Algorithmic HBM bytes of one GEMM / implicit-GEMM conv: A read once (a conv reads its
    input map once), W once, C written once, residuals read once (scales of fp8 operands add
    1/32 per element)."""
    M, N, K = d.m, d.n, d.k
    a = (d.conv_batch * d.conv_h * d.conv_w * d.conv_c) if d.conv else M * K
    c_esz = (4.0 if d.c_f32 else 2.0) if c_esz is None else c_esz
    b = a * esz + N * K * esz + M * N * c_esz
    if d.res:
        b += M * N * (4.0 if d.res_f32 else 2.0)
    if d.res2:
        b += M * N * 2.0
    if d.ln_part:          # LN-fold producer: the bf16 copy (unless it is the output) + chunk partials
        b += (M * N * 2.0 if d.c_f32 else 0.0) + M * (N // (d.ln_chunk or 64)) * 8.0
    if d.res_shift:
        b += M * 4.0
    if d.ln_rows:          # LN-fold consumer: row scales + column sums
        b += M * 8.0 + N * 4.0
    return b


def gemm(desc: GemmDesc) -> None:
    """i2pc_gemm_ws with a split-K workspace from torch's stream-ordered caching allocator when
    the call splits (inside a graph capture it comes from the graph's pool, so replays own it)."""
    nb = _lib.load().i2pc_gemm_workspace_bytes(ctypes.byref(desc))
    ws = _torch().empty(nb, dtype=_torch().uint8, device="cuda") if nb else None
    if profile is None:
        _lib.call("i2pc_gemm_ws", ctypes.byref(desc), _p(ws), nb, _stream())
        return
    with _Timed(gemm_kernel_label(desc), 2.0 * desc.m * desc.n * desc.k, gemm_bytes(desc)):
        _lib.call("i2pc_gemm_ws", ctypes.byref(desc), _p(ws), nb, _stream())


def _ceil(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def _pad_cols(t, cols: int):
    """A copy of the 2-D device tensor t [R, c] zero-padded to [R, cols] (same dtype)."""
    torch = _torch()
    o = torch.zeros((t.shape[0], cols), dtype=t.dtype, device=t.device)
    o[:, :t.shape[1]] = t
    return o


_PAD_CACHE = {}


def _padded_param(t, shape, fill_view):
    """Zero-padded copy of a parameter tensor, made once per (tensor, version) and cached (ADVICE
    r03: the padded GEMM / conv paths used to rebuild every weight and bias on each call, inside HIP
    graph captures too).  fill_view(padded) returns the view `t` is copied into."""
    import weakref
    torch = _torch()
    key = (id(t), tuple(shape))
    hit = _PAD_CACHE.get(key)
    if hit is not None and hit[0]() is t and hit[1] == t._version:
        return hit[2]
    o = torch.zeros(shape, dtype=t.dtype, device=t.device)
    fill_view(o).copy_(t.reshape(fill_view(o).shape))
    for k in [k for k, v in _PAD_CACHE.items() if v[0]() is None]:       # drop entries of freed tensors
        del _PAD_CACHE[k]
    _PAD_CACHE[key] = (weakref.ref(t), t._version, o)
    return o


def _linear_padded(x, w, bias, act, res, res2, out, out_f32, rows):
    """linear() for widths the GEMM engines do not take (K % 64, N % 32): the operands are
    zero-padded to K' = ceil64(K), N' = ceil32(N) (zero weights and bias add nothing), the HIP
    GEMM runs on the padded shapes and the first N columns are copied to `out`.  For checkpoints
    whose widths differ from the shipped models'; the shipped networks never take this path."""
    torch = _torch()
    M = rows if rows is not None else x.shape[0]
    N, K = w.shape
    Kp, Np = _ceil(K, 64), _ceil(N, 32)
    xp = _pad_cols(x[:M].reshape(M, -1)[:, :K], Kp) if Kp != K else x
    wp = _padded_param(w, (Np, Kp), lambda o: o[:N, :K])
    bp = _padded_param(bias, (Np,), lambda o: o[:N]) if bias is not None else None
    rp = _pad_cols(res[:M], Np) if res is not None else None
    r2p = _pad_cols(res2[:M], Np) if res2 is not None else None
    dt = out.dtype if out is not None else (torch.float32 if out_f32 else torch.bfloat16)
    op = torch.empty((M, Np), dtype=dt, device=x.device)
    linear(xp, wp, bias=bp, act=act, res=rp, res2=r2p, out=op, rows=M)
    if out is None:
        return op[:, :N].contiguous()
    out[:M, :N].copy_(op[:, :N])
    return out


def linear(x, w, bias=None, act=None, res=None, res2=None, out=None, out_f32=False,
           a_map=(0, 0, 0), out_map=(0, 0, 0), rows=None, row_bias=None, row_bias_group=1,
           table=None, table_rows=1, ldc=None, ln_rows=None, col_sum=None, ln_part=None, out_bf16=None,
           ln_shift=None, ln_chunk=64, res_shift=None):
    """out = act(x @ w.T + bias + row_bias + table) + res + res2.

    x: bf16 [*, K] (row stride x.stride(0)); w: bf16 [N, K]; rows = M (defaults to x rows).
    a_map / out_map = (group, group_stride, offset) row remaps (see i2pc.h).
    LayerNorm fold (i2pc.h): ln_rows fp32 [M, 2] (ln_rowstats) + col_sum fp32 [N] make this the
    consumer (out = act(rs.x * acc + rs.y * col_sum + bias)); ln_part fp32 [M, N / ln_chunk, 2] +
    out_bf16 bf16 [M, N] make an fp32-output call the producer (of out - ln_shift[row] when given;
    ln_chunk 64 or 32 columns per partial).  With a bf16 `out` and no out_bf16 the producer's only
    output is out = bf16(value - ln_shift[row]) (the shifted bf16 residual stream); a bf16 `res` is
    then read as res + res_shift[row] (the shift it was stored relative to).
    """
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    _check(w, torch.bfloat16, "w")
    M = rows if rows is not None else x.shape[0]
    N, K = w.shape
    if K % 64 or N % 32:
        plain = (a_map == (0, 0, 0) and out_map == (0, 0, 0) and row_bias is None and table is None and ldc is None
                 and ln_rows is None and ln_part is None)
        if not plain:
            raise _lib.I2PCError(f"linear: K={K} (% 64) / N={N} (% 32) are padded for plain calls only")
        return _linear_padded(x, w, bias, act, res, res2, out, out_f32, rows)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
    d = GemmDesc()
    d.a, d.lda, d.m, d.n, d.k = _p(x), x.stride(0), M, N, K
    d.a_group, d.a_group_stride, d.a_offset = a_map
    d.w, d.ldw = _p(w), w.stride(0)
    d.bias = _p(bias)
    d.row_bias, d.row_bias_group = _p(row_bias), row_bias_group
    d.table, d.table_rows = _p(table), table_rows
    d.act = ACT[act]
    if res is not None:
        d.res, d.res_f32, d.ldr = _p(res), int(res.dtype == torch.float32), res.stride(0)
    if res2 is not None:
        d.res2, d.ldr2 = _p(res2), res2.stride(0)
    d.c, d.c_f32 = _p(out), int(out.dtype == torch.float32)
    d.ldc = ldc if ldc is not None else out.stride(0)
    d.out_group, d.out_group_stride, d.out_offset = out_map
    if ln_rows is not None:
        _check(ln_rows, torch.float32, "ln_rows")
        _check(col_sum, torch.float32, "col_sum")
        d.ln_rows, d.col_sum = _p(ln_rows), _p(col_sum)
    if ln_part is not None:
        _check(ln_part, torch.float32, "ln_part")
        _check(out_bf16, torch.bfloat16, "out_bf16")
        if ln_chunk not in (32, 64):
            raise ValueError(f"ln_chunk={ln_chunk} must be 32 or 64")
        if out_bf16 is None and out.dtype != torch.bfloat16:
            raise ValueError("ln_part: an fp32 out needs out_bf16 (or pass a bf16 out: the shifted residual stream)")
        cb = out if out_bf16 is None else out_bf16
        if ln_part.numel() < 2 * M * (N // ln_chunk) or cb.shape[0] < M or cb.shape[-1] < N:
            raise ValueError("ln_part / out_bf16 too small for the call")
        if out_bf16 is not None:
            d.c_bf16, d.ldc_bf16 = _p(out_bf16), out_bf16.stride(0)
        d.ln_part = _p(ln_part)
        d.ln_chunk = ln_chunk
        if ln_shift is not None:
            _check(ln_shift, torch.float32, "ln_shift")
            d.ln_shift = _p(ln_shift)
    if res_shift is not None:
        _check(res_shift, torch.float32, "res_shift")
        d.res_shift = _p(res_shift)
    gemm(d)
    return out


def ln_rowstats(part, eps, out=None, shift_in=None, shift_out=None, chunk=64):
    """LayerNorm row statistics from producer partials: part fp32 [M, P, 2] of `chunk`-column
    chunks -> out fp32 [M, 2] = (rstd, -rstd * mean) (i2pc_ln_rowstats_w); shift_in: the
    producer's ln_shift (None = 0); shift_out fp32 [M] receives the rows' true means (may be shift_in)."""
    torch = _torch()
    _check(part, torch.float32, "part")
    _check(shift_in, torch.float32, "shift_in")
    _check(shift_out, torch.float32, "shift_out")
    M, P = part.shape[0], part.shape[1]
    if out is None:
        out = torch.empty((M, 2), dtype=torch.float32, device=part.device)
    nb = M * (P * 8.0 + 8.0 + (4.0 if shift_in is not None else 0.0) + (4.0 if shift_out is not None else 0.0))
    with _Timed("k_ln_rowstats", 0.0, nb):
        _lib.call("i2pc_ln_rowstats_w", _p(part), M, P, int(chunk), float(eps), _p(out), _p(shift_in), _p(shift_out),
                  _stream())
    return out


def ln_apply(x, rows_stats, gamma, beta, out=None):
    """LayerNorm of bf16 rows x [M, D] from ln_rowstats' (rstd, -rstd * mean) rows (i2pc_ln_apply):
    bf16(gamma * (rstd * x - rstd * mean) + beta)."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    _check(rows_stats, torch.float32, "rows_stats")
    M, D = x.shape
    if out is None:
        out = torch.empty((M, D), dtype=torch.bfloat16, device=x.device)
    with _Timed("k_ln_apply", 0.0, M * D * 4.0 + M * 8.0):
        _lib.call("i2pc_ln_apply", _p(x), x.stride(0), _p(rows_stats), _p(gamma), _p(beta), M, D, _p(out),
                  out.stride(0), _stream())
    return out


def ln_fold_weights(w, b, gamma, beta):
    """Weights of a LayerNorm-folded linear (i2pc.h): W' = bf16(W * gamma) [N, K], col_sum[n] =
    sum_k W'[n][k] (fp32, of the bf16 values the GEMM multiplies), bias' = b + W beta (fp32)."""
    torch = _torch()
    w32 = w.to(torch.float32)
    wg = (w32 * gamma.to(torch.float32)[None, :]).to(torch.bfloat16)
    col = wg.to(torch.float64).sum(1).to(torch.float32)
    bias = (b.to(torch.float64) + w32.to(torch.float64) @ beta.to(torch.float64)).to(torch.float32)
    return wg.contiguous(), col.contiguous(), bias.contiguous()


def conv2d(x, w, bias=None, k=3, stride=1, pad=1, relu_in=False, act=None, res=None, res2=None, out=None,
           out_hw=None):
    """NHWC bf16 conv via implicit GEMM.  w: bf16 [Co, k*k*Ci] in (ky, kx, ci) order.
    pad = top/left padding; out_hw overrides the output size (TF "SAME" stride-2 convs pad
    less on the top/left than on the bottom/right: the missing bottom/right taps read zero)."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    Co = w.shape[0]
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    if out_hw is not None:
        OH, OW = out_hw
    if C % 64 or Co % 32:
        # widths the engines do not take: zero-pad the input channels to ceil64(C) (the weights'
        # k*k*C axis with them) and the output channels to ceil32(Co), run the HIP conv, keep Co
        Cp, Cop = _ceil(C, 64), _ceil(Co, 32)
        xp = x
        if Cp != C:
            xp = torch.zeros((B, H, W, Cp), dtype=x.dtype, device=x.device)
            xp[..., :C] = x
        wp = _padded_param(w, (Cop, k * k, Cp), lambda o: o[:Co, :, :C])
        bp = _padded_param(bias, (Cop,), lambda o: o[:Co]) if bias is not None else None
        pad4 = lambda t: None if t is None else torch.nn.functional.pad(t, (0, Cop - Co))   # noqa: E731 (a copy)
        op = conv2d(xp, wp.reshape(Cop, k * k * Cp), bias=bp, k=k, stride=stride, pad=pad, relu_in=relu_in, act=act,
                    res=pad4(res), res2=pad4(res2), out_hw=(OH, OW))
        if out is None:
            return op[..., :Co].contiguous()
        out.copy_(op[..., :Co])
        return out
    if out is None:
        out = torch.empty((B, OH, OW, Co), dtype=torch.bfloat16, device=x.device)
    d = GemmDesc()
    d.a, d.lda, d.m, d.n, d.k = _p(x), C, B * OH * OW, Co, k * k * C
    if k == 1 and stride == 1 and pad == 0 and (OH, OW) == (H, W):
        pass    # a 1x1 conv is a plain GEMM over pixels
    else:
        d.conv, d.conv_batch, d.conv_h, d.conv_w, d.conv_c = 1, B, H, W, C
        d.conv_oh, d.conv_ow, d.conv_k, d.conv_stride, d.conv_pad = OH, OW, k, stride, pad
    d.conv_relu_in = int(relu_in)
    d.w, d.ldw = _p(w), w.stride(0)
    d.bias = _p(bias)
    d.act = ACT[act]
    if res is not None:
        d.res, d.res_f32, d.ldr = _p(res), int(res.dtype == torch.float32), Co
    if res2 is not None:
        d.res2, d.ldr2 = _p(res2), Co
    d.c, d.c_f32, d.ldc = _p(out), int(out.dtype == torch.float32), Co
    gemm(d)
    return out


def conv_transpose(x, w, bias_tiled, s, out=None):
    """ConvTranspose2d(kernel = stride = s) on NHWC bf16.  w: bf16 [s*s*Co, Ci] ((dy,dx,co) rows)."""
    torch = _torch()
    B, H, W, C = x.shape
    Co = w.shape[0] // (s * s)
    if out is None:
        out = torch.empty((B, H * s, W * s, Co), dtype=torch.bfloat16, device=x.device)
    d = GemmDesc()
    d.a, d.lda, d.m, d.n, d.k = _p(x), C, B * H * W, w.shape[0], C
    d.w, d.ldw = _p(w), w.stride(0)
    d.bias = _p(bias_tiled)
    d.c, d.c_f32, d.ldc = _p(out), 0, Co
    d.convt_s, d.convt_h, d.convt_w, d.convt_c = s, H, W, Co
    gemm(d)
    return out


def layernorm(x, gamma, beta, eps, out=None, mean_out=None):
    """nn.LayerNorm of fp32 rows -> bf16; mean_out (fp32 [rows]) also receives the row means."""
    torch = _torch()
    _check(x, torch.float32, "x")
    _check(mean_out, torch.float32, "mean_out")
    rows, dim = x.shape
    if out is None:
        out = torch.empty((rows, dim), dtype=torch.bfloat16, device=x.device)
    with _Timed("k_layernorm", 0.0, rows * dim * 6.0):
        if mean_out is not None:
            _lib.call("i2pc_layernorm_stats", _p(x), x.stride(0), _p(gamma), _p(beta), float(eps), rows, dim,
                      _p(out), out.stride(0), _p(mean_out), _stream())
        else:
            _lib.call("i2pc_layernorm", _p(x), x.stride(0), _p(gamma), _p(beta), float(eps), rows, dim,
                      _p(out), out.stride(0), _stream())
    return out


def attention(qkv, batch, tokens, heads, scale, out=None, q_log2=False):
    """Fused self-attention (i2pc_attention).  out: bf16 [batch*tokens, heads*64], or an Fp8 of that
    shape: the MX fp8 operand of the next GEMM written by the kernel's epilogue (i2pc_attention_fp8;
    the same bytes as quant_fp8 of the bf16 output).  q_log2: the Q block already holds
    q * scale * log2(e) (folded into the QKV weights, `fold_q_scale`); scale is then ignored and the
    threshold-rescale kernel runs (i2pc_attention_q2 / _q2_fp8)."""
    torch = _torch()
    _check(qkv, torch.bfloat16, "qkv")
    D = heads * 64
    if out is None:
        out = torch.empty((batch * tokens, D), dtype=torch.bfloat16, device=qkv.device)
    flops = 4.0 * batch * heads * tokens * tokens * 64
    if isinstance(out, Fp8):
        if tuple(out.data.shape) != (batch * tokens, D):
            raise ValueError(f"attention fp8 out {tuple(out.data.shape)} != {(batch * tokens, D)}")
        with _Timed("k_attention", flops, 2.0 * 3 * batch * tokens * D + (1.0 + 1.0 / 32) * batch * tokens * D):
            if q_log2:
                _lib.call("i2pc_attention_q2_fp8", _p(qkv), batch, tokens, heads, _p(out.data), D,
                          _p(out.scale), out.scale.shape[-1] // 4, _stream())
            else:
                _lib.call("i2pc_attention_fp8", _p(qkv), batch, tokens, heads, float(scale), _p(out.data), D,
                          _p(out.scale), out.scale.shape[-1] // 4, _stream())
        return out
    with _Timed("k_attention", flops, 2.0 * 4 * batch * tokens * D):
        if q_log2:
            _lib.call("i2pc_attention_q2", _p(qkv), batch, tokens, heads, _p(out), _stream())
        else:
            _lib.call("i2pc_attention", _p(qkv), batch, tokens, heads, float(scale), _p(out), _stream())
    return out


LOG2E = 1.4426950408889634


def fold_q_scale(w_qkv, b_qkv, scale):
    """The QKV weights and bias (fp32, Q | K | V row blocks of equal size) with the Q rows multiplied by
    scale * log2(e), in fp32 before any bf16 rounding: the product Q is then what
    attention(..., q_log2=True) takes (the softmax scale and the exp2 base conversion ride on the GEMM)."""
    c = float(scale) * LOG2E
    d = w_qkv.shape[0] // 3
    w = w_qkv.float().clone()
    b = b_qkv.float().clone()
    w[:d] *= c
    b[:d] *= c
    return w, b


def upsample2x(x, add=None, out=None, out_fp8=False):
    """Bilinear 2x (align_corners) of NHWC bf16 x (+ add); out_fp8: returned as Fp8 rows [B, 2H, 2W, C]
    (i2pc_upsample2x_fp8, the bytes quant_fp8 of the bf16 result would give)."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    if out_fp8:
        if out is None:
            out = empty_fp8((B, 2 * H, 2 * W, C), x.device)
        with _Timed("k_resize_fp8", 0.0, 2.0 * B * H * W * C + 4.0 * B * H * W * C * (1 + 1 / 32 + (2 if add is not None else 0))):
            _lib.call("i2pc_upsample2x_fp8", _p(x), B, H, W, C, _p(add), _p(out.data), out.data.shape[-1],
                      _p(out.scale), out.scale.shape[-1] // 4, _stream())
        return out
    if out is None:
        out = torch.empty((B, 2 * H, 2 * W, C), dtype=torch.bfloat16, device=x.device)
    with _Timed("k_resize", 0.0, 2.0 * B * H * W * C * (1 + 4 + (4 if add is not None else 0))):
        _lib.call("i2pc_upsample2x", _p(x), B, H, W, C, _p(add), _p(out), _stream())
    return out


def resize_bilinear(x, out_h, out_w, align_corners=True, add=None, out=None):
    """NHWC bf16 bilinear resize (torch upsample_bilinear2d index rules), optional + add."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty((B, out_h, out_w, C), dtype=torch.bfloat16, device=x.device)
    # algorithmic bytes: the input read once, the output written once, the addend read once (the
    # per-output taps re-read the input through the caches; that is traffic, not algorithm)
    with _Timed("k_resize", 0.0, 2.0 * B * C * (H * W + out_h * out_w * (1 + (1 if add is not None else 0)))):
        _lib.call("i2pc_resize_bilinear", _p(x), B, H, W, C, out_h, out_w, int(bool(align_corners)), _p(add),
                  _p(out), _stream())
    return out


def cls_pos(cls, pos0, x, batch, tokens, dim):
    _lib.call("i2pc_cls_pos", _p(cls), _p(pos0), batch, tokens, dim, _p(x), _stream())


def f32_to_bf16(x, out=None):
    torch = _torch()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    _lib.call("i2pc_f32_to_bf16", _p(x), x.numel(), _p(out), _stream())
    return out


def head_upconv(x, out_h, out_w, w2, b2, w4, b4: float, out=None, cin=None):
    """Fused head tail: align_corners resize to (out_h, out_w) -> 3x3 conv (C -> 32) + bias + ReLU
    -> 1x1 conv (32 -> 1) + bias + ReLU, without materialising the resized map.
    x: bf16 NHWC [B, h, w, C] (C % 8 == 0); w2: bf16 [32, 9*C]; b2, w4: fp32 [32]; cin: the
    channels used (default C, a multiple of 32; the rest are the zero padding of a narrower head)."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, h, w, C = x.shape
    cin = C if cin is None else int(cin)
    if tuple(w2.shape) != (32, 9 * C) or w2.dtype != torch.bfloat16:
        raise ValueError(f"head_upconv: w2 must be bf16 [32, {9 * C}], got {tuple(w2.shape)} {w2.dtype}")
    if out is None:
        out = torch.empty((B, out_h, out_w), dtype=torch.float32, device=x.device)
    flops = 2.0 * B * out_h * out_w * 32 * (9 * cin + 1)
    with _Timed("k_head_upconv", flops, 2.0 * B * h * w * cin + 4.0 * B * out_h * out_w):
        _lib.call("i2pc_head_upconv", _p(x), B, h, w, C, cin, out_h, out_w, _p(w2.contiguous()), _p(b2), _p(w4),
                  float(b4), _p(out), _stream())
    return out


def head_out(x, w, bias: float, out=None):
    torch = _torch()
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty((B, H, W), dtype=torch.float32, device=x.device)
    with _Timed("k_head_out", 2.0 * B * H * W * C, B * H * W * (2.0 * C + 4)):
        _lib.call("i2pc_head_out", _p(x), B * H * W, C, _p(w), float(bias), _p(out), _stream())
    return out


# ------------------------------------------------------------------ MX fp8 (DPT-Hybrid fp8 path)
class GemmFp8Desc(ctypes.Structure):
    _fields_ = [("g", GemmDesc), ("a_scale", c_void_p), ("lda_scale", c_int64), ("w_scale", c_void_p),
                ("ldw_scale", c_int64), ("c_scale", c_void_p), ("ldc_scale", c_int64), ("c_fp8", c_int32)]


_lib.register("i2pc_gemm_fp8", ctypes.c_int, [ctypes.POINTER(GemmFp8Desc), c_void_p])
_lib.register("i2pc_gemm_fp8_kernel_name", ctypes.c_char_p, [ctypes.POINTER(GemmFp8Desc)])
_lib.register("i2pc_quant_fp8", ctypes.c_int, [c_void_p, ctypes.c_int, c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_int64, c_void_p,
                                               c_int64, c_void_p])
_lib.register("i2pc_layernorm_fp8", ctypes.c_int, [c_void_p, c_int64, c_void_p, c_void_p, ctypes.c_float, ctypes.c_int,
                                                   ctypes.c_int, c_void_p, c_int64, c_void_p, c_int64, c_void_p])


class Fp8:
    """An MX fp8 operand: `data` uint8 e4m3fn [..., K] (rows or NHWC pixels) and `scale` uint8
    [..., K / 32] (E8M0 exponent + 127 of each 32-element block; viewed by the kernels as
    uint32 [..., K / 128])."""

    def __init__(self, data, scale):
        self.data, self.scale = data, scale

    @property
    def shape(self):
        return self.data.shape

    def rows(self):
        return self.data.numel() // self.data.shape[-1]

    def view(self, *shape):
        k = self.data.shape[-1]
        return Fp8(self.data.view(*shape), self.scale.view(*shape[:-1], k // 32))

    def dequantize(self):
        """fp32 values (test helper)."""
        torch = _torch()
        v = self.data.view(torch.float8_e4m3fn).float()
        e = (self.scale.to(torch.int32) - 127).repeat_interleave(32, dim=-1)
        return v * exp2i(e)


def empty_fp8(shape, device):
    torch = _torch()
    shape = tuple(shape)
    return Fp8(torch.empty(shape, dtype=torch.uint8, device=device),
               torch.empty(shape[:-1] + (shape[-1] // 32,), dtype=torch.uint8, device=device))


def mx_exponent(amax):
    """E8M0 exponent of blocks with max |v| = amax (torch, any device): the smallest e with
    amax / 2^e <= 448 -- the same rule as csrc/mx.h."""
    torch = _torch()
    m, ex = torch.frexp(amax)                 # amax = m * 2^ex, m in [0.5, 1)
    e = (ex - 1) - 8 + (m > 0.875).to(ex.dtype)
    e = torch.where(amax == 0, torch.full_like(e, -127), e)
    return e.clamp(-127, 127)


def exp2i(e):
    """Exact 2^e (float32) for an integer tensor e in [-127, 127], built from the exponent bits
    (torch's pow / ldexp on the device are not exact)."""
    torch = _torch()
    e = e.to(torch.int32)
    bits = ((e.clamp(min=-126) + 127) << 23).view(torch.float32)
    return torch.where(e >= -126, bits, torch.full_like(bits, 2.0 ** -127))


def round_e4m3(q):
    """Round fp32 values with |q| <= 448 to the e4m3fn grid, nearest, ties to even (what
    v_cvt_pk_fp8_f32 does; torch's own float8 cast does not break ties to even here)."""
    torch = _torch()
    a = q.abs()
    _, ex = torch.frexp(a)                                  # a = m * 2^ex, m in [0.5, 1)
    ulp_exp = torch.clamp(ex - 1, min=-6) - 3               # normal: 2^(E-3); subnormal: 2^-9
    # exact powers of two (exp2i): torch's device pow / ldexp are off by an ulp and move ties
    return torch.round(q * exp2i(-ulp_exp)) * exp2i(ulp_exp)            # round: half to even


def quantize_mx(w):
    """fp32 [..., K] -> Fp8 on w's device (weights: done once at load; K % 32 == 0).
    Same block rule and round-to-nearest-even as the device producers."""
    torch = _torch()
    w = w.float()
    K = w.shape[-1]
    blocks = w.reshape(*w.shape[:-1], K // 32, 32)
    e = mx_exponent(blocks.abs().amax(dim=-1))
    q = round_e4m3((blocks * exp2i(-e).unsqueeze(-1)).clamp(-448.0, 448.0))
    data = q.to(torch.float8_e4m3fn).view(torch.uint8).reshape(w.shape).contiguous()
    return Fp8(data, (e + 127).to(torch.uint8).contiguous())


def quant_fp8(x, relu=False, rows=None, a_map=(0, 0, 0), out=None):
    """bf16 / fp32 device rows [*, K] -> Fp8 [rows, K] (row r reads input row a_map(r))."""
    torch = _torch()
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    R = rows if rows is not None else x2.shape[0]
    if out is None:
        out = empty_fp8(tuple(x.shape) if rows is None else (R, K), x.device)
    with _Timed("k_quant_rows", 0.0, R * K * (x.element_size() + 1.0)):
        _lib.call("i2pc_quant_fp8", _p(x2), int(x.dtype == torch.float32), x2.stride(0), R, K, int(bool(relu)),
                  a_map[0], a_map[1], a_map[2], _p(out.data), out.data.shape[-1], _p(out.scale),
                  out.scale.shape[-1] // 4, _stream())
    return out


def layernorm_fp8(x, gamma, beta, eps, out=None):
    torch = _torch()
    _check(x, torch.float32, "x")
    rows, dim = x.shape
    if out is None:
        out = empty_fp8((rows, dim), x.device)
    with _Timed("k_layernorm_fp8", 0.0, rows * dim * 5.0):
        _lib.call("i2pc_layernorm_fp8", _p(x), x.stride(0), _p(gamma), _p(beta), float(eps), rows, dim,
                  _p(out.data), out.data.shape[-1], _p(out.scale), out.scale.shape[-1] // 4, _stream())
    return out


def gemm_fp8(d: GemmFp8Desc) -> None:
    if profile is None:
        _lib.call("i2pc_gemm_fp8", ctypes.byref(d), _stream())
        return
    label = _lib.load().i2pc_gemm_fp8_kernel_name(ctypes.byref(d)).decode()
    nbytes = gemm_bytes(d.g, esz=1.0 + 1.0 / 32, c_esz=(1.0 + 1.0 / 32) if d.c_fp8 else None)
    with _Timed(label, 2.0 * d.g.m * d.g.n * d.g.k, nbytes):
        _lib.call("i2pc_gemm_fp8", ctypes.byref(d), _stream())


def _fp8_out(d, out, out_fp8, M, N, device, shape=None):
    torch = _torch()
    if out_fp8:
        if out is None:
            out = empty_fp8(shape or (M, N), device)
        d.g.c, d.g.c_f32, d.g.ldc = _p(out.data), 0, out.data.shape[-1]
        d.c_scale, d.ldc_scale, d.c_fp8 = _p(out.scale), out.scale.shape[-1] // 4, 1
    else:
        if out is None:
            out = torch.empty(shape or (M, N), dtype=torch.bfloat16, device=device)
        d.g.c, d.g.c_f32, d.g.ldc = _p(out), int(out.dtype == torch.float32), out.shape[-1]
    return out


def linear_fp8(x: Fp8, w: Fp8, bias=None, act=None, res=None, out=None, out_fp8=False, row_bias=None,
               row_bias_group=1, table=None, table_rows=1):
    """out = act(x @ w.T + bias + row_bias + table) [+ res fp32] on MX fp8 operands.
    x: Fp8 [M, K]; w: Fp8 [N, K]; out bf16 [M, N], fp32 (with an fp32 res), or Fp8 (out_fp8)."""
    torch = _torch()
    M, K = x.rows(), x.shape[-1]
    N = w.shape[0]
    d = GemmFp8Desc()
    d.g.a, d.g.lda, d.g.m, d.g.n, d.g.k = _p(x.data), K, M, N, K
    d.a_scale, d.lda_scale = _p(x.scale), K // 128
    d.g.w, d.g.ldw = _p(w.data), w.shape[-1]
    d.w_scale, d.ldw_scale = _p(w.scale), w.shape[-1] // 128
    d.g.bias = _p(bias)
    d.g.row_bias, d.g.row_bias_group = _p(row_bias), row_bias_group
    d.g.table, d.g.table_rows = _p(table), table_rows
    d.g.act = ACT[act]
    if res is not None:
        d.g.res, d.g.res_f32, d.g.ldr = _p(res), int(res.dtype == torch.float32), res.stride(0)
    if out is None and res is not None and res.dtype == torch.float32:
        out = res
    out = _fp8_out(d, out, out_fp8, M, N, x.data.device)
    gemm_fp8(d)
    return out


def conv2d_fp8(x: Fp8, w: Fp8, bias=None, k=3, stride=1, pad=1, relu_in=False, act=None, res=None, res2=None,
               out=None, out_fp8=False):
    """NHWC implicit-GEMM conv on MX fp8: x Fp8 [B, H, W, C] (C % 128 == 0), w Fp8 [Co, k*k*C]
    packed (ky, kx, ci); out bf16 NHWC (+ bf16 residuals) or Fp8 NHWC (out_fp8)."""
    B, H, W, C = x.shape
    Co = w.shape[0]
    OH = (H + 2 * pad - k) // stride + 1
    OW = (W + 2 * pad - k) // stride + 1
    d = GemmFp8Desc()
    d.g.a, d.g.lda, d.g.m, d.g.n, d.g.k = _p(x.data), C, B * OH * OW, Co, k * k * C
    d.a_scale, d.lda_scale = _p(x.scale), C // 128
    if not (k == 1 and stride == 1 and pad == 0):
        d.g.conv, d.g.conv_batch, d.g.conv_h, d.g.conv_w, d.g.conv_c = 1, B, H, W, C
        d.g.conv_oh, d.g.conv_ow, d.g.conv_k, d.g.conv_stride, d.g.conv_pad = OH, OW, k, stride, pad
    d.g.conv_relu_in = int(relu_in)
    d.g.w, d.g.ldw = _p(w.data), w.shape[-1]
    d.w_scale, d.ldw_scale = _p(w.scale), w.shape[-1] // 128
    d.g.bias = _p(bias)
    d.g.act = ACT[act]
    if res is not None:
        d.g.res, d.g.res_f32, d.g.ldr = _p(res), 0, Co
    if res2 is not None:
        d.g.res2, d.g.ldr2 = _p(res2), Co
    out = _fp8_out(d, out, out_fp8, B * OH * OW, Co, x.data.device, shape=(B, OH, OW, Co))
    gemm_fp8(d)
    return out


# ------------------------------------------------------------------ BiT stem (DPT-Hybrid)
_lib.register("i2pc_bit_stem_im2col", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     c_void_p, c_void_p])
_lib.register("i2pc_groupnorm_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int])
_lib.register("i2pc_groupnorm_stats", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_float, c_void_p, c_void_p, ctypes.c_size_t, c_void_p])
_lib.register("i2pc_groupnorm_apply", ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                     c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_int, c_void_p, c_void_p])
_lib.register("i2pc_maxpool3s2", ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p])


def same_pad(size: int, k: int, s: int):
    """DynamicPad2d (modeling_bit.py:171-196): (output size, top/left pad) of TF "SAME" padding."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return out, total // 2


def stem_im2col(pixels, ksize=7, stride=2, k_pitch=None, out=None):
    """fp32 NCHW [B, 3, H, W] -> bf16 [B * OH * OW, k_pitch] rows of the stem conv (SAME pad)."""
    torch = _torch()
    _check(pixels, torch.float32, "pixels")
    assert stride == 2
    B, _, H, W = pixels.shape
    OH, pt = same_pad(H, ksize, stride)
    OW, pl = same_pad(W, ksize, stride)
    kp = k_pitch or (ksize * ksize * 3 + 63) // 64 * 64
    if out is None:
        out = torch.empty((B * OH * OW, kp), dtype=torch.bfloat16, device=pixels.device)
    with _Timed("k_stem_im2col", 0.0, pixels.numel() * 4.0 + out.numel() * 2.0):
        _lib.call("i2pc_bit_stem_im2col", _p(pixels), B, H, W, OH, OW, pt, pl, ksize, kp, _p(out), _stream())
    return out, (OH, OW)


def group_norm(x, gamma, beta, groups=32, eps=1e-5, relu=False, shortcut=None, acc=None, out=None):
    """act(GroupNorm(x) + shortcut) on NHWC bf16; shortcut = None | bf16 tensor | (tensor, gamma, beta)
    (normalised with its own statistics).  Returns bf16 NHWC."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    hw = H * W

    def stats(t):
        a = torch.empty((B, groups, 2), dtype=torch.float32, device=t.device)
        nb = _lib.load().i2pc_groupnorm_workspace_bytes(B, hw, groups)
        ws = torch.empty(max(nb, 4), dtype=torch.uint8, device=t.device)
        with _Timed("k_gn_stats", 0.0, t.numel() * 2.0):
            _lib.call("i2pc_groupnorm_stats", _p(t), B, hw, C, groups, float(eps), _p(a), _p(ws), nb, _stream())
        return a

    a = acc if acc is not None else stats(x)
    r = ra = rg = rb = None
    if isinstance(shortcut, tuple):
        r, rg, rb = shortcut
        ra = stats(r)
    elif shortcut is not None:
        r = shortcut
    if out is None:
        out = torch.empty_like(x)
    nbytes = x.numel() * 4.0 + (r.numel() * 2.0 if r is not None else 0.0)
    with _Timed("k_gn_apply", 0.0, nbytes):
        _lib.call("i2pc_groupnorm_apply", _p(x), _p(a), _p(gamma), _p(beta), _p(r), _p(ra), _p(rg), _p(rb), B, hw, C,
                  groups, int(bool(relu)), _p(out), _stream())
    return out


def maxpool3s2(x, out=None):
    """BitMaxPool2d(3, 2, dynamic SAME padding with 0) on NHWC bf16."""
    torch = _torch()
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    OH, pt = same_pad(H, 3, 2)
    OW, pl = same_pad(W, 3, 2)
    if out is None:
        out = torch.empty((B, OH, OW, C), dtype=torch.bfloat16, device=x.device)
    with _Timed("k_maxpool", 0.0, x.numel() * 2.0 + out.numel() * 2.0):
        _lib.call("i2pc_maxpool3s2", _p(x), B, H, W, C, OH, OW, pt, pl, _p(out), _stream())
    return out

"""CPU-side checks of the C ABI: the library builds/loads and exports every declared symbol."""
import ctypes
import os

import pytest

from image_to_pointcloud_amd import _lib


def test_header_declares_core_entry_points():
    syms = _lib.declared_symbols()
    for s in ("i2pc_unproject", "i2pc_unproject_workspace_bytes", "i2pc_last_error", "i2pc_abi_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built (run python -m image_to_pointcloud_amd.build)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in _lib.declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_no_gpu_calls_needed_for_metadata():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built")
    lib = _lib.load()
    assert lib.i2pc_abi_version() >= 1
    assert lib.i2pc_unproject_workspace_bytes(32, 1024, 1024, 0) > 0
    assert lib.i2pc_unproject_workspace_bytes(0, 1024, 1024, 0) == 0
    assert lib.i2pc_last_error() is not None


def test_missing_device_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("device present")
    from image_to_pointcloud_amd import geometry
    import numpy as np
    with pytest.raises(_lib.I2PCError):
        geometry.depth_to_point_cloud(np.zeros((4, 4, 3), np.uint8), np.zeros((4, 4), np.float32))


def test_kernel_selection_knobs_are_per_thread():
    """i2pc_gemm_set_engine / i2pc_set_tuning change the kernels of the CALLING thread only
    (include/i2pc.h: re-entrant across threads), checked through i2pc_gemm_kernel_name (no
    device work)."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built")
    import threading
    from image_to_pointcloud_amd import ops
    d = ops.GemmDesc()
    d.m, d.n, d.k, d.lda, d.ldw, d.ldc = 18464, 3072, 1024, 1024, 1024, 3072
    d.a = d.w = d.c = 16
    default = ops.gemm_kernel_label(d)
    seen = {}
    ready, done = threading.Event(), threading.Event()

    def other():
        ready.wait(10)
        seen["other"] = ops.gemm_kernel_label(d)      # while the main thread has engine 1 set
        done.set()

    t = threading.Thread(target=other)
    t.start()
    try:
        ops.set_gemm_engine(1)                          # tile kernel only, this thread
        seen["mine"] = ops.gemm_kernel_label(d)
        ready.set()
        done.wait(10)
    finally:
        ops.set_gemm_engine(0)
        t.join(10)
    assert seen["other"] == default
    assert seen["mine"] != default and seen["mine"].startswith("k_gemm<")
    assert ops.gemm_kernel_label(d) == default


def test_ln_fold_producer_plans():
    """The LN-fold producer plans (i2pc_gemm_kernel_name, no device work): 64-column partials need
    wave tiles of whole 64-column chunks, so Depth-Anything-V2-Small's 384-wide attention-out / FC2
    (M = 43840) falls back to 128 x 128 tiles with them and keeps its 384 x 192 tiles with 32-column
    partials (ln_chunk = 32); ln_chunk other than 0 / 32 / 64 is rejected."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built")
    from image_to_pointcloud_amd import ops

    def label(chunk):
        d = ops.GemmDesc()
        d.m, d.n, d.k, d.lda, d.ldw, d.ldc = 43840, 384, 1536, 1536, 1536, 384
        d.a = d.w = d.c = d.res = d.ln_part = d.c_bf16 = 16
        d.res_f32, d.ldr, d.c_f32, d.ldc_bf16, d.ln_chunk = 1, 384, 1, 384, chunk
        return ops.gemm_kernel_label(d)
    assert label(0).startswith("k_gemm<128, 128") and label(64) == label(0)
    assert label(32).startswith("k_gemm<384, 192")
    assert label(48) == "invalid"


def test_tuning_knob_names():
    """Every knob include/i2pc.h documents (ops.TUNING_KNOBS) is accepted by i2pc_set_tuning
    (host-side state only, no device work), the header and the unknown-knob error message list the
    same names, and an unknown name is an error (I2PCError)."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built")
    from image_to_pointcloud_amd import ops
    defaults = {"gemm_tail": 1, "gemm_bn128": 1, "gemm_splitk": 1, "gemm_split_tile": 0, "gemm_tile192": 1, "gemm_lnp_p": 0, "gemm_lnp_stream": 0, "conv_halo": 3, "gelu_tanh": 1, "gemm_resq": 2, "gemm_simple_epi": 1, "gemm_tail160": 1,
                "gemm_stagger": 1,
                "unp_rows": 1, "unp_nt": 1, "unp_rpt": 8, "sel_windows": 1, "sel_parts": 0, "sel_rows": 16,
                "sel_lband": -1, "sel_scratch": 0, "attn_lazy": 1, "attn_scalar": 1, "attn_rb": 1, "ln_f2": 1, "ln_apply_gs": 0, "resize_rows": 1}
    assert set(defaults) == set(ops.TUNING_KNOBS)
    header = open(os.path.join(os.path.dirname(__file__), "..", "include", "i2pc.h")).read()
    for name in ops.TUNING_KNOBS:
        assert f'"{name}"' in header, name
    for name, v in defaults.items():
        ops.set_tuning(name, v)
    with pytest.raises(_lib.I2PCError) as ei:
        ops.set_tuning("no_such_knob", 1)
    msg = str(ei.value)
    for name in ops.TUNING_KNOBS:
        assert name in msg, name

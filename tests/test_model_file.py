"""The prepared-network file of the native executor (model_file.py, csrc/model.cpp) on the CPU:
written from a Depth-Anything model built on the host, read back by Python and by libi2pc.so's
host-only i2pc_model_file_info; the header describes the network and input size, and every tensor
the executor's forward reads is present with the kernels' layout."""
import os

import pytest

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def da_file(tmp_path_factory):
    from image_to_pointcloud_amd import _lib, model_file
    from image_to_pointcloud_amd.depth_anything import DA_TINY, DepthAnythingModel, synthetic_state_dict
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libi2pc.so not built")
    m = DepthAnythingModel(DA_TINY, synthetic_state_dict(DA_TINY, 0), "cpu")
    path = str(tmp_path_factory.mktemp("net") / "da_tiny.i2pcnet")
    model_file.export_depth_anything(m, path, 100, 150)
    return m, path


def test_header_round_trip(da_file):
    from image_to_pointcloud_amd import model_file as mf
    from image_to_pointcloud_amd.preprocess import DEPTH_ANYTHING_PROCESSOR, output_size
    m, path = da_file
    h = mf.read_header(path)
    ints, floats, n = mf.file_info(path)           # the C reader
    assert ints == list(h["ints"]) and n == len(h["tensors"]) == ints[mf.I_NTENSORS]
    oh, ow = output_size(100, 150, DEPTH_ANYTHING_PROCESSOR)
    assert (ints[mf.I_IN_H], ints[mf.I_IN_W], ints[mf.I_OUT_H], ints[mf.I_OUT_W]) == (100, 150, oh, ow)
    assert (ints[mf.I_GH], ints[mf.I_GW]) == (oh // 14, ow // 14)
    assert ints[mf.I_FAMILY] == mf.FAMILY_DEPTH_ANYTHING and ints[mf.I_LAYERS] == m.spec.layers
    assert list(ints[mf.I_OUT0:mf.I_OUT0 + 4]) == list(m.spec.out_indices)
    assert list(ints[mf.I_FAC0:mf.I_FAC0 + 4]) == [4, 2, 1, -2]
    assert abs(floats[mf.F_EPS] - m.spec.eps) < 1e-12 and floats[mf.F_B_H3] == pytest.approx(m.b_h3)
    t = h["tensors"]
    assert t["pos.table"]["shape"] == ((oh // 14) * (ow // 14), m.spec.hidden)
    assert t["L0.w_qkv_f"]["dtype"] == 1 and t["L0.s_qkv"]["dtype"] == 0
    assert all(e["offset"] % 256 == 0 for e in t.values())


def test_tensor_bytes_are_the_models(da_file):
    """Spot-check that the data region holds the model's own prepared tensors."""
    from image_to_pointcloud_amd import model_file as mf
    m, path = da_file
    h = mf.read_header(path)
    raw = open(path, "rb").read()
    data0 = 8 + 128 + 64 + mf.ENTRY.size * len(h["tensors"])
    for name, ref in (("pe.w", m.w_pe), ("L1.s_1", m.layers[1]["s_1"]), ("H.w3", m.w_h3)):
        e = h["tensors"][name]
        got = raw[data0 + e["offset"]:data0 + e["offset"] + e["nbytes"]]
        want = ref.contiguous().view(torch.int16 if ref.dtype == torch.bfloat16 else torch.int32).numpy().tobytes()
        assert got == want, name


def test_bad_file_is_an_error(tmp_path):
    from image_to_pointcloud_amd import _lib, model_file as mf
    p = tmp_path / "junk"
    p.write_bytes(b"not a network")
    with pytest.raises(_lib.I2PCError, match="not an i2pc network file"):
        mf.file_info(str(p))


def _patched(path, tmp_path, fn, tag):
    """A copy of the file at `path` with its tensor table / header edited by fn(raw bytearray, header)."""
    from image_to_pointcloud_amd import model_file as mf
    raw = bytearray(open(path, "rb").read())
    fn(raw, mf.read_header(path))
    out = tmp_path / f"{tag}.i2pcnet"
    out.write_bytes(bytes(raw))
    return str(out)


def _entry_pos(h, name):
    from image_to_pointcloud_amd import model_file as mf
    return 8 + 128 + 64 + mf.ENTRY.size * list(h["tensors"]).index(name)


@pytest.mark.parametrize("case", ["nbytes", "dtype", "missing", "out_repeat", "out_range"])
def test_mismatched_file_is_rejected(da_file, tmp_path, case):
    """the reader checks every tensor the executor's forward reads (name, dtype, byte
    count implied by the header) and the out indices, so a mismatched file fails at create / info time
    instead of reading past a tensor on the GPU."""
    import struct
    from image_to_pointcloud_amd import _lib, model_file as mf
    _, path = da_file

    def edit(raw, h):
        if case in ("nbytes", "dtype", "missing"):
            pos = _entry_pos(h, "L1.w_o")
            name, dt, nd, d0, d1, d2, d3, off, nb = mf.ENTRY.unpack(bytes(raw[pos:pos + mf.ENTRY.size]))
            if case == "nbytes":
                nb, d0 = nb // 2, d0 // 2            # a truncated tensor, consistent with itself
            elif case == "dtype":
                dt = 0
            else:
                name = b"L1.w_o_renamed"
            raw[pos:pos + mf.ENTRY.size] = mf.ENTRY.pack(name, dt, nd, d0, d1, d2, d3, off, nb)
        else:
            ints = list(h["ints"])
            if case == "out_repeat":
                ints[mf.I_OUT0 + 3] = ints[mf.I_OUT0 + 2]
            else:
                ints[mf.I_OUT0] = ints[mf.I_LAYERS] + 1
            raw[8:8 + 128] = struct.pack("<32i", *ints)
    bad = _patched(path, tmp_path, edit, case)
    msg = {"nbytes": "header implies", "dtype": "header implies", "missing": "missing", "out_repeat": "repeat",
           "out_range": "outside"}[case]
    with pytest.raises(_lib.I2PCError, match=msg):
        mf.file_info(bad)

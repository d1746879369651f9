"""CPU: the C-ABI library loads, exports every function include/ore.h declares, and its host-only
geometry (shape inference, padding resolution, error reporting) matches the oracle's
restatement of the reference.  No kernel is launched here."""
import ctypes
import itertools
import os
import re

import numpy as np
import pytest

import oracle
import ore
from ore import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(HERE), "include", "ore.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ore_\w+)\s*\(", src)))


def test_library_exports_header():
    L = ore.load()
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), f"libore.so does not export {n}"
    assert sorted(_lib.EXPORTED) == names
    assert L.ore_abi_version() == 1


def test_library_is_gfx950():
    """The code object embedded in libore.so targets gfx950 only (no other offload arch)."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert other not in data


CASES = list(itertools.product([7, 14, 15, 28, 54, 224], [1, 3, 5, 7], [1, 2, 3], ["SAME_UPPER", "SAME_LOWER", "VALID"]))


@pytest.mark.parametrize("H,k,s,auto_pad", CASES)
def test_conv_shape_matches_oracle(H, k, s, auto_pad):
    W = H + 1
    try:
        p_ref, ho, wo = oracle.resolve_window(auto_pad, None, H, W, k, k, s, s)
    except oracle.OracleError:
        with pytest.raises(ore.OreError):
            ore.conv_out_shape((2, 3, H, W), (4, 3, k, k), auto_pad=auto_pad, strides=(s, s))
        return
    yd, p = ore.conv_out_shape((2, 3, H, W), (4, 3, k, k), auto_pad=auto_pad, strides=(s, s))
    assert yd == (2, 4, ho, wo)
    assert p == tuple(p_ref)


@pytest.mark.parametrize("pads", [[0, 0, 0, 0], [1, 1, 1, 1], [0, 0, 1, 1], [2, 1, 0, 3]])
def test_notset_shapes(pads):
    yd, p = ore.conv_out_shape((1, 2, 10, 9), (3, 2, 3, 3), auto_pad="VALID", pads=pads, strides=(2, 2))
    eff = "NOTSET" if any(pads) else "VALID"  # positive pads force NOTSET for Conv (:169-173)
    p_ref, ho, wo = oracle.resolve_window(eff, pads, 10, 9, 3, 3, 2, 2)
    assert yd[2:] == (ho, wo) and p == tuple(p_ref)
    # MaxPool honours pads only under an explicit NOTSET (max_pool_op.rs:88, 248)
    yv, _ = ore.pool_out_shape((1, 2, 10, 9), (3, 3), (2, 2), auto_pad="VALID", pads=pads)
    _, hv, wv = oracle.resolve_window("VALID", None, 10, 9, 3, 3, 2, 2)
    assert yv[2:] == (hv, wv)
    yn, pn = ore.pool_out_shape((1, 2, 10, 9), (3, 3), (2, 2), auto_pad="NOTSET", pads=pads)
    assert yn[2:] == (ho, wo) and pn == tuple(p_ref)


def test_squeezenet_pool_geometry():
    assert ore.pool_out_shape((1, 96, 109, 109), (3, 3), (2, 2), "NOTSET", [0, 0, 0, 0])[0] == (1, 96, 54, 54)
    assert ore.pool_out_shape((1, 256, 54, 54), (3, 3), (2, 2), "NOTSET", [0, 0, 1, 1])[0] == (1, 256, 27, 27)
    assert ore.pool_out_shape((1, 512, 27, 27), (3, 3), (2, 2), "NOTSET", [0, 0, 0, 0])[0] == (1, 512, 13, 13)


def test_errors_without_gpu():
    with pytest.raises(ore.OreError, match="group"):
        ore.conv_out_shape((1, 3, 8, 8), (4, 3, 3, 3), strides=(1, 1), group=3)
    with pytest.raises(ore.OreError, match="dilation"):
        ore.conv_out_shape((1, 3, 8, 8), (4, 3, 3, 3), strides=(1, 1), dilations=(2, 2))
    with pytest.raises(ore.OreError):
        ore.conv_out_shape((1, 3, 8, 8), (4, 3, 3, 3), auto_pad="NOTSET", pads=None, strides=(1, 1))
    with pytest.raises(ore.OreError):
        ore.pool_out_shape((1, 3, 2, 2), (3, 3), (1, 1), "VALID")
    L = ore.load()
    assert L.ore_model_step_count(None) == 0
    assert L.ore_sync(None) == 1 and b"null" in L.ore_last_error(None)


def test_reshape_host_only():
    t = _lib.Tensor()
    t.data = 0x1000
    t.ndim = 4
    for i, d in enumerate((4, 2, 2, 3)):
        t.dims[i] = d
    out = _lib.Tensor()
    shape = (ctypes.c_int64 * 2)(16, 3)
    assert ore.load().ore_reshape(ctypes.byref(t), shape, 2, ctypes.byref(out)) == 0
    assert (out.dims[0], out.dims[1], out.data) == (16, 3, 0x1000)
    bad = (ctypes.c_int64 * 2)(5, 3)
    assert ore.load().ore_reshape(ctypes.byref(t), bad, 2, ctypes.byref(out)) == 1
    three = (ctypes.c_int64 * 3)(4, 2, 6)
    assert ore.load().ore_reshape(ctypes.byref(t), three, 3, ctypes.byref(out)) == 2


def test_ctx_create_reports_missing_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    st = ore.load().ore_ctx_create(0, ctypes.byref(h))
    assert st == 3  # ORE_ERR_HIP, no crash
    assert np.isscalar(st)

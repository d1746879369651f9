"""ctypes binding of the C oracle (TEST INFRASTRUCTURE ONLY — see package docstring)."""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

AUTO_PAD = {"NOTSET": 0, "NOT_SET": 0, "SAME_UPPER": 1, "SAME_LOWER": 2, "VALID": 3}

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, f32, vp, ci = ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_int
        L.oref_ndarray_sum.restype = f32
        L.oref_ndarray_sum.argtypes = [_f32p, i64]
        L.oref_resolve_window.restype = ci
        L.oref_resolve_window.argtypes = [ci, _i64p, ci, i64, i64, i64, i64, i64, i64, _i64p, _i64p, _i64p]
        L.oref_conv2d.restype = ci
        L.oref_conv2d.argtypes = [_f32p, i64, i64, i64, i64, _f32p, i64, i64, i64, _f32p, _i64p, i64, i64,
                                  i64, i64, _f32p, ci]
        L.oref_maxpool2d.restype = ci
        L.oref_maxpool2d.argtypes = [_f32p, i64, i64, i64, i64, i64, i64, _i64p, i64, i64, i64, i64, _f32p, ci]
        L.oref_relu.argtypes = [_f32p, i64, _f32p]
        L.oref_add_bcast.restype = ci
        L.oref_add_bcast.argtypes = [_f32p, _i64p, ci, _f32p, _i64p, ci, _f32p]
        L.oref_softmax_rows.argtypes = [_f32p, i64, i64, _f32p]
        L.oref_matmul.argtypes = [_f32p, _f32p, i64, i64, i64, _f32p]
        L.oref_gap.argtypes = [_f32p, i64, i64, i64, _f32p]
        L.oref_concat2.restype = ci
        L.oref_concat2.argtypes = [_f32p, _i64p, _f32p, _i64p, ci, _f32p]
        L.oref_model_load.restype = vp
        L.oref_model_load.argtypes = [ctypes.c_char_p, i64]
        L.oref_model_free.argtypes = [vp]
        L.oref_model_run.restype = ci
        L.oref_model_run.argtypes = [vp, _f32p, i64, _f32p, i64, ci]
        L.oref_model_out_elems.restype = i64
        L.oref_model_out_elems.argtypes = [vp]
        L.oref_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def _ip(a: np.ndarray):
    return a.ctypes.data_as(_i64p)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleError(RuntimeError):
    pass


def _check(rc: int):
    if rc != 0:
        raise OracleError(lib().oref_last_error().decode())


def ndarray_sum(x) -> np.float32:
    x = _f32(x)
    return np.float32(lib().oref_ndarray_sum(_fp(x), x.size))


def resolve_window(auto_pad: str, pads: Optional[Sequence[int]], H, W, kh, kw, sh, sw):
    """-> (pads_tlbr, Ho, Wo), following get_padding_size / the H' formulas of the reference."""
    pa = np.asarray(pads if pads is not None else [], dtype=np.int64)
    out = np.zeros(4, dtype=np.int64)
    ho, wo = ctypes.c_int64(), ctypes.c_int64()
    _check(lib().oref_resolve_window(AUTO_PAD[auto_pad], _ip(pa) if pa.size else None, pa.size,
                                     H, W, kh, kw, sh, sw, _ip(out), ctypes.byref(ho), ctypes.byref(wo)))
    return out, ho.value, wo.value


def conv2d(x, w, bias=None, auto_pad="NOTSET", pads=(0, 0, 0, 0), strides=(1, 1), faithful=False):
    """ONNX Conv with the reference's semantics; pads in ONNX order [hb, wb, he, we]."""
    x, w = _f32(x), _f32(w)
    N, C, H, W = x.shape
    M, Cw, kh, kw = w.shape
    assert Cw == C
    if auto_pad in ("NOTSET", "NOT_SET", "VALID") and pads is not None and any(p > 0 for p in pads):
        auto_pad = "NOTSET"
    p, Ho, Wo = resolve_window(auto_pad, pads, H, W, kh, kw, strides[0], strides[1])
    y = np.empty((N, M, Ho, Wo), dtype=np.float32)
    b = _f32(bias) if bias is not None else None
    _check(lib().oref_conv2d(_fp(x), N, C, H, W, _fp(w), M, kh, kw, _fp(b) if b is not None else None,
                             _ip(p), strides[0], strides[1], Ho, Wo, _fp(y), int(faithful)))
    return y


def maxpool2d(x, kernel, strides, auto_pad="VALID", pads=None):
    x = _f32(x)
    N, C, H, W = x.shape
    p, Ho, Wo = resolve_window(auto_pad, pads, H, W, kernel[0], kernel[1], strides[0], strides[1])
    y = np.empty((N, C, Ho, Wo), dtype=np.float32)
    _check(lib().oref_maxpool2d(_fp(x), N, C, H, W, kernel[0], kernel[1], _ip(p), strides[0], strides[1],
                                Ho, Wo, _fp(y), 0))
    return y


def relu(x):
    x = _f32(x)
    y = np.empty_like(x)
    lib().oref_relu(_fp(x), x.size, _fp(y))
    return y


def add(a, b):
    a, b = _f32(a), _f32(b)
    ad = np.asarray(a.shape, dtype=np.int64)
    bd = np.asarray(b.shape, dtype=np.int64)
    y = np.empty_like(a)
    _check(lib().oref_add_bcast(_fp(a), _ip(ad), a.ndim, _fp(b), _ip(bd), b.ndim, _fp(y)))
    return y


def softmax(x):
    """softmax_wrapper: flatten to (N, C*H*W), softmax over axis 1."""
    x = _f32(x)
    rows = x.shape[0]
    D = x.size // rows
    y = np.empty((rows, D), dtype=np.float32)
    lib().oref_softmax_rows(_fp(x), rows, D, _fp(y))
    return y


def matmul(a, b):
    a, b = _f32(a), _f32(b)
    y = np.empty((a.shape[0], b.shape[1]), dtype=np.float32)
    lib().oref_matmul(_fp(a), _fp(b), a.shape[0], a.shape[1], b.shape[1], _fp(y))
    return y


def gap(x):
    x = _f32(x)
    N, C, H, W = x.shape
    y = np.empty((N, C, 1, 1), dtype=np.float32)
    lib().oref_gap(_fp(x), N, C, H * W, _fp(y))
    return y


def concat(a, b, axis=1):
    a, b = _f32(a), _f32(b)
    shape = list(a.shape)
    shape[axis] += b.shape[axis]
    y = np.empty(shape, dtype=np.float32)
    _check(lib().oref_concat2(_fp(a), _ip(np.asarray(a.shape, dtype=np.int64)), _fp(b),
                              _ip(np.asarray(b.shape, dtype=np.int64)), axis, _fp(y)))
    return y


class Model:
    """Whole-graph restatement of inference() over an ONNX ModelProto byte string."""

    def __init__(self, onnx_bytes: bytes):
        self._bytes = onnx_bytes
        h = lib().oref_model_load(onnx_bytes, len(onnx_bytes))
        if not h:
            raise OracleError(lib().oref_last_error().decode())
        self._h = h

    def run(self, x, out_elems_per_image: int, faithful: bool = False) -> np.ndarray:
        x = _f32(x)
        n = x.shape[0]
        out = np.empty(n * out_elems_per_image, dtype=np.float32)
        _check(lib().oref_model_run(self._h, _fp(x), n, _fp(out), out.size, int(faithful)))
        got = lib().oref_model_out_elems(self._h)
        return out[: n * got].reshape(n, got)

    def close(self):
        if self._h:
            lib().oref_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

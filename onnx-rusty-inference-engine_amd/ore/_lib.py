"""ctypes loader for the in-tree C-ABI library `lib/libore.so` (include/ore.h).

The library is the product: there is no CPU fallback.  If it is missing the import of any
entry point raises, so a GPU run never silently computes through something else.
"""
from __future__ import annotations

import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ORE_LIB selects another build of the same library (tools/build_exp.sh A/B variants)
LIB_PATH = os.environ.get("ORE_LIB") or os.path.join(PKG_ROOT, "lib", "libore.so")

ORE_OK = 0
STATUS_NAMES = {0: "ORE_OK", 1: "ORE_ERR_INVALID", 2: "ORE_ERR_UNSUPPORTED", 3: "ORE_ERR_HIP",
                4: "ORE_ERR_OOM", 5: "ORE_ERR_PARSE"}

# ore_model_set_fusion flags (include/ore.h)
FUSE_CONV_RELU, FUSE_CONCAT, FUSE_ALIAS, KEEP_VALUES, FUSE_CONV_POOL = 1, 2, 4, 8, 32
FUSE_FIRE, FUSE_CONCAT_POOL, FUSE_FIRE_POOL, FUSE_FIRST_SQUEEZE, FUSE_POOL_SQUEEZE = 64, 128, 256, 512, 1024
FUSE_CONV_GAP, FUSE_POOL_EXPAND = 4096, 8192
FUSE_EAGER = 2048  # tests: every eligible fusion regardless of the size heuristics
FUSE_ALL = 14311
LOAD_F16 = 1  # ore_model_load_ex flag: the fp16 variant
LOAD_NO_WINOGRAD = 4  # ore_model_load_ex flag: 3x3 stride-1 convs on the direct kernels only
LOAD_RETIRED_MASK = 10  # ABI 1's LOAD_X3 / LOAD_X3_ALL: rejected (ORE_ERR_UNSUPPORTED) since ABI 2
ABI_VERSION = 2  # ORE_ABI_VERSION this binding was written against
CONV_ALGO_DIRECT, CONV_ALGO_WINOGRAD = 0, 1  # ore_ctx_set_conv_algo (per-op ore_conv2d_f32)
PAD = {"NOTSET": 0, "NOT_SET": 0, "SAME_UPPER": 1, "SAME_LOWER": 2, "VALID": 3}

# every symbol include/ore.h declares (checked by tests/test_abi.py on CPU)
EXPORTED = [
    "ore_abi_version", "ore_ctx_create", "ore_ctx_destroy", "ore_ctx_set_stream", "ore_ctx_get_stream",
    "ore_ctx_set_conv_algo", "ore_ctx_set_conv_tile", "ore_ctx_set_pool_variant", "ore_sync", "ore_last_error", "ore_malloc", "ore_free", "ore_upload", "ore_download",
    "ore_conv_out_shape", "ore_pool_out_shape", "ore_conv2d_f32", "ore_maxpool2d_f32", "ore_relu_f32",
    "ore_add_f32", "ore_softmax_f32", "ore_matmul_f32", "ore_gap_f32", "ore_concat_f32", "ore_dropout_f32",
    "ore_reshape", "ore_model_parse", "ore_model_load", "ore_model_load_ex", "ore_model_destroy", "ore_model_set_fusion", "ore_model_input_dims",
    "ore_model_output_elems", "ore_model_run", "ore_model_read_value", "ore_model_autotune",
    "ore_model_step_tile", "ore_model_set_step_tile", "ore_model_step_mfma_flops", "ore_model_set_streams",
    "ore_model_graph_capture", "ore_model_graph_launch", "ore_model_enable_timing",
    "ore_model_step_count", "ore_model_step_info", "ore_model_step_times", "ore_model_run_batch",
]


class OreError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Tensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("ndim", ctypes.c_int32), ("dims", ctypes.c_int64 * 4),
                ("nstride", ctypes.c_int64)]


class ConvAttrs(ctypes.Structure):
    _fields_ = [("auto_pad", ctypes.c_int32), ("n_pads", ctypes.c_int32), ("pads", ctypes.c_int64 * 4),
                ("strides", ctypes.c_int64 * 2), ("dilations", ctypes.c_int64 * 2), ("group", ctypes.c_int64),
                ("fuse_relu", ctypes.c_int32)]


class PoolAttrs(ctypes.Structure):
    _fields_ = [("auto_pad", ctypes.c_int32), ("n_pads", ctypes.c_int32), ("pads", ctypes.c_int64 * 4),
                ("kernel", ctypes.c_int64 * 2), ("strides", ctypes.c_int64 * 2)]


_lib = None


def load():
    """Load libore.so (raises if it has not been built: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built; run `make -C {PKG_ROOT}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, cs = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_char_p
    T = ctypes.POINTER(Tensor)
    I64P = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "ore_abi_version": (i32, []),
        "ore_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "ore_ctx_destroy": (i32, [vp]),
        "ore_ctx_set_stream": (i32, [vp, vp]),
        "ore_ctx_get_stream": (vp, [vp]),
        "ore_ctx_set_conv_algo": (i32, [vp, i32]),
        "ore_ctx_set_conv_tile": (i32, [vp, i32]),
        "ore_ctx_set_pool_variant": (i32, [vp, i32]),
        "ore_sync": (i32, [vp]),
        "ore_last_error": (cs, [vp]),
        "ore_malloc": (i32, [vp, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "ore_free": (i32, [vp, vp]),
        "ore_upload": (i32, [vp, vp, vp, ctypes.c_size_t]),
        "ore_download": (i32, [vp, vp, vp, ctypes.c_size_t]),
        "ore_conv_out_shape": (i32, [I64P, I64P, ctypes.POINTER(ConvAttrs), I64P, I64P]),
        "ore_pool_out_shape": (i32, [I64P, ctypes.POINTER(PoolAttrs), I64P, I64P]),
        "ore_conv2d_f32": (i32, [vp, T, T, T, ctypes.POINTER(ConvAttrs), T]),
        "ore_maxpool2d_f32": (i32, [vp, T, ctypes.POINTER(PoolAttrs), T]),
        "ore_relu_f32": (i32, [vp, T, T]),
        "ore_add_f32": (i32, [vp, T, T, T]),
        "ore_softmax_f32": (i32, [vp, T, T]),
        "ore_matmul_f32": (i32, [vp, T, T, T]),
        "ore_gap_f32": (i32, [vp, T, T]),
        "ore_concat_f32": (i32, [vp, T, T, i64, T]),
        "ore_dropout_f32": (i32, [vp, T, T]),
        "ore_reshape": (i32, [T, I64P, i32, T]),
        "ore_model_parse": (i32, [ctypes.c_char_p, ctypes.c_size_t]),
        "ore_model_load": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, i64, ctypes.POINTER(vp)]),
        "ore_model_load_ex": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, i64, i32, ctypes.POINTER(vp)]),
        "ore_model_destroy": (i32, [vp]),
        "ore_model_set_fusion": (i32, [vp, i32]),
        "ore_model_input_dims": (i32, [vp, I64P]),
        "ore_model_output_elems": (i32, [vp, I64P]),
        "ore_model_run": (i32, [vp, vp, i64, vp]),
        "ore_model_read_value": (i32, [vp, cs, vp, ctypes.c_size_t, I64P, ctypes.POINTER(i32)]),
        "ore_model_enable_timing": (i32, [vp, i32]),
        "ore_model_set_streams": (i32, [vp, i32]),
        "ore_model_autotune": (i32, [vp, vp, i64, vp, i32]),
        "ore_model_step_tile": (i32, [vp, i32]),
        "ore_model_set_step_tile": (i32, [vp, i32, i32]),
        "ore_model_step_mfma_flops": (i32, [vp, i32, ctypes.POINTER(ctypes.c_double)]),
        "ore_model_graph_capture": (i32, [vp, vp, i64, vp]),
        "ore_model_graph_launch": (i32, [vp]),
        "ore_model_step_count": (i32, [vp]),
        "ore_model_run_batch": (i64, [vp]),
        "ore_model_step_info": (i32, [vp, i32, ctypes.POINTER(cs), ctypes.POINTER(cs),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
        "ore_model_step_times": (i32, [vp, ctypes.POINTER(ctypes.c_float), i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, ctx=None):
    if status != ORE_OK:
        msg = load().ore_last_error(ctx)
        raise OreError(status, msg.decode() if msg else "")

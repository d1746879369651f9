"""Host-side mirror of the reference's operator interface over the C ABI (include/ore.h).

Names follow the reference: one function per `node_inference` arm
(/root/reference/src/inference_engine/model_inference.rs:137-161) —
`convolution`, `max_pool`, `relu`, `add`, `softmax`, `mul`, `global_average_pool`,
`concatenation`, `drop_out`, `reshape` — and `inference()` for the graph walker
(model_inference.rs:29-120).  Tensors are torch CUDA tensors (PyTorch is only the device
memory / stream plumbing); every computation is a HIP kernel in libore.so.  Errors the
reference reports by panicking raise `OreError`.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import LOAD_F16, LOAD_NO_WINOGRAD, ConvAttrs, OreError, PoolAttrs, Tensor, check, load

__all__ = ["Context", "Model", "OreError", "convolution", "max_pool", "relu", "add", "softmax", "mul",
           "global_average_pool", "concatenation", "drop_out", "reshape", "inference", "conv_out_shape",
           "pool_out_shape"]


def _torch():
    import torch
    return torch


class Context:
    """One device + one HIP stream (ore_ctx).  Not thread-safe; one per host thread/device."""

    def __init__(self, device: int = 0, use_torch_stream: bool = True):
        L = load()
        h = ctypes.c_void_p()
        check(L.ore_ctx_create(int(device), ctypes.byref(h)))
        self.h = h
        self.device = device
        if use_torch_stream:
            torch = _torch()
            self.set_stream(torch.cuda.current_stream(device).cuda_stream)

    def set_stream(self, stream_ptr: Optional[int]):
        check(load().ore_ctx_set_stream(self.h, ctypes.c_void_p(stream_ptr or None)), self.h)

    def set_conv_algo(self, algo: int):
        """ore_ctx_set_conv_algo: the per-op convolution()'s algorithm (CONV_ALGO_DIRECT, the
        reference's k order; CONV_ALGO_WINOGRAD, F(2x2, 3x3) on eligible 3x3 stride-1 convs)."""
        check(load().ore_ctx_set_conv_algo(self.h, int(algo)), self.h)

    def set_conv_tile(self, tile: int = -1):
        """ore_ctx_set_conv_tile: force a tile id on every conv planned on this context afterwards
        (per-op calls and models loaded later); -1 = the per-layer heuristic.  Results do not depend
        on it (parity tests sweep it)."""
        check(load().ore_ctx_set_conv_tile(self.h, int(tile)), self.h)

    def set_pool_variant(self, variant: int = 0):
        """ore_ctx_set_pool_variant: force a MaxPool kernel (2 direct, 3 column strip, 4 plane-staged,
        5 chunk-staged; 0 = by layout)."""
        check(load().ore_ctx_set_pool_variant(self.h, int(variant)), self.h)

    @property
    def stream(self) -> int:
        return load().ore_ctx_get_stream(self.h) or 0

    def sync(self):
        check(load().ore_sync(self.h), self.h)

    def close(self):
        if getattr(self, "h", None):
            load().ore_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _desc(t, ndim: Optional[int] = None) -> Tensor:
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32:
        raise OreError(1, "expected a float32 CUDA tensor")
    if not t.is_contiguous():
        raise OreError(1, "expected a contiguous tensor")
    d = Tensor()
    d.data = t.data_ptr()
    d.ndim = t.dim() if ndim is None else ndim
    for i, s in enumerate(t.shape):
        d.dims[i] = int(s)
    d.nstride = 0
    return d


def _conv_attrs(auto_pad, pads, strides, dilations, group, fuse_relu) -> ConvAttrs:
    a = ConvAttrs()
    a.auto_pad = _lib.PAD[auto_pad]
    pads = list(pads) if pads is not None else []
    a.n_pads = min(len(pads), 4)
    for i in range(a.n_pads):
        a.pads[i] = int(pads[i])
    a.strides[0], a.strides[1] = int(strides[0]), int(strides[1])
    a.dilations[0], a.dilations[1] = int(dilations[0]), int(dilations[1])
    a.group = int(group)
    a.fuse_relu = 1 if fuse_relu else 0
    return a


def _pool_attrs(kernel_shape, strides, auto_pad, pads) -> PoolAttrs:
    a = PoolAttrs()
    a.auto_pad = _lib.PAD[auto_pad]
    pads = list(pads) if pads is not None else []
    a.n_pads = min(len(pads), 4)
    for i in range(a.n_pads):
        a.pads[i] = int(pads[i])
    a.kernel[0], a.kernel[1] = int(kernel_shape[0]), int(kernel_shape[1])
    a.strides[0], a.strides[1] = int(strides[0]), int(strides[1])
    return a


def conv_out_shape(x_shape, w_shape, auto_pad="VALID", pads=None, strides=(1, 1), dilations=(1, 1), group=1):
    """-> (y_dims, pads_tlbr) as the reference resolves them (host-only, no GPU needed)."""
    a = _conv_attrs(auto_pad, pads, strides, dilations, group, False)
    xd = (ctypes.c_int64 * 4)(*x_shape)
    wd = (ctypes.c_int64 * 4)(*w_shape)
    yd = (ctypes.c_int64 * 4)()
    p = (ctypes.c_int64 * 4)()
    check(load().ore_conv_out_shape(xd, wd, ctypes.byref(a), yd, p))
    return tuple(yd), tuple(p)


def pool_out_shape(x_shape, kernel_shape, strides, auto_pad="VALID", pads=None):
    a = _pool_attrs(kernel_shape, strides, auto_pad, pads)
    xd = (ctypes.c_int64 * 4)(*x_shape)
    yd = (ctypes.c_int64 * 4)()
    p = (ctypes.c_int64 * 4)()
    check(load().ore_pool_out_shape(xd, ctypes.byref(a), yd, p))
    return tuple(yd), tuple(p)


# ------------------------------------------------------------------------------ op arms
def convolution(ctx: Context, x, w, bias=None, auto_pad="VALID", pads=None, strides=(1, 1), dilations=(1, 1),
                group=1, fuse_relu=False):
    """convolution_op.rs:94-193."""
    torch = _torch()
    yd, _ = conv_out_shape(tuple(x.shape), tuple(w.shape), auto_pad, pads, strides, dilations, group)
    y = torch.empty(yd, dtype=torch.float32, device=x.device)
    a = _conv_attrs(auto_pad, pads, strides, dilations, group, fuse_relu)
    b = ctypes.byref(_desc(bias)) if bias is not None else None
    check(load().ore_conv2d_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(_desc(w)), b, ctypes.byref(a),
                                ctypes.byref(_desc(y))), ctx.h)
    return y


def max_pool(ctx: Context, x, kernel_shape, strides, auto_pad="VALID", pads=None):
    """max_pool_op.rs:65-129."""
    torch = _torch()
    yd, _ = pool_out_shape(tuple(x.shape), kernel_shape, strides, auto_pad, pads)
    y = torch.empty(yd, dtype=torch.float32, device=x.device)
    a = _pool_attrs(kernel_shape, strides, auto_pad, pads)
    check(load().ore_maxpool2d_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(a), ctypes.byref(_desc(y))), ctx.h)
    return y


def relu(ctx: Context, x):
    """relu_op.rs:11-33."""
    y = _torch().empty_like(x)
    check(load().ore_relu_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(_desc(y))), ctx.h)
    return y


def add(ctx: Context, a, b):
    """add_op.rs:16-107 (b broadcast onto a)."""
    y = _torch().empty_like(a)
    check(load().ore_add_f32(ctx.h, ctypes.byref(_desc(a)), ctypes.byref(_desc(b)), ctypes.byref(_desc(y))), ctx.h)
    return y


def softmax(ctx: Context, x):
    """softmax_op.rs:45-57: (N, C*H*W) rows."""
    torch = _torch()
    rows = x.shape[0]
    y = torch.empty((rows, x.numel() // max(rows, 1)), dtype=torch.float32, device=x.device)
    check(load().ore_softmax_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(_desc(y))), ctx.h)
    return y


def mul(ctx: Context, a, b):
    """MatMul, mul_op.rs:11-32."""
    torch = _torch()
    y = torch.empty((a.shape[0], b.shape[1]), dtype=torch.float32, device=a.device)
    check(load().ore_matmul_f32(ctx.h, ctypes.byref(_desc(a)), ctypes.byref(_desc(b)), ctypes.byref(_desc(y))), ctx.h)
    return y


def global_average_pool(ctx: Context, x):
    """global_average_pool_op.rs:11-51."""
    torch = _torch()
    y = torch.empty((x.shape[0], x.shape[1], 1, 1), dtype=torch.float32, device=x.device)
    check(load().ore_gap_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(_desc(y))), ctx.h)
    return y


def concatenation(ctx: Context, a, b, axis: int = 1):
    """concatenate_op.rs:11-41."""
    torch = _torch()
    shape = list(a.shape)
    shape[axis] += b.shape[axis]
    y = torch.empty(shape, dtype=torch.float32, device=a.device)
    check(load().ore_concat_f32(ctx.h, ctypes.byref(_desc(a)), ctypes.byref(_desc(b)), int(axis),
                                ctypes.byref(_desc(y))), ctx.h)
    return y


def drop_out(ctx: Context, x, ratio: Optional[float] = None):
    """dropout_op.rs:12-89: identity at inference."""
    y = _torch().empty_like(x)
    check(load().ore_dropout_f32(ctx.h, ctypes.byref(_desc(x)), ctypes.byref(_desc(y))), ctx.h)
    return y


def reshape(x, shape: Sequence[int]):
    """reshape_op.rs:16-92: metadata-only 2-D view."""
    s = (ctypes.c_int64 * len(shape))(*shape)
    y = Tensor()
    check(load().ore_reshape(ctypes.byref(_desc(x)), s, len(shape), ctypes.byref(y)))
    return x.view(int(y.dims[0]), int(y.dims[1]))


# ------------------------------------------------------------------------------ graph walker
class Model:
    """ore_model: the device-resident walker over one ONNX graph."""

    def __init__(self, ctx: Context, onnx_bytes: bytes, max_batch: int, precision: str = "f32",
                 winograd: bool = True):
        """precision "f32": convs on the f32-input MFMA; "f16": the fp16 variant (ORE_LOAD_F16).
        Input / output stay f32.  winograd (f32 only): 3x3 stride-1 pad-1 convs that no direct-kernel
        fusion takes run Winograd F(2x2, 3x3) in f32; False = ORE_LOAD_NO_WINOGRAD (direct kernels
        only).  Any max_batch loads: batches past run_batch run in image chunks (ore_model_run)."""
        if precision not in ("f32", "f16"):
            raise OreError(1, f"precision must be 'f32' or 'f16', not {precision!r}")
        self.ctx = ctx
        self.precision = precision
        h = ctypes.c_void_p()
        flags = {"f32": 0, "f16": LOAD_F16}[precision]
        if not winograd:
            flags |= LOAD_NO_WINOGRAD
        check(load().ore_model_load_ex(ctx.h, onnx_bytes, len(onnx_bytes), int(max_batch), flags, ctypes.byref(h)),
              ctx.h)
        self.h = h
        self.max_batch = max_batch
        # images per pass of the graph: larger batches run in image chunks inside ore_model_run
        self.run_batch = int(load().ore_model_run_batch(h))
        d = (ctypes.c_int64 * 4)()
        check(load().ore_model_input_dims(self.h, d), ctx.h)
        self.input_dims = tuple(d)[1:]
        e = ctypes.c_int64()
        check(load().ore_model_output_elems(self.h, ctypes.byref(e)), ctx.h)
        self.output_elems = e.value

    def set_fusion(self, flags: int):
        check(load().ore_model_set_fusion(self.h, int(flags)), self.ctx.h)

    def _check_io(self, x, out):
        """The walker reads x and writes out through raw device pointers: both must be contiguous
        float32 tensors on this context's device, x [n, C, H, W] with n <= max_batch and out holding
        n * output_elems floats (the same contract _desc() enforces for the per-op entries)."""
        torch = _torch()
        for name, t in (("x", x), ("out", out)):
            if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32:
                raise OreError(1, f"{name}: expected a float32 CUDA tensor")
            if t.device.index != self.ctx.device:
                raise OreError(1, f"{name}: on cuda:{t.device.index}, the context is on cuda:{self.ctx.device}")
            if not t.is_contiguous():
                raise OreError(1, f"{name}: expected a contiguous tensor")
        n = x.shape[0]
        if tuple(x.shape[1:]) != self.input_dims:
            raise OreError(1, f"input dims {tuple(x.shape[1:])} != model {self.input_dims}")
        if out.numel() < n * self.output_elems:
            raise OreError(1, f"out holds {out.numel()} floats, {n} images need {n * self.output_elems}")
        return n

    def run_into(self, x, out):
        """Asynchronous on the context stream; x [n, C, H, W], out [n, output_elems] (CUDA)."""
        n = self._check_io(x, out)
        check(load().ore_model_run(self.h, ctypes.c_void_p(x.data_ptr()), int(n), ctypes.c_void_p(out.data_ptr())),
              self.ctx.h)
        return out

    def run(self, x):
        torch = _torch()
        out = torch.empty((x.shape[0], self.output_elems), dtype=torch.float32, device=x.device)
        return self.run_into(x, out)

    def read_value(self, name: str) -> np.ndarray:
        dims = (ctypes.c_int64 * 4)()
        nd = ctypes.c_int32()
        check(load().ore_model_read_value(self.h, name.encode(), None, 0, dims, ctypes.byref(nd)), self.ctx.h)
        shape = tuple(dims)[: nd.value]
        buf = np.empty(shape, dtype=np.float32)
        check(load().ore_model_read_value(self.h, name.encode(), buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                          dims, ctypes.byref(nd)), self.ctx.h)
        return buf

    def autotune(self, x, out, reps: int = 3):
        """Per-layer block-tile search on a real run (ore_model_autotune); synchronous."""
        self._check_io(x, out)
        check(load().ore_model_autotune(self.h, ctypes.c_void_p(x.data_ptr()), int(x.shape[0]),
                                        ctypes.c_void_p(out.data_ptr()), int(reps)), self.ctx.h)

    # tile ids (ore_model_step_tile); None = a retired id (kernels removed after measuring slower)
    TILE_NAMES = ["128x128", "96x128", "64x128", "32x256",
                  None, None, None, None,  # 4-7: the LDS-free direct conv
                  None, None, None, None,  # 8-11: the warp-specialised conv_gemm_kernel
                  "stream 64x128", "stream 32x256", "stream 16x256", "stream 48x128", "stream 64x64",
                  "stream 128x64", "stream 64x64 d8", "stream 32x128", "stream 48x64", "fire",
                  "epool patch", "epool walk48", "epool walk96", "epool walk64",
                  "epool walk64 b3", None,  # 27: the 2-band walker
                  None, None, None, None, None, None, None, None,  # 28-35: ABI 1's bf16x3 kernels
                  "wino 32x32 d4", "wino 32x32 d2", "wino16 32x16", "wino16 16x32",
                  "wino lds", None,  # 41: the Winograd fire module (retired)
                  "fire f16", "first conv pool f16", "epool window f32", "fire pool f32",
                  "stream1x1 persist 32x128", "stream1x1 persist 64x64", "stream1x1 persist 16x256",
                  "conv1x1 gap f16", "conv1x1 gap f32", "epool band f32", "epool band f16"]

    def tiles(self):
        """Block tile per exec step (-1 for non-conv steps); names in TILE_NAMES."""
        return [load().ore_model_step_tile(self.h, i) for i in range(load().ore_model_step_count(self.h))]

    def set_tile(self, step: int, tile: int):
        """ore_model_set_step_tile: run exec step `step` on tile id `tile` (one of its autotune
        candidates; e.g. to restore a saved autotune result)."""
        check(load().ore_model_set_step_tile(self.h, int(step), int(tile)), self.ctx.h)

    def set_streams(self, streams: int):
        """2: run independent neighbouring steps (the fire modules' expand branches) on a side
        stream (ore_model_set_streams)."""
        check(load().ore_model_set_streams(self.h, int(streams)), self.ctx.h)

    def capture(self, x, out):
        """Capture run_into(x, out) as a HIP graph on the context stream (ore_model_graph_capture);
        replay() re-runs it on whatever x / out hold then."""
        n = self._check_io(x, out)
        self._graph_bufs = (x, out)  # the graph holds these pointers
        check(load().ore_model_graph_capture(self.h, ctypes.c_void_p(x.data_ptr()), int(n),
                                             ctypes.c_void_p(out.data_ptr())), self.ctx.h)
        return out

    def replay(self):
        check(load().ore_model_graph_launch(self.h), self.ctx.h)
        return self._graph_bufs[1]

    def enable_timing(self, on: bool = True):
        check(load().ore_model_enable_timing(self.h, 1 if on else 0), self.ctx.h)

    def steps(self):
        L = load()
        out = []
        for i in range(L.ore_model_step_count(self.h)):
            op, name = ctypes.c_char_p(), ctypes.c_char_p()
            fl, by = ctypes.c_double(), ctypes.c_double()
            check(L.ore_model_step_info(self.h, i, ctypes.byref(op), ctypes.byref(name), ctypes.byref(fl),
                                        ctypes.byref(by)), self.ctx.h)
            mf = ctypes.c_double()
            check(L.ore_model_step_mfma_flops(self.h, i, ctypes.byref(mf)), self.ctx.h)
            out.append({"op": op.value.decode(), "name": name.value.decode(), "flops": fl.value, "bytes": by.value,
                        "mfma_flops": mf.value})
        return out

    def step_times_ms(self):
        n = load().ore_model_step_count(self.h)
        buf = (ctypes.c_float * max(n, 1))()
        check(load().ore_model_step_times(self.h, buf, n), self.ctx.h)
        return list(buf)[:n]

    def close(self):
        if getattr(self, "h", None):
            load().ore_model_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def inference(onnx_bytes: bytes, input_data, input_tensor_name=None, device: int = 0) -> np.ndarray:
    """inference() (model_inference.rs:29-120) on the GPU: returns graph.output[0] for the batch
    (the reference only prints it).  input_data: array [n, C, H, W] or the flat per-image vector
    the reference takes (then n = 1).  input_tensor_name is accepted for signature parity; the
    seeded input is the graph input that is not an initializer (utils.rs:29-45)."""
    torch = _torch()
    ctx = Context(device)
    try:
        x = np.asarray(input_data, dtype=np.float32)
        m = Model(ctx, onnx_bytes, max_batch=max(1, x.shape[0] if x.ndim == 4 else 1))
        if x.ndim != 4:
            x = x.reshape((1,) + tuple(m.input_dims))
        xd = torch.from_numpy(np.ascontiguousarray(x)).to(f"cuda:{device}")
        y = m.run(xd)
        torch.cuda.synchronize(device)
        out = y.cpu().numpy()
        m.close()
        return out
    finally:
        ctx.close()

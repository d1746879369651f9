"""Float64 executor of the ONNX graphs used here (SqueezeNet-1.0 / MNIST-8 op subset), for
accuracy budgets: how far the oracle (f32, the reference's summation order), the f32-MFMA path and
the x3 path each are from the exact result.  Test infrastructure only.

Op semantics follow the reference as restated in oracle/ref_ops.c: Conv with zero padding
(convolution_op.rs:224-517), MaxPool padding with 0 and starting from -FLT_MAX
(max_pool_op.rs:265-276, :337), GlobalAveragePool, Softmax over axis 1, Concat, Dropout = identity,
Add, Reshape, MatMul.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "onnx-rusty-inference-engine_amd"))

from ore import onnx_wire  # noqa: E402

FLT_MAX = float(np.finfo(np.float32).max)


def _pads(a, H, W, kh, kw, sh, sw):
    auto = a["auto_pad"].s.decode() if "auto_pad" in a else "NOTSET"
    if auto in ("SAME_UPPER", "SAME_LOWER"):
        Ho, Wo = -(-H // sh), -(-W // sw)
        ph = max((Ho - 1) * sh + kh - H, 0)
        pw = max((Wo - 1) * sw + kw - W, 0)
        # the reference puts the larger half top/left for both (convolution_op.rs:547-556)
        return [ph - ph // 2, pw - pw // 2, ph // 2, pw // 2]
    p = list(a["pads"].ints) if "pads" in a else [0, 0, 0, 0]
    return p if len(p) == 4 else [0, 0, 0, 0]


def _windows(xp, kh, kw, sh, sw, Ho, Wo):
    N, C = xp.shape[:2]
    cols = np.empty((N, C, kh, kw, Ho, Wo), dtype=xp.dtype)
    for r in range(kh):
        for s in range(kw):
            cols[:, :, r, s] = xp[:, :, r:r + sh * (Ho - 1) + 1:sh, s:s + sw * (Wo - 1) + 1:sw]
    return cols


def run(model_bytes, x):
    """Run graph.output[0] in float64 on x (numpy [N, ...]); returns float64."""
    g = onnx_wire.decode_model(model_bytes).graph
    env = {t.name: t.to_numpy().astype(np.float64) if t.to_numpy().dtype != np.int64 else t.to_numpy()
           for t in g.initializer}
    inputs = [v.name for v in g.input if v.name not in env]
    env[inputs[0]] = np.asarray(x, dtype=np.float64)
    consts = set(env) - {inputs[0]}
    for n in g.node:
        a = n.attrs()
        ins = [env[i] for i in n.input]
        op = n.op_type
        if op == "Conv":
            xx, w = ins[0], ins[1]
            b = ins[2] if len(ins) > 2 else None
            M, C, kh, kw = w.shape
            sh, sw = a["strides"].ints
            pt, pl, pb, pr = _pads(a, xx.shape[2], xx.shape[3], kh, kw, sh, sw)
            xp = np.pad(xx, ((0, 0), (0, 0), (pt, pb), (pl, pr)))
            Ho = (xp.shape[2] - kh) // sh + 1
            Wo = (xp.shape[3] - kw) // sw + 1
            cols = _windows(xp, kh, kw, sh, sw, Ho, Wo).reshape(xx.shape[0], C * kh * kw, Ho * Wo)
            y = np.einsum("mk,nkp->nmp", w.reshape(M, -1), cols).reshape(xx.shape[0], M, Ho, Wo)
            if b is not None:
                y = y + b.reshape(1, M, 1, 1)
        elif op == "Relu":
            y = np.maximum(ins[0], 0.0)
        elif op == "MaxPool":
            xx = ins[0]
            kh, kw = a["kernel_shape"].ints
            sh, sw = a["strides"].ints
            auto = a["auto_pad"].s.decode() if "auto_pad" in a else "VALID"
            if auto == "NOTSET":
                pt, pl, pb, pr = list(a["pads"].ints) if "pads" in a else [0, 0, 0, 0]
            elif auto in ("SAME_UPPER", "SAME_LOWER"):
                pt, pl, pb, pr = _pads(a, xx.shape[2], xx.shape[3], kh, kw, sh, sw)
            else:
                pt = pl = pb = pr = 0
            xp = np.pad(xx, ((0, 0), (0, 0), (pt, pb), (pl, pr)))  # the reference pads with 0
            Ho = (xp.shape[2] - kh) // sh + 1
            Wo = (xp.shape[3] - kw) // sw + 1
            y = np.maximum(_windows(xp, kh, kw, sh, sw, Ho, Wo).max(axis=(2, 3)), -FLT_MAX)
        elif op == "Concat":
            y = np.concatenate(ins[:2], axis=a["axis"].i if "axis" in a else 1)
        elif op == "Dropout":
            y = ins[0]
        elif op == "GlobalAveragePool":
            y = ins[0].mean(axis=(2, 3), keepdims=True)
        elif op == "Softmax":
            z = ins[0].reshape(ins[0].shape[0], -1)
            z = np.exp(z - z.max(axis=1, keepdims=True))
            y = z / z.sum(axis=1, keepdims=True)
        elif op == "Add":
            y = ins[0] + ins[1]
        elif op == "Reshape":
            shape = [int(s) for s in ins[1]]
            shape = [ins[0].shape[i] if s == 0 else s for i, s in enumerate(shape)]
            if n.input[0] in consts:  # an initializer: reshaped as is (reshape_op.rs:66-92)
                y = ins[0].reshape(shape)
            else:  # an activation: per image (the batch dim leads)
                y = ins[0].reshape(ins[0].shape[0], -1)
        elif op == "MatMul":
            y = ins[0] @ ins[1]
        else:
            raise NotImplementedError(op)
        if op == "Reshape" and n.input[0] in consts:
            consts.add(n.output[0])
        env[n.output[0]] = y
    out = env[g.output[0].name]
    return out.reshape(out.shape[0], -1)

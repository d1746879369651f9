"""Float64 reference helpers for the conv parity tests (no GPU): a direct convolution with the
per-output magnitude sum |w x| that the f32 tolerance 2e-6 * sum|w x| is written against, and a
one-Conv ONNX model builder."""
import numpy as np


def conv_f64(x, w, b, pads, strides):
    """Direct convolution in float64 (zero padding, pads t, l, b, r) and sum |w x| per output."""
    x = x.astype(np.float64)
    w = w.astype(np.float64)
    N, C, H, W = x.shape
    M, _, kh, kw = w.shape
    pt, pl, pb, pr = pads
    sh, sw = strides
    xp = np.zeros((N, C, H + pt + pb, W + pl + pr))
    xp[:, :, pt:pt + H, pl:pl + W] = x
    Ho = (H + pt + pb - kh) // sh + 1
    Wo = (W + pl + pr - kw) // sw + 1
    cols = np.empty((N, C, kh, kw, Ho, Wo))
    for r in range(kh):
        for s in range(kw):
            cols[:, :, r, s] = xp[:, :, r:r + sh * (Ho - 1) + 1:sh, s:s + sw * (Wo - 1) + 1:sw]
    cols = cols.reshape(N, C * kh * kw, Ho * Wo)
    wm = w.reshape(M, -1)
    y = np.einsum("mk,nkp->nmp", wm, cols).reshape(N, M, Ho, Wo)
    mag = np.einsum("mk,nkp->nmp", np.abs(wm), np.abs(cols)).reshape(N, M, Ho, Wo)
    if b is not None:
        y += b.astype(np.float64)[None, :, None, None]
        mag += np.abs(b.astype(np.float64))[None, :, None, None]
    return y, mag


def _conv_model(x_shape, w, b, pads, strides):
    from ore import onnx_wire as wr
    ins = ["x", "w"] + (["b"] if b is not None else [])
    nodes = [wr.encode_node("Conv", ins, ["y"], attrs=[wr.encode_attr_ints("pads", pads),
                                                       wr.encode_attr_ints("strides", strides)])]
    inits = [wr.encode_tensor("w", w)] + ([wr.encode_tensor("b", b)] if b is not None else [])
    vinfo = [wr.encode_value_info("x", x_shape), wr.encode_value_info("w", w.shape)]
    if b is not None:
        vinfo.append(wr.encode_value_info("b", b.shape))
    return wr.encode_model("c", nodes, inits, vinfo, [wr.encode_value_info("y", (1, 1, 1, 1))])

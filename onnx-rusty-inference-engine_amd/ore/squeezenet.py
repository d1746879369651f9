"""Deterministic synthetic SqueezeNet-1.0 (ONNX model-zoo `squeezenet1.0-8.onnx` topology).

The real model file is not available here (stripped from the reference mirror,
/root/reference/.MISSING_LARGE_BLOBS:1), so the benchmark and the parity tests use this graph:
the zoo's 66-node topology (26 Conv, 26 Relu, 3 MaxPool, 8 Concat, 1 Dropout,
1 GlobalAveragePool, 1 Softmax), its value names (`data_0` -> `softmaxout_1`), opset 8, IR 3
(initializers listed in graph.input, as utils.rs:53-97 requires), Caffe-style explicit pads,
and seeded weights: He-normal N(0, 2/fan_in) (seed 1234) and biases U(-0.1, 0.1).

Pool4 carries pads [0,0,1,1] with auto_pad "NOTSET" (Caffe ceil mode: 54 -> 27, final map
13x13, 818.9 M MAC per 224x224 image).  The reference honours MaxPool pads only under an
explicit NOTSET (max_pool_op.rs:88-99, 248); see DESIGN.md for this choice.
"""
from __future__ import annotations

import numpy as np

from . import onnx_wire as w

# conv10's weight gain of the zoo-calibrated variant: with it the softmax of the zoo image
# (squeezenet_data_0.pb) peaks at 0.074, as squeezenet_output_0.pb does for the real weights (0.0742);
# the plain He-normal graph (gain 1) peaks at 0.62-0.95, where f32 rounding in any summation order,
# the reference's own included, already moves the probabilities by up to ~1e-5
ZOO_LOGIT_GAIN = 0.167

# (name, squeeze, expand) for fire2..fire9; a MaxPool follows fire4 and fire8
FIRES = [("fire2", 16, 64), ("fire3", 16, 64), ("fire4", 32, 128), ("fire5", 32, 128),
         ("fire6", 48, 192), ("fire7", 48, 192), ("fire8", 64, 256), ("fire9", 64, 256)]


def _conv_params(rng, cout, cin, k):
    fan_in = cin * k * k
    wt = rng.standard_normal((cout, cin, k, k)).astype(np.float32) * np.float32(np.sqrt(2.0 / fan_in))
    b = rng.uniform(-0.1, 0.1, size=(cout,)).astype(np.float32)
    return wt, b


def build(input_hw: int = 224, seed: int = 1234, num_classes: int = 1000, logit_gain: float = 1.0,
          pool4_ceil: bool = True) -> bytes:
    """Return the ONNX ModelProto bytes of a SqueezeNet-1.0 with seeded weights."""
    rng = np.random.default_rng(seed)
    nodes, inits, inputs = [], [], []

    def add_init(name, arr):
        inits.append(w.encode_tensor(name, arr))
        inputs.append(w.encode_value_info(name, arr.shape))

    def conv(prefix, x, cin, cout, k, stride, pad, gain=1.0):
        wt, b = _conv_params(rng, cout, cin, k)
        if gain != 1.0:
            wt = (wt * np.float32(gain)).astype(np.float32)
        add_init(f"{prefix}_w_0", wt)
        add_init(f"{prefix}_b_0", b)
        y = f"{prefix}_1"
        nodes.append(w.encode_node("Conv", [x, f"{prefix}_w_0", f"{prefix}_b_0"], [y], name=prefix, attrs=[
            w.encode_attr_ints("kernel_shape", [k, k]), w.encode_attr_ints("pads", [pad] * 4),
            w.encode_attr_ints("strides", [stride, stride])]))
        r = f"{prefix}_2"
        nodes.append(w.encode_node("Relu", [y], [r], name=f"{prefix}_relu"))
        return r

    def maxpool(name, x, pads):
        y = f"{name}_1"
        nodes.append(w.encode_node("MaxPool", [x], [y], name=name, attrs=[
            w.encode_attr_ints("kernel_shape", [3, 3]), w.encode_attr_ints("pads", pads),
            w.encode_attr_ints("strides", [2, 2]), w.encode_attr_string("auto_pad", "NOTSET")]))
        return y

    x = conv("conv1", "data_0", 3, 96, 7, 2, 0)
    x = maxpool("pool1", x, [0, 0, 0, 0])
    cin = 96
    for name, s, e in FIRES:
        sq = conv(f"{name}/squeeze1x1", x, cin, s, 1, 1, 0)
        e1 = conv(f"{name}/expand1x1", sq, s, e, 1, 1, 0)
        e3 = conv(f"{name}/expand3x3", sq, s, e, 3, 1, 1)
        x = f"{name}/concat_1"
        nodes.append(w.encode_node("Concat", [e1, e3], [x], name=f"{name}/concat", attrs=[w.encode_attr_int("axis", 1)]))
        cin = 2 * e
        if name == "fire4":
            x = maxpool("pool3", x, [0, 0, 1, 1] if pool4_ceil else [0, 0, 0, 0])
        elif name == "fire8":
            x = maxpool("pool5", x, [0, 0, 0, 0])
    nodes.append(w.encode_node("Dropout", [x], ["fire9/concat_2", "_fire9/concat_mask"], name="drop9",
                               attrs=[w.encode_attr_float("ratio", 0.5)]))
    x = conv("conv10", "fire9/concat_2", cin, num_classes, 1, 1, 0, gain=logit_gain)
    nodes.append(w.encode_node("GlobalAveragePool", [x], ["pool10_1"], name="pool10"))
    nodes.append(w.encode_node("Softmax", ["pool10_1"], ["softmaxout_1"], name="softmax"))

    graph_inputs = [w.encode_value_info("data_0", (1, 3, input_hw, input_hw))] + inputs
    outputs = [w.encode_value_info("softmaxout_1", (1, num_classes, 1, 1))]
    return w.encode_model("squeezenet1.0-synthetic", nodes, inits, graph_inputs, outputs, opset=8)


def build_calibrated(input_hw: int = 224) -> bytes:
    """The zoo-calibrated SqueezeNet-1.0: build() with conv10's weights scaled by ZOO_LOGIT_GAIN (same
    topology, same work per image; bench.py's model and the strict-parity fixtures)."""
    return build(input_hw, logit_gain=ZOO_LOGIT_GAIN)


def macs_per_image(input_hw: int = 224) -> int:
    """Analytic multiply-accumulates of the 26 convolutions for one image (818.9 M at 224)."""
    def out(h, k, s, p_lo, p_hi):
        return (h + p_lo + p_hi - k) // s + 1
    h = out(input_hw, 7, 2, 0, 0)
    total = 96 * h * h * 3 * 49
    h = out(h, 3, 2, 0, 0)
    cin = 96
    for name, s, e in FIRES:
        total += s * h * h * cin + e * h * h * s + e * h * h * s * 9
        cin = 2 * e
        if name == "fire4":
            h = out(h, 3, 2, 0, 1)
        elif name == "fire8":
            h = out(h, 3, 2, 0, 0)
    total += 1000 * h * h * cin
    return total


def synthetic_input(n: int, input_hw: int = 224, seed: int = 0) -> np.ndarray:
    """U(-50, 50) images: the range of the zoo's squeezenet_data_0.pb (-48.9 .. 44.1)."""
    rng = np.random.default_rng(seed)
    return rng.uniform(-50.0, 50.0, size=(n, 3, input_hw, input_hw)).astype(np.float32)

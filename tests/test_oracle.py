"""CPU: pin the oracle (the C restatement of the reference) against the reference's own golden
vectors and known-answer tests before trusting it as the GPU checker."""
import os

import numpy as np
import pytest

import oracle
from ore import onnx_wire

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def test_mnist_golden():
    """models/mnist-8.onnx + mnist_data_0.pb -> mnist_output_0.pb (the reference's manual
    integration check, main.rs:11-14/39-41)."""
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        m = oracle.Model(f.read())
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_output_0.pb")).to_numpy()
    y = m.run(x, 10)
    assert np.abs(y - g).max() <= 1e-6 * np.abs(g).max()
    assert y.argmax() == 2


def test_mnist_faithful_equals_fast():
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        m = oracle.Model(f.read())
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy()
    assert np.array_equal(m.run(x, 10), m.run(x, 10, faithful=True))


def _direct_conv64(x, w, pads_tlbr, strides):
    x = x.astype(np.float64)
    w = w.astype(np.float64)
    t, l, b, r = pads_tlbr
    xp = np.pad(x, ((0, 0), (0, 0), (t, b), (l, r)))
    N, C, H, W = xp.shape
    M, _, kh, kw = w.shape
    Ho, Wo = (H - kh) // strides[0] + 1, (W - kw) // strides[1] + 1
    y = np.zeros((N, M, Ho, Wo))
    for i in range(Ho):
        for j in range(Wo):
            patch = xp[:, :, i * strides[0]:i * strides[0] + kh, j * strides[1]:j * strides[1] + kw]
            y[:, :, i, j] = np.einsum("nchw,mchw->nm", patch, w)
    return y


def test_conv_reference_kats():
    """Inputs of test_convolution_* (convolution_op.rs:729-832): integer data, so the expected
    output is exact; checks the [1,0,3,2] permute + ker2col/im2col row pairing."""
    x1 = np.arange(1, 31, dtype=np.float32).reshape(1, 1, 5, 6)
    w1 = np.arange(1, 11, dtype=np.float32).reshape(1, 1, 5, 2)
    x2 = np.arange(1, 61, dtype=np.float32).reshape(1, 2, 5, 6)
    w2 = np.repeat(np.array([1, 2, 3, 4], dtype=np.float32), 12).reshape(2, 2, 3, 4)
    x3 = np.arange(0, 35, dtype=np.float32).reshape(1, 1, 7, 5)
    w3 = np.arange(1, 25, dtype=np.float32).reshape(2, 1, 3, 4)
    for x, w in ((x1, w1), (x2, w2), (x3, w3)):
        y = oracle.conv2d(x, w, None, auto_pad="NOTSET", pads=[0, 0, 0, 0], strides=(1, 1))
        np.testing.assert_array_equal(y, _direct_conv64(x, w, (0, 0, 0, 0), (1, 1)).astype(np.float32))


@pytest.mark.parametrize("auto_pad,strides", [("SAME_UPPER", (1, 1)), ("SAME_LOWER", (2, 2)), ("VALID", (2, 1))])
def test_conv_random_vs_float64(auto_pad, strides):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 5, 11, 13)).astype(np.float32)
    w = rng.standard_normal((7, 5, 4, 3)).astype(np.float32)
    b = rng.standard_normal(7).astype(np.float32)
    p, Ho, Wo = oracle.resolve_window(auto_pad, None, 11, 13, 4, 3, *strides)
    ref = _direct_conv64(x, w, p, strides)[:, :, :Ho, :Wo] + b[None, :, None, None]
    y = oracle.conv2d(x, w, b, auto_pad=auto_pad, strides=strides)
    assert y.shape == ref.shape
    assert np.abs(y - ref).max() <= 1e-5


def test_same_padding_quirk():
    """get_padding_size puts the larger half at the top/left for SAME_UPPER and SAME_LOWER
    alike (convolution_op.rs:547-556)."""
    p, Ho, Wo = oracle.resolve_window("SAME_UPPER", None, 15, 14, 4, 4, 2, 2)
    # H: 15 % 2 = 1 -> pad 4 - 1 = 3 -> top 2, bottom 1; W: 14 % 2 = 0 -> pad 2 -> 1/1
    assert tuple(p) == (2, 1, 1, 1) and (Ho, Wo) == (8, 7)
    p2, _, _ = oracle.resolve_window("SAME_LOWER", None, 15, 14, 4, 4, 2, 2)
    assert tuple(p2) == tuple(p)
    with pytest.raises(oracle.OracleError):  # kernel < stride: usize underflow in the reference
        oracle.resolve_window("SAME_UPPER", None, 8, 8, 1, 1, 2, 2)


def test_maxpool_reference_kat():
    """test_max_pool (max_pool_op.rs:452-472): 4x4 = 1..16, 3x3, stride 1, VALID."""
    x = np.arange(1, 17, dtype=np.float32).reshape(1, 1, 4, 4)
    y = oracle.maxpool2d(x, (3, 3), (1, 1), auto_pad="VALID")
    np.testing.assert_array_equal(y.ravel(), [11, 12, 15, 16])


def test_maxpool_zero_padding():
    """The reference pads with 0, not -inf (max_pool_op.rs:265-276)."""
    x = -np.ones((1, 1, 3, 3), np.float32)
    y = oracle.maxpool2d(x, (2, 2), (2, 2), auto_pad="NOTSET", pads=[0, 0, 1, 1])
    np.testing.assert_array_equal(y.ravel(), [-1, 0, 0, 0])
    yv = oracle.maxpool2d(x, (2, 2), (2, 2), auto_pad="VALID", pads=[0, 0, 1, 1])  # pads ignored
    assert yv.shape == (1, 1, 1, 1)


def test_relu_reference_kat():
    x = np.arange(0, 35, dtype=np.float32)
    x[17] = -17.0
    e = np.arange(0, 35, dtype=np.float32)
    e[17] = 0.0
    np.testing.assert_array_equal(oracle.relu(x.reshape(1, 1, 7, 5)).ravel(), e)


def test_softmax_reference_kat():
    x = np.array([118.85734, 5640.1426, 2., 3., 1000., 1001., 1002., 1003.], np.float32).reshape(1, 1, 2, 4)
    y = oracle.softmax(x)
    x64 = x.reshape(1, -1).astype(np.float64)
    ref = np.exp(x64 - x64.max()) / np.exp(x64 - x64.max()).sum()
    assert np.abs(y - ref).max() <= 1e-7
    assert y.argmax() == 1


def test_gap_reference_kat():
    x = np.tile(np.arange(1, 17, dtype=np.float32), 2).reshape(1, 2, 4, 4)
    np.testing.assert_array_equal(oracle.gap(x).ravel(), [8.5, 8.5])


def test_ndarray_sum_order():
    """unrolled_fold: 8 partial sums, combined (p0+p4),(p1+p5),(p2+p6),(p3+p7), then the tail."""
    xs = np.array([1e8, 1, 1, 1, -1e8, 1, 1, 1, 1], np.float32)
    p = [np.float32(0)] * 8
    for i in range(8):
        p[i] = np.float32(p[i] + xs[i])
    acc = np.float32(0)
    for a, b in ((0, 4), (1, 5), (2, 6), (3, 7)):
        acc = np.float32(acc + np.float32(p[a] + p[b]))
    acc = np.float32(acc + xs[8])
    assert oracle.ndarray_sum(xs) == acc == np.float32(7.0)
    assert np.float32(sum(np.float32(v) for v in xs)) != acc  # sequential order differs here


def test_concat_and_add():
    a = np.ones((1, 2, 2, 2), np.float32)
    b = np.zeros((1, 3, 2, 2), np.float32)
    y = oracle.concat(a, b, 1)
    assert y.shape == (1, 5, 2, 2) and y[0, :2].sum() == 8 and y[0, 2:].sum() == 0
    c = np.arange(2, dtype=np.float32).reshape(2, 1, 1)
    np.testing.assert_array_equal(oracle.add(a, c)[0, :, 0, 0], [1, 2])


def test_model_errors():
    from ore import onnx_wire as w
    mb = w.encode_model("t", [w.encode_node("Sigmoid", ["x"], ["y"])], [],
                        [w.encode_value_info("x", (1, 1, 2, 2))], [w.encode_value_info("y", (1, 1, 2, 2))])
    m = oracle.Model(mb)
    with pytest.raises(oracle.OracleError, match="NOT FOUND"):
        m.run(np.zeros((1, 1, 2, 2), np.float32), 4)

"""Per-op parity: every node_inference arm through the C ABI (libore.so, HIP on gfx950) against
the CPU restatement of the reference (oracle/) on the same seeded inputs.

Tolerances: bit-exact for Relu, MaxPool, Concat, Dropout, Reshape, Add (single rounding), GAP
(same sequential order); Conv / MatMul within 2e-6 * sum|a*b| per output (the MFMA result is a
k-ordered f32 fma chain, the reference sums per-channel 8-partial ndarray sums); Softmax within
2e-7 absolute (expf ulp differences; same max and same 8-partial denominator order)."""
import zlib

import numpy as np
import pytest

from _knobs import conv_tile, pool_variant

import oracle

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _conv_bound(x, w, pads_tlbr, strides, Ho, Wo):
    """sum |x| * |w| per output (float64), the scale of the rounding error of one output."""
    import torch
    xt = torch.from_numpy(np.abs(x).astype(np.float64))
    wt = torch.from_numpy(np.abs(w).astype(np.float64))
    t, l, b, r = pads_tlbr
    xt = torch.nn.functional.pad(xt, (l, r, t, b))
    y = torch.nn.functional.conv2d(xt, wt, stride=tuple(strides))
    return y[:, :, :Ho, :Wo].numpy()


CONV_CASES = [
    # N, C, H, W, M, kh, kw, auto_pad, pads, strides, bias
    (1, 3, 17, 19, 8, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], True),
    (2, 5, 16, 16, 40, 3, 3, "SAME_UPPER", None, [1, 1], True),
    (3, 4, 15, 14, 24, 4, 4, "SAME_UPPER", None, [2, 2], False),   # asymmetric SAME split
    (2, 4, 15, 14, 24, 4, 2, "SAME_LOWER", None, [2, 3], True),
    (2, 7, 23, 23, 96, 7, 7, "VALID", None, [2, 2], True),          # conv1-like
    (3, 96, 13, 13, 16, 1, 1, "VALID", None, [1, 1], True),         # squeeze (1x1 path)
    (2, 16, 9, 9, 64, 1, 1, "NOTSET", [0, 0, 0, 0], [1, 1], True),  # expand1x1
    (2, 16, 9, 9, 64, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], True),  # expand3x3
    (2, 64, 5, 5, 200, 1, 1, "VALID", None, [1, 1], True),          # conv10-like, M % 128 != 0
    (1, 1, 28, 28, 8, 5, 5, "SAME_UPPER", None, [1, 1], False),     # MNIST conv 1
    (1, 8, 14, 14, 16, 5, 5, "SAME_UPPER", None, [1, 1], False),    # MNIST conv 2
    (2, 3, 11, 9, 33, 2, 3, "NOTSET", [2, 0, 1, 3], [3, 1], True),  # uneven explicit pads
    (5, 17, 7, 7, 130, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], False),
    (2, 33, 6, 10, 48, 1, 1, "NOTSET", [1, 0, 0, 1], [1, 2], True),  # 1x1 with pads/stride -> generic path
    # planes >= 512 pixels: window-staged kernel (plan_conv in ore_conv.hip)
    (2, 16, 54, 54, 64, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], True),     # fire2 expand3x3
    (2, 32, 54, 54, 128, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], False),   # fire4 expand3x3
    (2, 48, 27, 27, 192, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], True),    # fire6 expand3x3
    (1, 64, 27, 27, 256, 3, 3, "NOTSET", [1, 1, 1, 1], [1, 1], True),    # fire8 expand3x3
    (1, 3, 224, 224, 96, 7, 7, "VALID", None, [2, 2], True),             # conv1, 4 loads per window row
    (2, 3, 64, 64, 96, 7, 7, "VALID", None, [2, 2], True),
    (2, 13, 40, 37, 20, 3, 3, "SAME_UPPER", None, [1, 1], True),         # 32x256 tile, ragged channel stage
    (2, 7, 30, 150, 33, 5, 3, "NOTSET", [2, 1, 0, 3], [1, 2], False),    # 3 loads per row, uneven pads
    (3, 5, 33, 31, 40, 2, 4, "SAME_LOWER", None, [1, 1], True),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("fuse_relu", [False, True])
def test_conv2d(gpu_ctx, case, fuse_relu):
    import ore
    N, C, H, W, M, kh, kw, auto_pad, pads, strides, with_bias = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()))
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, kh, kw)).astype(np.float32)
    b = rng.standard_normal((M,)).astype(np.float32) if with_bias else None
    ref = oracle.conv2d(x, w, b, auto_pad=auto_pad, pads=pads, strides=strides)
    if fuse_relu:
        ref = oracle.relu(ref)
    y = ore.convolution(gpu_ctx, _t(x), _t(w), _t(b) if b is not None else None, auto_pad=auto_pad, pads=pads,
                        strides=strides, fuse_relu=fuse_relu)
    got = _np(y)
    assert got.shape == ref.shape
    eff = auto_pad
    if pads is not None and any(p > 0 for p in pads):
        eff = "NOTSET"
    p, Ho, Wo = oracle.resolve_window(eff, pads, H, W, kh, kw, strides[0], strides[1])
    bound = _conv_bound(x, w, p, strides, Ho, Wo) + (np.abs(b)[None, :, None, None] if b is not None else 0)
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    assert np.all(err <= 2e-6 * bound + 1e-30), f"max err {err.max()} vs bound {(2e-6 * bound).max()}"


@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("case", CONV_CASES[::2] + CONV_CASES[14:16])
def test_conv2d_tiles_bit_identical(gpu_ctx, case, tile):
    """The LDS-staged kernel's block tiles (ore_ctx_set_conv_tile) run the same k-ordered MFMA chain
    per output as tile 0: bit-identical outputs, and within tolerance of the oracle.  (Tile ids 4-11,
    the retired direct / warp-specialised variants, are refused.)"""
    import ore
    N, C, H, W, M, kh, kw, auto_pad, pads, strides, with_bias = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()) ^ 0x5a5a)
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, kh, kw)).astype(np.float32)
    b = rng.standard_normal((M,)).astype(np.float32) if with_bias else None
    outs = []
    for t in (0, tile):
        with conv_tile(gpu_ctx, t):
            outs.append(_np(ore.convolution(gpu_ctx, _t(x), _t(w), _t(b) if b is not None else None, auto_pad=auto_pad,
                                            pads=pads, strides=strides, fuse_relu=True)))
    np.testing.assert_array_equal(outs[1], outs[0])
    ref = oracle.relu(oracle.conv2d(x, w, b, auto_pad=auto_pad, pads=pads, strides=strides))
    assert np.abs(outs[1] - ref).max() <= 1e-4 * (np.abs(ref).max() + 1.0)
    for retired in (4, 8, 11):
        with pytest.raises(ore.OreError):
            gpu_ctx.set_conv_tile(retired)


STREAM_CASES = [
    # N, C, H, W, M, k, pad, bias: 16-B aligned output planes (Ho*Wo % 4 == 0), C*k*k % 16 == 0
    (3, 96, 12, 12, 16, 1, 0, True),     # squeeze
    (2, 16, 8, 8, 64, 1, 0, True),       # expand1x1, K = 16 (the ring's prologue only)
    (2, 64, 4, 6, 200, 1, 0, False),     # M % 64 != 0: ragged channel tile
    (5, 32, 10, 10, 40, 1, 0, True),     # 500 columns: ragged pixel tile
    (1, 512, 6, 6, 1000, 1, 0, True),    # conv10-like
    (3, 32, 16, 16, 16, 1, 0, True),     # 768 columns over 3 images
    (2, 48, 7, 4, 48, 1, 0, True),       # fewer columns than one wave tile
    (2, 16, 13, 13, 24, 1, 0, True),     # 169-pixel planes: not eligible, falls back to tile 0
    (3, 16, 64, 64, 1024, 1, 0, True),   # more pixel tiles than resident waves per m tile: the
                                         # persistent tiles (46-48) walk 2 tiles per wave
    (2, 16, 12, 12, 64, 3, 1, True),     # expand3x3 (STAPS): zero-padded taps, row wraps
    (3, 32, 10, 10, 128, 3, 1, False),   # 300 columns over 3 images
    (1, 48, 7, 8, 192, 3, 1, True),      # W = 8: 4-pixel groups straddle rows
    (2, 64, 6, 6, 256, 3, 1, True),
    (2, 16, 9, 12, 40, 3, 0, True),      # VALID 3x3: Wo != W -> falls back
]


@pytest.mark.parametrize("tile", list(range(12, 21)) + [46, 47, 48])
@pytest.mark.parametrize("case", STREAM_CASES)
def test_conv_stream_bit_identical(gpu_ctx, case, tile):
    """The LDS-free streaming kernel (ore_conv_stream.hip, 16x16x4 MFMA, tiles 12-20: 1x1 and 3x3
    'same' convs; 46-48: the persistent 1x1 variant, which walks several pixel tiles per wave) runs
    the same k-ordered fmaf chain per output as the LDS-staged kernel: bit-identical to tile 0, and
    within the conv tolerance of the oracle (the persistent tiles fall back to tile 0 on 3x3 layers)."""
    import ore
    N, C, H, W, M, k, pad, with_bias = case
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()) ^ 0x1111)
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, k, k)).astype(np.float32)
    b = rng.standard_normal((M,)).astype(np.float32) if with_bias else None
    pads = [pad] * 4
    # x 256 B into a 4 KiB page: the 3x3 stream kernel reads up to (W + 1) floats before x (masked),
    # which the per-op path allows only inside x's own page
    import torch
    buf = torch.zeros(x.size + 1024 + 64, dtype=torch.float32, device="cuda")
    xd = buf[1024 + 64:].view(x.shape)
    xd.copy_(_t(x))
    outs = []
    for t in (0, tile):
        with conv_tile(gpu_ctx, t):
            for relu in (False, True):
                outs.append(_np(ore.convolution(gpu_ctx, xd, _t(w), _t(b) if b is not None else None,
                                                auto_pad="NOTSET", pads=pads, strides=(1, 1), fuse_relu=relu)))
    np.testing.assert_array_equal(outs[2], outs[0])
    np.testing.assert_array_equal(outs[3], outs[1])
    ref = oracle.conv2d(x, w, b, auto_pad="NOTSET", pads=pads, strides=(1, 1))
    Ho, Wo = ref.shape[2], ref.shape[3]
    bound = _conv_bound(x, w, pads, (1, 1), Ho, Wo) + (np.abs(b)[None, :, None, None] if b is not None else 0)
    err = np.abs(outs[2].astype(np.float64) - ref.astype(np.float64))
    assert np.all(err <= 2e-6 * bound + 1e-30), f"max err {err.max()}"
    np.testing.assert_array_equal(outs[3], np.maximum(outs[2], 0))


def test_conv_integer_exact(gpu_ctx):
    """Small-integer data: every partial sum is exact in f32, so GPU == oracle bit for bit."""
    import ore
    rng = np.random.default_rng(7)
    x = rng.integers(-4, 5, size=(3, 12, 10, 11)).astype(np.float32)
    w = rng.integers(-3, 4, size=(70, 12, 3, 3)).astype(np.float32)
    b = rng.integers(-5, 6, size=(70,)).astype(np.float32)
    ref = oracle.conv2d(x, w, b, auto_pad="SAME_UPPER", strides=(1, 1))
    got = _np(ore.convolution(gpu_ctx, _t(x), _t(w), _t(b), auto_pad="SAME_UPPER", strides=(1, 1)))
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 12])
def test_conv_integer_exact_tiles(gpu_ctx, tile):
    """A 3x3 'same' layer on every LDS-staged tile and the streaming kernel: small-integer data, so each
    equals the oracle bit for bit."""
    import ore
    rng = np.random.default_rng(11)
    x = rng.integers(-4, 5, size=(2, 19, 30, 29)).astype(np.float32)
    w = rng.integers(-3, 4, size=(100, 19, 3, 3)).astype(np.float32)
    b = rng.integers(-5, 6, size=(100,)).astype(np.float32)
    ref = oracle.conv2d(x, w, b, pads=[1, 1, 1, 1], strides=(1, 1))
    with conv_tile(gpu_ctx, tile):
        got = _np(ore.convolution(gpu_ctx, _t(x), _t(w), _t(b), pads=[1, 1, 1, 1], strides=(1, 1)))
    np.testing.assert_array_equal(got, ref)


def test_conv_reference_kats(gpu_ctx):
    """The reference's own conv test inputs (convolution_op.rs:729-832), integer-exact."""
    import ore
    x1 = np.arange(1, 31, dtype=np.float32).reshape(1, 1, 5, 6)
    w1 = np.arange(1, 11, dtype=np.float32).reshape(1, 1, 5, 2)
    x2 = np.arange(1, 61, dtype=np.float32).reshape(1, 2, 5, 6)
    w2 = np.repeat(np.array([1, 2, 3, 4], dtype=np.float32), 12).reshape(2, 2, 3, 4)
    x3 = np.arange(0, 35, dtype=np.float32).reshape(1, 1, 7, 5)
    w3 = np.arange(1, 25, dtype=np.float32).reshape(2, 1, 3, 4)
    for x, w in ((x1, w1), (x2, w2), (x3, w3)):
        ref = oracle.conv2d(x, w, None, auto_pad="NOTSET", pads=[0, 0, 0, 0], strides=(1, 1))
        got = _np(ore.convolution(gpu_ctx, _t(x), _t(w), None, auto_pad="NOTSET", pads=[0, 0, 0, 0],
                                  strides=(1, 1)))
        np.testing.assert_array_equal(got, ref)


POOL_CASES = [
    # N, C, H, W, k, s, auto_pad, pads
    (2, 5, 9, 9, (3, 3), (2, 2), "VALID", None),
    (1, 96, 109, 109, (3, 3), (2, 2), "NOTSET", [0, 0, 0, 0]),   # pool1
    (2, 16, 54, 54, (3, 3), (2, 2), "NOTSET", [0, 0, 1, 1]),     # pool4 (ceil via pads)
    (2, 16, 54, 54, (3, 3), (2, 2), "VALID", [0, 0, 1, 1]),      # pads ignored without NOTSET
    (1, 8, 28, 28, (2, 2), (2, 2), "NOTSET", [0, 0, 0, 0]),      # MNIST pool 1
    (1, 16, 14, 14, (3, 3), (3, 3), "NOTSET", [0, 0, 0, 0]),     # MNIST pool 2
    (3, 4, 10, 7, (3, 2), (2, 1), "SAME_UPPER", None),
    (3, 4, 10, 7, (4, 4), (3, 2), "SAME_LOWER", None),
    # 3x3 stride-2 rows: the column-strip kernel (bands of 8 output rows)
    (3, 7, 27, 27, (3, 3), (2, 2), "NOTSET", [0, 0, 0, 0]),      # pool8 shape, 13 columns per plane
    (2, 3, 20, 17, (3, 3), (2, 1), "SAME_LOWER", None),
    (2, 5, 35, 30, (3, 3), (2, 3), "NOTSET", [1, 2, 1, 0]),
    (1, 2, 40, 9, (3, 3), (2, 2), "SAME_UPPER", None),
]


@pytest.mark.parametrize("variant", [0, 2, 3, 4, 5])
@pytest.mark.parametrize("case", POOL_CASES)
def test_maxpool(gpu_ctx, case, variant):
    """Every MaxPool kernel (ore_ctx_set_pool_variant: by layout, direct, column strip, plane-LDS,
    chunk-LDS; a variant that does not apply to a shape falls through to the direct kernel)."""
    import ore
    N, C, H, W, k, s, auto_pad, pads = case
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((N, C, H, W)) - 2.0).astype(np.float32)  # mostly negative: zero padding shows
    ref = oracle.maxpool2d(x, k, s, auto_pad=auto_pad, pads=pads)
    with pool_variant(gpu_ctx, variant):
        got = _np(ore.max_pool(gpu_ctx, _t(x), k, s, auto_pad=auto_pad, pads=pads))
    np.testing.assert_array_equal(got, ref)
    with pytest.raises(ore.OreError):
        gpu_ctx.set_pool_variant(1)  # the retired band kernel


def test_relu_reference_kat(gpu_ctx):
    """relu_op.rs:36-50: the only reference test with an expected array."""
    import ore
    x = np.arange(0, 35, dtype=np.float32)
    x[17] = -17.0
    x = x.reshape(1, 1, 7, 5)
    expected = np.arange(0, 35, dtype=np.float32)
    expected[17] = 0.0
    got = _np(ore.relu(gpu_ctx, _t(x)))
    np.testing.assert_array_equal(got.ravel(), expected)


@pytest.mark.parametrize("n", [1, 7, 4096, 4099, 1 << 20])
def test_relu(gpu_ctx, n):
    import ore
    x = np.random.default_rng(n).standard_normal(n).astype(np.float32).reshape(1, 1, 1, n)
    np.testing.assert_array_equal(_np(ore.relu(gpu_ctx, _t(x))), oracle.relu(x))


def test_add(gpu_ctx):
    import ore
    rng = np.random.default_rng(11)
    a = rng.standard_normal((3, 8, 5, 6)).astype(np.float32)
    b = rng.standard_normal((8, 1, 1)).astype(np.float32)
    np.testing.assert_array_equal(_np(ore.add(gpu_ctx, _t(a), _t(b))), oracle.add(a, b))
    a2 = rng.standard_normal((4, 10)).astype(np.float32)
    b2 = rng.standard_normal((1, 10)).astype(np.float32)
    np.testing.assert_array_equal(_np(ore.add(gpu_ctx, _t(a2), _t(b2))), oracle.add(a2, b2))
    with pytest.raises(ore.OreError):
        ore.add(gpu_ctx, _t(a), _t(rng.standard_normal((3, 1, 1)).astype(np.float32)))


def test_softmax_reference_kat(gpu_ctx):
    import ore
    x = np.array([118.85734, 5640.1426, 2., 3., 1000., 1001., 1002., 1003.], dtype=np.float32).reshape(1, 1, 2, 4)
    got = _np(ore.softmax(gpu_ctx, _t(x)))
    ref = oracle.softmax(x)
    np.testing.assert_allclose(got, ref, atol=2e-7, rtol=0)


@pytest.mark.parametrize("rows,d", [(1, 1000), (256, 1000), (3, 7), (5, 8), (2, 17), (3, 64), (3, 255), (3, 256), (3, 257),
                                    (5, 1020), (5, 1024), (5, 1025), (4, 5000), (2, 20000)])
def test_softmax(gpu_ctx, rows, d):
    import ore
    x = (np.random.default_rng(d).standard_normal((rows, d, 1, 1)) * 5).astype(np.float32)
    got = _np(ore.softmax(gpu_ctx, _t(x)))
    ref = oracle.softmax(x)
    assert np.abs(got - ref).max() <= 2e-7
    assert np.array_equal(got.argmax(1), ref.argmax(1))


@pytest.mark.parametrize("m,k,n", [(1, 256, 10), (37, 256, 10), (256, 256, 10), (5, 3, 129)])
def test_matmul(gpu_ctx, m, k, n):
    import ore
    rng = np.random.default_rng(m * 7 + n)
    a = rng.standard_normal((m, k)).astype(np.float32)
    b = rng.standard_normal((k, n)).astype(np.float32)
    ref = oracle.matmul(a, b)
    got = _np(ore.mul(gpu_ctx, _t(a), _t(b)))
    bound = np.abs(a).astype(np.float64) @ np.abs(b).astype(np.float64)
    assert np.all(np.abs(got - ref) <= 2e-6 * bound + 1e-30)


@pytest.mark.parametrize("shape", [(1, 2, 4, 4), (2, 1000, 13, 13), (3, 7, 1, 1), (2, 5, 129, 130)])
def test_gap(gpu_ctx, shape):
    import ore
    x = np.random.default_rng(5).standard_normal(shape).astype(np.float32)
    np.testing.assert_array_equal(_np(ore.global_average_pool(gpu_ctx, _t(x))), oracle.gap(x))


@pytest.mark.parametrize("axis", [1, 2, 3, 0])
def test_concat(gpu_ctx, axis):
    import ore
    rng = np.random.default_rng(axis)
    sa = [2, 3, 4, 5]
    sb = list(sa)
    sb[axis] = 6
    a = rng.standard_normal(sa).astype(np.float32)
    b = rng.standard_normal(sb).astype(np.float32)
    np.testing.assert_array_equal(_np(ore.concatenation(gpu_ctx, _t(a), _t(b), axis)), oracle.concat(a, b, axis))


def test_dropout_reshape(gpu_ctx):
    import ore
    x = np.random.default_rng(1).standard_normal((4, 2, 2, 3)).astype(np.float32)
    np.testing.assert_array_equal(_np(ore.drop_out(gpu_ctx, _t(x), 0.5)), x)
    xt = _t(x)
    y = ore.reshape(xt, [16, 3])   # reshape_op.rs:95-107
    assert tuple(y.shape) == (16, 3) and y.data_ptr() == xt.data_ptr()
    y0 = ore.reshape(xt, [0, 12])  # 0 copies the input dim
    assert tuple(y0.shape) == (4, 12)
    with pytest.raises(ore.OreError):
        ore.reshape(xt, [5, 3])


def test_error_behaviour(gpu_ctx):
    import ore
    x = _t(np.zeros((1, 3, 8, 8), np.float32))
    w = _t(np.zeros((4, 2, 3, 3), np.float32))
    with pytest.raises(ore.OreError, match="group"):          # Cin mismatch (assert, :252)
        ore.convolution(gpu_ctx, x, w, strides=(1, 1))
    w3 = _t(np.zeros((4, 3, 3, 3), np.float32))
    with pytest.raises(ore.OreError):
        ore.convolution(gpu_ctx, x, w3, strides=(1, 1), dilations=(2, 2))
    with pytest.raises(ore.OreError):
        ore.convolution(gpu_ctx, x, w3, strides=(1, 1), group=3)
    with pytest.raises(ore.OreError):                          # bias of the wrong size (:710)
        ore.convolution(gpu_ctx, x, w3, bias=_t(np.zeros(5, np.float32)), strides=(1, 1))
    with pytest.raises(ore.OreError):                          # NOTSET without pads
        ore.max_pool(gpu_ctx, x, (3, 3), (1, 1), auto_pad="NOTSET", pads=None)

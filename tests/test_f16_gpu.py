"""fp16 variant (ORE_LOAD_F16) against the f32 oracle.

The reference has no f16 path, so the bar is the one §8(f)3 states: "tolerance stated against
fp32, plus top-1 agreement".
  * Exactness of the kernels (channels-last layout, gathers, packing, epilogue): small-integer
    data whose every product, partial sum and output is exact in f16/f32 -> the f16 path equals
    the f32 oracle bit for bit (Conv via 1x1, 3x3 and 7x7/s2 geometry; f32 NCHW-input, 16-B NHWC
    and per-element NHWC gathers; all four block tiles; MaxPool; GAP).  read_value returns NCHW.
  * SqueezeNet-1.0 @224 vs the oracle fixture: |p16 - p32| <= 1.5e-2 on the probabilities
    (measured 7.0e-3 at a top probability of 0.62, i.e. ~0.03 on the logits: f16 activations
    carry 2^-11 relative rounding per layer over 26 conv layers) and the same top-1; at batch
    256 vs the f32 GPU path: top-1 agreement >= 97 %.
  * fused == unfused bit for bit (the unfused f16 Relu / Concat / copy kernels are exact)."""
import os

import numpy as np
import pytest

from _knobs import C1_POOL_F16, EPOOL_PATCH, conv_tile, force_tiles

import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _chain_model(x_shape, layers, pool=None):
    """Conv(+Relu) layers [(w, b, pads, strides, relu)], optional MaxPool after the first, then
    GlobalAveragePool (an f16 model's output must be f32)."""
    from ore import onnx_wire as w
    nodes, inits, vinfo = [], [], [w.encode_value_info("x", x_shape)]
    cur = "x"
    for i, (wt, b, pads, strides, relu) in enumerate(layers):
        ins = [cur, f"w{i}"] + ([f"b{i}"] if b is not None else [])
        inits.append(w.encode_tensor(f"w{i}", wt))
        vinfo.append(w.encode_value_info(f"w{i}", wt.shape))
        if b is not None:
            inits.append(w.encode_tensor(f"b{i}", b))
            vinfo.append(w.encode_value_info(f"b{i}", b.shape))
        nodes.append(w.encode_node("Conv", ins, [f"c{i}"], attrs=[w.encode_attr_ints("pads", pads),
                                                                   w.encode_attr_ints("strides", strides)]))
        cur = f"c{i}"
        if relu:
            nodes.append(w.encode_node("Relu", [cur], [f"r{i}"]))
            cur = f"r{i}"
        if i == 0 and pool is not None:
            nodes.append(w.encode_node("MaxPool", [cur], ["p0"], attrs=[
                w.encode_attr_ints("kernel_shape", [3, 3]), w.encode_attr_ints("strides", [2, 2]),
                w.encode_attr_string("auto_pad", "NOTSET"), w.encode_attr_ints("pads", pool)]))
            cur = "p0"
    nodes.append(w.encode_node("GlobalAveragePool", [cur], ["y"]))
    return w.encode_model("t", nodes, inits, vinfo, [w.encode_value_info("y", (1, 1, 1, 1))])


def _ints(rng, lo, hi, shape):
    return rng.integers(lo, hi + 1, size=shape).astype(np.float32)


def _sparse(rng, shape, nonzeros):
    """weights in {-1, 0, 1} with ~`nonzeros` non-zero taps per output channel, so every conv
    output stays a small integer (exact in f16 up to 2048)."""
    fan_in = int(np.prod(shape[1:]))
    keep = rng.random(shape) < min(1.0, nonzeros / fan_in)
    return (rng.choice([-1.0, 1.0], size=shape) * keep).astype(np.float32)


@pytest.mark.parametrize("case", [
    # N, C, H, W, M1, k1, s1, p1, M2, k2   (conv1 reads the f32 input; conv2 reads conv1's f16 output)
    (2, 3, 23, 23, 96, 7, 2, 0, 16, 1),    # conv1-like (96-row tile) -> squeeze 1x1 (32x256 tile)
    (2, 5, 17, 19, 64, 3, 1, 1, 128, 3),   # 64-row tile -> 3x3 gather, 128-row tile
    (3, 8, 9, 9, 20, 1, 1, 0, 130, 3),     # 1x1 on f32 input -> 3x3 on C % 8 != 0 (per-element NHWC), M % 8 != 0
    (2, 3, 31, 29, 8, 3, 2, 1, 40, 3),     # 3x3/s2 -> 3x3 on C = 8 (K = 72: a partial last k stage)
    (1, 4, 12, 12, 24, 5, 1, 2, 16, 3),    # 5x5 pad 2 on 4 channels (odd kw: the PAIR padding tap)
])
def test_f16_conv_exact_integers(gpu_ctx, case):
    """The conv on the f32 input takes the NHWC4 tap-pair gather for C <= 4 (cases 1, 4, 5) and the
    per-element NCHW gather above (cases 2, 3); the second conv the 16-B NHWC LDS-DMA kernel or the
    per-element NHWC gather (C % 8 != 0)."""
    import ore
    N, C, H, W, M1, k1, s1, p1, M2, k2 = case
    rng = np.random.default_rng(hash(case) & 0xffff)
    x = _ints(rng, -2, 2, (N, C, H, W))
    w1, b1 = _sparse(rng, (M1, C, k1, k1), 12), _ints(rng, -4, 4, (M1,))
    w2, b2 = _sparse(rng, (M2, M1, k2, k2), 12), _ints(rng, -4, 4, (M2,))
    p2 = (k2 - 1) // 2
    mb = _chain_model((1, C, H, W), [(w1, b1, [p1] * 4, [s1, s1], False), (w2, b2, [p2] * 4, [1, 1], False)])
    m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f16")
    m.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
    xt = _t(x)
    _np(m.run(xt))
    c0 = oracle.conv2d(x, w1, b1, pads=[p1] * 4, strides=(s1, s1))
    c1 = oracle.conv2d(c0, w2, b2, pads=[p2] * 4, strides=(1, 1))
    assert np.abs(c1).max() < 2048  # every value exact in f16
    np.testing.assert_array_equal(m.read_value("c0"), c0)
    np.testing.assert_array_equal(m.read_value("c1"), c1)
    m.close()


def test_f16_pool_relu_gap_exact(gpu_ctx):
    import ore
    rng = np.random.default_rng(5)
    x = _ints(rng, -3, 3, (2, 4, 29, 29))
    w1, b1 = _ints(rng, -1, 1, (32, 4, 3, 3)), _ints(rng, -8, 8, (32,))
    w2 = _sparse(rng, (8, 32, 1, 1), 8)
    mb = _chain_model((1, 4, 29, 29), [(w1, b1, [1] * 4, [1, 1], True), (w2, None, [0] * 4, [1, 1], False)],
                      pool=[0, 0, 1, 1])
    for fusion in (ore.FUSE_ALL | ore.KEEP_VALUES, ore.KEEP_VALUES, ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES):
        m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f16")
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        r0 = oracle.relu(oracle.conv2d(x, w1, b1, pads=[1] * 4, strides=(1, 1)))
        p0 = oracle.maxpool2d(r0, (3, 3), (2, 2), auto_pad="NOTSET", pads=[0, 0, 1, 1])
        c1 = oracle.conv2d(p0, w2, None, pads=[0] * 4, strides=(1, 1))
        np.testing.assert_array_equal(m.read_value("p0"), p0)
        np.testing.assert_array_equal(m.read_value("c1"), c1)
        np.testing.assert_array_equal(y.reshape(2, 8), oracle.gap(c1).reshape(2, 8))  # exact: f32 sums of ints
        m.close()


@pytest.mark.parametrize("m2", [8, 7])
def test_f16_gap_sequential_sum(gpu_ctx, m2):
    """The f16 GlobalAveragePool is the reference's sequential f32 sum (global_average_pool_op.rs:44-48)
    over the f16 values, bit for bit, on non-integer data (an order-sensitive check)."""
    import ore
    rng = np.random.default_rng(11)
    x = rng.standard_normal((2, 4, 29, 29)).astype(np.float32)
    w1 = (rng.standard_normal((32, 4, 3, 3)) * 0.3).astype(np.float32)
    b1 = rng.standard_normal((32,)).astype(np.float32)
    w2 = (rng.standard_normal((m2, 32, 1, 1)) * 0.2).astype(np.float32)
    mb = _chain_model((1, 4, 29, 29), [(w1, b1, [1] * 4, [1, 1], True), (w2, None, [0] * 4, [1, 1], False)],
                      pool=[0, 0, 1, 1])
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f16")
    m.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
    y = _np(m.run(_t(x))).reshape(2, m2)
    c1 = m.read_value("c1").astype(np.float32)  # the f16 values the GAP reads, [2, m2, 15, 15]
    ref = np.zeros((2, m2), np.float32)
    for n in range(2):
        for c in range(m2):
            s = np.float32(0.0)
            for v in c1[n, c].reshape(-1):
                s = np.float32(s + v)
            ref[n, c] = np.float32(s / np.float32(c1.shape[2] * c1.shape[3]))
    np.testing.assert_array_equal(y, ref)
    m.close()


@pytest.fixture(scope="module")
def squeeze_f16(gpu_ctx):
    import ore
    from ore import squeezenet
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=256, precision="f16")
    yield m
    m.close()


def test_f16_squeezenet_vs_f32_oracle(squeeze_f16):
    from golden.make_golden import squeezenet_inputs
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    y = _np(squeeze_f16.run(_t(squeezenet_inputs())))
    assert y.shape == ref.shape == (2, 1000)
    err = np.abs(y - ref).max()
    print(f"f16 vs f32 oracle: max |dp| = {err:.3e}, max p = {ref.max():.3e}")
    assert err <= 1.5e-2
    assert np.array_equal(y.argmax(1), ref.argmax(1))
    assert np.abs(y.sum(1) - 1.0).max() <= 1e-5


def test_f16_squeezenet_batch256_top1(gpu_ctx, squeeze_f16):
    import ore
    from ore import squeezenet
    x = _t(squeezenet.synthetic_input(256, 224, seed=77))
    y16 = _np(squeeze_f16.run(x))
    m32 = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=256)
    y32 = _np(m32.run(x))
    m32.close()
    agree = float((y16.argmax(1) == y32.argmax(1)).mean())
    print(f"f16 vs f32 top-1 agreement at B=256: {agree:.4f}, max |dp| = {np.abs(y16 - y32).max():.3e}")
    assert agree >= 0.97
    assert np.isfinite(y16).all() and np.abs(y16.sum(1) - 1.0).max() <= 1e-5
    # batching only tiles N: image i alone == image i in the batch, bit for bit
    yi = _np(squeeze_f16.run(x[5:6].contiguous()))
    assert np.array_equal(yi[0], y16[5])


def test_f16_fused_equals_unfused(gpu_ctx):
    import ore
    from ore import squeezenet
    mb = squeezenet.build(64)
    x = _t(squeezenet.synthetic_input(3, 64, seed=9))
    outs = []
    for fusion in (ore.FUSE_ALL, 0):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("shape", [(3, 128, 7, 7, 200, True), (2, 64, 16, 16, 96, False), (1, 192, 1, 1, 33, True),
                                   (2, 128, 13, 13, 1000, True), (1, 64, 11, 11, 130, False), (2, 64, 3, 3, 40, True)])
def test_f16_conv_gap_fused_equals_unfused(gpu_ctx, shape):
    """ORE_FUSE_CONV_GAP (conv1x1_gap_f16_kernel: 1x1 conv + Relu + GlobalAveragePool in one launch) is
    bit-identical to conv_f16 + gap_nhwc_kernel: partial 128-channel blocks, 1-8 pixel fragments, no Relu."""
    import ore
    N, C, H, W, M, relu = shape
    rng = np.random.default_rng(C + M)
    x = rng.standard_normal((N, 8, H, W)).astype(np.float32)
    w0 = (rng.standard_normal((C, 8, 1, 1)) * 0.5).astype(np.float32)
    b0 = rng.standard_normal((C,)).astype(np.float32)
    w1 = (rng.standard_normal((M, C, 1, 1)) * 0.2).astype(np.float32)
    b1 = rng.standard_normal((M,)).astype(np.float32)
    mb = _chain_model((1, 8, H, W), [(w0, b0, [0] * 4, [1, 1], True), (w1, b1, [0] * 4, [1, 1], relu)])
    outs, tiles = [], []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_CONV_GAP):
        m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f16")
        m.set_fusion(fusion)
        outs.append(_np(m.run(_t(x))).reshape(N, M))
        tiles.append([ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0])
        m.close()
    assert "conv1x1 gap f16" in tiles[0] and "conv1x1 gap f16" not in tiles[1]
    np.testing.assert_array_equal(outs[0], outs[1])


def test_f16_conv_gap_squeezenet224(gpu_ctx):
    """SqueezeNet @224 f16: conv10 + relu10 + pool10 fused == unfused, bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(4, 224, seed=21))
    outs = []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_CONV_GAP):
        m = ore.Model(gpu_ctx, mb, max_batch=4, precision="f16")
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def test_f16_rejects_f32_only_ops(gpu_ctx):
    import ore
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        mb = f.read()
    with pytest.raises(ore.OreError, match="f16"):  # Add on a conv output
        ore.Model(gpu_ctx, mb, max_batch=1, precision="f16")
    with pytest.raises(ore.OreError):
        ore.Model(gpu_ctx, mb, max_batch=1, precision="bf16")


@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
def test_f16_tiles_bit_identical(gpu_ctx, cfg):
    """Every block tile of the f16 conv kernels (ore_ctx_set_conv_tile) runs the same MFMA chain as
    the heuristic plan's: equal outputs and intermediate values."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(64)
    x = _t(squeezenet.synthetic_input(3, 64, seed=4))
    outs = []
    for tile in (-1, cfg):
        with conv_tile(gpu_ctx, tile):
            m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
        outs.append((_np(m.run(x)), m.read_value("fire9/concat_1")))
        m.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


def _fire_model_f16(C, H, W, S1, E1, E3, S2, ints=False, seed=0, pool=None):
    # S2 None: no squeeze after the Concat (GAP reads it)
    """squeeze (C -> S1) -> expand 1x1 (E1) / 3x3 pad 1 (E3) -> Concat [-> 3x3 / stride-2 MaxPool with
    pads `pool`] -> squeeze (S2) -> GAP, all Relu; ints: sparse {-1, 0, 1} weights and small integer
    biases (every value exact in f16).  Returns (model bytes, {name: (w, b)})."""
    from ore import onnx_wire as wr
    rng = np.random.default_rng(seed + C * 7 + H + W + S1 + E1 + E3 + (S2 or 0))
    shapes = {"wq": (S1, C, 1, 1), "w1": (E1, S1, 1, 1), "w3": (E3, S1, 3, 3)}
    if S2 is not None:
        shapes["wn"] = (S2, E1 + E3, 1, 1)
    params, inits, vinfo = {}, [], [wr.encode_value_info("x", (1, C, H, W))]
    for n, shp in shapes.items():
        if ints:
            w, b = _sparse(rng, shp, 8), _ints(rng, -4, 4, (shp[0],))
        else:
            fan = shp[1] * shp[2] * shp[3]
            w = (rng.standard_normal(shp) * np.sqrt(2.0 / fan)).astype(np.float32)
            b = rng.uniform(-0.1, 0.1, shp[0]).astype(np.float32)
        params[n] = (w, b)
        inits += [wr.encode_tensor(n, w), wr.encode_tensor("b" + n, b)]
        vinfo += [wr.encode_value_info(n, w.shape), wr.encode_value_info("b" + n, b.shape)]
    conv = lambda i, w, o, pads: wr.encode_node("Conv", [i, w, "b" + w], [o], attrs=[
        wr.encode_attr_ints("pads", pads), wr.encode_attr_ints("strides", [1, 1])])
    nodes = [conv("x", "wq", "q", [0] * 4), wr.encode_node("Relu", ["q"], ["qr"]),
             conv("qr", "w1", "e1", [0] * 4), wr.encode_node("Relu", ["e1"], ["e1r"]),
             conv("qr", "w3", "e3", [1] * 4), wr.encode_node("Relu", ["e3"], ["e3r"]),
             wr.encode_node("Concat", ["e1r", "e3r"], ["cat"], attrs=[wr.encode_attr_int("axis", 1)])]
    if pool is not None:
        nodes.append(wr.encode_node("MaxPool", ["cat"], ["pc"], attrs=[
            wr.encode_attr_ints("kernel_shape", [3, 3]), wr.encode_attr_ints("strides", [2, 2]),
            wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pool)]))
    if S2 is None:  # the Concat read by something other than a squeeze (GAP): fire_f16_kernel's Concat form
        nodes.append(wr.encode_node("GlobalAveragePool", ["cat"], ["y"]))
        return wr.encode_model("fire", nodes, inits, vinfo, [wr.encode_value_info("y", (1, E1 + E3, 1, 1))]), params
    nodes += [conv("pc" if pool is not None else "cat", "wn", "n", [0] * 4), wr.encode_node("Relu", ["n"], ["nr"]),
              wr.encode_node("GlobalAveragePool", ["nr"], ["y"])]
    return wr.encode_model("fire", nodes, inits, vinfo, [wr.encode_value_info("y", (1, S2, 1, 1))]), params


FIRE_F16_CASES = [
    # C, H, W, S1, E1, E3, S2 -> fire_f16_kernel<S1 / 16, ceil(S2 / 32)>
    (16, 12, 12, 16, 64, 64, 16),     # fire2 -> squeeze3 family, one tile per image
    (32, 9, 8, 32, 128, 128, 48),     # fire5 -> squeeze6 (48 of 64 squeeze rows), W = 8
    (24, 8, 7, 48, 192, 192, 64),     # fire7 -> squeeze8, W = 7
    (16, 13, 13, 64, 64, 128, 32),    # C = 64, unequal expands, 13 x 13
    (8, 54, 54, 16, 64, 64, 32),      # SqueezeNet fire3 plane: 12 tiles per image, tile edges mid-row
    (16, 27, 27, 48, 192, 192, 48),   # fire6 plane: 3 tiles, the last partial
]


@pytest.mark.parametrize("case", FIRE_F16_CASES)
def test_f16_fire_fusion_bit_identical(gpu_ctx, case):
    """f16 models: expand 1x1 + expand 3x3 + Concat + the next squeeze in one fire_f16_kernel launch
    equals the three separate conv_f16_kernel launches bit for bit; the concat is never stored."""
    import ore
    C, H, W = case[:3]
    mb, _ = _fire_model_f16(*case)
    x = np.random.default_rng(sum(case)).standard_normal((3, C, H, W)).astype(np.float32)
    vals = []
    for fusion in (ore.FUSE_ALL | ore.KEEP_VALUES, (ore.FUSE_ALL & ~ore.FUSE_FIRE) | ore.KEEP_VALUES):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("nr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert ("fire f16" in names) == bool(fusion & ore.FUSE_FIRE)
        if fusion & ore.FUSE_FIRE:
            with pytest.raises(ore.OreError):
                m.read_value("cat")  # never materialised
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    assert np.abs(vals[0][1]).max() > 0  # not a dead (all-Relu-zero) module


FIRE_F16_CONCAT_CASES = [
    # C, H, W, S1, E1, E3 -> fire_f16_kernel<S1 / 16, 0> (no squeeze: the kernel stores the Concat)
    (8, 13, 13, 16, 64, 96),      # S1 = 16, unequal expands, 169 pixels (one partial 256-pixel tile)
    (16, 10, 11, 32, 128, 64),    # S1 = 32, E1 > E3, 110 pixels
    (24, 9, 7, 48, 96, 192),      # S1 = 48, W = 7, 63 pixels
    (16, 27, 27, 64, 128, 256),   # S1 = 64 (SqueezeNet fire9's instance), 3 tiles per image, the last partial
]


@pytest.mark.parametrize("case", FIRE_F16_CONCAT_CASES)
def test_f16_fire_concat_form_bit_identical(gpu_ctx, case):
    """fire_f16_kernel's no-squeeze form (planner pass 6b) -- expands + Concat in one launch,
    the Concat read by a non-squeeze (GAP here, conv10 in SqueezeNet) -- equals the two separate
    conv_f16 launches bit for bit (the Concat itself and the GAP of it), at every squeeze width 16 / 32 /
    48 / 64, unequal expands and plane sizes that are not a multiple of the 256-pixel tile."""
    import ore
    C, H, W, S1, E1, E3 = case
    mb, _ = _fire_model_f16(C, H, W, S1, E1, E3, None)
    x = np.random.default_rng(sum(case)).standard_normal((3, C, H, W)).astype(np.float32)
    vals = []
    for fusion in (ore.FUSE_ALL | ore.KEEP_VALUES, (ore.FUSE_ALL & ~ore.FUSE_FIRE) | ore.KEEP_VALUES):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        vals.append((y, m.read_value("cat"), names))
        m.close()
    assert "fire f16" in vals[0][2] and "fire f16" not in vals[1][2], (vals[0][2], vals[1][2])
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    assert np.isfinite(vals[0][0]).all() and vals[0][1].shape == (3, E1 + E3, H, W)


@pytest.mark.parametrize("case", [FIRE_F16_CASES[1], FIRE_F16_CASES[4]])
def test_f16_fire_fusion_exact_integers(gpu_ctx, case):
    """Small-integer weights / biases / input: every product and sum of the fused module is exact in
    f16 / f32, so the fused f16 kernel equals the f32 oracle bit for bit (checks the permuted
    packings, the halo staging and the tap offsets independently of the unfused kernels)."""
    import ore
    C, H, W, S1, E1, E3, S2 = case
    mb, prm = _fire_model_f16(*case, ints=True, seed=3)
    x = _ints(np.random.default_rng(11), -2, 2, (2, C, H, W))
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f16")
    m.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
    _np(m.run(_t(x)))
    assert "fire f16" in [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
    q = oracle.relu(oracle.conv2d(x, *prm["wq"], pads=[0] * 4, strides=(1, 1)))
    e1 = oracle.relu(oracle.conv2d(q, *prm["w1"], pads=[0] * 4, strides=(1, 1)))
    e3 = oracle.relu(oracle.conv2d(q, *prm["w3"], pads=[1] * 4, strides=(1, 1)))
    n = oracle.relu(oracle.conv2d(np.concatenate([e1, e3], 1), *prm["wn"], pads=[0] * 4, strides=(1, 1)))
    assert np.abs(n).max() < 2048 and np.abs(n).max() > 0
    np.testing.assert_array_equal(m.read_value("nr"), n)
    m.close()


def test_f16_squeezenet_fire_fusion(gpu_ctx):
    """SqueezeNet-1.0 @224, f16: the five fire + squeeze pairs run fire_f16_kernel, fire4 / fire8 with
    their MaxPool and the next squeeze fire_pool_f16_kernel, fire9 (read by conv10, no squeeze)
    fire_f16_kernel's Concat-writing form, and the probabilities equal the unfused graph's bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=21))
    outs = []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_FIRE):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        n = sum(1 for t in m.tiles() if t >= 0 and ore.Model.TILE_NAMES[t] == "fire f16")
        assert n == (8 if fusion & ore.FUSE_FIRE else 0)  # + fire4 -> pool3 -> fire5, fire8 -> pool5 -> fire9, fire9
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


FIRE_POOL_F16_CASES = [
    # C, H, W, S1, E1, E3, S2, pool pads
    (16, 54, 54, 32, 128, 128, 32, [0, 0, 1, 1]),   # SqueezeNet fire4 -> pool3 -> fire5
    (32, 27, 27, 64, 256, 256, 64, [0, 0, 1, 1]),   # fire8 -> pool5 -> fire9
    (8, 13, 15, 16, 64, 96, 48, [1, 1, 1, 1]),      # padded on all sides, unequal expands, 48 squeeze rows
    (8, 9, 8, 48, 32, 64, 16, [0, 0, 0, 0]),        # floor-mode pool, C = 48
    (8, 38, 33, 32, 64, 64, 24, [0, 0, 1, 1]),      # 4 bands of 5 pooled rows, the last 4
]


@pytest.mark.parametrize("case", FIRE_POOL_F16_CASES)
def test_f16_fire_pool_fusion_bit_identical(gpu_ctx, case):
    """f16: expand 1x1 + expand 3x3 + Concat + MaxPool + the next squeeze in one fire_pool_f16_kernel
    launch equals the separate kernels bit for bit; neither the concat nor the pooled map is stored."""
    import ore
    C, H, W = case[:3]
    mb, _ = _fire_model_f16(*case[:7], pool=case[7])
    x = np.random.default_rng(sum(case[:7])).standard_normal((3, C, H, W)).astype(np.float32)
    vals = []
    for fusion in (ore.FUSE_ALL | ore.KEEP_VALUES, (ore.FUSE_ALL & ~ore.FUSE_FIRE) | ore.KEEP_VALUES):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("nr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert ("fire f16" in names) == bool(fusion & ore.FUSE_FIRE)
        if fusion & ore.FUSE_FIRE:
            for v in ("cat", "pc"):
                with pytest.raises(ore.OreError):
                    m.read_value(v)  # never materialised
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    assert np.abs(vals[0][1]).max() > 0


@pytest.mark.parametrize("case", [FIRE_POOL_F16_CASES[0], FIRE_POOL_F16_CASES[2]])
def test_f16_fire_pool_fusion_exact_integers(gpu_ctx, case):
    """Small-integer data: the pooled fused kernel equals the f32 oracle (conv, Relu, Concat, the
    reference's MaxPool, conv) bit for bit."""
    import ore
    C, H, W, S1, E1, E3, S2, pads = case
    mb, prm = _fire_model_f16(*case[:7], ints=True, seed=5, pool=pads)
    x = _ints(np.random.default_rng(13), -2, 2, (2, C, H, W))
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f16")
    m.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
    _np(m.run(_t(x)))
    assert "fire f16" in [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
    q = oracle.relu(oracle.conv2d(x, *prm["wq"], pads=[0] * 4, strides=(1, 1)))
    e1 = oracle.relu(oracle.conv2d(q, *prm["w1"], pads=[0] * 4, strides=(1, 1)))
    e3 = oracle.relu(oracle.conv2d(q, *prm["w3"], pads=[1] * 4, strides=(1, 1)))
    pc = oracle.maxpool2d(np.concatenate([e1, e3], 1), (3, 3), (2, 2), auto_pad="NOTSET", pads=pads)
    n = oracle.relu(oracle.conv2d(pc, *prm["wn"], pads=[0] * 4, strides=(1, 1)))
    assert np.abs(n).max() < 2048 and np.abs(n).max() > 0
    np.testing.assert_array_equal(m.read_value("nr"), n)
    m.close()


C1POOL_CASES = [
    # N, C, H, W, M, k, stride, pad, pool pads
    (2, 3, 67, 71, 96, 7, 2, 0, [0, 0, 0, 0]),   # SqueezeNet conv1 + pool1 geometry, partial tiles
    (3, 1, 40, 33, 64, 7, 2, 0, [0, 0, 1, 1]),   # one channel, ceil-mode pool
    (2, 4, 29, 30, 40, 3, 2, 2, [1, 1, 1, 1]),   # 3x3 (PAIR padding tap), M % 32 != 0, padded pool
    (1, 3, 47, 45, 128, 3, 2, 2, [0, 0, 1, 1]),  # 4 channel fragments (3x3: the weights fit LDS)
]


@pytest.mark.parametrize("case", C1POOL_CASES)
def test_f16_first_conv_pool_fused_bit_identical(gpu_ctx, case):
    """f16 first conv (f32 NCHW input, <= 4 channels) + Relu + 3x3/s2 MaxPool: the one-launch kernel
    (conv_pair_pool_f16_kernel, reads the f32 input itself) equals the two-launch path (NHWC4
    conversion + conv_f16_kernel with the pooled epilogue) bit for bit."""
    import ore
    N, C, H, W, M, k, st, pd, pp = case
    rng = np.random.default_rng(sum(case[:8]))
    x = (rng.standard_normal((N, C, H, W)) * 20).astype(np.float32)
    w1 = (rng.standard_normal((M, C, k, k)) * np.sqrt(2.0 / (C * k * k))).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    w2 = (rng.standard_normal((16, M, 1, 1)) * np.sqrt(2.0 / M)).astype(np.float32)
    mb = _chain_model((1, C, H, W), [(w1, b1, [pd] * 4, [st, st], True), (w2, None, [0] * 4, [1, 1], False)], pool=pp)
    vals = []
    for on in ("1", "0"):
        m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f16")
        m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)  # eager: pooled epilogue at small planes
        assert force_tiles(m, C1_POOL_F16 if on == "1" else EPOOL_PATCH) == 1  # one launch / conversion + patch
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("p0"), m.read_value("c1")))
        assert ("first conv pool f16" in [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]) == (on == "1")
        m.close()
    for a, b in zip(vals[0], vals[1]):
        np.testing.assert_array_equal(a, b)
    assert np.abs(vals[0][1]).max() > 0


def test_f16_first_conv_pool_exact_integers(gpu_ctx):
    """Small integers: the one-launch first conv + pool equals the f32 oracle bit for bit."""
    import ore
    rng = np.random.default_rng(8)
    x = _ints(rng, -3, 3, (2, 3, 51, 49))
    w1, b1 = _sparse(rng, (96, 3, 7, 7), 16), _ints(rng, -8, 8, (96,))
    w2 = _sparse(rng, (8, 96, 1, 1), 8)
    mb = _chain_model((1, 3, 51, 49), [(w1, b1, [0] * 4, [2, 2], True), (w2, None, [0] * 4, [1, 1], False)],
                      pool=[0, 0, 1, 1])
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f16")
    m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)
    _np(m.run(_t(x)))
    assert ore.Model.TILE_NAMES[m.tiles()[0]] == "first conv pool f16"
    r0 = oracle.relu(oracle.conv2d(x, w1, b1, pads=[0] * 4, strides=(2, 2)))
    p0 = oracle.maxpool2d(r0, (3, 3), (2, 2), auto_pad="NOTSET", pads=[0, 0, 1, 1])
    np.testing.assert_array_equal(m.read_value("p0"), p0)
    m.close()


def test_f16_squeezenet_first_conv_pool_fused(gpu_ctx):
    """SqueezeNet-1.0 @224 f16: probabilities with the one-launch conv1 + pool1 equal the two-launch
    path's bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=23))
    outs = []
    for on in ("1", "0"):
        m = ore.Model(gpu_ctx, mb, max_batch=3, precision="f16")
        if on == "0":  # the two-launch first conv (and so no squeeze inside it)
            m.set_fusion(ore.FUSE_ALL & ~ore.FUSE_FIRST_SQUEEZE)
            assert force_tiles(m, EPOOL_PATCH) == 1
        outs.append(_np(m.run(x)))
        assert (ore.Model.TILE_NAMES[m.tiles()[0]] == "first conv pool f16") == (on == "1")
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("case", [
    # N, H, W, M, pool pads, squeeze channels
    (2, 67, 71, 96, [0, 0, 0, 0], 16),   # SqueezeNet conv1 + pool1 + fire2/squeeze1x1 family
    (3, 40, 33, 64, [0, 0, 1, 1], 32),   # two channel fragments in, 32 out, ceil-mode pool
    (2, 45, 52, 96, [1, 1, 1, 1], 24),   # padded pool, 24 squeeze channels (a partial store group)
])
def test_f16_first_conv_pool_squeeze_fused(gpu_ctx, case):
    """The first conv + Relu + MaxPool + the next 1x1 conv + Relu in one launch (the pooled map never
    stored) equals the two-launch first conv + the separate squeeze bit for bit."""
    import ore
    N, H, W, M, pp, Q = case
    rng = np.random.default_rng(sum(case[:4]) + Q)
    x = (rng.standard_normal((N, 3, H, W)) * 20).astype(np.float32)
    w1 = (rng.standard_normal((M, 3, 7, 7)) * np.sqrt(2.0 / 147)).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    w2 = (rng.standard_normal((Q, M, 1, 1)) * np.sqrt(2.0 / M)).astype(np.float32)
    b2 = rng.uniform(-0.1, 0.1, Q).astype(np.float32)
    mb = _chain_model((1, 3, H, W), [(w1, b1, [0] * 4, [2, 2], True), (w2, b2, [0] * 4, [1, 1], True)], pool=pp)
    vals = []
    for on in ("1", "0"):
        m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f16")
        fusion = ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_FIRST_SQUEEZE
        m.set_fusion(fusion | ore.FUSE_EAGER | ore.KEEP_VALUES)
        if on == "0":
            assert force_tiles(m, EPOOL_PATCH) == 1  # the two-launch first conv
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("r1")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        if on == "1":
            assert names == ["first conv pool f16"], names  # one conv launch: the squeeze is inside
            with pytest.raises(ore.OreError):
                m.read_value("p0")  # the pooled map is never stored
        else:
            assert len(names) == 2, names
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    assert np.abs(vals[0][1]).max() > 0


@pytest.mark.parametrize("case", [
    # N, H, W, squeeze channels
    (3, 224, 224, 16),   # SqueezeNet conv1 + pool1 + fire2/squeeze1x1 (28 steps, the last with one conv row)
    (2, 113, 100, 32),   # odd conv rows / columns, 32 squeeze channels (two store groups)
    (300, 64, 72, 24),   # more images than workgroups (a workgroup walks several), 24 channels (a partial group)
])
def test_f16_conv1_band_bit_identical(gpu_ctx, case):
    """Round 6: the f16 band walker (conv_band_pool_f16_kernel, tile "epool band f16") equals the patch kernel
    ("first conv pool f16") bit for bit on the fused first conv + Relu + MaxPool + squeeze + Relu: the same
    operands, k order and MFMA chains, the max of the same nine f16 values, the same squeeze chain."""
    import ore
    N, H, W, Q = case
    rng = np.random.default_rng(N + H + W + Q)
    x = (rng.standard_normal((N, 3, H, W)) * 20).astype(np.float32)
    w1 = (rng.standard_normal((96, 3, 7, 7)) * np.sqrt(2.0 / 147)).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, 96).astype(np.float32)
    w2 = (rng.standard_normal((Q, 96, 1, 1)) * np.sqrt(2.0 / 96)).astype(np.float32)
    b2 = rng.uniform(-0.1, 0.1, Q).astype(np.float32)
    mb = _chain_model((1, 3, H, W), [(w1, b1, [0] * 4, [2, 2], True), (w2, b2, [0] * 4, [1, 1], True)], pool=[0] * 4)
    vals = []
    for name in ("first conv pool f16", "epool band f16"):
        m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f16")
        m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)
        m.set_tile(0, ore.Model.TILE_NAMES.index(name))
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("r1")))
        assert [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0] == [name]
        m.close()
    np.testing.assert_array_equal(vals[1][1], vals[0][1])
    np.testing.assert_array_equal(vals[1][0], vals[0][0])
    assert np.abs(vals[0][1]).max() > 0


def test_f16_squeezenet_conv1_band(gpu_ctx):
    """SqueezeNet-1.0 @224 f16 at max_batch 256 (config 5's plan): the untuned plan takes the band walker for
    conv1 + pool1 + fire2/squeeze1x1, and the probabilities equal the patch kernel's bit for bit."""
    import ore
    import torch
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(4, 224, seed=29))
    x = torch.cat([x] * 64).contiguous()
    outs = []
    for name in ("epool band f16", "first conv pool f16"):
        m = ore.Model(gpu_ctx, mb, max_batch=256, precision="f16")
        if name == "first conv pool f16":
            m.set_tile(0, ore.Model.TILE_NAMES.index(name))
        outs.append(_np(m.run(x)))
        assert ore.Model.TILE_NAMES[m.tiles()[0]] == name, ore.Model.TILE_NAMES[m.tiles()[0]]
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])

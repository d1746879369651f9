"""Graph-level parity: the device walker (ore_model_*, replacing inference()/node_inference())
against the reference's golden vectors and the oracle's committed fixtures.

  MNIST-8 (real CNTK weights) vs mnist_output_0.pb: |d| <= 1e-6 * max|y| (1-4 ulp of the logits)
  synthetic SqueezeNet-1.0 @224 vs oracle fixture: <= 1e-5 max-abs on the softmax probabilities
  full-size properties at batch 256: rows sum to 1, per-image results bit-identical to the same
  images run alone (no cross-image arithmetic), fused == unfused bit for bit."""
import functools
import os

import numpy as np
import pytest

from ore import FUSE_ALL, FUSE_EAGER, FUSE_FIRE

from _knobs import (EPOOL_PATCH, EPOOL_WALK48, EPOOL_WALK64, EPOOL_WALK64_B3, EPOOL_WALK96, EPOOL_WINDOW, conv_tile,
                    force_tiles)

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


def _model(ctx, mb, *args, **kw):
    """These tests pin the direct kernels and their fusions (bit-identical to the unfused graph): every
    model loads with ORE_LOAD_NO_WINOGRAD.  The Winograd 3x3 path, on by default for f32 models, has
    its own parity tests (tests/test_wino_gpu.py)."""
    import ore
    return ore.Model(ctx, mb, *args, winograd=False, **kw)


def _mnist_bytes():
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def squeeze224(gpu_ctx):
    import ore
    from ore import squeezenet
    m = _model(gpu_ctx, squeezenet.build(224), max_batch=256)
    yield m
    m.close()


@pytest.mark.parametrize("fusion", [FUSE_ALL | FUSE_EAGER, FUSE_ALL, 7, 0])  # 7: relu + concat + alias; 0 unfused
def test_mnist_golden(gpu_ctx, fusion):
    import ore
    from ore import onnx_wire
    m = _model(gpu_ctx, _mnist_bytes(), max_batch=4)
    m.set_fusion(fusion)
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_output_0.pb")).to_numpy()
    y = _np(m.run(_t(x)))
    assert y.shape == (1, 10)
    assert np.abs(y - g).max() <= 1e-6 * np.abs(g).max()
    assert y.argmax() == g.argmax() == 2
    m.close()


def test_mnist_oracle_batch(gpu_ctx):
    import ore
    from golden.make_golden import mnist_inputs
    ref = np.load(os.path.join(GOLD, "mnist_oracle.npz"))["output"]
    m = _model(gpu_ctx, _mnist_bytes(), max_batch=8)
    y = _np(m.run(_t(mnist_inputs())))
    assert np.abs(y - ref).max() <= 1e-6 * np.abs(ref).max()
    m.close()


def test_inference_entry_point():
    """ore.inference() mirrors the reference's inference(model, input_data, names)."""
    import ore
    from ore import onnx_wire
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy().ravel()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_output_0.pb")).to_numpy()
    y = ore.inference(_mnist_bytes(), x, ["Input3", "Parameter193"])
    assert np.abs(y - g).max() <= 1e-6 * np.abs(g).max()


def test_squeezenet_synth_vs_oracle(squeeze224):
    from golden.make_golden import squeezenet_inputs
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    y = _np(squeeze224.run(_t(squeezenet_inputs())))
    assert y.shape == ref.shape == (2, 1000)
    assert np.abs(y - ref).max() <= 1e-5
    assert np.array_equal(y.argmax(1), ref.argmax(1))


@pytest.mark.parametrize("fusion", [FUSE_ALL | FUSE_EAGER, FUSE_ALL, 7, 0, 1, 2, 4, 32, FUSE_ALL & ~FUSE_FIRE])
def test_squeezenet_mini_vs_oracle(gpu_ctx, fusion):
    import ore
    from ore import squeezenet
    from golden.make_golden import mini_inputs
    ref = np.load(os.path.join(GOLD, "squeezenet_mini_oracle.npz"))["output"]
    m = _model(gpu_ctx, squeezenet.build(64), max_batch=4)
    m.set_fusion(fusion)
    y = _np(m.run(_t(mini_inputs())))
    assert np.abs(y - ref).max() <= 1e-5
    m.close()


def test_squeezenet_node_level_parity(gpu_ctx):
    """Unfused run: every intermediate value vs the oracle op applied to the GPU's own input of
    that node (isolates each op's error from the accumulated one)."""
    import ore
    import oracle
    from ore import onnx_wire, squeezenet
    from golden.make_golden import mini_inputs
    mb = squeezenet.build(64)
    model = onnx_wire.decode_model(mb)
    inits = {t.name: t.to_numpy() for t in model.graph.initializer}
    m = _model(gpu_ctx, mb, max_batch=4)
    m.set_fusion(ore.KEEP_VALUES)  # unfused, and no storage reuse so every value can be read back
    xt = _t(mini_inputs()[:2])  # kept alive: read_value of the model input reads this buffer
    _np(m.run(xt))
    for node in model.graph.node:
        a = node.attrs()
        x = m.read_value(node.input[0])
        y = m.read_value(node.output[0])
        if node.op_type == "Conv":
            w, b = inits[node.input[1]], inits[node.input[2]]
            ref = oracle.conv2d(x, w, b, pads=a["pads"].ints, strides=a["strides"].ints)
            scale = np.abs(ref).max() + 1.0
            assert np.abs(y - ref).max() <= 1e-5 * scale, node.name
        elif node.op_type == "Relu":
            np.testing.assert_array_equal(y, oracle.relu(x))
        elif node.op_type == "MaxPool":
            ref = oracle.maxpool2d(x, a["kernel_shape"].ints, a["strides"].ints, auto_pad=a["auto_pad"].s.decode(),
                                   pads=a["pads"].ints)
            np.testing.assert_array_equal(y, ref)
        elif node.op_type == "Concat":
            np.testing.assert_array_equal(y, oracle.concat(x, m.read_value(node.input[1]), 1))
        elif node.op_type == "Dropout":
            np.testing.assert_array_equal(y, x)
        elif node.op_type == "GlobalAveragePool":
            np.testing.assert_array_equal(y, oracle.gap(x))
        elif node.op_type == "Softmax":
            assert np.abs(y - oracle.softmax(x)).max() <= 2e-7
    m.close()


@pytest.mark.parametrize("hw", [64, 224])
def test_fused_padded_layout_values(gpu_ctx, hw):
    """Fused graph (conv->relu epilogue, concat in place, 128-B padded channel planes): every
    value it materialises equals the unfused dense run's value bit for bit."""
    import ore
    from ore import onnx_wire, squeezenet
    mb = squeezenet.build(hw)
    model = onnx_wire.decode_model(mb)
    xt = _t(squeezenet.synthetic_input(3, hw, seed=31))
    ref = _model(gpu_ctx, mb, max_batch=3)
    ref.set_fusion(ore.KEEP_VALUES)
    _np(ref.run(xt))
    fused = _model(gpu_ctx, mb, max_batch=3)
    fused.set_fusion(ore.FUSE_ALL | ore.KEEP_VALUES)
    _np(fused.run(xt))
    checked = 0
    for node in model.graph.node:
        try:
            y = fused.read_value(node.output[0])
        except ore.OreError:
            continue  # fused away (conv output feeding its relu)
        np.testing.assert_array_equal(y, ref.read_value(node.output[0]), err_msg=node.output[0])
        checked += 1
    # @224 conv1's relu output is fused into pool1, pool1 into fire2's squeeze and fire4's expand
    # outputs and concat into pool3; pool5 (both sizes) into fire9's squeeze
    assert checked >= (33 if hw == 224 else 37)
    ref.close()
    fused.close()


def test_squeezenet_batch256_properties(squeeze224):
    """Full benchmark size: size-independent properties (no oracle run at B=256)."""
    import torch
    from ore import squeezenet
    x = squeezenet.synthetic_input(256, 224, seed=123)
    xt = _t(x)
    y = _np(squeeze224.run(xt))
    assert y.shape == (256, 1000) and np.isfinite(y).all()
    assert np.abs(y.sum(1) - 1.0).max() <= 1e-5
    # image i of the batch == image i run alone, bit for bit (batch only tiles the N dim)
    for i in (0, 1, 128, 255):
        yi = _np(squeeze224.run(xt[i:i + 1].contiguous()))
        assert np.array_equal(yi[0], y[i]), i
    # fused and unfused graphs compute identical values
    import ore
    squeeze224.set_fusion(0)
    y0 = _np(squeeze224.run(xt))
    squeeze224.set_fusion(ore.FUSE_ALL)
    assert np.array_equal(y0, y)
    torch.cuda.synchronize()


@pytest.mark.parametrize("precision", ["f32", "f16"])
@pytest.mark.parametrize("hw", [64, 224])
def test_forced_tiles_bit_identical(gpu_ctx, precision, hw):
    """Every conv tile forced through ore_ctx_set_conv_tile (the four LDS-staged tiles, and for f32 two
    streaming ones) gives the heuristic plan's results bit for bit, eager fusions included."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(hw)
    x = _t(squeezenet.synthetic_input(3, hw, seed=13))
    outs = []
    tiles = [None, 2, 3, 1, 0] + ([12, 14] if precision == "f32" else [])
    for tile in tiles:
        with conv_tile(gpu_ctx, -1 if tile is None else tile):
            m = _model(gpu_ctx, mb, max_batch=3, precision=precision)
        m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER)
        outs.append(_np(m.run(x)))
        m.close()
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])
    with pytest.raises(ore.OreError):
        gpu_ctx.set_conv_tile(5)  # a retired tile id


@pytest.mark.parametrize("precision", ["f32", "f16"])
def test_autotune_keeps_results(gpu_ctx, precision):
    """ore_model_autotune only changes block tiles: outputs stay bit-identical."""
    import torch
    import ore
    from ore import squeezenet
    m = _model(gpu_ctx, squeezenet.build(224), max_batch=8, precision=precision)
    x = _t(squeezenet.synthetic_input(8, 224, seed=21))
    before = _np(m.run(x))
    tiles0 = m.tiles()
    out = torch.empty_like(torch.from_numpy(before)).cuda()
    m.autotune(x, out, reps=2)
    np.testing.assert_array_equal(_np(out), before)  # the autotune pass leaves a real result
    np.testing.assert_array_equal(_np(m.run(x)), before)
    tiles1 = m.tiles()
    # f32 at batch 8: 25 conv launches (conv1 + pool1 + fire2's squeeze in one; the fire fusion waits
    # for >= 65536 columns); f16: 10 (conv1 + pool1 + fire2's squeeze, 5 fused fire modules, 2 fire +
    # pool + squeeze, fire9's expands + Concat, conv10 + relu10 + pool10)
    assert len(tiles1) == len(tiles0) and sum(t >= 0 for t in tiles1) == (25 if precision == "f32" else 10)
    m.set_fusion(ore.FUSE_ALL)  # the choice survives re-planning
    a, b = [t for t in tiles1 if t >= 0], [t for t in m.tiles() if t >= 0]
    # convs with a pooled epilogue (conv1 + pool1, fire4 / fire8 expands + pool3 / pool5): their kernel
    # choice (patch vs row walk) has no unfused counterpart
    ep = ore.Model.TILE_NAMES.index("epool patch")
    assert len(a) == len(b) and [x for x, y in zip(a, b) if x < ep] == [y for x, y in zip(a, b) if x < ep]
    np.testing.assert_array_equal(_np(m.run(x)), before)
    m.close()


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(HERE), "models", "squeezenet1.0-8.onnx")),
                    reason="real squeezenet1.0-8.onnx is not in the repo (stripped from the reference mirror)")
def test_real_squeezenet_golden(gpu_ctx):
    import ore
    from ore import onnx_wire
    path = os.path.join(os.path.dirname(HERE), "models", "squeezenet1.0-8.onnx")
    with open(path, "rb") as f:
        m = _model(gpu_ctx, f.read(), max_batch=1)
    x = onnx_wire.load_tensor(os.path.join(GOLD, "squeezenet_data_0.pb")).to_numpy()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "squeezenet_output_0.pb")).to_numpy().reshape(1, -1)
    y = _np(m.run(_t(x)))
    assert np.abs(y - g).max() <= 1e-5


def test_model_errors(gpu_ctx):
    import ore
    from ore import onnx_wire as w
    def model(nodes, inits=(), extra_inputs=()):
        return w.encode_model("t", nodes, [w.encode_tensor(n, a) for n, a in inits],
                              [w.encode_value_info("x", (1, 2, 4, 4))] + list(extra_inputs),
                              [w.encode_value_info("y", (1, 2, 4, 4))])
    with pytest.raises(ore.OreError, match="NOT FOUND"):
        _model(gpu_ctx, model([w.encode_node("Sigmoid", ["x"], ["y"])]), 1)
    with pytest.raises(ore.OreError, match="CONCATENATE"):
        _model(gpu_ctx, model([w.encode_node("Concat", ["x", "x"], ["y"], attrs=[w.encode_attr_int("bogus", 1)])]), 1)
    wt = np.zeros((2, 2, 3, 3), np.float32)
    with pytest.raises(ore.OreError, match="Auto Pad"):  # Conv accepts NOT_SET, not NOTSET
        _model(gpu_ctx, model([w.encode_node("Conv", ["x", "w"], ["y"], attrs=[
            w.encode_attr_string("auto_pad", "NOTSET"), w.encode_attr_ints("strides", [1, 1])])], [("w", wt)]), 1)
    with pytest.raises(ore.OreError):
        _model(gpu_ctx, b"\xff\xff\xff", 1)


def _conv_pool_model(x_shape, w, b, conv_pads, conv_strides, relu, pool_k, pool_s, pool_pads, pre_relu=False):
    """x [-> Relu] -> Conv [-> Relu] -> MaxPool -> GAP.  pre_relu puts the conv input in the walker's
    arena (mapped bytes before it, as for every inner layer of a real graph)."""
    from ore import onnx_wire as wr
    nodes = [wr.encode_node("Relu", ["x"], ["xr"])] if pre_relu else []
    nodes.append(wr.encode_node("Conv", ["xr" if pre_relu else "x", "w", "b"], ["c"], attrs=[
        wr.encode_attr_ints("pads", conv_pads), wr.encode_attr_ints("strides", conv_strides)]))
    cur = "c"
    if relu:
        nodes.append(wr.encode_node("Relu", ["c"], ["r"]))
        cur = "r"
    nodes.append(wr.encode_node("MaxPool", [cur], ["p"], attrs=[
        wr.encode_attr_ints("kernel_shape", pool_k), wr.encode_attr_ints("strides", pool_s),
        wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pool_pads)]))
    nodes.append(wr.encode_node("GlobalAveragePool", ["p"], ["y"]))
    inits = [wr.encode_tensor("w", w), wr.encode_tensor("b", b)]
    vinfo = [wr.encode_value_info("x", x_shape), wr.encode_value_info("w", w.shape), wr.encode_value_info("b", b.shape)]
    return wr.encode_model("cp", nodes, inits, vinfo, [wr.encode_value_info("y", (1, 1, 1, 1))])


@pytest.mark.parametrize("case", [
    # C, H, M, k, conv stride, conv pad, relu, pool k, pool s, pool pads
    (3, 45, 96, 7, 2, 0, True, 3, 2, [0, 0, 0, 0]),     # conv1 + pool1 shape family (96-row tile)
    (5, 40, 40, 3, 1, 1, True, 3, 2, [0, 0, 1, 1]),     # ceil-mode pad on the pool, 96-row tile on M = 40
    (8, 33, 130, 1, 1, 0, False, 3, 2, [1, 1, 1, 1]),   # 1x1 conv, no relu (negative values vs the 0 pad), M > 128
    (4, 30, 24, 5, 1, 2, True, 3, 2, [1, 0, 0, 1]),     # asymmetric pool pads, 32-row tile
    (6, 20, 16, 3, 2, 1, True, 2, 2, [0, 0, 0, 0]),     # 2x2 pool: not fused (the epilogue takes 3x3/s2)
])
@pytest.mark.parametrize("precision", ["f32", "f16"])
def test_conv_pool_fusion_bit_identical(gpu_ctx, case, precision):
    """ORE_FUSE_CONV_POOL: the pooled epilogue equals the separate conv + pool kernels bit for bit
    (forced with ORE_FUSE_EAGER so the small planes qualify).  f16 models: the conv values are
    rounded to f16 before the max, as the separate conv stores them (NHWC f16)."""
    import ore
    C, H, M, k, cs, cp, relu, pk, ps, ppads = case
    rng = np.random.default_rng(sum(case[:6]))
    w = (rng.standard_normal((M, C, k, k)) * 0.3).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, M).astype(np.float32)
    x = rng.standard_normal((3, C, H, H)).astype(np.float32)
    mb = _conv_pool_model((1, C, H, H), w, b, [cp] * 4, [cs, cs], relu, [pk, pk], [ps, ps], ppads)
    vals = []
    eager = ore.FUSE_EAGER | ore.KEEP_VALUES
    for fusion in (ore.FUSE_ALL | eager, (ore.FUSE_ALL & ~ore.FUSE_CONV_POOL) | eager):
        m = _model(gpu_ctx, mb, max_batch=3, precision=precision)
        m.set_fusion(fusion)
        _np(m.run(_t(x)))
        vals.append(m.read_value("p"))
        if fusion & ore.FUSE_CONV_POOL and pk == 3 and ps == 2:
            with pytest.raises(ore.OreError):
                m.read_value("r" if relu else "c")  # fused away: the pre-pool tensor is never stored
        m.close()
    np.testing.assert_array_equal(vals[0], vals[1])
    import oracle
    c = oracle.conv2d(x, w, b, pads=[cp] * 4, strides=(cs, cs))
    ref = oracle.maxpool2d(oracle.relu(c) if relu else c, (pk, pk), (ps, ps), auto_pad="NOTSET", pads=ppads)
    tol = 1e-5 if precision == "f32" else 2e-2 * (np.abs(ref).max() + 1.0)  # f16 storage: ~3 significant digits
    np.testing.assert_allclose(vals[0], ref, rtol=tol if precision == "f16" else 1e-5, atol=tol)


@pytest.mark.parametrize("case", [
    # C, H, M, k: stride-2 'valid' conv + Relu + 3x3 / stride-2 pool (the row-walking kernel's family)
    (3, 45, 96, 7),    # conv1 shape family: Ho 20, 5 quads per row, two 48-channel tiles
    (3, 64, 96, 7),    # Ho 29: a 64-quad step spans a row boundary mid-row
    (3, 31, 40, 5),    # M = 40: one 48-channel tile, channels 40..47 masked
    (2, 50, 100, 4),   # kw = 4 (one tap carry per k-step), M = 100: a 4-channel last tile
    (4, 23, 20, 7),    # M = 20: 32-channel tiles (MF = 2), Ho 9 -> a single step per image
    (3, 113, 64, 7),   # Ho 54 (even), 14 quads per row, pooled 26 x 26
    (1, 40, 128, 7),   # one input channel, 4 channel fragments (window kernel)
    (4, 37, 72, 7),    # four input channels, M = 72: a partial third fragment (window kernel)
])
def test_conv_pool_walk_bit_identical(gpu_ctx, case):
    """The row-walking conv + pool kernels (ore_conv_pool.hip, LDS-ring pooled epilogue with ds_max on
    the f32 bits; "epool walk48": 48 channels x 64 quads per block, "walk96": 96 x 128) and the
    window kernel ("epool window f32", ore_conv1_f32.hip: 7x7 / stride 2, C in {1, 3, 4}, 32 < M <= 128)
    forced with ore_model_set_step_tile equal the patch-epilogue kernel and the separate conv + Relu +
    MaxPool kernels bit for bit, and the oracle within the conv tolerance."""
    import ore
    C, H, M, k = case
    rng = np.random.default_rng(sum(case))
    w = (rng.standard_normal((M, C, k, k)) * 0.3).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, M).astype(np.float32)
    x = rng.standard_normal((3, C, H, H)).astype(np.float32)
    mb = _conv_pool_model((1, C, H, H), w, b, [0] * 4, [2, 2], True, [3, 3], [2, 2], [0, 0, 0, 0])
    vals = []
    names = ore.Model.TILE_NAMES
    for tile, fusion in ((EPOOL_WALK48, ore.FUSE_ALL), (EPOOL_PATCH, ore.FUSE_ALL), (EPOOL_WALK96, ore.FUSE_ALL),
                         (EPOOL_WINDOW, ore.FUSE_ALL), (EPOOL_WALK48, ore.FUSE_ALL & ~ore.FUSE_CONV_POOL)):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(fusion | ore.FUSE_EAGER | ore.KEEP_VALUES)
        forced = force_tiles(m, tile)
        _np(m.run(_t(x)))
        vals.append(m.read_value("p"))
        if tile == EPOOL_WINDOW and k == 7 and C in (1, 3, 4) and 32 < M <= 128:  # the window kernel ran
            assert forced == 1 and [names[t] for t in m.tiles() if t >= 0] == ["epool window f32"]
        m.close()
    for v in vals[1:]:
        np.testing.assert_array_equal(vals[0], v)
    import oracle
    ref = oracle.maxpool2d(oracle.relu(oracle.conv2d(x, w, b, pads=[0] * 4, strides=(2, 2))), (3, 3), (2, 2),
                           auto_pad="NOTSET", pads=[0, 0, 0, 0])
    np.testing.assert_allclose(vals[0], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("H", [40, 79])
@pytest.mark.parametrize("relu", [False, True])
def test_conv_pool_window_variants(gpu_ctx, H, relu):
    """The window kernel's compile-time forms (round 4): Relu or not (Relu and the zero outside the conv
    plane as one v_med3_f32, else a select), and IN -- every tile's input window inside the image, loads
    at a scalar tile origin -- (H = 79: 18 x 18 pooled = 3 x 2 whole tiles, the last window ending on the
    last row / column) or per-element bounds (H = 40).  Bit for bit the patch-epilogue kernel's output,
    and the oracle within the conv tolerance."""
    import ore
    C, M, k = 3, 96, 7
    rng = np.random.default_rng(H + relu)
    w = (rng.standard_normal((M, C, k, k)) * 0.3).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, M).astype(np.float32)
    x = rng.standard_normal((3, C, H, H)).astype(np.float32)
    mb = _conv_pool_model((1, C, H, H), w, b, [0] * 4, [2, 2], relu, [3, 3], [2, 2], [0, 0, 0, 0])
    names = ore.Model.TILE_NAMES
    vals = []
    for tile in (EPOOL_PATCH, EPOOL_WINDOW):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)
        forced = force_tiles(m, tile)
        _np(m.run(_t(x)))
        vals.append(m.read_value("p"))
        if tile == EPOOL_WINDOW:
            assert forced == 1 and [names[t] for t in m.tiles() if t >= 0] == ["epool window f32"]
        m.close()
    np.testing.assert_array_equal(vals[0], vals[1])
    import oracle
    c = oracle.conv2d(x, w, b, pads=[0] * 4, strides=(2, 2))
    ref = oracle.maxpool2d(oracle.relu(c) if relu else c, (3, 3), (2, 2), auto_pad="NOTSET", pads=[0, 0, 0, 0])
    np.testing.assert_allclose(vals[1], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", [
    # C, H, M, k, conv pad, pool pads: stride-1 convs + Relu + 3x3 / stride-2 pool (operand modes 1x1 / 3x3)
    (32, 54, 128, 1, 0, [0, 0, 1, 1]),   # fire4 expand1x1 -> pool3 (ceil-mode bottom / right pad)
    (32, 54, 128, 3, 1, [0, 0, 1, 1]),   # fire4 expand3x3 -> pool3
    (64, 27, 256, 3, 1, [0, 0, 0, 0]),   # fire8 expand3x3 -> pool5
    (64, 27, 256, 1, 0, [0, 0, 0, 0]),   # fire8 expand1x1 -> pool5
    (5, 21, 40, 3, 1, [0, 0, 1, 1]),     # odd width (quad padding inside a window), masked channel tail
    (6, 18, 20, 1, 0, [0, 0, 0, 0]),     # 32-channel tiles
    (16, 9, 64, 3, 1, [0, 0, 1, 1]),     # 3 quads per row: a step spans many rows
    (7, 9, 64, 3, 1, [0, 0, 1, 1]),      # 9 C % 16 != 0: the walker declines (patch kernel)
])
def test_conv_pool_walk_stride1_bit_identical(gpu_ctx, case):
    """The row-walking conv + pool kernel's stride-1 operand modes (1x1; 3x3 'same' with per-element
    tap masks) for every block shape equal the patch-epilogue kernel and the separate kernels bit for
    bit, ceil-mode pool pads included."""
    import ore
    C, H, M, k, cp, ppads = case
    rng = np.random.default_rng(C * H + M + k)
    w = (rng.standard_normal((M, C, k, k)) * 0.3).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, M).astype(np.float32)
    x = rng.standard_normal((3, C, H, H)).astype(np.float32)
    mb = _conv_pool_model((1, C, H, H), w, b, [cp] * 4, [1, 1], True, [3, 3], [2, 2], ppads, pre_relu=True)
    vals = []
    names = ore.Model.TILE_NAMES
    for tile, fusion in ((EPOOL_PATCH, ore.FUSE_ALL), (EPOOL_WALK48, ore.FUSE_ALL), (EPOOL_WALK96, ore.FUSE_ALL),
                         (EPOOL_WALK64, ore.FUSE_ALL), (EPOOL_WALK64_B3, ore.FUSE_ALL),
                         (EPOOL_PATCH, ore.FUSE_ALL & ~ore.FUSE_CONV_POOL)):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(fusion | ore.FUSE_EAGER | ore.KEEP_VALUES)
        force_tiles(m, tile)
        _np(m.run(_t(x)))
        vals.append(m.read_value("p"))
        walkable = (k == 1 and C % 16 == 0) or (k == 3 and 9 * C % 16 == 0)  # whole ring rounds per step
        if (fusion & ore.FUSE_CONV_POOL and tile in (EPOOL_WALK48, EPOOL_WALK64, EPOOL_WALK64_B3) and M >= 48 and
                (tile != EPOOL_WALK64_B3 or H >= 12) and walkable):
            ran = [names[t] for t in m.tiles() if t >= names.index("epool patch")]  # the forced walker ran
            assert ran == [names[tile]], ran
        m.close()
    for v in vals[1:]:
        np.testing.assert_array_equal(vals[0], v)
    import oracle
    ref = oracle.maxpool2d(oracle.relu(oracle.conv2d(oracle.relu(x), w, b, pads=[cp] * 4, strides=(1, 1))), (3, 3),
                           (2, 2), auto_pad="NOTSET", pads=ppads)
    np.testing.assert_allclose(vals[0], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("hw", [64, 224])
def test_squeezenet_concat_pool_fusion(gpu_ctx, hw):
    """ORE_FUSE_CONCAT_POOL (in FUSE_ALL; by default fire4 -> pool3 only, here forced onto fire8 ->
    pool5 too with ORE_FUSE_EAGER: the pools computed in the expand convs'
    epilogues, the expand outputs and their concat never stored): every value the fused graph
    materialises -- pool3 / pool5 included -- and the probabilities equal the unfused run's bit
    for bit; the row-walking kernel runs for the pooled expands."""
    import ore
    from ore import onnx_wire, squeezenet
    mb = squeezenet.build(hw)
    model = onnx_wire.decode_model(mb)
    xt = _t(squeezenet.synthetic_input(3, hw, seed=41))
    ref = _model(gpu_ctx, mb, max_batch=3)
    ref.set_fusion(ore.KEEP_VALUES)
    y0 = _np(ref.run(xt))
    fused = _model(gpu_ctx, mb, max_batch=3)
    # fire4 -> pool3 stays with the walkers (no fire_pool_kernel); eager: fire8 -> pool5 too (27 x 27)
    fused.set_fusion((ore.FUSE_ALL & ~ore.FUSE_FIRE_POOL) | ore.FUSE_EAGER | ore.KEEP_VALUES)
    force_tiles(fused, EPOOL_WALK64)  # the 64-channel walker (auto takes it from batch 128)
    y1 = _np(fused.run(xt))
    np.testing.assert_array_equal(y0, y1)
    for v in ("pool3", "pool5"):
        name = [n.output[0] for n in model.graph.node if n.name == v][0]
        np.testing.assert_array_equal(fused.read_value(name), ref.read_value(name), err_msg=v)
    names = ore.Model.TILE_NAMES
    walk = [names[t] for t in fused.tiles() if t >= names.index("epool walk48")]
    assert len(walk) >= 4, walk  # fire4 / fire8 expand1x1 + expand3x3 (+ conv1 @224)
    ref.close()
    fused.close()


@pytest.mark.parametrize("hw", [64, 224])
@pytest.mark.parametrize("precision", ["f32", "f16"])
def test_squeezenet_conv_pool_fusion(gpu_ctx, hw, precision):
    """SqueezeNet with conv1 + pool1 fused (the only pair under the default work bound at 224):
    probabilities bit-identical to the unfused pool, in the f32 and the f16 model."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(hw)
    x = _t(squeezenet.synthetic_input(3, hw, seed=17))
    outs = []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_CONV_POOL):
        m = _model(gpu_ctx, mb, max_batch=3, precision=precision)
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def _fire_model(C, H, W, S1, E1, E3, S2):
    """squeeze (C -> S1) -> expand 1x1 (E1) / 3x3 pad 1 (E3) -> Concat -> squeeze (S2) -> GAP, all Relu."""
    from ore import onnx_wire as wr
    rng = np.random.default_rng(C * 7 + H + W + S1 + E1 + E3 + S2)
    shapes = {"wq": (S1, C, 1, 1), "w1": (E1, S1, 1, 1), "w3": (E3, S1, 3, 3), "wn": (S2, E1 + E3, 1, 1)}
    inits, vinfo = [], [wr.encode_value_info("x", (1, C, H, W))]
    for n, shp in shapes.items():
        fan = shp[1] * shp[2] * shp[3]
        w = (rng.standard_normal(shp) * np.sqrt(2.0 / fan)).astype(np.float32)
        b = rng.uniform(-0.1, 0.1, shp[0]).astype(np.float32)
        inits += [wr.encode_tensor(n, w), wr.encode_tensor("b" + n, b)]
        vinfo += [wr.encode_value_info(n, w.shape), wr.encode_value_info("b" + n, b.shape)]
    conv = lambda i, w, o, pads: wr.encode_node("Conv", [i, w, "b" + w], [o], attrs=[
        wr.encode_attr_ints("pads", pads), wr.encode_attr_ints("strides", [1, 1])])
    nodes = [conv("x", "wq", "q", [0] * 4), wr.encode_node("Relu", ["q"], ["qr"]),
             conv("qr", "w1", "e1", [0] * 4), wr.encode_node("Relu", ["e1"], ["e1r"]),
             conv("qr", "w3", "e3", [1] * 4), wr.encode_node("Relu", ["e3"], ["e3r"]),
             wr.encode_node("Concat", ["e1r", "e3r"], ["cat"], attrs=[wr.encode_attr_int("axis", 1)]),
             conv("cat", "wn", "n", [0] * 4), wr.encode_node("Relu", ["n"], ["nr"]),
             wr.encode_node("GlobalAveragePool", ["nr"], ["y"])]
    return wr.encode_model("fire", nodes, inits, vinfo, [wr.encode_value_info("y", (1, S2, 1, 1))])


@pytest.mark.parametrize("case", [
    # C, H, W, S1, E1, E3, S2: the fused fire kernel's shapes (16-B planes: H*W % 4 == 0 after padding)
    (16, 12, 12, 16, 64, 64, 16),     # fire2 -> squeeze3 shape family
    (32, 9, 8, 32, 128, 128, 48),     # fire5 -> squeeze6 (MFS = 3), W = 8: row wraps inside a pixel group
    (24, 8, 7, 48, 192, 192, 64),     # fire7 -> squeeze8 (MFS = 4), W = 7
    (16, 13, 13, 16, 64, 128, 32),    # unequal expands, fire9-like 13 x 13 planes
])
def test_fire_fusion_bit_identical(gpu_ctx, case):
    """ORE_FUSE_FIRE: expand 1x1 + expand 3x3 + Concat + the next squeeze in one launch equals the
    separate kernels bit for bit (forced with ORE_FUSE_EAGER at these small sizes), and the
    oracle within the conv tolerance."""
    import ore
    import oracle
    C, H, W, S1, E1, E3, S2 = case
    mb = _fire_model(*case)
    x = np.random.default_rng(sum(case)).standard_normal((5, C, H, W)).astype(np.float32)
    vals = []
    eager = ore.FUSE_EAGER | ore.KEEP_VALUES
    for fusion in (ore.FUSE_ALL | eager, (ore.FUSE_ALL & ~ore.FUSE_FIRE) | eager):
        m = _model(gpu_ctx, mb, max_batch=5)
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("nr")))
        if fusion & ore.FUSE_FIRE:
            assert "fire" in [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
            with pytest.raises(ore.OreError):
                m.read_value("cat")  # never materialised
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, S2)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("hw", [64, 224])
def test_squeezenet_fire_fusion(gpu_ctx, hw):
    """SqueezeNet with the five fire + squeeze pairs fused (ORE_FUSE_EAGER so batch 3 fuses; the fire +
    pool + squeeze fusion off): probabilities bit-identical to the separate kernels."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(hw)
    x = _t(squeezenet.synthetic_input(3, hw, seed=19))
    outs = []
    base = (ore.FUSE_ALL & ~ore.FUSE_FIRE_POOL) | ore.FUSE_EAGER
    for fusion in (base, base & ~ore.FUSE_FIRE):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        if fusion & ore.FUSE_FIRE:
            # @64 the 7 x 7 planes of fire5-8 cannot take 16-B padding: fire2 and fire3 only
            assert sum(1 for t in m.tiles() if t >= 0 and ore.Model.TILE_NAMES[t] == "fire") == (5 if hw == 224 else 2)
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def test_model_io_checks_gpu(gpu_ctx):
    """an f16 / f64 output or input, or a non-contiguous one, is refused before the
    walker sees the pointer (an f16 out would otherwise take 2x its size in f32 stores)."""
    import torch
    import ore
    m = _model(gpu_ctx, _mnist_bytes(), max_batch=4)
    x = torch.zeros((2, 1, 28, 28), device="cuda")
    out = torch.zeros((2, 10), device="cuda")
    m.run_into(x, out)
    for fn in (m.run_into, m.autotune, m.capture):
        with pytest.raises(ore.OreError, match="float32 CUDA"):
            fn(x, out.half())
        with pytest.raises(ore.OreError, match="float32 CUDA"):
            fn(x.double(), out)
        with pytest.raises(ore.OreError, match="contiguous"):
            fn(torch.zeros((2, 1, 28, 56), device="cuda")[..., ::2], out)
        with pytest.raises(ore.OreError, match="holds"):
            fn(x, torch.zeros((1, 10), device="cuda"))
    m.close()


def test_read_value_refuses_overwritten(gpu_ctx):
    """without ORE_KEEP_VALUES the arena reuses slots, so an early intermediate whose
    bytes a later value overwrote is refused (not returned stale); the graph output and, with
    KEEP_VALUES, every value stay readable."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(64)
    x = _t(squeezenet.synthetic_input(2, 64, seed=3))
    m = _model(gpu_ctx, mb, max_batch=2)
    m.set_fusion(0)  # op by op: every node's output is a value of its own
    y = _np(m.run(x))
    from ore import onnx_wire
    g = onnx_wire.decode_model(mb).graph
    names = [n.output[0] for n in g.node]
    refused = 0
    for nm in names[:10]:
        try:
            m.read_value(nm)
        except ore.OreError as e:
            assert "overwritten" in str(e)
            refused += 1
    assert refused > 0  # op-by-op SqueezeNet reuses the early slots
    keep = _model(gpu_ctx, mb, max_batch=2)
    keep.set_fusion(ore.KEEP_VALUES)
    np.testing.assert_array_equal(_np(keep.run(x)), y)
    for nm in names[:10]:
        keep.read_value(nm)
    m.close()
    keep.close()


def test_two_contexts_large_lds_variant():
    """the 152 KiB row-walking conv1 + pool1 variant raises its dynamic-LDS limit per
    device (not once per process); two contexts driven from two host threads both run the
    batch-128 conv1 + pool1 step and agree bit for bit."""
    import threading
    import torch
    import ore
    C, H, M, k = 3, 45, 96, 7
    rng = np.random.default_rng(5)
    w = (rng.standard_normal((M, C, k, k)) * 0.3).astype(np.float32)
    b = rng.uniform(-0.5, 0.5, M).astype(np.float32)
    mb = _conv_pool_model((1, C, H, H), w, b, [0] * 4, [2, 2], True, [3, 3], [2, 2], [0, 0, 0, 0])
    x = torch.from_numpy(rng.standard_normal((128, C, H, H)).astype(np.float32)).cuda()
    res, errs = [None, None], []

    def work(i):
        try:
            torch.cuda.set_device(0)
            ctx = ore.Context(0, use_torch_stream=False)
            m = _model(ctx, mb, max_batch=128)
            m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)
            force_tiles(m, EPOOL_WALK96)  # 96 channels x 128 quads, 152 KiB of LDS
            out = torch.empty((128, m.output_elems), device="cuda")
            m.run_into(x, out)
            ctx.sync()
            res[i] = m.read_value("p")
            assert "epool walk96" in [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
            m.close()
            ctx.close()
        except Exception as e:  # surfaced below
            errs.append(e)

    ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    np.testing.assert_array_equal(res[0], res[1])


def _conv_pool_squeeze_model(H, W, M, Q, pool_pads):
    """x (3 channels) -> Conv 7x7 / 2 + Relu -> MaxPool 3x3 / 2 -> Conv 1x1 (Q) + Relu -> GAP."""
    from ore import onnx_wire as wr
    rng = np.random.default_rng(H * 31 + W + M + Q)
    w1 = (rng.standard_normal((M, 3, 7, 7)) * np.sqrt(2.0 / 147)).astype(np.float32)
    b1 = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    w2 = (rng.standard_normal((Q, M, 1, 1)) * np.sqrt(2.0 / M)).astype(np.float32)
    b2 = rng.uniform(-0.1, 0.1, Q).astype(np.float32)
    nodes = [wr.encode_node("Conv", ["x", "w1", "b1"], ["c"], attrs=[wr.encode_attr_ints("strides", [2, 2]),
                                                                      wr.encode_attr_ints("pads", [0] * 4)]),
             wr.encode_node("Relu", ["c"], ["r"]),
             wr.encode_node("MaxPool", ["r"], ["p"], attrs=[
                 wr.encode_attr_ints("kernel_shape", [3, 3]), wr.encode_attr_ints("strides", [2, 2]),
                 wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pool_pads)]),
             wr.encode_node("Conv", ["p", "w2", "b2"], ["q"], attrs=[wr.encode_attr_ints("strides", [1, 1]),
                                                                     wr.encode_attr_ints("pads", [0] * 4)]),
             wr.encode_node("Relu", ["q"], ["qr"]),
             wr.encode_node("GlobalAveragePool", ["qr"], ["y"])]
    inits = [wr.encode_tensor(n, a) for n, a in (("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2))]
    vinfo = [wr.encode_value_info("x", (1, 3, H, W))] + [wr.encode_value_info(n, a.shape) for n, a in
                                                          (("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2))]
    return wr.encode_model("cps", nodes, inits, vinfo, [wr.encode_value_info("y", (1, Q, 1, 1))])


@pytest.mark.parametrize("case", [(67, 71, 16, [0, 0, 0, 0]), (40, 45, 12, [0, 0, 1, 1])])
def test_conv_pool_squeeze_fused_bit_identical(gpu_ctx, case):
    """f32: conv1 + Relu + pool1 + the next 1x1 conv + Relu in one window-kernel launch (pooled-conv
    variant 7 with the squeeze inside, the pooled map never stored) equals the separate launches
    (without ORE_FUSE_FIRST_SQUEEZE) bit for bit, and the oracle within the conv tolerance."""
    import ore
    import oracle
    H, W, Q, pads = case
    mb = _conv_pool_squeeze_model(H, W, 96, Q, pads)
    x = (np.random.default_rng(H + W).standard_normal((3, 3, H, W)) * 20).astype(np.float32)
    vals = []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=3)
        fusion = ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_FIRST_SQUEEZE
        m.set_fusion(fusion | ore.FUSE_EAGER | ore.KEEP_VALUES)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("qr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        if on == "1":
            assert names == ["epool window f32"], names
            with pytest.raises(ore.OreError):
                m.read_value("p")  # never stored
        else:
            assert len(names) == 2, names
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, Q)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", [(224, 224, 16, [0, 0, 0, 0], 2), (61, 224, 13, [0, 0, 1, 1], 3),
                                  (23, 216, 16, [1, 1, 1, 1], 2), (40, 212, 9, [0, 0, 0, 0], 5),
                                  (15, 224, 16, [1, 1, 0, 0], 1)])
def test_conv1_band_bit_identical(gpu_ctx, case):
    """The band walker (pooled-conv variant 8, "epool band f32": conv rows walked in steps of 256 column
    pairs, pooling by DPP + LDS max, completed pooled rows squeezed) equals the window kernel (variant 7)
    bit for bit on the squeeze output, over heights that give 1-13 bands per image, pool pads on every
    side and widths down to the eligibility edge (52 column pairs per conv row); and the oracle within
    the conv tolerance."""
    import ore
    import oracle
    H, W, Q, pads, B = case
    mb = _conv_pool_squeeze_model(H, W, 96, Q, pads)
    x = (np.random.default_rng(H * 7 + W).standard_normal((B, 3, H, W)) * 20).astype(np.float32)
    band = ore.Model.TILE_NAMES.index("epool band f32")
    vals = []
    for tile in (None, band):
        m = _model(gpu_ctx, mb, max_batch=B)
        m.set_fusion(ore.FUSE_ALL | ore.FUSE_EAGER | ore.KEEP_VALUES)
        if tile is not None:
            m.set_tile(0, tile)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("qr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert names == ["epool band f32" if tile is not None else "epool window f32"], names
        m.close()
    np.testing.assert_array_equal(vals[1][1], vals[0][1])
    np.testing.assert_array_equal(vals[1][0], vals[0][0])
    ref = oracle.Model(mb).run(x, Q)
    np.testing.assert_allclose(vals[1][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


def test_conv1_band_units_per_workgroup(gpu_ctx):
    """Batch 300 at 224 x 224: more (image, band) units than workgroups (one per CU), so workgroups walk
    a second unit after their first (the ring and window reused across units); equal to the window
    kernel bit for bit."""
    import ore
    B = 300
    mb = _conv_pool_squeeze_model(224, 224, 96, 16, [0, 0, 0, 0])
    x = (np.random.default_rng(300).standard_normal((B, 3, 224, 224)) * 20).astype(np.float32)
    outs = []
    for name in ("epool window f32", "epool band f32"):
        m = _model(gpu_ctx, mb, max_batch=B)
        m.set_tile(0, ore.Model.TILE_NAMES.index(name))
        outs.append(_np(m.run(_t(x))))
        assert ore.Model.TILE_NAMES[m.tiles()[0]] == name
        m.close()
    np.testing.assert_array_equal(outs[1], outs[0])


def test_squeezenet_conv1_band(gpu_ctx):
    """SqueezeNet-1.0 @224 f32 with conv1 + pool1 + fire2/squeeze1x1 on the band walker: probabilities
    equal the window kernel's plan bit for bit (batch 3: 13 bands per image, and batch 256's one band
    per image via a 260-image chunk-free run is covered by the benched-plan parity tests)."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=37))
    band = ore.Model.TILE_NAMES.index("epool band f32")
    outs = []
    for tile in (None, band):
        m = _model(gpu_ctx, mb, max_batch=3)
        if tile is not None:
            m.set_tile(0, tile)
        outs.append(_np(m.run(x)))
        assert ore.Model.TILE_NAMES[m.tiles()[0]] == ("epool band f32" if tile is not None else "epool window f32")
        m.close()
    np.testing.assert_array_equal(outs[1], outs[0])


def test_squeezenet_conv1_squeeze_fused(gpu_ctx):
    """SqueezeNet-1.0 @224 f32: conv1 + pool1 + fire2/squeeze1x1 in one launch; probabilities equal the
    plan without that fusion bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=29))
    outs = []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_FIRST_SQUEEZE)
        outs.append(_np(m.run(x)))
        first = ore.Model.TILE_NAMES[m.tiles()[0]]
        assert (first == "epool window f32") == (on == "1"), first
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def _pool_squeeze_model(C, H, W, M, pool_pads, relu=True):
    """x -> Relu -> MaxPool 3x3 / 2 -> Conv 1x1 (M) [+ Relu] -> GAP (the pooled map's only reader is the conv)."""
    from ore import onnx_wire as wr
    rng = np.random.default_rng(C + H * 3 + W + M)
    w = (rng.standard_normal((M, C, 1, 1)) * np.sqrt(2.0 / C)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    nodes = [wr.encode_node("Relu", ["x"], ["xr"]),
             wr.encode_node("MaxPool", ["xr"], ["p"], attrs=[
                 wr.encode_attr_ints("kernel_shape", [3, 3]), wr.encode_attr_ints("strides", [2, 2]),
                 wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pool_pads)]),
             wr.encode_node("Conv", ["p", "w", "b"], ["q"], attrs=[wr.encode_attr_ints("strides", [1, 1]),
                                                                   wr.encode_attr_ints("pads", [0] * 4)])]
    out = "q"
    if relu:
        nodes.append(wr.encode_node("Relu", ["q"], ["qr"]))
        out = "qr"
    nodes.append(wr.encode_node("GlobalAveragePool", [out], ["y"]))
    inits = [wr.encode_tensor("w", w), wr.encode_tensor("b", b)]
    vinfo = [wr.encode_value_info("x", (1, C, H, W)), wr.encode_value_info("w", w.shape), wr.encode_value_info("b", b.shape)]
    return wr.encode_model("ps", nodes, inits, vinfo, [wr.encode_value_info("y", (1, M, 1, 1))]), out


@pytest.mark.parametrize("case", [
    (512, 27, 27, 64, [0, 0, 0, 0], True),   # SqueezeNet pool5 + fire9/squeeze1x1
    (64, 20, 31, 48, [0, 0, 1, 1], True),    # ceil-mode pads, 16 pooled columns, M = 48
    (32, 9, 7, 10, [1, 1, 1, 1], False),     # padded on all sides, no Relu (negative outputs), M = 10
    (256, 54, 54, 32, [0, 0, 1, 1], True),   # SqueezeNet pool3 + fire5/squeeze1x1: 27 pooled columns (2 fragments)
    (64, 40, 61, 24, [1, 1, 1, 1], False),   # 31 pooled columns, padded on all sides
])
def test_pool_squeeze_fused_bit_identical(gpu_ctx, case):
    """f32: a 3x3 / stride-2 MaxPool and the 1x1 conv that is its only reader in one launch
    (pool_conv1x1_f32_kernel, the pooled map never stored) equal maxpool_kernel + the separate conv
    (without ORE_FUSE_POOL_SQUEEZE) bit for bit, and the oracle within the conv tolerance."""
    import ore
    import oracle
    C, H, W, M, pads, relu = case
    mb, out = _pool_squeeze_model(C, H, W, M, pads, relu)
    x = np.random.default_rng(C + H).standard_normal((3, C, H, W)).astype(np.float32)
    vals = []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion((ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_POOL_SQUEEZE) | ore.KEEP_VALUES)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value(out)))
        if on == "1":
            with pytest.raises(ore.OreError):
                m.read_value("p")  # never stored
        else:
            assert m.read_value("p").shape[1] == C
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, M)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


def test_squeezenet_pool_squeeze_fused(gpu_ctx):
    """SqueezeNet-1.0 @224 f32: pool5 + fire9/squeeze1x1 in one launch; probabilities equal the plan
    without that fusion bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=31))
    outs, nsteps = [], []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=3)
        base = ore.FUSE_ALL & ~ore.FUSE_POOL_EXPAND  # (with it, fire8's expand1x1 would join as well)
        m.set_fusion(base if on == "1" else base & ~ore.FUSE_POOL_SQUEEZE)
        outs.append(_np(m.run(x)))
        nsteps.append(len(m.tiles()))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    assert nsteps[0] == nsteps[1] - 1  # pool5 is no longer a launch of its own


def _fire_pool_model(C, H, W, S1, E1, E3, S2, pool_pads):
    """squeeze (C -> S1) -> expand 1x1 (E1) / 3x3 pad 1 (E3) -> Concat -> MaxPool 3x3 / 2 (pool_pads)
    -> squeeze (S2) -> GAP, all Relu (SqueezeNet's fire4 -> pool3 -> fire5/squeeze1x1 family)."""
    from ore import onnx_wire as wr
    rng = np.random.default_rng(C * 5 + H + W + S1 + E1 + E3 + S2)
    shapes = {"wq": (S1, C, 1, 1), "w1": (E1, S1, 1, 1), "w3": (E3, S1, 3, 3), "wn": (S2, E1 + E3, 1, 1)}
    inits, vinfo = [], [wr.encode_value_info("x", (1, C, H, W))]
    for n, shp in shapes.items():
        fan = shp[1] * shp[2] * shp[3]
        w = (rng.standard_normal(shp) * np.sqrt(2.0 / fan)).astype(np.float32)
        b = rng.uniform(-0.1, 0.1, shp[0]).astype(np.float32)
        inits += [wr.encode_tensor(n, w), wr.encode_tensor("b" + n, b)]
        vinfo += [wr.encode_value_info(n, w.shape), wr.encode_value_info("b" + n, b.shape)]
    conv = lambda i, w, o, pads: wr.encode_node("Conv", [i, w, "b" + w], [o], attrs=[
        wr.encode_attr_ints("pads", pads), wr.encode_attr_ints("strides", [1, 1])])
    nodes = [conv("x", "wq", "q", [0] * 4), wr.encode_node("Relu", ["q"], ["qr"]),
             conv("qr", "w1", "e1", [0] * 4), wr.encode_node("Relu", ["e1"], ["e1r"]),
             conv("qr", "w3", "e3", [1] * 4), wr.encode_node("Relu", ["e3"], ["e3r"]),
             wr.encode_node("Concat", ["e1r", "e3r"], ["cat"], attrs=[wr.encode_attr_int("axis", 1)]),
             wr.encode_node("MaxPool", ["cat"], ["p"], attrs=[
                 wr.encode_attr_ints("kernel_shape", [3, 3]), wr.encode_attr_ints("strides", [2, 2]),
                 wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pool_pads)]),
             conv("p", "wn", "n", [0] * 4), wr.encode_node("Relu", ["n"], ["nr"]),
             wr.encode_node("GlobalAveragePool", ["nr"], ["y"])]
    return wr.encode_model("firepool", nodes, inits, vinfo, [wr.encode_value_info("y", (1, S2, 1, 1))])


@pytest.mark.parametrize("case", [
    # C, H, W, S1, E1, E3, S2, pool pads (expand planes with H * W % 4 == 0: 16-B input planes)
    (16, 54, 54, 32, 128, 128, 32, [0, 0, 1, 1]),  # SqueezeNet fire4 -> pool3 (ceil) -> fire5 squeeze: 4 rows / band
    (16, 20, 21, 16, 64, 64, 48, [1, 1, 1, 1]),    # padded on all sides, odd W (row wraps in a pixel quad), MFS = 3
    (32, 9, 8, 32, 128, 64, 16, [0, 0, 0, 0]),     # 'valid' pool, W = 8, unequal expands
    (16, 30, 17, 16, 64, 128, 64, [0, 0, 1, 1]),   # MFS = 4, short last band
])
def test_fire_pool_fusion_bit_identical(gpu_ctx, case):
    """f32: fire module + 3x3 / stride-2 MaxPool + the next squeeze in one launch (fire_pool_kernel;
    the expand outputs, their concat and the pooled map never stored) equal the pooled-epilogue
    expands + the separate squeeze (without ORE_FUSE_FIRE_POOL) bit for bit, and the oracle within the
    conv tolerance."""
    import ore
    import oracle
    C, H, W, S1, E1, E3, S2, pads = case
    mb = _fire_pool_model(*case)
    x = np.random.default_rng(sum(case[:7])).standard_normal((5, C, H, W)).astype(np.float32)
    vals = []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=5)
        fusion = ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_FIRE_POOL
        m.set_fusion(fusion | ore.FUSE_EAGER | ore.KEEP_VALUES)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("nr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert ("fire pool f32" in names) == (on == "1"), names
        if on == "1":
            for v in ("cat", "p"):
                with pytest.raises(ore.OreError):
                    m.read_value(v)  # never materialised
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, S2)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-6)


def test_squeezenet_fire_pool_fused(gpu_ctx):
    """SqueezeNet-1.0 @224 f32: fire4 + pool3 + fire5/squeeze1x1 and (eager: 27 x 27 planes too) fire8 +
    pool5 + fire9/squeeze1x1 in one launch each (ORE_FUSE_EAGER so batch 3 fuses); probabilities
    equal the plan without ORE_FUSE_FIRE_POOL bit for bit."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=37))
    outs, nsteps = [], []
    for on in ("1", "0"):
        m = _model(gpu_ctx, mb, max_batch=3)
        m.set_fusion((ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_FIRE_POOL) | ore.FUSE_EAGER)
        outs.append(_np(m.run(x)))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert names.count("fire pool f32") == (2 if on == "1" else 0), names
        nsteps.append(len(m.tiles()))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    assert nsteps[0] == nsteps[1] - 4  # per pair: two expand walkers + the squeeze -> fire_pool_kernel


@pytest.mark.parametrize("case", [
    # C, H, W, S1, E1, E3, S2, pool pads (S1 = C1 of the recomputed expand1x1: 32 or 64)
    (16, 54, 54, 32, 128, 128, 32, [0, 0, 1, 1]),  # SqueezeNet fire4 -> pool3 (ceil) -> fire5 squeeze (NF = 2)
    (32, 27, 27, 64, 256, 256, 64, [0, 0, 0, 0]),  # fire8 -> pool5 -> fire9 squeeze (C1 = 64, NF = 1)
    (16, 20, 21, 32, 64, 64, 48, [1, 1, 1, 1]),    # padded on all sides, odd W: band pixels wrap rows in a fragment
    (16, 9, 8, 64, 48, 80, 16, [0, 0, 0, 0]),      # E1 = 48 (3 recomputed chunks), E3 = 80, W = 8
    (16, 30, 17, 32, 32, 96, 64, [0, 0, 1, 1]),    # one recomputed chunk, short last band
])
def test_pool_expand_fused_bit_identical(gpu_ctx, case):
    """ORE_FUSE_POOL_EXPAND: the pooled squeeze (pool_conv1x1_f32_kernel) recomputes the Concat's
    expand1x1 slice from the fire module's squeeze output instead of reading it back; the output
    equals the plan without that bit (expand1x1 as its own launch, its map stored) bit for bit, the
    step count drops by one, and the oracle agrees within the conv tolerance.  Winograd and direct
    expand3x3 plans (the direct one with the 54 x 54 case taken by the Concat + pool fusion instead)."""
    import ore
    import oracle
    C, H, W, S1, E1, E3, S2, pads = case
    mb = _fire_pool_model(*case)
    x = np.random.default_rng(sum(case[:7]) + 3).standard_normal((5, C, H, W)).astype(np.float32)
    outs, nsteps = [], []
    ref = oracle.Model(mb).run(x, S2)
    for wino in (True, False):
        outs, nsteps = [], []
        # C1 = 64 runs only under ORE_FUSE_EAGER (slower at B = 256), which skips the Winograd pool split
        # and would give the pattern to the fire + pool fusions first: the direct plan without those
        base = ore.FUSE_ALL if S1 == 32 else (ore.FUSE_ALL & ~ore.FUSE_FIRE_POOL & ~ore.FUSE_CONCAT_POOL) | ore.FUSE_EAGER
        if S1 == 64 and wino:
            continue
        for on in ("1", "0"):
            m = ore.Model(gpu_ctx, mb, max_batch=5, winograd=wino)
            m.set_fusion(base if on == "1" else base & ~ore.FUSE_POOL_EXPAND)
            outs.append(_np(m.run(_t(x))))
            nsteps.append(len(m.tiles()))
            m.close()
        if wino or H * W < 1024 or S1 == 64:
            assert nsteps[0] == nsteps[1] - 1, (wino, nsteps)  # the expand1x1 launch is gone
        np.testing.assert_array_equal(outs[0], outs[1])
        np.testing.assert_allclose(outs[0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


def test_pool_expand_shared_concat_not_fused(gpu_ctx):
    """ORE_FUSE_POOL_EXPAND leaves e1's Concat slice unwritten, so it must not fire when the Concat has
    another reader: here GlobalAveragePool(cat) joins the graph output.  The plan keeps
    expand1x1 as its own launch (same step count with and without the bit), and the whole output,
    including the GAP of the Concat, matches the oracle."""
    import ore
    import oracle
    from ore import onnx_wire as wr
    C, H, W, S1, E1, E3, S2, pads = (16, 54, 54, 32, 128, 128, 32, [0, 0, 1, 1])
    rng = np.random.default_rng(77)
    shapes = {"wq": (S1, C, 1, 1), "w1": (E1, S1, 1, 1), "w3": (E3, S1, 3, 3), "wn": (S2, E1 + E3, 1, 1)}
    inits, vinfo = [], [wr.encode_value_info("x", (1, C, H, W))]
    for n, shp in shapes.items():
        fan = shp[1] * shp[2] * shp[3]
        w = (rng.standard_normal(shp) * np.sqrt(2.0 / fan)).astype(np.float32)
        b = rng.uniform(-0.1, 0.1, shp[0]).astype(np.float32)
        inits += [wr.encode_tensor(n, w), wr.encode_tensor("b" + n, b)]
        vinfo += [wr.encode_value_info(n, w.shape), wr.encode_value_info("b" + n, b.shape)]
    conv = lambda i, w, o, p: wr.encode_node("Conv", [i, w, "b" + w], [o], attrs=[
        wr.encode_attr_ints("pads", p), wr.encode_attr_ints("strides", [1, 1])])
    nodes = [conv("x", "wq", "q", [0] * 4), wr.encode_node("Relu", ["q"], ["qr"]),
             conv("qr", "w1", "e1", [0] * 4), wr.encode_node("Relu", ["e1"], ["e1r"]),
             conv("qr", "w3", "e3", [1] * 4), wr.encode_node("Relu", ["e3"], ["e3r"]),
             wr.encode_node("Concat", ["e1r", "e3r"], ["cat"], attrs=[wr.encode_attr_int("axis", 1)]),
             wr.encode_node("MaxPool", ["cat"], ["p"], attrs=[
                 wr.encode_attr_ints("kernel_shape", [3, 3]), wr.encode_attr_ints("strides", [2, 2]),
                 wr.encode_attr_string("auto_pad", "NOTSET"), wr.encode_attr_ints("pads", pads)]),
             conv("p", "wn", "n", [0] * 4), wr.encode_node("Relu", ["n"], ["nr"]),
             wr.encode_node("GlobalAveragePool", ["nr"], ["y1"]),
             wr.encode_node("GlobalAveragePool", ["cat"], ["g2"]),
             wr.encode_node("Concat", ["y1", "g2"], ["y"], attrs=[wr.encode_attr_int("axis", 1)])]
    mb = wr.encode_model("firepool_shared", nodes, inits, vinfo, [wr.encode_value_info("y", (1, S2 + E1 + E3, 1, 1))])
    x = np.random.default_rng(5).standard_normal((3, C, H, W)).astype(np.float32)
    ref = oracle.Model(mb).run(x, S2 + E1 + E3)
    outs, nsteps = [], []
    for on in (True, False):
        m = ore.Model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(ore.FUSE_ALL if on else ore.FUSE_ALL & ~ore.FUSE_POOL_EXPAND)
        outs.append(_np(m.run(_t(x))))
        nsteps.append(len(m.tiles()))
        assert not any("expand1x1+" in st["name"] for st in m.steps()), [st["name"] for st in m.steps()]
        m.close()
    assert nsteps[0] == nsteps[1], nsteps
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_allclose(outs[0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B", [3, 256])
def test_squeezenet_pool_expand_fused(gpu_ctx, B):
    """SqueezeNet-1.0 @224 f32 (Winograd plan): fire4/expand1x1 inside pool3 + fire5/squeeze1x1
    (fire8's C1 = 64 case stays separate outside ORE_FUSE_EAGER); probabilities equal the plan without
    ORE_FUSE_POOL_EXPAND bit for bit, with one launch fewer (B = 256: the headline plan, 2 streams)."""
    import ore
    import torch
    from ore import squeezenet
    mb = squeezenet.build_calibrated(224)
    x = _t(squeezenet.synthetic_input(min(B, 4), 224, seed=41))
    if B > 4:
        x = torch.cat([x] * (B // 4 + 1))[:B].contiguous()
    outs, nsteps, names = [], [], []
    for on in ("1", "0"):
        m = ore.Model(gpu_ctx, mb, max_batch=B)  # the default (Winograd) plan
        m.set_fusion(ore.FUSE_ALL if on == "1" else ore.FUSE_ALL & ~ore.FUSE_POOL_EXPAND)
        m.set_streams(2)
        outs.append(_np(m.run(x)))
        nsteps.append(len(m.tiles()))
        names.append([st["name"] for st in m.steps()])
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    assert nsteps[0] == nsteps[1] - 1, (nsteps, names)
    assert "fire4/expand1x1+pool3+fire5/squeeze1x1" in names[0], names[0]


def test_abi2_retired_values(gpu_ctx):
    """ABI 2 (include/ore.h): ABI 1's retired values fail with ORE_ERR_UNSUPPORTED and a message
    naming the retirement -- the bf16x3 load flags (2, 8) and tiles 28-35, fusion bit 16
    (ORE_FUSE_POOL_CONV), MaxPool variant 1 and tiles 4-11."""
    import ctypes
    import ore
    from ore import _lib, squeezenet
    L = ore.load()
    for t in (4, 11, 28, 35):
        assert L.ore_ctx_set_conv_tile(gpu_ctx.h, t) == 2 and b"retired" in L.ore_last_error(gpu_ctx.h)
    assert L.ore_ctx_set_conv_tile(gpu_ctx.h, -1) == 0
    assert L.ore_ctx_set_pool_variant(gpu_ctx.h, 1) == 2 and b"retired" in L.ore_last_error(gpu_ctx.h)
    mb = squeezenet.build(32)
    h = ctypes.c_void_p()
    for flags in (2, 8, 2 | 8):
        assert L.ore_model_load_ex(gpu_ctx.h, mb, len(mb), 2, flags, ctypes.byref(h)) == 2
        assert b"retired" in L.ore_last_error(gpu_ctx.h)
    assert _lib.LOAD_RETIRED_MASK == 10
    m = ore.Model(gpu_ctx, mb, max_batch=2)
    assert L.ore_model_set_fusion(m.h, ore.FUSE_ALL | 16) == 2 and b"retired" in L.ore_last_error(gpu_ctx.h)
    m.close()

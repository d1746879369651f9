"""The Winograd F(2x2, 3x3) path (csrc/ore_conv_wino.hip): 3x3 / stride-1 / pad-1 convs in f32 with
2.25x fewer MFMAs than the direct conv.  On by default for f32 models (every such conv no direct-kernel
fusion takes), per-op through ore_ctx_set_conv_algo(ORE_CONV_ALGO_WINOGRAD).

Parity bar, written per test:
  * each output within 2e-6 * sum|w x| of a float64 direct convolution (the bar the direct f32
    kernels meet, tests/test_ops_gpu.py), and the Winograd error no larger than 2x the direct f32
    kernel's own error on the same data (+1e-7 of slack): it is the same f32 accuracy class;
  * exact on small integers (every transform and product is exact in f32 there);
  * tile independence: every Winograd tile gives the same bits;
  * end to end: synthetic SqueezeNet @224 vs the oracle fixture (<= 1e-5 max-abs, same argmax) with
    the default plan and with every expand3x3 on Winograd (fusion off), the B = 256 properties, and
    MNIST (no eligible conv: untouched).
"""
import os

import numpy as np
import pytest

from test_x3_gpu import _conv_model, conv_f64

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


@pytest.fixture(autouse=True)
def default_algo(monkeypatch):
    monkeypatch.delenv("ORE_NO_WINOGRAD", raising=False)
    monkeypatch.delenv("ORE_WINO_TILE", raising=False)
    monkeypatch.delenv("ORE_FIRE_WINO", raising=False)


# N, C, H, W, M: the SqueezeNet expand3x3 families and ragged edges (odd planes, 1-pixel planes,
# partial 32-channel tiles, a tile group spanning images)
CASES = [
    (3, 16, 54, 54, 64),    # fire2 / fire3
    (2, 32, 54, 54, 128),   # fire4
    (3, 48, 27, 27, 192),   # fire6 / fire7
    (2, 64, 27, 27, 256),   # fire8
    (3, 64, 13, 13, 256),   # fire9
    (2, 16, 5, 7, 40),      # odd plane, partial channel tile
    (3, 16, 1, 1, 32),      # 1 x 1 plane: only the centre tap
    (2, 32, 2, 3, 24),
    (1, 16, 9, 1, 16),      # one column
    (5, 32, 6, 6, 33),      # 33 channels: one live row in the last tile
]


def _conv(ctx, algo, x, w, b, relu=False):
    import ore
    ctx.set_conv_algo(algo)
    try:
        return _np(ore.convolution(ctx, _t(x), _t(w), _t(b) if b is not None else None, auto_pad="NOTSET",
                                   pads=[1, 1, 1, 1], strides=(1, 1), fuse_relu=relu))
    finally:
        ctx.set_conv_algo(ore.CONV_ALGO_DIRECT)


@pytest.mark.parametrize("case", CASES)
def test_wino_conv_vs_f64(gpu_ctx, case):
    """Per-op ABI: Winograd vs float64 and vs the direct f32 kernel's own error."""
    import ore
    N, C, H, W, M = case
    rng = np.random.default_rng(sum(case))
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = (rng.standard_normal((M, C, 3, 3)) * np.sqrt(2.0 / (C * 9))).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    ref, mag = conv_f64(x, w, b, [1] * 4, (1, 1))
    yw = _conv(gpu_ctx, ore.CONV_ALGO_WINOGRAD, x, w, b)
    yd = _conv(gpu_ctx, ore.CONV_ALGO_DIRECT, x, w, b)
    ew = np.abs(yw.astype(np.float64) - ref) / (mag + 1e-30)
    ed = np.abs(yd.astype(np.float64) - ref) / (mag + 1e-30)
    assert ew.max() <= 2e-6, ew.max()
    assert ew.max() <= 2.0 * ed.max() + 1e-7, (ew.max(), ed.max())
    assert not np.array_equal(yw, yd) or H * W == 1  # the Winograd kernel really ran


def test_wino_relu_and_no_bias(gpu_ctx):
    import ore
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, 16, 11, 12)).astype(np.float32)
    w = rng.standard_normal((48, 16, 3, 3)).astype(np.float32)
    ref, mag = conv_f64(x, w, None, [1] * 4, (1, 1))
    y = _conv(gpu_ctx, ore.CONV_ALGO_WINOGRAD, x, w, None, relu=True)
    assert (y >= 0).all()
    err = np.abs(y.astype(np.float64) - np.maximum(ref, 0)) / (mag + 1e-30)
    assert err.max() <= 2e-6, err.max()


def test_wino_exact_on_small_integers(gpu_ctx):
    """Small integers: U = G g G^T is exact in quarters, V and every partial sum are small
    integers or quarters, so the Winograd conv equals the float64 result bit for bit."""
    import ore
    rng = np.random.default_rng(7)
    x = rng.integers(-8, 9, (2, 32, 14, 13)).astype(np.float32)
    w = rng.integers(-4, 5, (64, 32, 3, 3)).astype(np.float32)
    b = rng.integers(-3, 4, 64).astype(np.float32)
    ref, _ = conv_f64(x, w, b, [1] * 4, (1, 1))
    y = _conv(gpu_ctx, ore.CONV_ALGO_WINOGRAD, x, w, b)
    np.testing.assert_array_equal(y, ref.astype(np.float32))


@pytest.mark.parametrize("ci", [0, 3, 4, 5, 9])
def test_wino_tiles_bit_identical(gpu_ctx, ci, monkeypatch):
    """Every Winograd tile (ORE_WINO_TILE=0..4; 4 = the LDS-staged kernel) computes each output the
    same way: identical bits;
    the model reports the tile it ran."""
    import ore
    N, C, H, W, M = CASES[ci]
    rng = np.random.default_rng(3)
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, 3, 3)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    mb = _conv_model((1, C, H, W), w, b, [1] * 4, [1, 1])
    base = ore.Model.TILE_NAMES.index("wino 32x32 d4")
    outs = []
    for t in range(5):
        monkeypatch.setenv("ORE_WINO_TILE", str(t))
        m = ore.Model(gpu_ctx, mb, max_batch=N)
        outs.append(_np(m.run(_t(x))))
        assert m.tiles()[0] == base + t, (m.tiles(), base + t)
        m.close()
    for o in outs[1:]:
        np.testing.assert_array_equal(outs[0], o)


def test_wino_model_choice(gpu_ctx):
    """The model takes Winograd for eligible convs only (C % 16 == 0, 3x3, stride 1, pad 1) and never
    with winograd=False; the per-op and model paths agree bit for bit."""
    import ore
    names = ore.Model.TILE_NAMES
    rng = np.random.default_rng(9)
    for C, pads, st, want in ((16, [1] * 4, [1, 1], True), (12, [1] * 4, [1, 1], False),
                              (16, [0] * 4, [1, 1], False), (16, [1] * 4, [2, 2], False)):
        w = rng.standard_normal((32, C, 3, 3)).astype(np.float32)
        b = rng.standard_normal(32).astype(np.float32)
        x = rng.standard_normal((2, C, 10, 10)).astype(np.float32)
        mb = _conv_model((1, C, 10, 10), w, b, pads, st)
        for wg in (True, False):
            m = ore.Model(gpu_ctx, mb, max_batch=2, winograd=wg)
            y = _np(m.run(_t(x)))
            assert names[m.tiles()[0]].startswith("wino") == (want and wg), (C, pads, st, wg, names[m.tiles()[0]])
            if want and wg:
                yo = _conv(gpu_ctx, ore.CONV_ALGO_WINOGRAD, x, w, b)
                np.testing.assert_array_equal(y.reshape(yo.shape), yo)
            m.close()


@pytest.mark.parametrize("fusion", [None, 0])
def test_squeezenet_synth_vs_oracle_wino(gpu_ctx, fusion):
    """The default f32 plan (Winograd where no direct fusion takes the conv) and the unfused graph
    (every expand3x3 on Winograd) vs the oracle fixture: <= 1e-5 max-abs, same argmax."""
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=2)
    if fusion is not None:
        m.set_fusion(fusion)
    names = [ore.Model.TILE_NAMES[t] if t >= 0 else "" for t in m.tiles()]
    nw = sum(n.startswith("wino") for n in names)
    assert nw == 8 if fusion == 0 else nw >= 2, names  # default: fire8 / fire9 expand3x3 at least
    y = _np(m.run(_t(squeezenet_inputs())))
    m.close()
    assert np.abs(y - ref).max() <= 1e-5, np.abs(y - ref).max()
    assert np.array_equal(y.argmax(1), ref.argmax(1))


def test_squeezenet_wino_batch256_properties(gpu_ctx):
    """B = 256 with the default plan: rows sum to 1, each image bit-identical to itself run alone,
    top-1 equal to the direct-kernel model's and probabilities within 2e-5 of it (each path is within
    1e-5 of the oracle, test_squeezenet_synth_vs_oracle_wino; their errors need not cancel)."""
    import ore
    from ore import squeezenet
    x = _t(squeezenet.synthetic_input(256, 224, seed=123))
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=256)
    y = _np(m.run(x))
    assert np.isfinite(y).all() and np.abs(y.sum(1) - 1.0).max() <= 1e-5
    for i in (0, 77, 255):
        assert np.array_equal(_np(m.run(x[i:i + 1].contiguous()))[0], y[i]), i
    m.close()
    d = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=256, winograd=False)
    yd = _np(d.run(x))
    d.close()
    assert np.array_equal(y.argmax(1), yd.argmax(1))
    assert np.abs(y - yd).max() <= 2e-5


def test_mnist_untouched(gpu_ctx):
    """MNIST's convs are 5x5: no Winograd plan, results equal with and without the flag."""
    import ore
    from ore import onnx_wire
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        mb = f.read()
    x = _t(onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy())
    ys = []
    for wg in (True, False):
        m = ore.Model(gpu_ctx, mb, max_batch=1, winograd=wg)
        ys.append(_np(m.run(x)))
        m.close()
    np.testing.assert_array_equal(ys[0], ys[1])


def test_set_conv_algo_rejects_unknown(gpu_ctx):
    import ore
    with pytest.raises(ore.OreError):
        gpu_ctx.set_conv_algo(7)


@pytest.mark.parametrize("case", [
    # C, H, W, S1, E1, E3, S2 (as tests/test_model_gpu.py::test_fire_fusion_bit_identical)
    (16, 12, 12, 16, 64, 64, 16),     # fire2 -> squeeze3 family
    (32, 9, 8, 32, 128, 128, 48),     # fire5 -> squeeze6 (MFS = 3), W = 8
    (24, 8, 7, 48, 192, 192, 64),     # fire7 -> squeeze8 (MFS = 4), odd W: right-edge tiles half outside
    (16, 13, 13, 16, 64, 128, 32),    # unequal expands, 13 x 13 planes (odd H and W)
])
def test_fire_wino_fusion_bit_identical(gpu_ctx, case, monkeypatch):
    """The fused fire module with its expand3x3 by Winograd ("fire wino", opt-in ORE_FIRE_WINO=1) equals
    the separate kernels (Winograd expand3x3) bit for bit, and the oracle within the conv tolerance."""
    import ore
    import oracle
    from test_model_gpu import _fire_model
    monkeypatch.setenv("ORE_FIRE_MIN_COLS", "0")
    monkeypatch.setenv("ORE_FIRE_WINO", "1")
    C, H, W, S1, E1, E3, S2 = case
    mb = _fire_model(*case)
    x = np.random.default_rng(sum(case)).standard_normal((5, C, H, W)).astype(np.float32)
    vals = []
    for fusion in (ore.FUSE_ALL | ore.KEEP_VALUES, (ore.FUSE_ALL & ~ore.FUSE_FIRE) | ore.KEEP_VALUES):
        m = ore.Model(gpu_ctx, mb, max_batch=5)
        m.set_fusion(fusion)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("nr")))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        if fusion & ore.FUSE_FIRE:
            assert "fire wino" in names, names
        else:
            assert any(n.startswith("wino") for n in names), names
        m.close()
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, S2)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("hw", [64, 224])
def test_squeezenet_fire_wino_fusion(gpu_ctx, hw, monkeypatch):
    """SqueezeNet with the fire + squeeze pairs fused on the Winograd fire kernel: probabilities
    bit-identical to the separate (Winograd) kernels."""
    import ore
    from ore import squeezenet
    monkeypatch.setenv("ORE_FIRE_MIN_COLS", "0")
    monkeypatch.setenv("ORE_FIRE_WINO", "1")
    mb = squeezenet.build(hw)
    x = _t(squeezenet.synthetic_input(3, hw, seed=19))
    outs = []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_FIRE):
        m = ore.Model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        if fusion & ore.FUSE_FIRE:
            n = sum(1 for t in m.tiles() if t >= 0 and ore.Model.TILE_NAMES[t] == "fire wino")
            assert n == (5 if hw == 224 else 2), n
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("case", [
    # C, H, W, S1, E1 = E3, S2 (the expands read the S1-channel squeeze output)
    (16, 12, 12, 16, 64, 64, 16),     # fire2 family
    (32, 9, 8, 32, 128, 128, 48),     # even W, row wraps inside a tile group
    (16, 13, 13, 64, 256, 256, 64),   # fire9 family: odd H and W (half-outside edge tiles)
    (16, 6, 7, 48, 40, 40, 8),        # 40 channels: a partial 32-channel m tile, odd W
    (16, 1, 1, 16, 32, 32, 8),        # 1 x 1 plane: the centre tap only
])
def test_wino_e1_fusion_bit_identical(gpu_ctx, case, monkeypatch):
    """(3b), opt-in ORE_WINO_E1=1: the expand1x1 beside a Winograd expand3x3 runs inside the Winograd
    launch (conv_wino16_kernel E1, tile "wino16 32x16"): the Concat it writes equals the separate 1x1
    conv's bit for bit (ORE_WINO_E1=0), the model launches one conv fewer, and the oracle agrees
    within the conv tolerance."""
    import ore
    import oracle
    from test_model_gpu import _fire_model
    C, H, W, S1, E1, E3, S2 = case
    mb = _fire_model(*case)
    x = np.random.default_rng(sum(case) + 1).standard_normal((5, C, H, W)).astype(np.float32)
    names_all, vals = [], []
    for flag in ("1", "0"):
        monkeypatch.setenv("ORE_WINO_E1", flag)
        m = ore.Model(gpu_ctx, mb, max_batch=5)
        m.set_fusion((ore.FUSE_ALL & ~ore.FUSE_FIRE) | ore.KEEP_VALUES)
        y = _np(m.run(_t(x)))
        vals.append((y, m.read_value("cat")))
        names_all.append([ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0])
        m.close()
    fused, plain = names_all
    assert len(fused) == len(plain) - 1, (fused, plain)
    assert "wino16 32x16" in fused, fused
    np.testing.assert_array_equal(vals[0][1], vals[1][1])
    np.testing.assert_array_equal(vals[0][0], vals[1][0])
    ref = oracle.Model(mb).run(x, S2)
    np.testing.assert_allclose(vals[0][0].reshape(ref.shape), ref, rtol=1e-5, atol=1e-6)


def test_wino_e1_needs_equal_channels(gpu_ctx, monkeypatch):
    """Unequal expands (E1 != E3) keep the separate 1x1 conv."""
    import ore
    from test_model_gpu import _fire_model
    monkeypatch.setenv("ORE_WINO_E1", "1")
    mb = _fire_model(16, 8, 8, 16, 32, 64, 8)
    m = ore.Model(gpu_ctx, mb, max_batch=2)
    m.set_fusion(ore.FUSE_ALL & ~ore.FUSE_FIRE)
    names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
    m.close()
    assert sum(n.startswith("wino") for n in names) == 1 and len(names) == 4, names


def test_squeezenet_wino_e1_fusion(gpu_ctx, monkeypatch):
    """SqueezeNet @224 default plan at B = 3 (too few columns for the fused fire kernels, so every
    fire module's expands run separately): each expand1x1 inside its Winograd expand3x3 launch,
    probabilities bit-identical to ORE_WINO_E1=0."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(3, 224, seed=29))
    outs, counts = [], []
    for flag in ("1", "0"):
        monkeypatch.setenv("ORE_WINO_E1", flag)
        m = ore.Model(gpu_ctx, mb, max_batch=3)
        outs.append(_np(m.run(x)))
        counts.append(sum(1 for t in m.tiles() if t >= 0))
        if flag == "1":
            names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
            nf = names.count("wino16 32x16")
            assert nf >= 2, names  # fire8 / fire9 at least
        m.close()
    assert counts[0] == counts[1] - nf, counts
    np.testing.assert_array_equal(outs[0], outs[1])

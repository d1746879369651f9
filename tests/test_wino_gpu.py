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

from _knobs import conv_tile

from _convref import _conv_model, conv_f64

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


@pytest.mark.parametrize("ci", list(range(10)))
def test_wino_tiles_bit_identical(gpu_ctx, ci):
    """Every Winograd tile (ore_ctx_set_conv_tile, "wino 32x32 d4" .. "wino16 16x32", "wino lds")
    computes each output the same way: identical bits; the model reports the tile it ran."""
    import ore
    N, C, H, W, M = CASES[ci]
    rng = np.random.default_rng(3)
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, 3, 3)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    mb = _conv_model((1, C, H, W), w, b, [1] * 4, [1, 1])
    base = ore.Model.TILE_NAMES.index("wino 32x32 d4")
    outs = []
    for t in range(5):  # 4: the LDS-staged kernel
        with conv_tile(gpu_ctx, base + t):
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


@pytest.mark.parametrize("tile", [None, 4])
def test_wino_output_past_2gib(gpu_ctx, tile):
    """A Winograd conv whose output passes 2 GiB (fire8 / expand3x3 geometry at batch 2900: 2.16 GB
    out, 0.54 GB in): the launch is split into image chunks (32-bit buffer offsets), so the first
    and the last images equal the same images run on their own, bit for bit."""
    import torch
    import ore
    from _knobs import conv_tile
    N, C, H, W, M = 2900, 64, 27, 27, 256
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.randn((N, C, H, W), generator=g, device="cuda")
    w = torch.randn((M, C, 3, 3), generator=g, device="cuda") * 0.05
    b = torch.randn((M,), generator=g, device="cuda") * 0.1
    assert N * M * H * W * 4 > 2 ** 31
    gpu_ctx.set_conv_algo(ore.CONV_ALGO_WINOGRAD)
    try:
        def conv(t):
            kw = dict(auto_pad="NOTSET", pads=[1, 1, 1, 1], strides=(1, 1))
            if tile is None:
                return ore.convolution(gpu_ctx, t, w, b, **kw)
            with conv_tile(gpu_ctx, 36 + tile):
                return ore.convolution(gpu_ctx, t, w, b, **kw)
        y = conv(x)
        for sl in (slice(0, 2), slice(N - 3, N)):
            ys = conv(x[sl].contiguous())
            torch.cuda.synchronize()
            assert torch.equal(y[sl], ys)
        del y
    finally:
        gpu_ctx.set_conv_algo(ore.CONV_ALGO_DIRECT)
        torch.cuda.empty_cache()

"""The f32x3 path (ORE_LOAD_X3, csrc/ore_conv_x3.hip): f32 Conv / MatMul on the BF16 matrix cores
through an exact three-way bf16 split of both operands (six part products, f32 accumulation).

Parity bar, written per test:
  * each conv output within 2e-6 * sum|w x| of a float64 direct convolution (the bar the f32-MFMA
    kernels meet in test_ops_gpu.py), and the x3 error no larger than 2x the f32-MFMA kernels'
    own error on the same data (both are f32-accurate; their summation orders differ);
  * tile independence: every x3 tile gives the same bits;
  * end to end: MNIST-8 vs the reference's golden output (<= 1e-6 max|y|), synthetic
    SqueezeNet @224 vs the oracle fixture (<= 1e-5 max-abs, same argmax), B=256 properties.
"""
import os

import numpy as np
import pytest

from _knobs import conv_tile

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


X3_ALL = True


@pytest.fixture(autouse=True)
def x3_all(request):
    """Kernel-level tests put every conv on x3 (ORE_LOAD_X3_ALL); tests marked `hybrid` keep the
    default ORE_LOAD_X3 policy (x3 where it wins, the f32-MFMA fusions elsewhere)."""
    global X3_ALL
    X3_ALL = "hybrid" not in request.keywords
    yield
    X3_ALL = True


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


CASES = [
    # N, C, H, W, M, k, stride, pad: SqueezeNet families and ragged edges
    (2, 3, 45, 45, 96, 7, 2, 0),     # conv1 family (7x7 / s2, 49 taps: the 64-bit tap mask)
    (3, 16, 27, 27, 64, 3, 1, 1),    # expand3x3 family
    (2, 32, 13, 13, 128, 3, 1, 1),   # 13 x 13 planes (169 pixels per image: ragged tiles)
    (2, 96, 27, 27, 16, 1, 1, 0),    # squeeze 1x1
    (2, 48, 13, 13, 1000, 1, 1, 0),  # conv10 family: M = 1000 (partial M tile), K = 48 (K % 32 != 0)
    (3, 13, 10, 11, 40, 1, 1, 0),    # K = 13 (a partial k-group), odd plane (no 16-B epilogue)
    (1, 1, 28, 28, 8, 5, 1, 2),      # MNIST conv 1 (SAME-style pads, C = 1)
    (2, 5, 9, 7, 20, 3, 2, 1),       # strided 3x3, odd sizes
    # the window-staged kernel (stride 1, C % 8 == 0): channel-group / chunk / tap-padding cases
    (2, 48, 27, 27, 192, 3, 1, 1),   # fire6 family: G = 2, three 16-channel chunks
    (2, 64, 13, 13, 256, 3, 1, 1),   # fire9 family: G = 4, two chunks, 13 x 13 (128 x 64 window tiles)
    (3, 32, 54, 54, 128, 3, 1, 1),   # fire4 family: one 32-channel chunk, 6-row windows
    (2, 8, 14, 14, 16, 5, 1, 2),     # MNIST conv 2 family: 5 x 5, 25 taps x G = 2 (13 k-steps, padded)
]
WINDOW = {8, 9, 10, 11, 1, 2}  # case indices the window kernel takes


@pytest.mark.parametrize("case", CASES)
def test_x3_conv_vs_f64(gpu_ctx, case):
    """x3 conv within 2e-6 * sum|w x| of float64, and within 2x (+1 ulp-scale slack) of the
    f32-MFMA kernels' own error on the same data."""
    import ore
    N, C, H, W, M, k, st, pd = case
    rng = np.random.default_rng(sum(case))
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = (rng.standard_normal((M, C, k, k)) * np.sqrt(2.0 / (C * k * k))).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    mb = _conv_model((1, C, H, W), w, b, [pd] * 4, [st, st])
    ref, mag = conv_f64(x, w, b, [pd] * 4, (st, st))
    errs = {}
    for prec in ("f32", "f32x3"):
        m = ore.Model(gpu_ctx, mb, max_batch=N, precision=prec)
        y = _np(m.run(_t(x))).reshape(ref.shape)
        m.close()
        errs[prec] = np.abs(y.astype(np.float64) - ref) / (mag + 1e-30)
    assert errs["f32x3"].max() <= 2e-6, errs["f32x3"].max()
    assert errs["f32x3"].max() <= 2.0 * errs["f32"].max() + 1e-7, (errs["f32x3"].max(), errs["f32"].max())


def test_x3_exact_on_small_integers(gpu_ctx):
    """Small-integer operands: every part product and partial sum is exact, so the x3 conv equals
    the float64 result bit for bit (the split's hi part carries the whole value)."""
    import ore
    rng = np.random.default_rng(7)
    x = rng.integers(-8, 9, (2, 12, 14, 14)).astype(np.float32)
    w = rng.integers(-4, 5, (24, 12, 3, 3)).astype(np.float32)
    b = rng.integers(-3, 4, 24).astype(np.float32)
    mb = _conv_model((1, 12, 14, 14), w, b, [1, 1, 1, 1], [1, 1])
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f32x3", x3_all=X3_ALL)
    y = _np(m.run(_t(x)))
    m.close()
    ref, _ = conv_f64(x, w, b, [1] * 4, (1, 1))
    np.testing.assert_array_equal(y.reshape(ref.shape), ref.astype(np.float32))


def test_x3_split_is_exact_for_wide_exponents(gpu_ctx):
    """Operands spanning many binades (1e-20 .. 1e20 with full 24-bit significands): the split
    loses nothing, so a 1x1 conv with one-hot weights returns x exactly (times the weight)."""
    import ore
    rng = np.random.default_rng(11)
    mant = rng.uniform(1.0, 2.0, (2, 8, 6, 8))
    ex = rng.integers(-60, 60, mant.shape)
    x = (mant * np.exp2(ex) * rng.choice([-1, 1], mant.shape)).astype(np.float32)
    w = np.zeros((8, 8, 1, 1), np.float32)
    for i in range(8):
        w[i, (i * 3) % 8, 0, 0] = 1.0
    mb = _conv_model((1, 8, 6, 8), w, None, [0, 0, 0, 0], [1, 1])
    m = ore.Model(gpu_ctx, mb, max_batch=2, precision="f32x3", x3_all=X3_ALL)
    y = _np(m.run(_t(x))).reshape(2, 8, 6, 8)
    m.close()
    for i in range(8):
        np.testing.assert_array_equal(y[:, i], x[:, (i * 3) % 8])


@pytest.mark.parametrize("ci", [0, 1, 4, 8, 9])
def test_x3_tiles_bit_identical(gpu_ctx, ci):
    """Every x3 tile of a kernel family (ore_ctx_set_conv_tile: the gather kernel's, or the window
    kernel's for stride-1 geometries) runs the same per-output sequence: identical bits."""
    import ore
    case = CASES[ci]
    N, C, H, W, M, k, st, pd = case
    rng = np.random.default_rng(3)
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = rng.standard_normal((M, C, k, k)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    mb = _conv_model((1, C, H, W), w, b, [pd] * 4, [st, st])
    outs = []
    base = ore.Model.TILE_NAMES.index("x3w 128x128" if ci in WINDOW else "x3 128x128")
    for t in range(4):
        with conv_tile(gpu_ctx, base + t):
            m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f32x3", x3_all=X3_ALL)
        outs.append(_np(m.run(_t(x))))
        assert m.tiles()[0] == base + t, (m.tiles(), base + t)
        m.close()
    for o in outs[1:]:
        np.testing.assert_array_equal(outs[0], o)


@pytest.mark.parametrize("ci", sorted(WINDOW))
def test_x3_window_vs_gather(gpu_ctx, ci):
    """The window kernel (k order (tap, channel)) and the gather kernel (k order (channel, tap)) on
    the same stride-1 conv: both within the f32 bar of float64 (different summation orders)."""
    import ore
    N, C, H, W, M, k, st, pd = CASES[ci]
    rng = np.random.default_rng(ci)
    x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
    w = (rng.standard_normal((M, C, k, k)) * np.sqrt(2.0 / (C * k * k))).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
    mb = _conv_model((1, C, H, W), w, b, [pd] * 4, [st, st])
    ref, mag = conv_f64(x, w, b, [pd] * 4, (st, st))
    names = ore.Model.TILE_NAMES
    for win in ("0", "1"):  # 0: a gather tile forced (ore_ctx_set_conv_tile), 1: the default window kernel
        with conv_tile(gpu_ctx, names.index("x3 128x128") if win == "0" else -1):
            m = ore.Model(gpu_ctx, mb, max_batch=N, precision="f32x3", x3_all=X3_ALL)
        y = _np(m.run(_t(x))).reshape(ref.shape)
        assert names[m.tiles()[0]].startswith("x3w" if win == "1" else "x3 "), names[m.tiles()[0]]
        m.close()
        assert (np.abs(y - ref) / (mag + 1e-30)).max() <= 2e-6, win


def test_x3_mnist_golden(gpu_ctx):
    """MNIST-8 (real weights; its MatMul runs on the x3 kernel too) vs mnist_output_0.pb."""
    import ore
    from ore import onnx_wire
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        m = ore.Model(gpu_ctx, f.read(), max_batch=4, precision="f32x3", x3_all=X3_ALL)
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_output_0.pb")).to_numpy()
    y = _np(m.run(_t(x)))
    assert np.abs(y - g).max() <= 1e-6 * np.abs(g).max()
    assert y.argmax() == g.argmax() == 2
    assert all(t >= ore.Model.TILE_NAMES.index("x3 128x128") for t in m.tiles() if t >= 0)
    m.close()


@pytest.mark.hybrid
def test_x3_hybrid_mnist_golden(gpu_ctx):
    """MNIST-8 with the default x3 policy: conv 2 (5x5, 8 channels) on the window kernel, the rest
    on the f32-MFMA kernels; still within 1e-6 max|y| of mnist_output_0.pb."""
    import ore
    from ore import onnx_wire
    with open(os.path.join(GOLD, "mnist-8.onnx"), "rb") as f:
        m = ore.Model(gpu_ctx, f.read(), max_batch=4, precision="f32x3", x3_all=X3_ALL)
    x = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_data_0.pb")).to_numpy()
    g = onnx_wire.load_tensor(os.path.join(GOLD, "mnist_output_0.pb")).to_numpy()
    y = _np(m.run(_t(x)))
    assert np.abs(y - g).max() <= 1e-6 * np.abs(g).max()
    names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
    assert sum(n.startswith("x3w") for n in names) == 1, names
    m.close()


def _x3_model(gpu_ctx, hybrid, max_batch):
    import ore
    from ore import squeezenet
    return ore.Model(gpu_ctx, squeezenet.build(224), max_batch=max_batch, precision="f32x3", x3_all=not hybrid)


@pytest.mark.parametrize("hybrid", [True, False])
def test_x3_squeezenet_synth_vs_oracle_and_f64(gpu_ctx, hybrid):
    """Synthetic SqueezeNet @224: <= 1e-5 max-abs of the oracle (the bar), same argmax, and no
    farther from the float64 result than the oracle itself is (block summation makes the x3 convs
    more accurate than an f32 fma chain)."""
    from golden.make_golden import squeezenet_inputs
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    f64 = np.load(os.path.join(GOLD, "squeezenet_synth_f64.npz"))["output"]
    m = _x3_model(gpu_ctx, hybrid, 2)
    y = _np(m.run(_t(squeezenet_inputs())))
    m.close()
    assert np.abs(y - ref).max() <= 1e-5
    assert np.array_equal(y.argmax(1), ref.argmax(1))
    assert np.abs(y - f64).max() <= np.abs(ref - f64).max() * 1.5


@pytest.mark.parametrize("hybrid", [True, False])
def test_x3_squeezenet_batch256_properties(gpu_ctx, hybrid):
    """B = 256: rows sum to 1, each image equals itself run alone bit for bit, and the autotuned
    tiles change no bit."""
    import torch
    from ore import squeezenet
    m = _x3_model(gpu_ctx, hybrid, 256)
    x = squeezenet.synthetic_input(256, 224, seed=123)
    xt = _t(x)
    y = _np(m.run(xt))
    assert y.shape == (256, 1000) and np.isfinite(y).all()
    assert np.abs(y.sum(1) - 1.0).max() <= 1e-5
    for i in (0, 77, 255):
        yi = _np(m.run(xt[i:i + 1].contiguous()))
        assert np.array_equal(yi[0], y[i]), i
    out = torch.empty((256, 1000), device="cuda")
    m.autotune(xt, out)
    assert np.array_equal(_np(m.run(xt)), y)
    names = [ore_tile_name(t) for t in m.tiles() if t >= 0]
    m.close()
    if hybrid:  # conv1 + pool1 on the f32-MFMA walker, the expand3x3s and conv10 on x3
        assert names[0].startswith("epool") and sum(n.startswith("x3") for n in names) >= 6, names
    else:
        assert all(n.startswith("x3") for n in names), names


def ore_tile_name(t):
    import ore
    return ore.Model.TILE_NAMES[t]


def test_x3_node_level_parity(gpu_ctx):
    """Unfused x3 SqueezeNet @64: each conv node vs the oracle op on the GPU's own input."""
    import ore
    import oracle
    from ore import onnx_wire, squeezenet
    from golden.make_golden import mini_inputs
    mb = squeezenet.build(64)
    model = onnx_wire.decode_model(mb)
    inits = {t.name: t.to_numpy() for t in model.graph.initializer}
    m = ore.Model(gpu_ctx, mb, max_batch=4, precision="f32x3", x3_all=X3_ALL)
    m.set_fusion(ore.KEEP_VALUES)
    xt = _t(mini_inputs()[:2])
    _np(m.run(xt))
    n = 0
    for node in model.graph.node:
        if node.op_type != "Conv":
            continue
        a = node.attrs()
        x = m.read_value(node.input[0])
        y = m.read_value(node.output[0])
        w, b = inits[node.input[1]], inits[node.input[2]]
        ref, mag = conv_f64(x, w, b, a["pads"].ints, a["strides"].ints)
        assert (np.abs(y - ref) / (mag + 1e-30)).max() <= 2e-6, node.name
        n += 1
    assert n == 26
    m.close()

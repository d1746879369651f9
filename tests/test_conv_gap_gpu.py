"""f32 conv + GlobalAveragePool in one launch (ORE_FUSE_CONV_GAP on an f32 model: conv1x1_gap_f32_kernel,
SqueezeNet's conv10 -> relu10 -> pool10; reference convolution_op.rs:94-517, relu_op.rs:31-33,
global_average_pool_op.rs:33-51).

The fused launch must equal the unfused streaming conv + gap_kernel bit for bit (same operands, the same
k order and f32 fma chain, the same sequential pixel sum), on 16-B aligned padded planes (the LDS-DMA
stage) and on unpadded planes straight from the graph input (the plain-load stage), with partial
128-channel blocks, 1..8 32-pixel fragments and no Relu; and stay within f32 rounding of a float64
restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _gap_model(x_shape, layers):
    """Conv(+Relu) layers [(w, b, relu)] (1x1, stride 1, no pads), then GlobalAveragePool."""
    from ore import onnx_wire as w
    nodes, inits, vinfo = [], [], [w.encode_value_info("x", x_shape)]
    cur = "x"
    for i, (wt, b, relu) in enumerate(layers):
        ins = [cur, f"w{i}"] + ([f"b{i}"] if b is not None else [])
        inits.append(w.encode_tensor(f"w{i}", wt))
        vinfo.append(w.encode_value_info(f"w{i}", wt.shape))
        if b is not None:
            inits.append(w.encode_tensor(f"b{i}", b))
            vinfo.append(w.encode_value_info(f"b{i}", b.shape))
        nodes.append(w.encode_node("Conv", ins, [f"c{i}"], attrs=[w.encode_attr_ints("pads", [0] * 4),
                                                                   w.encode_attr_ints("strides", [1, 1])]))
        cur = f"c{i}"
        if relu:
            nodes.append(w.encode_node("Relu", [cur], [f"r{i}"]))
            cur = f"r{i}"
    nodes.append(w.encode_node("GlobalAveragePool", [cur], ["y"]))
    return w.encode_model("t", nodes, inits, vinfo, [w.encode_value_info("y", (1, 1, 1, 1))])


def _ref(x, layers):
    """float64 restatement: 1x1 convs (+ Relu), then the mean over the pixels."""
    a = x.astype(np.float64)
    for wt, b, relu in layers:
        a = np.einsum("mc,nchw->nmhw", wt[:, :, 0, 0].astype(np.float64), a)
        if b is not None:
            a = a + b.astype(np.float64)[None, :, None, None]
        if relu:
            a = np.maximum(a, 0.0)
    return a.mean(axis=(2, 3))


# (N, C, H, W, M, relu, direct): direct = the fused conv reads the graph input (unpadded planes)
CASES = [
    (3, 512, 13, 13, 1000, True, False),  # SqueezeNet conv10: 172-float planes, 8 m-blocks (last 104 wide)
    (2, 64, 13, 13, 200, True, True),     # 169-float planes from the input: plain-load stage
    (2, 32, 1, 1, 10, False, False),      # one pixel, no Relu
    (2, 96, 16, 16, 130, True, False),    # P = 256: eight fragments; 130 = 128 + 2
    (5, 64, 7, 5, 40, True, True),        # P = 35: two fragments, odd plane from the input
    (4, 128, 6, 6, 256, False, False),    # P = 36, two full m-blocks
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:5])) + ("r" if c[5] else "") + ("d" if c[6] else ""))
def test_conv_gap_f32_fused_equals_unfused(gpu_ctx, case):
    import ore
    N, C, H, W, M, relu, direct = case
    rng = np.random.default_rng(C * 7 + M)
    layers = []
    if direct:
        x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    else:
        x = rng.standard_normal((N, 8, H, W)).astype(np.float32)
        layers.append(((rng.standard_normal((C, 8, 1, 1)) * 0.5).astype(np.float32),
                       rng.standard_normal((C,)).astype(np.float32), True))
    layers.append(((rng.standard_normal((M, C, 1, 1)) * (1.0 / np.sqrt(C))).astype(np.float32),
                   rng.standard_normal((M,)).astype(np.float32), relu))
    mb = _gap_model((1,) + x.shape[1:], layers)
    outs, tiles = [], []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_CONV_GAP):
        m = ore.Model(gpu_ctx, mb, max_batch=N)
        m.set_fusion(fusion)
        outs.append(_np(m.run(_t(x))).reshape(N, M))
        tiles.append([ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0])
        m.close()
    assert "conv1x1 gap f32" in tiles[0] and "conv1x1 gap f32" not in tiles[1]
    np.testing.assert_array_equal(outs[0], outs[1])
    ref = _ref(x, layers)
    err = np.abs(outs[0] - ref).max()
    assert err <= 1e-5 * max(1.0, np.abs(ref).max()), err  # f32 accumulation over C <= 512 terms


def test_conv_gap_f32_unpadded_layout(gpu_ctx):
    """With ORE_FUSE_CONCAT off every plane is dense (169 floats at 13x13): the plain-load stage, still
    equal to the unfused launches."""
    import ore
    rng = np.random.default_rng(5)
    x = rng.standard_normal((3, 16, 13, 13)).astype(np.float32)
    layers = [((rng.standard_normal((64, 16, 1, 1)) * 0.3).astype(np.float32), rng.standard_normal(64).astype(np.float32), True),
              ((rng.standard_normal((300, 64, 1, 1)) * 0.1).astype(np.float32), rng.standard_normal(300).astype(np.float32), True)]
    mb = _gap_model((1, 16, 13, 13), layers)
    outs = []
    for fusion in (ore.FUSE_ALL & ~ore.FUSE_CONCAT, ore.FUSE_ALL & ~ore.FUSE_CONCAT & ~ore.FUSE_CONV_GAP):
        m = ore.Model(gpu_ctx, mb, max_batch=3)
        m.set_fusion(fusion)
        outs.append(_np(m.run(_t(x))).reshape(3, 300))
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("winograd", [True, False])
def test_conv_gap_f32_squeezenet224(gpu_ctx, winograd):
    """SqueezeNet @224 f32: conv10 + relu10 + pool10 fused == unfused, bit for bit, and the fused step
    is the one the benched plan runs."""
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = _t(squeezenet.synthetic_input(4, 224, seed=21))
    outs = []
    for fusion in (ore.FUSE_ALL, ore.FUSE_ALL & ~ore.FUSE_CONV_GAP):
        m = ore.Model(gpu_ctx, mb, max_batch=4, winograd=winograd)
        m.set_fusion(fusion)
        outs.append(_np(m.run(x)))
        names = [ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0]
        assert ("conv1x1 gap f32" in names) == (fusion == ore.FUSE_ALL)
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])

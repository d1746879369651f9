"""Config 2 (BASELINE.json configs[1]): SqueezeNet-1.0 at batch 1, the reference's own batch size
(convolution_op.rs:480 writes image 0 only), on the exact plan bench.py times as `b1_latency_ms`:
max_batch = 1 (so the fire fusions' size thresholds leave the separate kernels in place), conv tiles
autotuned at batch 1, issued three ways -- plain launches, one HIP-graph replay, and a graph with the
fire branches on two streams.  Each fixture image runs alone and must match the oracle's committed
output (tests/golden/squeezenet_synth_oracle.npz) within 1e-5 max-abs with the same argmax.

The real zoo weights (squeezenet1.0-8.onnx) are absent, so the reference's own golden pair
squeezenet_data_0.pb -> squeezenet_output_0.pb stays unpinned here; the zoo
image is fixture image 0 on the synthetic weights."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture()
def stream_ctx():
    import torch
    import ore
    s = torch.cuda.Stream()
    ctx = ore.Context(0, use_torch_stream=False)  # graph capture needs a non-null stream
    ctx.set_stream(s.cuda_stream)
    yield ctx, s
    s.synchronize()
    ctx.close()


@pytest.mark.parametrize("winograd", [True, False])
@pytest.mark.parametrize("mode", ["plain", "graph", "graph_2streams"])
def test_squeezenet_b1_plan_vs_oracle(stream_ctx, mode, winograd):
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs
    ctx, s = stream_ctx
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    x = squeezenet_inputs()
    m = ore.Model(ctx, squeezenet.build(224), max_batch=1, winograd=winograd)
    m.set_streams(2 if mode == "graph_2streams" else 1)
    xb = torch.empty((1, 3, 224, 224), device="cuda")
    out = torch.empty((1, m.output_elems), device="cuda")
    xb.copy_(torch.from_numpy(x[:1]))
    torch.cuda.synchronize()
    m.autotune(xb, out)  # batch-1 tiles, as bench.py's b1_latency
    tiles = [t for t in m.tiles() if t >= 0]
    names = {ore.Model.TILE_NAMES[t] for t in tiles}
    assert not any(n.startswith("fire") for n in names), names  # max_batch 1: the unfused fire kernels
    if mode != "plain":
        m.capture(xb, out)
    for i in range(2):  # each image alone, through the same buffers (the graph reads them at replay)
        xb.copy_(torch.from_numpy(x[i:i + 1]))
        torch.cuda.synchronize()
        if mode == "plain":
            m.run_into(xb, out)
        else:
            m.replay()
        s.synchronize()
        y = out.cpu().numpy()
        err = float(np.abs(y - ref[i:i + 1]).max())
        assert err <= 1e-5, (mode, i, err)
        assert y.argmax() == ref[i].argmax()
    m.close()


def test_squeezenet_b1_equals_batched_rows(stream_ctx):
    """The batch-1 plan (winograd off: every kernel in the reference's k order) and the headline
    max_batch-256 plan (fused kernels) give each image bit-identical probabilities: the fusions,
    tiles and batching change how outputs are issued, never an output's arithmetic."""
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs
    ctx, s = stream_ctx
    mb = squeezenet.build(224)
    x = torch.from_numpy(squeezenet_inputs()).cuda()
    big = ore.Model(ctx, mb, max_batch=256, winograd=False)
    yb = torch.empty((2, big.output_elems), device="cuda")
    torch.cuda.synchronize()
    big.run_into(x, yb)
    s.synchronize()
    one = ore.Model(ctx, mb, max_batch=1, winograd=False)
    for i in range(2):
        y1 = torch.empty((1, one.output_elems), device="cuda")
        xi = x[i:i + 1].contiguous()
        torch.cuda.synchronize()
        one.run_into(xi, y1)
        s.synchronize()
        np.testing.assert_array_equal(y1.cpu().numpy(), yb[i:i + 1].cpu().numpy())
    big.close()
    one.close()

"""Branch concurrency (ore_model_set_streams) and HIP-graph replay
(ore_model_graph_capture / _launch): both must leave every result bit-identical to the plain
single-stream run -- they only change how the same kernels are issued."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture()
def stream_ctx():
    import torch
    import ore
    s = torch.cuda.Stream()
    ctx = ore.Context(0, use_torch_stream=False)
    ctx.set_stream(s.cuda_stream)
    yield ctx, s
    s.synchronize()
    ctx.close()


@pytest.mark.parametrize("precision", ["f32", "f16"])
@pytest.mark.parametrize("batch", [1, 3])
def test_two_streams_bit_identical(stream_ctx, precision, batch):
    import torch
    import ore
    from ore import squeezenet
    ctx, s = stream_ctx
    mb = squeezenet.build(64)
    x = torch.from_numpy(squeezenet.synthetic_input(batch, 64, seed=4)).cuda()
    outs = []
    for streams in (1, 2):
        m = ore.Model(ctx, mb, max_batch=batch, precision=precision)
        m.set_streams(streams)
        out = torch.empty((batch, m.output_elems), device="cuda")
        torch.cuda.synchronize()
        m.run_into(x, out)
        s.synchronize()
        outs.append(out.cpu().numpy())
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


def test_two_streams_headline_plan(stream_ctx):
    """The bench's headline plan (SqueezeNet @224, batch 256, Winograd, the split fire modules whose
    expand1x1 / Winograd expand3x3 pairs run on two streams): bit-identical to one stream."""
    import torch
    import ore
    from ore import squeezenet
    ctx, s = stream_ctx
    mb = squeezenet.build(224)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.rand((256, 3, 224, 224), generator=g, device="cuda") * 100.0 - 50.0
    outs, paired = [], []
    for streams in (1, 2):
        m = ore.Model(ctx, mb, max_batch=256)
        m.set_streams(streams)
        out = torch.empty((256, m.output_elems), device="cuda")
        torch.cuda.synchronize()
        m.run_into(x, out)
        s.synchronize()
        outs.append(out.cpu().numpy())
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("streams", [1, 2])
def test_graph_replay_matches_run(stream_ctx, streams):
    import torch
    import ore
    from ore import squeezenet
    ctx, s = stream_ctx
    mb = squeezenet.build(224)
    m = ore.Model(ctx, mb, max_batch=2)
    m.set_streams(streams)
    x = torch.from_numpy(squeezenet.synthetic_input(2, 224, seed=1)).cuda()
    ref = torch.empty((2, m.output_elems), device="cuda")
    torch.cuda.synchronize()
    m.run_into(x, ref)
    s.synchronize()
    ref1 = ref.cpu().numpy()
    out = torch.empty_like(ref)
    m.capture(x, out)  # capture only: nothing runs yet
    m.replay()
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref1)
    # the graph reads whatever the captured input buffer holds at replay time
    x.copy_(torch.from_numpy(squeezenet.synthetic_input(2, 224, seed=2)).cuda())
    torch.cuda.synchronize()
    m.replay()
    s.synchronize()
    m.run_into(x, ref)
    s.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref.cpu().numpy())
    assert not np.array_equal(out.cpu().numpy(), ref1)
    m.close()


def test_graph_capture_errors(gpu_ctx):
    import torch
    import ore
    from ore import squeezenet
    m = ore.Model(gpu_ctx, squeezenet.build(64), max_batch=1)
    with pytest.raises(ore.OreError):
        m.replay()  # nothing captured
    with pytest.raises(ore.OreError):
        m.set_streams(3)
    m.close()

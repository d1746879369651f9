"""CPU: the synthetic SqueezeNet-1.0 graph, the ONNX wire codec, and the batch-extended oracle
walker on the benchmark topology."""
import os

import numpy as np

import oracle
from ore import onnx_wire, squeezenet

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def test_squeezenet_topology():
    m = onnx_wire.decode_model(squeezenet.build(224))
    ops = [n.op_type for n in m.graph.node]
    assert len(ops) == 66
    assert {o: ops.count(o) for o in set(ops)} == {"Conv": 26, "Relu": 26, "MaxPool": 3, "Concat": 8,
                                                   "Dropout": 1, "GlobalAveragePool": 1, "Softmax": 1}
    assert m.graph.input[0].name == "data_0" and m.graph.input[0].shape == [1, 3, 224, 224]
    assert m.graph.output[0].name == "softmaxout_1"
    n_weights = sum(int(np.prod(t.dims)) for t in m.graph.initializer)
    assert abs(n_weights * 4 / 1e6 - 4.994) < 0.01      # zoo file ~4.9 MB of f32 weights
    init_names = {t.name for t in m.graph.initializer}
    assert init_names <= {v.name for v in m.graph.input}  # IR-3 style: listed in graph.input


def test_macs():
    assert squeezenet.macs_per_image(224) == 818924576


def test_deterministic():
    assert squeezenet.build(64) == squeezenet.build(64)
    assert squeezenet.build(64, seed=1) != squeezenet.build(64)


def test_wire_roundtrip():
    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    t = onnx_wire.decode_tensor(onnx_wire.encode_tensor("a", a))
    assert t.name == "a" and t.dims == [3, 4] and np.array_equal(t.to_numpy(), a)
    s = np.array([1, 256], np.int64)
    t = onnx_wire.decode_tensor(onnx_wire.encode_tensor("s", s, use_raw=False))
    assert np.array_equal(t.to_numpy(), s)
    t = onnx_wire.decode_tensor(onnx_wire.encode_tensor("f", a, use_raw=False))
    assert np.array_equal(t.to_numpy(), a)


def test_golden_pb_files():
    x = onnx_wire.load_tensor(os.path.join(GOLD, "squeezenet_data_0.pb")).to_numpy()
    y = onnx_wire.load_tensor(os.path.join(GOLD, "squeezenet_output_0.pb")).to_numpy()
    assert x.shape == (1, 3, 224, 224) and y.shape == (1, 1000, 1, 1)
    assert int(y.argmax()) == 549 and abs(float(y.sum()) - 1.0) < 1e-5


def test_oracle_batch_extension_is_per_image():
    """Batch-N oracle == N independent batch-1 runs (the reference's per-image algorithm)."""
    mb = squeezenet.build(32)
    m = oracle.Model(mb)
    x = squeezenet.synthetic_input(3, 32, seed=2)
    y = m.run(x, 1000)
    for i in range(3):
        assert np.array_equal(m.run(x[i:i + 1], 1000)[0], y[i])
    assert np.abs(y.sum(1) - 1).max() < 1e-5


def test_committed_fixtures_reproduce():
    ref = np.load(os.path.join(GOLD, "squeezenet_mini_oracle.npz"))["output"]
    from golden.make_golden import mini_inputs
    y = oracle.Model(squeezenet.build(64)).run(mini_inputs(), 1000)
    assert np.array_equal(y, ref)

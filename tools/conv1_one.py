#!/usr/bin/env python3
"""Runs SqueezeNet's conv1 + Relu + pool1 (fused: the row-walking conv_pool_stream_kernel) a few times
at batch 256 through the walker, for rocprofv3 counter passes on one kernel.
usage: python tools/conv1_one.py [--reps 5] [--batch 256]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))

import numpy as np  # noqa: E402


def graph():
    from ore import onnx_wire as w
    rng = np.random.default_rng(0)
    wt = (rng.standard_normal((96, 3, 7, 7)) * np.sqrt(2.0 / 147)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, 96).astype(np.float32)
    nodes = [w.encode_node("Conv", ["x", "w", "b"], ["c"], attrs=[w.encode_attr_ints("strides", [2, 2])]),
             w.encode_node("Relu", ["c"], ["r"]),
             w.encode_node("MaxPool", ["r"], ["y"], attrs=[w.encode_attr_ints("kernel_shape", [3, 3]),
                                                         w.encode_attr_ints("strides", [2, 2])])]
    return w.encode_model("c1", nodes, [w.encode_tensor("w", wt), w.encode_tensor("b", b)],
                          [w.encode_value_info("x", (1, 3, 224, 224)), w.encode_value_info("w", wt.shape),
                           w.encode_value_info("b", b.shape)], [w.encode_value_info("y", (1, 96, 54, 54))])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import ore
    ctx = ore.Context(0)
    x = (torch.rand((a.batch, 3, 224, 224), device="cuda") * 100 - 50).contiguous()
    m = ore.Model(ctx, graph(), max_batch=a.batch)
    out = torch.empty((a.batch, m.output_elems), device="cuda")
    m.autotune(x, out)
    for _ in range(a.reps):
        m.run_into(x, out)
    torch.cuda.synchronize()
    print([ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0])
    m.close()
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Kernel-level timing of single-node graphs (one Conv(+Relu) or MaxPool node) through the
device walker, so weights are packed once and only the op's kernel is timed (HIP events on the
context stream).  Shapes default to the SqueezeNet-1.0 layers at batch 256.
usage: python tools/bench_ops.py [--batch 256] [--only conv|pool] [--names f8.e3,..] [--reps 20] [--tile T]
       [--pool-variant V]
(--tile / --pool-variant: ore_ctx_set_conv_tile / ore_ctx_set_pool_variant)"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))

import numpy as np  # noqa: E402

# name, Cin, H, Cout, k, stride, pad
CONVS = [("conv1", 3, 224, 96, 7, 2, 0), ("f2.sq", 96, 54, 16, 1, 1, 0), ("f2.e1", 16, 54, 64, 1, 1, 0),
         ("f2.e3", 16, 54, 64, 3, 1, 1), ("f4.sq", 128, 54, 32, 1, 1, 0), ("f4.e1", 32, 54, 128, 1, 1, 0),
         ("f4.e3", 32, 54, 128, 3, 1, 1), ("f6.sq", 256, 27, 48, 1, 1, 0), ("f6.e3", 48, 27, 192, 3, 1, 1),
         ("f8.e3", 64, 27, 256, 3, 1, 1), ("f9.e3", 64, 13, 256, 3, 1, 1), ("conv10", 512, 13, 1000, 1, 1, 0)]
POOLS = [("pool1", 96, 109, [0, 0, 0, 0]), ("pool3", 256, 54, [0, 0, 1, 1]), ("pool5", 512, 27, [0, 0, 0, 0])]


def conv_graph(cin, h, cout, k, stride, pad):
    from ore import onnx_wire as w
    rng = np.random.default_rng(0)
    wt = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, cout).astype(np.float32)
    nodes = [w.encode_node("Conv", ["x", "w", "b"], ["c"], attrs=[
        w.encode_attr_ints("pads", [pad] * 4), w.encode_attr_ints("strides", [stride, stride])]),
        w.encode_node("Relu", ["c"], ["y"])]
    ho = (h + 2 * pad - k) // stride + 1
    return w.encode_model("c", nodes, [w.encode_tensor("w", wt), w.encode_tensor("b", b)],
                          [w.encode_value_info("x", (1, cin, h, h)), w.encode_value_info("w", wt.shape),
                           w.encode_value_info("b", b.shape)], [w.encode_value_info("y", (1, cout, ho, ho))])


def pool_graph(c, h, pads):
    from ore import onnx_wire as w
    nodes = [w.encode_node("MaxPool", ["x"], ["y"], attrs=[
        w.encode_attr_ints("kernel_shape", [3, 3]), w.encode_attr_ints("pads", pads),
        w.encode_attr_ints("strides", [2, 2]), w.encode_attr_string("auto_pad", "NOTSET")])]
    return w.encode_model("p", nodes, [], [w.encode_value_info("x", (1, c, h, h))],
                          [w.encode_value_info("y", (1, c, 1, 1))])


def time_model(ctx, mb, x, reps):
    import ore
    import torch
    m = ore.Model(ctx, mb, max_batch=x.shape[0])
    out = torch.empty((x.shape[0], m.output_elems), device="cuda")
    for _ in range(3):
        m.run_into(x, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        m.run_into(x, out)
    e1.record()
    torch.cuda.synchronize()
    m.close()
    return e0.elapsed_time(e1) / reps * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tile", type=int, default=-1)
    ap.add_argument("--pool-variant", type=int, default=0)
    ap.add_argument("--names", default="", help="comma-separated layer names (default: all)")
    a = ap.parse_args()
    keep = set(a.names.split(",")) if a.names else None
    import torch
    import ore
    ctx = ore.Context(0)
    ctx.set_conv_tile(a.tile)
    ctx.set_pool_variant(a.pool_variant)
    tag = f"tile={a.tile} pool={a.pool_variant}"
    B = a.batch
    if a.only in ("", "conv"):
        for name, cin, h, cout, k, s, p in CONVS:
            if keep is not None and name not in keep:
                continue
            x = torch.randn((B, cin, h, h), device="cuda")
            us = time_model(ctx, conv_graph(cin, h, cout, k, s, p), x, a.reps)
            ho = (h + 2 * p - k) // s + 1
            tf = 2.0 * B * cout * ho * ho * cin * k * k / (us * 1e-6) / 1e12
            print(f"{tag} {name:8s} {us:9.1f} us {tf:7.1f} TF/s", flush=True)
    if a.only in ("", "pool"):
        for name, c, h, pads in POOLS:
            if keep is not None and name not in keep:
                continue
            x = torch.randn((B, c, h, h), device="cuda")
            us = time_model(ctx, pool_graph(c, h, pads), x, a.reps)
            ho = (h + pads[2] - 3) // 2 + 1
            gbs = 4.0 * B * c * (h * h + ho * ho) / (us * 1e-6) / 1e9
            print(f"{tag} {name:8s} {us:9.1f} us {gbs:7.1f} GB/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Standalone timing of SqueezeNet's 1x1 conv shapes (B = 256) per forced conv tile
(ORE_CONV_CFG), through single-node graphs (tools/bench_ops.py), with the achieved HBM rate of
the algorithmic bytes (input + output, f32).
usage: python tools/bench_1x1.py [--tiles 0,3,12,13,14,15,16] [--reps 20]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

# name, Cin, H, Cout
SHAPES = [("f2.sq", 96, 54, 16), ("f3.sq", 128, 54, 16), ("f4.sq", 128, 54, 32), ("f5.sq", 256, 27, 32),
          ("f6.sq", 256, 27, 48), ("f7.sq", 384, 27, 48), ("f8.sq", 384, 27, 64), ("f9.sq", 512, 13, 64),
          ("f2.e1", 16, 54, 64), ("f4.e1", 32, 54, 128), ("f6.e1", 48, 27, 192), ("f8.e1", 64, 27, 256),
          ("conv10", 512, 13, 1000)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="3,12,13,14,15,16,19")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import torch
    import ore
    from bench_ops import conv_graph, time_model
    ctx = ore.Context(0)
    B = a.batch
    for name, cin, h, cout in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn((B, cin, h, h), device="cuda")
        res = []
        for t in a.tiles.split(","):
            os.environ["ORE_CONV_CFG"] = t
            us = time_model(ctx, conv_graph(cin, h, cout, 1, 1, 0), x, a.reps)
            gbs = 4.0 * B * h * h * (cin + cout) / (us * 1e-6) / 1e9
            res.append(f"{t}:{us:7.1f}us {gbs / 1000:4.2f}TB/s")
        print(f"{name:7s} " + "  ".join(res), flush=True)
    os.environ.pop("ORE_CONV_CFG", None)
    ctx.close()


if __name__ == "__main__":
    main()

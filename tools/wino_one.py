#!/usr/bin/env python3
"""Runs one Conv + Relu node (default: SqueezeNet fire8/expand3x3 at batch 256) a few times through
the walker, for rocprofv3 counter passes on a single kernel.  usage: python tools/wino_one.py
[--c 64 --h 27 --m 256] [--tile T] [--direct] [--reps 5]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from bench_ops import conv_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c", type=int, default=64)
    ap.add_argument("--h", type=int, default=27)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tile", type=int, default=-1)
    ap.add_argument("--direct", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if a.tile >= 0:
        os.environ["ORE_WINO_TILE"] = str(a.tile)
    import torch
    import ore
    ctx = ore.Context(0)
    x = torch.randn((a.batch, a.c, a.h, a.h), device="cuda")
    m = ore.Model(ctx, conv_graph(a.c, a.h, a.m, 3, 1, 1), max_batch=a.batch, winograd=not a.direct)
    out = torch.empty((a.batch, m.output_elems), device="cuda")
    for _ in range(a.reps):
        m.run_into(x, out)
    torch.cuda.synchronize()
    print(ore.Model.TILE_NAMES[m.tiles()[0]])
    m.close()
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Times the pooled 1x1 conv (MaxPool 3x3/2 + Conv 1x1 + Relu, the pool reading a Relu) on its two
kernels at B = 256: SqueezeNet pool5 + fire9/squeeze (512 x 27 x 27 -> 64) and pool3 + fire5/squeeze
(256 x 54 x 54 -> 32), model = Relu -> MaxPool -> Conv -> Relu -> GAP (HIP events per run; the Relu and
GAP launches included).  usage: python tools/pool_sq_probe.py [--reps 20]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import ore
    from test_model_gpu import _pool_squeeze_model
    ctx = ore.Context(0)
    names = ore.Model.TILE_NAMES
    for (C, H, W, M, pads) in ((512, 27, 27, 64, [0, 0, 0, 0]), (256, 54, 54, 32, [0, 0, 1, 1])):
        mb, _ = _pool_squeeze_model(C, H, W, M, pads)
        x = torch.randn((256, C, H, W), device="cuda")
        ys = {}
        for tile in ("pool squeeze lds", "pool squeeze stream"):
            m = ore.Model(ctx, mb, max_batch=256)
            k = [i for i, t in enumerate(m.tiles()) if t >= 0 and names[t].startswith("pool squeeze")][0]
            m.set_tile(k, names.index(tile))
            out = torch.empty((256, m.output_elems), device="cuda")
            for _ in range(3):
                m.run_into(x, out)
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(a.reps):
                m.run_into(x, out)
            ev[1].record()
            torch.cuda.synchronize()
            ys[tile] = out.clone()
            print(f"C{C} {H}x{W} M{M} {tile}: {1000 * ev[0].elapsed_time(ev[1]) / a.reps:.1f} us/run", flush=True)
            m.close()
        print("  equal:", bool(torch.equal(ys["pool squeeze lds"], ys["pool squeeze stream"])))
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Times the fused first conv + pool1 + squeeze (SqueezeNet conv1 geometry, B = 256 @224) on the window
kernel and on the band walker: conv1 -> Relu -> MaxPool -> Conv 1x1 (16) -> Relu -> GAP, per-launch HIP
event time of the whole model (the GAP is ~10 us).  ORE_LIB selects an experiment build.
usage: python tools/band_probe.py [--reps 20]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import ctypes
    import numpy as np
    import torch
    import ore
    lib = ctypes.CDLL(ore._lib.LIB_PATH)
    from test_model_gpu import _conv_pool_squeeze_model
    mb = _conv_pool_squeeze_model(224, 224, 96, 16, [0, 0, 0, 0])
    ctx = ore.Context(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.rand((a.batch, 3, 224, 224), generator=g, device="cuda") * 100.0 - 50.0
    ys = {}
    for name in ("epool window f32", "epool band f32"):
        m = ore.Model(ctx, mb, max_batch=a.batch)
        m.set_tile(0, ore.Model.TILE_NAMES.index(name))
        out = torch.empty((a.batch, m.output_elems), device="cuda")
        for _ in range(3):
            m.run_into(x, out)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.reps):
            m.run_into(x, out)
        ev[1].record()
        torch.cuda.synchronize()
        ys[name] = out.clone()
        if name == "epool band f32" and hasattr(lib, "ore_debug_stamps_band"):  # a stamps build
            st = np.zeros((1024, 8), dtype=np.uint64)
            assert lib.ore_debug_stamps_band(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes)) == 0
            st = st[: min(a.batch, 256)].astype(np.float64)
            tot = st.sum(1).mean()
            names = ["barrier T + top", "K loops", "epilogues", "-", "barrier E", "squeeze", "window store", "tail"]
            print("wave-0 phase shares (s_memtime):", ", ".join(f"{n} {100 * st[:, k].mean() / tot:.1f}%"
                                                               for k, n in enumerate(names)), f"total {tot:.0f}")
        print(f"{name}: {1000 * ev[0].elapsed_time(ev[1]) / a.reps:.1f} us/run "
              f"(ran {ore.Model.TILE_NAMES[m.tiles()[0]]})", flush=True)
        m.close()
    print("equal:", bool(torch.equal(ys["epool window f32"], ys["epool band f32"])))
    ctx.close()


if __name__ == "__main__":
    main()

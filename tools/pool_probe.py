#!/usr/bin/env python3
"""Phase shares of the fused expand1x1 + pool3 + fire5/squeeze launch (pool_conv1x1_f32_kernel with e1
recomputed) from wave-0 s_memtime stamps: experiment build only (PATCHES=tools/patches/pool_stamps.patch
tools/build_exp.sh pool_stamps -DORE_STAMPS ore_pool_conv; ORE_LIB=lib/exp/libore_pool_stamps.so).
usage: python tools/pool_probe.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))


def main():
    import numpy as np
    import torch
    import ore
    from ore import squeezenet
    lib = ctypes.CDLL(ore._lib.LIB_PATH)
    ctx = ore.Context(0)
    B = 256
    m = ore.Model(ctx, squeezenet.build_calibrated(224), max_batch=B)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    x = torch.rand((B, 3, 224, 224), generator=g, device="cuda") * 100.0 - 50.0
    out = torch.empty((B, m.output_elems), device="cuda")
    for _ in range(3):
        m.run_into(x, out)
    torch.cuda.synchronize()
    st = np.zeros((4096, 16), dtype=np.uint64)
    assert lib.ore_debug_stamps_ps(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes)) == 0
    st = st[: B * 14].astype(np.float64)
    tot = st[:, 12].mean()
    names = ["barrier A", "e1 / LDS write", "barrier B", "loads + pool", "barrier C", "squeeze"]
    for kind, off in (("e1 chunks", 0), ("loaded chunks", 6)):
        print(kind + ":", ", ".join(f"{n} {100 * st[:, off + k].mean() / tot:.1f}%" for k, n in enumerate(names)))
    print(f"workgroup total {tot:.0f} ticks (median {np.median(st[:, 12]):.0f})")
    m.close()
    ctx.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Phase timing from s_memtime stamps (experiment build only: PATCHES=tools/patches/stamps.patch tools/build_exp.sh stamps "-DORE_STAMPS"
"ore_conv_wino ore_conv1_f32", run with ORE_LIB=lib/exp/libore_stamps.so).  Wave 0 of each workgroup
stamps kernel entry, the end of its prologue, its K loop(s) and its exit; the hardware ids say which
CU it ran on.  Prints per-phase medians and how many workgroups overlapped on a CU.
usage: python tools/stamps.py [--batch 256]"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402


def cu_key(hw, xcc):
    return (int(xcc) & 15, (int(hw) >> 13) & 7, (int(hw) >> 8) & 15)


def overlap_stats(starts, ends, keys):
    """mean number of workgroups resident on the same CU at the start of each workgroup"""
    by = {}
    for s, e, k in zip(starts, ends, keys):
        by.setdefault(k, []).append((s, e))
    conc = []
    for iv in by.values():
        for s, e in iv:
            conc.append(sum(1 for s2, e2 in iv if s2 <= s < e2))
    return float(np.mean(conc)), len(by)


def wino(lib, ctx, name, tile=40, batch=256):
    import torch
    import ore
    from bench_ops import CONVS, conv_graph
    spec = [c for c in CONVS if c[0] == name][0]
    _, cin, h, cout, k, s, pad = spec
    ctx.set_conv_tile(tile)
    m = ore.Model(ctx, conv_graph(cin, h, cout, k, s, pad), max_batch=batch)
    x = torch.randn(batch, cin, h, h, device="cuda")
    out = torch.empty((batch, m.output_elems), device="cuda")
    for _ in range(2):
        m.run_into(x, out)
    torch.cuda.synchronize()
    assert lib.ore_debug_stamps_wino_clear() == 0
    m.run_into(x, out)
    torch.cuda.synchronize()
    st = np.zeros(1 << 17, dtype=np.uint64)
    assert lib.ore_debug_stamps_wino(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes)) == 0
    m.close()
    ctx.set_conv_tile(-1)
    st = st.reshape(-1, 8).astype(np.int64)
    st = st[st[:, 3] > 0]
    t0 = st[:, 0].min()
    pro, kl, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    keys = [cu_key(a, b) for a, b in zip(st[:, 4], st[:, 5])]
    conc, ncu = overlap_stats(st[:, 0], st[:, 3], keys)
    nks = cin // 4
    print(f"{name}: {len(st)} WGs on {ncu} CUs, span {(st[:, 3].max() - t0)} cyc; per WG median: prologue+first DMA "
          f"{int(np.median(pro))}, K loop {int(np.median(kl))} (MFMA content {nks * 32 * 32} per wave), epilogue "
          f"{int(np.median(epi))}, total {int(np.median(st[:, 3] - st[:, 0]))}; p90 total "
          f"{int(np.percentile(st[:, 3] - st[:, 0], 90))}; resident WGs per CU at a WG's start {conc:.2f}")
    if (st[:, 7] > 0).all():  # tools/patches/wino_stamps_prologue.patch: slot 7 just before the first stage's DMAs
        ix = st[:, 7] - st[:, 0]
        print(f"{name}: prologue = index arithmetic + LDS zero / bias {int(np.median(ix))} + first stage DMA to landed "
              f"{int(np.median(st[:, 1] - st[:, 7]))} cycles, median")
    if (st[:, 6] > 0).all():  # tools/patches/wino_stamps_drain.patch: slot 6 after the stores' vmcnt(0)
        dr = st[:, 6] - st[:, 3]
        print(f"{name}: epilogue = transform + store issue {int(np.median(epi))} + store drain {int(np.median(dr))} "
              f"(p10 {int(np.percentile(dr, 10))}, p90 {int(np.percentile(dr, 90))}) cycles, median")


def conv1(lib, ctx, batch=256):
    import torch
    import ore
    from ore import squeezenet
    m = ore.Model(ctx, squeezenet.build(224), max_batch=batch)
    x = torch.from_numpy(squeezenet.synthetic_input(batch, 224, seed=3)).cuda()
    out = torch.empty((batch, m.output_elems), device="cuda")
    m.autotune(x, out, reps=2)
    names = [ore.Model.TILE_NAMES[t] if t >= 0 else "-" for t in m.tiles()]
    for _ in range(2):
        m.run_into(x, out)
    torch.cuda.synchronize()
    st = np.zeros(1 << 16, dtype=np.uint64)
    assert lib.ore_debug_stamps_c3(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes)) == 0
    m.close()
    st = st.reshape(-1, 128).astype(np.int64)
    st = st[st[:, 31] > 0]
    st = st.reshape(-1, 128).astype(np.int64) if st.shape[1] != 128 else st
    # the epilogue after K loop 3, every wave: j = 0 K loop end; fragment i: 1 + 5 i conv tile written,
    # 2 + 5 i past its barrier, 3 + 5 i pooled block written, 4 + 5 i past its barrier, 5 + 5 i squeeze
    labels = []
    for i in range(3):
        labels += [f"f{i}.ctw", f"f{i}.ctbar", f"f{i}.poolw", f"f{i}.poolbar", f"f{i}.sq"]
    d = st[st[:, 3] > 4]
    for w in range(4):
        s = d[:, 32 + 16 * w: 32 + 16 * w + 16]
        seg = s[:, 1:] - s[:, :-1]
        print(f"  wave {w} mean: " + ", ".join(f"{lb} {int(np.mean(seg[:, j]))}" for j, lb in enumerate(labels)))
    print(f"conv1 plan tile: {names[0]}; {len(st)} WGs")
    kls, epis, firsts = [], [], []
    for r in st:
        nt = int(r[3])
        firsts.append(r[4] - r[0])
        for i in range(min(nt, 13)):
            s, ke = r[4 + 2 * i], r[5 + 2 * i]
            nxt = r[4 + 2 * (i + 1)] if i + 1 < min(nt, 13) else (r[31] if i + 1 == nt else None)
            kls.append(ke - s)
            if nxt is not None:
                epis.append(nxt - ke)
    nt0 = min(int(st[:, 3].min()), 13)
    kl_i = [int(np.median(st[:, 5 + 2 * i] - st[:, 4 + 2 * i])) for i in range(nt0)]
    ep_i = [int(np.median(st[:, 4 + 2 * (i + 1)] - st[:, 5 + 2 * i])) for i in range(nt0 - 1)]
    print("conv1 per tile index: K loop", kl_i, "epilogue", ep_i)
    keys = [cu_key(a, b) for a, b in zip(st[:, 1], st[:, 2])]
    conc, ncu = overlap_stats(st[:, 0], st[:, 31], keys)
    print(f"conv1: tiles per WG {int(np.median(st[:, 3]))}, span {st[:, 31].max() - st[:, 0].min()} cyc; median "
          f"prologue+first window {int(np.median(firsts))}, K loop {int(np.median(kls))} (MFMA content "
          f"{74 * 6 * 64} per wave), epilogue {int(np.median(epis))} (p10 {int(np.percentile(epis, 10))}, p90 "
          f"{int(np.percentile(epis, 90))}); WGs per CU {conc:.2f} on {ncu} CUs")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    print(f"== {a.tag or os.environ.get('ORE_LIB', '')}")
    import torch
    torch.cuda.init()  # before the library's own HIP registration
    import ore
    lib = ctypes.CDLL(ore._lib.LIB_PATH)
    ctx = ore.Context(0)
    if hasattr(lib, "ore_debug_stamps_conv1"):  # built with the conv1 stamps too
        conv1(lib, ctx, a.batch)
    for name in ("f4.e3", "f6.e3", "f8.e3", "f9.e3"):
        wino(lib, ctx, name, batch=a.batch)


if __name__ == "__main__":
    main()

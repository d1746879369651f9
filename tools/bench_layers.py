#!/usr/bin/env python3
"""Per-step device times of the SqueezeNet-1.0 walker (HIP events around every step,
ore_model_enable_timing), median over reps, for quick A/B of kernel variants: run it once per
library (ORE_LIB=lib/exp/libore_X.so) in one GPU call.
usage: python tools/bench_layers.py [--precision f16] [--batch 256] [--reps 10] [--tag NAME]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("ORE_LIB", "libore.so")))
    ap.add_argument("--fusion", type=int, default=None, help="ore_model_set_fusion flags (default: the model's)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import ore
    from ore import squeezenet
    ctx = ore.Context(0)
    m = ore.Model(ctx, squeezenet.build(224), max_batch=a.batch, precision=a.precision)
    x = torch.from_numpy(squeezenet.synthetic_input(a.batch, 224, seed=0)).cuda()
    out = torch.empty((a.batch, m.output_elems), device="cuda")
    if a.fusion is not None:
        m.set_fusion(a.fusion)
    m.autotune(x, out)
    m.enable_timing(True)
    for _ in range(2):
        m.run_into(x, out)
    torch.cuda.synchronize()
    times = []
    for _ in range(a.reps):
        m.run_into(x, out)
        torch.cuda.synchronize()
        times.append(m.step_times_ms())
    steps = m.steps()
    med = np.median(np.array(times), axis=0)
    tiles = m.tiles()
    total = float(med.sum())
    print(f"[{a.tag}] {a.precision} B={a.batch} total {total:.3f} ms = {a.batch / total * 1e3:.0f} img/s")
    for st, t, tl in zip(steps, med, tiles):
        tn = ore.Model.TILE_NAMES[tl] if 0 <= tl < len(ore.Model.TILE_NAMES) else ""
        tf = st["flops"] * a.batch / (t * 1e-3) / 1e12 if t > 0 else 0.0
        print(f"  {st['name']:24s} {st['op']:18s} {t * 1e3:8.1f} us {tf:7.1f} TF/s {tn}")
    m.close()
    ctx.close()


if __name__ == "__main__":
    main()

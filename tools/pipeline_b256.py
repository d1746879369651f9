#!/usr/bin/env python3
"""Batch-split pipelining experiment: the 256-image step as P independent walkers of 256/P images
each on P HIP streams (one ore_ctx + arena per part), the later parts started with a time offset so
that different layer types (MFMA-bound 3x3 convs, HBM-bound squeezes / pools) run side by side.
Prints ms per 256-image step for P = 1, 2, 4 and each offset.
usage: python tools/pipeline_b256.py [--steps 20]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import ore
    from ore import squeezenet
    mb = squeezenet.build(224)
    x = torch.from_numpy(squeezenet.synthetic_input(256, 224, seed=0)).cuda()
    ref = None
    for parts in (1, 2, 4):
        B = 256 // parts
        streams = [torch.cuda.Stream() for _ in range(parts)]
        ctxs, models, xs, outs = [], [], [], []
        for i in range(parts):
            c = ore.Context(0, use_torch_stream=False)
            c.set_stream(streams[i].cuda_stream)
            m = ore.Model(c, mb, max_batch=B)
            xi = x[i * B:(i + 1) * B].contiguous()
            o = torch.empty((B, m.output_elems), device="cuda")
            m.autotune(xi, o)
            ctxs.append(c)
            models.append(m)
            xs.append(xi)
            outs.append(o)
        torch.cuda.synchronize()
        for offset_ms in ((0.0,) if parts == 1 else (0.0, 1.0, 2.0)):
            for _ in range(3):
                for i in range(parts):
                    models[i].run_into(xs[i], outs[i])
            torch.cuda.synchronize()
            # stagger: part i spins i * offset / parts ms on its stream before its first step
            for i in range(1, parts):
                with torch.cuda.stream(streams[i]):
                    torch.cuda._sleep(int(offset_ms * 1e-3 * 2.4e9 * i / parts))
            t0 = time.perf_counter()
            for _ in range(a.steps):
                for i in range(parts):
                    models[i].run_into(xs[i], outs[i])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            y = torch.cat(outs).cpu()
            if ref is None:
                ref = y
            same = bool(torch.equal(y, ref))
            print(f"parts={parts} offset={offset_ms} ms: {dt:.3f} ms/step (the offset spin included once) "
                  f"= {256 / dt * 1e3:.0f} img/s, outputs identical to P=1: {same}", flush=True)
        for m in models:
            m.close()
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()

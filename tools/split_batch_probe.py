#!/usr/bin/env python3
"""Experiment: the B = 256 step as S independent sub-batches on S HIP streams (one ore_ctx + model each),
launched back to back so their kernels can share the CUs, against the one-model headline plan.
usage: python tools/split_batch_probe.py [--splits 1 2 4] [--steps 20]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--streams-per-model", type=int, default=2)
    a = ap.parse_args()
    import torch
    import ore
    from ore import squeezenet
    mb = squeezenet.build_calibrated(224)
    g = torch.Generator(device="cuda")
    g.manual_seed(1000)
    x = torch.rand((a.batch, 3, 224, 224), generator=g, device="cuda") * 100.0 - 50.0
    ref = None
    for S in a.splits:
        n = a.batch // S
        streams = [torch.cuda.Stream() for _ in range(S)]
        ctxs, models, outs, xs = [], [], [], []
        for i in range(S):
            c = ore.Context(0, use_torch_stream=False)
            c.set_stream(streams[i].cuda_stream)
            m = ore.Model(c, mb, max_batch=n)
            m.set_streams(a.streams_per_model)
            xi = x[i * n:(i + 1) * n].contiguous()
            o = torch.empty((n, m.output_elems), device="cuda")
            m.autotune(xi, o)
            ctxs.append(c); models.append(m); outs.append(o); xs.append(xi)
        torch.cuda.synchronize()

        def step():
            for m, xi, o in zip(models, xs, outs):
                m.run_into(xi, o)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        y = torch.cat(outs).cpu()
        if ref is None:
            ref = y
        same = bool(torch.equal(y, ref))
        print(f"splits {S}: {1000 * dt:.4f} ms/step = {a.batch / dt:.0f} img/s (rows equal to splits {a.splits[0]}: {same})",
              flush=True)
        for m in models:
            m.close()
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does a squeeze 1x1 conv run slower right after its input was rewritten?  Times the fire3
squeeze shape standalone (B = 256) with and without a preceding full rewrite of its input
(a device copy), HIP events around the conv only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-rusty-inference-engine_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    import torch
    import ore
    from bench_ops import conv_graph
    ctx = ore.Context(0)
    B = 256
    for cin, h, cout in ((96, 54, 16), (128, 54, 16), (128, 54, 32)):
        x = torch.randn((B, cin, h, h), device="cuda")
        x2 = torch.randn_like(x)
        m = ore.Model(ctx, conv_graph(cin, h, cout, 1, 1, 0), max_batch=B)
        out = torch.empty((B, m.output_elems), device="cuda")
        for _ in range(3):
            m.run_into(x, out)
        torch.cuda.synchronize()
        res = {}
        for mode in ("cold", "rewritten", "cold", "rewritten"):
            ts = []
            for _ in range(10):
                if mode == "rewritten":
                    x.copy_(x2)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m.run_into(x, out)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000)
            ts.sort()
            res.setdefault(mode, []).append(ts[len(ts) // 2])
        print(f"{cin}->{cout} @{h}: " + "  ".join(f"{k} {min(v):.1f} us" for k, v in res.items()), flush=True)
        m.close()
    ctx.close()


if __name__ == "__main__":
    main()

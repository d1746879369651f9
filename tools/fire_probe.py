import os, sys, time
sys.path.insert(0, 'onnx-rusty-inference-engine_amd')
import numpy as np, torch, ore
from ore import squeezenet
ctx = ore.Context(0)
mb = squeezenet.build(224)
for B in (3, 256):
    x = torch.from_numpy(squeezenet.synthetic_input(B, 224, seed=5)).cuda()
    outs = {}
    for name, fl in (("base", ore.FUSE_ALL), ("fire", ore.FUSE_ALL | ore.FUSE_FIRE)):
        m = ore.Model(ctx, mb, max_batch=B)
        m.set_fusion(fl)
        o = torch.empty((B, m.output_elems), device="cuda")
        m.autotune(x, o)
        for _ in range(3): m.run_into(x, o)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20): m.run_into(x, o)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20 * 1e3
        outs[name] = o.cpu().numpy()
        print(f"B={B} {name}: {dt:.3f} ms/step, tiles {m.tiles()}", flush=True)
        m.close()
    d = np.abs(outs["base"] - outs["fire"]).max()
    print(f"B={B} max |fire - base| = {d}, identical: {np.array_equal(outs['base'], outs['fire'])}", flush=True)

"""Diagnostic: per Winograd tile, error vs float64 and the mismatch pattern against tile 0 (one case)."""
import sys, os
import numpy as np
import torch
torch.cuda.init()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onnx-rusty-inference-engine_amd"))
import ore
from _convref import _conv_model, conv_f64

N, C, H, W, M = [int(v) for v in sys.argv[1:6]]
rng = np.random.default_rng(3)
x = rng.uniform(-50, 50, (N, C, H, W)).astype(np.float32)
w = rng.standard_normal((M, C, 3, 3)).astype(np.float32)
b = rng.uniform(-0.1, 0.1, M).astype(np.float32)
ref = conv_f64(x, w, b, [1] * 4, [1, 1])
ctx = ore.Context(0)
mb = _conv_model((1, C, H, W), w, b, [1] * 4, [1, 1])
base = ore.Model.TILE_NAMES.index("wino 32x32 d4")
outs = []
for t in range(5):
    ctx.set_conv_tile(base + t)
    m = ore.Model(ctx, mb, max_batch=N)
    y = m.run(torch.from_numpy(x).cuda()); torch.cuda.synchronize()
    outs.append(y.cpu().numpy().reshape(N, M, H, W)); print("tile", m.tiles()); m.close()
for t, o in enumerate(outs):
    e = np.abs(o - ref).max()
    bad = np.argwhere(o != outs[0])
    print(t, "maxerr", e, "mismatch", len(bad))
    if len(bad):
        for ax, nm in enumerate("nmyx"):
            u, c = np.unique(bad[:, ax], return_counts=True)
            print("  ", nm, list(zip(u[:12].tolist(), c[:12].tolist())))

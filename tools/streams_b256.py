import sys, os, time
sys.path.insert(0, 'onnx-rusty-inference-engine_amd')
import torch, ore
from ore import squeezenet
ctx = ore.Context(0)
m = ore.Model(ctx, squeezenet.build(224), max_batch=256)
x = torch.from_numpy(squeezenet.synthetic_input(256, 224, seed=0)).cuda()
out = torch.empty((256, m.output_elems), device='cuda')
m.autotune(x, out)
for streams in (1, 2, 1, 2):
    m.set_streams(streams)
    for _ in range(3): m.run_into(x, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): m.run_into(x, out)
    e1.record(); torch.cuda.synchronize()
    print(f"streams={streams}: {e0.elapsed_time(e1)/20:.3f} ms/step", flush=True)

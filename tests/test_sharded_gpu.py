"""SURVEY.md §8(e) correctness check on the HIP path: a global batch split unevenly (3 / 2 images)
over 2 ranks (two processes on GPU 0), each rank running its slice through the HIP model, must gather
to exactly the rows of a single-process HIP run of the whole batch, bit for bit.  The collective here
is ore.parallel.run_sharded / gather_rows over gloo on host tensors (uneven blocks, padded); bench.py's
per-step gather_rows_into (all_gather_into_tensor, even blocks) runs over gloo in
tests/test_config4_gpu.py::test_bench_world2_gloo.  The RCCL all-gather of device tensors needs one
GPU per rank and is not covered on the one-GPU test box.  Uses the headline plan (max_batch 256:
fused kernels, Winograd on) in every process."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
N_IMAGES = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch():
    from ore import squeezenet
    return squeezenet.synthetic_input(N_IMAGES, 224, seed=11)


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "onnx-rusty-inference-engine_amd"))
    import torch
    import torch.distributed as dist
    import ore
    from ore import squeezenet
    from ore.parallel import run_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = ore.Context(0)
    model = ore.Model(ctx, squeezenet.build(224), max_batch=256)

    def run(xs):  # this rank's slice through the HIP model; rows back on the host for gloo
        if xs.shape[0] == 0:
            return torch.zeros((0, model.output_elems))
        y = model.run(xs.cuda().contiguous())
        torch.cuda.synchronize()
        return y.cpu()

    y = run_sharded(run, torch.from_numpy(_global_batch()))
    if rank == 0:
        np.save(out_path, y.numpy())
    dist.barrier()
    model.close()
    ctx.close()
    dist.destroy_process_group()


def test_hip_sharded_gather_matches_single_process(tmp_path, gpu_ctx):
    import torch
    import ore
    from ore import squeezenet
    out = str(tmp_path / "y.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=256)
    ref = m.run(torch.from_numpy(_global_batch()).cuda())
    torch.cuda.synchronize()
    ref = ref.cpu().numpy()
    m.close()
    assert got.shape == ref.shape == (N_IMAGES, 1000)
    np.testing.assert_array_equal(got, ref)

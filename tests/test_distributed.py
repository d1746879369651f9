"""CPU, world_size 2 (gloo): the batch-shard + logits-gather path that bench.py runs over RCCL.
Each rank computes its slice with the oracle (a CPU stand-in for the HIP model) and the gathered
rows must equal a single-process run bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ore.parallel import shard_bounds

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_bounds():
    for n in (0, 1, 7, 256, 2048, 2049):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "onnx-rusty-inference-engine_amd"))
    import torch
    import torch.distributed as dist
    import oracle
    from ore import squeezenet
    from ore.parallel import run_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = oracle.Model(squeezenet.build(32))
    x = torch.from_numpy(squeezenet.synthetic_input(n, 32, seed=4))

    def run(xs):
        return torch.from_numpy(model.run(xs.numpy(), 1000)) if xs.shape[0] else torch.zeros((0, 1000))

    y = run_sharded(run, x)
    if rank == 0:
        np.save(out_path, y.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [4, 5])
def test_sharded_gather_matches_single_process(tmp_path, n):
    import oracle
    from ore import squeezenet
    out = str(tmp_path / "y.npy")
    mp.spawn(_worker, args=(2, _free_port(), n, out), nprocs=2, join=True)
    got = np.load(out)
    ref = oracle.Model(squeezenet.build(32)).run(squeezenet.synthetic_input(n, 32, seed=4), 1000)
    assert np.array_equal(got, ref)


def _bench_leg_worker(rank, world, port, G, out_path):
    """bench.py's N > 1 data path with the oracle standing in for the HIP model: one seeded global
    batch, this rank's shard_bounds slice, gather_rows_into the preallocated [G, D] rows."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "onnx-rusty-inference-engine_amd"))
    import torch
    import torch.distributed as dist
    import oracle
    from ore import squeezenet
    from ore.parallel import gather_rows_into, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    xg = squeezenet.synthetic_input(G, 32, seed=6)
    lo, hi = shard_bounds(G, world, rank)
    out = torch.from_numpy(oracle.Model(squeezenet.build(32)).run(xg[lo:hi], 1000))
    gathered = torch.empty((G, 1000))
    gather_rows_into(gathered, out)
    with pytest.raises(ValueError):
        gather_rows_into(torch.empty((G + 1, 1000)), out)
    if rank == 0:
        np.save(out_path, gathered.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_bench_gather_leg(tmp_path):
    import oracle
    from ore import squeezenet
    out = str(tmp_path / "g.npy")
    mp.spawn(_bench_leg_worker, args=(2, _free_port(), 4, out), nprocs=2, join=True)
    got = np.load(out)
    ref = oracle.Model(squeezenet.build(32)).run(squeezenet.synthetic_input(4, 32, seed=6), 1000)
    assert np.array_equal(got, ref)

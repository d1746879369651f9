"""Batch sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Images are independent, so a global batch is split into contiguous per-rank slices with no
data-path collective; the only exchange is gathering the [n, classes] output rows (BASELINE.json
north_star: "RCCL over xGMI only to gather the final logits").  The reference has no
multi-device path at all: this is new, and `run_sharded` is what bench.py and
the world_size-2 gloo tests exercise.
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_bounds(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of rank's images (the first n % world ranks get one more)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local, n_total: int, group=None):
    """All-gather per-rank row blocks [n_r, D] (uneven n_r allowed) into [n_total, D] on every
    rank, in rank order.  Blocks are padded to ceil(n_total / world) rows for the collective."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rows = -(-n_total // world)
    D = local.shape[1]
    padded = torch.zeros((rows, D), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    out = torch.empty((world * rows, D), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, padded, group=group)
    parts = []
    for r in range(world):
        s, e = shard_bounds(n_total, world, r)
        parts.append(out[r * rows: r * rows + (e - s)])
    return torch.cat(parts, dim=0)


def gather_rows_into(gathered, local, group=None):
    """The per-step collective of bench.py: every rank holds an equal [n, D] block (n_total divisible
    by the world size, shard_bounds then gives rank r rows [r n, (r + 1) n)), all-gathered in rank
    order into the preallocated [world * n, D] `gathered` -- one all_gather_into_tensor (RCCL on
    device tensors, gloo on host tensors), no allocation per step."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if gathered.shape[0] != world * local.shape[0] or tuple(gathered.shape[1:]) != tuple(local.shape[1:]):
        raise ValueError(f"gathered {tuple(gathered.shape)} != world {world} x local {tuple(local.shape)}")
    dist.all_gather_into_tensor(gathered, local, group=group)
    return gathered


def run_sharded(run_fn: Callable, x_global, group=None):
    """Run `run_fn(x_slice) -> [n_slice, D]` on this rank's slice of x_global and return the
    gathered [n_total, D] on every rank."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    s, e = shard_bounds(x_global.shape[0], world, rank)
    local = run_fn(x_global[s:e])
    return gather_rows(local, x_global.shape[0], group)

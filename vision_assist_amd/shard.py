"""Multi-GPU sharding of the per-frame hot path.

Frames are independent: one process per GPU, frame i goes to rank i % world
(round-robin, like a video read by one reader and dealt to workers), and there
is NO collective on the data path.  torch.distributed is used only around the
timed region (barrier, max of the elapsed times over ranks) and to gather small
per-frame results on rank 0.

Each process has its own PathFinder angle cache (PathFinder.py:32 is
process-global), so a shard's A* results equal the reference run over that
shard's frames in order -- tests/test_shard.py checks exactly that with
world_size 2 over gloo.
"""
from __future__ import annotations

import os
import time
from typing import Callable

import torch


def dist_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_indices(n_frames: int, world: int, rank: int) -> list[int]:
    """Frames of `rank`: i % world == rank, in stream order."""
    return list(range(rank, n_frames, world))


def timed(fn: Callable[[], object], world: int, sync: Callable[[], None] | None = None) -> tuple[object, float]:
    """Run fn between barriers (+ device sync) and return (result, max elapsed seconds over ranks)."""
    import torch.distributed as dist
    on = world > 1 and dist.is_available() and dist.is_initialized()
    if sync:
        sync()
    if on:
        dist.barrier()
    t0 = time.perf_counter()
    out = fn()
    if sync:
        sync()
    if on:
        dist.barrier()
    el = time.perf_counter() - t0
    if on:
        backend = dist.get_backend()
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return out, el


def gather_by_frame(local: dict[int, object], world: int) -> dict[int, object] | None:
    """Gather {frame index: small result} from every rank onto rank 0 (None elsewhere)."""
    import torch.distributed as dist
    if world == 1 or not (dist.is_available() and dist.is_initialized()):
        return dict(local)
    parts = [None] * world if dist.get_rank() == 0 else None
    dist.gather_object(local, parts, dst=0)
    if dist.get_rank() != 0:
        return None
    out = {}
    for p in parts:
        out.update(p)
    return out

"""world_size-2 CPU (gloo) test of the multi-GPU sharding path used by bench.py.

Each rank takes its round-robin shard of a frame stream and runs the grid-level
path with its OWN angle-cache state (the oracle stands in for the device
pipeline: no GPU here); rank 0 gathers and checks that every frame's A* result
equals replaying that rank's shard, in order, through a fresh process state --
the multi-GPU parity definition of SURVEY.md §8e -- and that the timed region
reports the max over ranks.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

N_FRAMES = 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame_result(g, pf):
    from oracle import nav as onav
    from workloads.corridors import cells_rect, cells_to_mask
    out = onav.frame_nav(cells_to_mask(g), cells_rect(g), 640, 640, pf)
    return [[(c.coords.x, c.coords.y) for c in q[2]] for q in out["queries"]], sorted(pf.angle_cache)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from oracle import nav as onav
    from vision_assist_amd.shard import dist_env, gather_by_frame, shard_indices, timed
    from workloads.corridors import corridor_cells
    dist.init_process_group("gloo")
    w, r, _ = dist_env()
    assert (w, r) == (world, rank)
    mine = shard_indices(N_FRAMES, w, r)
    pf = onav.PathFinderOracle()  # per-process angle cache

    def work():
        return {i: _frame_result(corridor_cells(4000 + i), pf) for i in mine}

    local, elapsed = timed(work, w)
    allres = gather_by_frame(local, w)
    if r == 0:
        q.put((allres, elapsed))
    dist.destroy_process_group()


def test_two_rank_sharding_matches_per_shard_replay():
    from vision_assist_amd.shard import shard_indices
    from oracle import nav as onav
    from workloads.corridors import corridor_cells
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    allres, elapsed = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(allres) == list(range(N_FRAMES))
    assert elapsed > 0
    for r in range(world):
        pf = onav.PathFinderOracle()
        for i in shard_indices(N_FRAMES, world, r):
            assert allres[i] == tuple(_frame_result(corridor_cells(4000 + i), pf)) or \
                list(allres[i]) == list(_frame_result(corridor_cells(4000 + i), pf))


def test_shard_indices_partition():
    from vision_assist_amd.shard import shard_indices
    for world in (1, 2, 4, 8):
        seen = sorted(i for r in range(world) for i in shard_indices(37, world, r))
        assert seen == list(range(37))

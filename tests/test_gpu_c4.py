"""C4 (BASELINE.json configs[3]): YOLOv8s-seg 640x640, ONE frame per GPU per step, frames dealt round-robin to
the ranks (the reference processes frames one at a time, main.py:62-82), the network's own
masks -- not planted ones -- through post-processing, the mask choice and the grid / A* stage.

Two ranks on the one test GPU (on a node each rank takes its own GPU; the code path is the same), gloo for the
barrier and the result gather only.  Each rank runs a batch-1 FramePipeline over its shard, frame after frame,
with its own PathFinder angle cache.  Rank 0 gathers every frame's detections, chosen instance, rect, cells, A*
paths and costs; they are compared with each shard's frames replayed in order through the oracle chain
(tests/chain_util.py) with a fresh PathFinder state per shard -- the per-shard definition of the reference's
output -- whose outputs are the committed fixture tests/golden/chain_oracle.json.gz["c4/*"]
(tests/golden/gen_chain_fixtures.py).

Regimes: 'sparse' (1-5 compact detections per frame: a trained model's frames) and 'dense_box' (300 solid box
masks).  f32 (the reference's precision) must agree: every detection matched in 'sparse' (>= 98 % at the
300-detection max_det cut, where the two roundings break ties differently), the same chosen instance, cells
within one sample, identical A* paths and costs on identical cells.  bf16 agreement is measured and held to
floors (below).
"""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_FRAMES = 8
WORLD = 2
CONFIGS = [(dt, rg) for rg in ("sparse", "dense_box") for dt in ("f32", "bf16")]
# bf16 floors: measured agreement rates (gpurun_out/c4_agreement.json) rounded down
BF16_FLOOR = {"sparse": {"chosen": 0.75, "cells": 0.75, "paths": 0.75},      # measured 0.875 each
              "dense_box": {"chosen": 0.75, "cells": 0.75, "paths": 0.75}}  # measured 0.875 each


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame(i):
    from tests.chain_util import frame_batch
    return frame_batch(7000 + i, 1)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from tests.chain_util import weights
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.shard import dist_env, gather_by_frame, shard_indices, timed
    dist.init_process_group("gloo")
    w, r, local = dist_env()
    torch.cuda.set_device(local % torch.cuda.device_count())
    mine = shard_indices(N_FRAMES, w, r)
    frames = {i: _frame(i).cuda() for i in mine}
    out = {}
    for dtype, regime in CONFIGS:
        arch, fw = weights(regime)
        pipe = FramePipeline(arch, fw, 1, 640, 640, dtype=dtype)  # one frame per GPU per step
        local_res = {}

        def steps():
            for i in mine:
                res = pipe.run(frames[i], plant_mode=PLANT_NEVER)
                nf = res.frame(0)
                det, _ = pipe.post.det_tensor(0)
                chosen = int(pipe.post.chosen[0])
                # plain numpy through the gather and the queue (a torch tensor would travel as a shared-memory
                # handle that dies with this process)
                local_res[i] = {"det": det.numpy(), "chosen": chosen, "rect": pipe.post.rects[0].cpu().tolist(),
                                "cells": pipe.post.cells[0].cpu().numpy(), "status": nf.status,
                                "queries": [(qq["path"], float(qq["cost"]).hex() if qq["path"] else None)
                                            for qq in nf.queries]}

        _, elapsed = timed(steps, w, sync=torch.cuda.synchronize)
        allres = gather_by_frame(local_res, w)
        if r == 0:
            out[(dtype, regime)] = (allres, elapsed)
        del pipe
        torch.cuda.empty_cache()
    if r == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_c4_one_frame_per_rank_network_masks_vs_per_shard_oracle_replay():
    import torch

    from tests.chain_util import compare, load_fixture, rates
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    # the per-shard oracle-chain replay: tests/golden/chain_oracle.json.gz["c4/<regime>"]
    # (tests/golden/gen_chain_fixtures.py runs exactly this replay: frames 7000 + i, a fresh PathFinder per shard)
    want = {(regime, i): rec for regime in ("sparse", "dense_box")
            for i, rec in enumerate(load_fixture(f"c4/{regime}"))}
    out = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    report, bad = {}, []
    for dtype, regime in CONFIGS:
        allres, elapsed = out[(dtype, regime)]
        assert sorted(allres) == list(range(N_FRAMES)) and elapsed > 0
        cmps = []
        for i in range(N_FRAMES):
            g = allres[i]
            ok = g["status"] == 0
            got = {"det": torch.from_numpy(g["det"]), "chosen": g["chosen"], "rect": tuple(g["rect"]) if g["chosen"] >= 0 else None,
                   "cells": g["cells"] if g["chosen"] >= 0 else None,
                   "paths": [p for p, _ in g["queries"]] if ok else None,
                   "costs": [c for _, c in g["queries"]] if ok else None}
            w = want[(regime, i)]
            c = compare(got, w, f32=dtype == "f32")
            cmps.append(c)
            if dtype == "f32":  # checked after the report is written out
                frac = 1.0 if regime == "sparse" else 0.98
                if c["matched"] < frac * max(c["ndet"]):
                    bad.append((regime, i, "detections", c))
                if not c["chosen"]:
                    bad.append((regime, i, "chosen", c))
                if c["cells_mismatch"] != 0 or not c["rect"]:
                    bad.append((regime, i, "cells / rect", c))
                if not c["paths"]:
                    bad.append((regime, i, "A* paths or costs differ", c))
        report[f"{dtype}/{regime}"] = {**rates(cmps), "frames_per_s_2ranks_one_gpu": round(N_FRAMES / elapsed, 1)}
        if dtype == "f32" and report[f"{dtype}/{regime}"]["frames_with_mask"] < N_FRAMES // 2:
            bad.append((regime, "frames_with_mask", report[f"{dtype}/{regime}"]))
    d = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "c4_agreement.json"), "w") as f:
            json.dump(report, f, indent=1)
    print(json.dumps(report))
    assert not bad, bad
    for dtype, regime in CONFIGS:
        if dtype == "bf16":
            rr = report[f"{dtype}/{regime}"]
            for k, floor in BF16_FLOOR[regime].items():
                assert rr[k] >= floor, (regime, k, rr[k], floor)

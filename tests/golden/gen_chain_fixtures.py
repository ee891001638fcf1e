"""Oracle-chain fixtures for the chain tests (tests/test_gpu_chain.py, tests/test_gpu_c4.py).

The oracle chain (tests/chain_util.py: oracle/yolo_ref.predict -> select_cells -> oracle/nav.frame_nav) spends
~10 s per frame of a 300-detection regime in the pure-Python findContours restatement, so the GPU tests read
its outputs from here instead of recomputing them on the GPU box.  Inputs are fully determined by seeds (torch
CPU generator frames, seeded synthetic weights), so the fixture is a function of this script.

Sets:
  chain/<regime>: frames frame_batch(21, 32), one PathFinder state across the 32 frames, regimes
                  sparse / dense / dense_box (s-seg 640);
  c4/<regime>:    frames frame_batch(7000 + i, 1), i < 8, dealt round-robin to 2 ranks; one PathFinder state
                  per shard, frames in shard order (SURVEY.md §8e per-shard replay); regimes sparse / dense_box.
  c5/<regime>:    YOLOv8m-seg at 1280 x 1280 (BASELINE configs[4]), frames frame_batch(8000, 8, 1280), one
                  PathFinder state; regimes sparse / dense_box (the fp8 chain test's reference).
  c2/<regime>:    YOLOv8n-seg 640 (BASELINE configs[1]), frames frame_batch(9000 + i, 1), i < 16, one at a time
                  with one PathFinder state (C2's batch-1 plan, tests/test_gpu_chain.py); regime sparse.

Per frame: det float32 [k, 6] (x1 y1 x2 y2 score cls, base64), chosen index, rect, cells uint8 [32, 32]
(base64), A* paths and float64 costs (hex).  Re-run:  python tests/golden/gen_chain_fixtures.py  (~5 min, 8 CPUs)
"""
from __future__ import annotations

import base64
import gzip
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
OUT = os.path.join(HERE, "chain_oracle.json.gz")
CHAIN_FRAMES, C4_FRAMES, C4_WORLD, C5_FRAMES, C2_FRAMES = 32, 8, 2, 8, 16


def _enc(rec: dict) -> dict:
    """One oracle record; cells travel as raw bytes with their shape."""
    det = rec["det"].numpy().astype(np.float32)
    out = {"det": base64.b64encode(det.tobytes()).decode(), "ndet": int(det.shape[0]), "chosen": int(rec["chosen"]),
           "rect": list(rec["rect"]) if rec["rect"] is not None else None, "paths": rec["paths"], "costs": rec["costs"]}
    out["cells"] = base64.b64encode(np.ascontiguousarray(rec["cells"], np.uint8).tobytes()).decode() \
        if rec["cells"] is not None else None
    out["cells_shape"] = list(rec["cells"].shape) if rec["cells"] is not None else None
    return out


def _job(args):
    import torch
    from oracle import nav as onav
    from tests.chain_util import frame_batch, oracle_frame, oracle_sequence, weights
    from vision_assist_amd.shard import shard_indices
    kind, regime = args
    torch.set_num_threads(2)
    arch, fw = weights(regime)
    if kind == "chain":
        return f"chain/{regime}", [_enc(r) for r in oracle_sequence(arch, fw, frame_batch(21, CHAIN_FRAMES))]
    if kind == "c5":
        arch, fw = weights(regime, scale="m")
        torch.set_num_threads(4)
        return f"c5/{regime}", [_enc(r) for r in oracle_sequence(arch, fw, frame_batch(8000, C5_FRAMES, 1280))]
    if kind == "c2":
        arch, fw = weights(regime, scale="n")
        pf = onav.PathFinderOracle()
        return f"c2/{regime}", [_enc(oracle_frame(arch, fw, frame_batch(9000 + i, 1), pf)) for i in range(C2_FRAMES)]
    recs = [None] * C4_FRAMES
    for r in range(C4_WORLD):
        pf = onav.PathFinderOracle()
        for i in shard_indices(C4_FRAMES, C4_WORLD, r):
            recs[i] = _enc(oracle_frame(arch, fw, frame_batch(7000 + i, 1), pf))
    return f"c4/{regime}", recs


def main():
    only = sys.argv[1:]  # optional set names to (re)generate, the rest kept from the existing file
    jobs = [("chain", r) for r in ("sparse", "dense", "dense_box")] + [("c4", r) for r in ("sparse", "dense_box")] + \
        [("c5", r) for r in ("sparse", "dense_box")] + [("c2", "sparse")]
    old = {}
    if only and os.path.exists(OUT):
        with gzip.open(OUT, "rt") as f:
            old = json.load(f)
        jobs = [j for j in jobs if f"{j[0]}/{j[1]}" in only]
    with ProcessPoolExecutor(max_workers=len(jobs)) as ex:
        out = {**old, **dict(ex.map(_job, jobs))}
    with gzip.open(OUT, "wt") as f:
        json.dump(out, f)
    print("wrote", OUT, {k: [r["ndet"] for r in v] for k, v in out.items()})


if __name__ == "__main__":
    main()

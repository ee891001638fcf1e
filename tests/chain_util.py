"""Shared pieces of the chain tests: the oracle chain the reference runs per frame and the comparison of one device
frame record against it.

Oracle chain (fp32, the reference's precision, args.yaml:43 `half: false`): oracle/yolo_ref.predict (Ultralytics'
predict restated: preprocess, forward, decode, NMS, process_mask) -> select_cells (FrameProcessor.py:67-97 on
OpenCV's findContours / contourArea / boundingRect / fillPoly, oracle/contours.py) -> oracle/nav.frame_nav
(FrameProcessor.py:50-271 + PathFinder.find_path, one PathFinder angle cache per process, in frame order).
"""
from __future__ import annotations

import base64
import functools
import gzip
import json

import numpy as np
import torch

from oracle import nav as onav
from oracle import yolo_ref as Y

# regime -> synthetic_state_dict keyword arguments (vision_assist_amd/seg_arch.py)
REGIMES = {
    "sparse": {"sparse": 640},                      # 1-5 compact detections per frame (a trained model's frames)
    "mid": {"cls_bias": 0.0},                       # every class at bias 0: the random weights saturate max_det
    "dense": {"cls_bias": 4.0},                     # 300 noise-mask detections
    "dense_box": {"cls_bias": 4.0, "solid_masks": True},  # 300 solid box masks
}


def weights(regime: str, scale: str = "s"):
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(scale)
    kw = dict(REGIMES[regime])
    if "sparse" in kw and scale == "m":
        kw["sparse"] = 1280
    return arch, fold(arch, synthetic_state_dict(arch, seed=0, **kw))


def frame_batch(seed: int, n: int, res: int = 640) -> torch.Tensor:
    return torch.randint(0, 256, (n, res, res, 3), generator=torch.Generator().manual_seed(seed), dtype=torch.uint8)


def oracle_frame(arch, fw, frame_u8: torch.Tensor, pf) -> dict:
    """One frame [1, H, W, 3] through the oracle chain with the PathFinder state pf (advanced in place)."""
    H, W = frame_u8.shape[1:3]
    with torch.no_grad():
        det, masks = Y.predict(arch, fw, frame_u8)[0]
    k, _pts, rect, cells = Y.select_cells(masks)
    rec = {"det": det[:, :6].clone(), "chosen": k, "rect": None, "cells": None, "paths": None, "costs": None}
    if k >= 0:
        rec["rect"] = tuple(int(v) for v in rect)
        rec["cells"] = cells
        mn = np.kron(cells, np.ones((20, 20), np.uint8))
        nav = onav.frame_nav(mn, rect, H, W, pf)
        rec["paths"] = [[(c.coords.x, c.coords.y) for c in q[2]] for q in nav["queries"]]
        rec["costs"] = [float(q[3]).hex() if q[2] else None for q in nav["queries"]]
    return rec


def oracle_sequence(arch, fw, frames: torch.Tensor, pf=None) -> list[dict]:
    """The frames in order through the oracle chain with one PathFinder state (fresh unless given)."""
    pf = pf if pf is not None else onav.PathFinderOracle()
    return [oracle_frame(arch, fw, frames[i:i + 1], pf) for i in range(frames.shape[0])]


def match(g: torch.Tensor, r: torch.Tensor, tol_box=1e-2, tol_score=1e-4):
    """Greedy one-to-one matching of two detection lists [k, 6] (score order): same class, boxes within tol_box,
    scores within tol_score.  Near-tied scores may come out in either order (the two networks round
    differently), so order is not required.  -> (matched pairs {g index: r index}, unmatched g, unmatched r)."""
    used, pairs = set(), {}
    for i in range(g.shape[0]):
        for j in range(r.shape[0]):
            if j in used or int(g[i, 5]) != int(r[j, 5]):
                continue
            if abs(float(g[i, 4] - r[j, 4])) <= tol_score and float((g[i, :4] - r[j, :4]).abs().max()) <= tol_box:
                used.add(j)
                pairs[i] = j
                break
    return pairs, [i for i in range(g.shape[0]) if i not in pairs], [j for j in range(r.shape[0]) if j not in used]


def device_record(det: torch.Tensor, chosen: int, rect, cells: np.ndarray, nf) -> dict:
    """A device frame in the oracle record's form (det [k, 6] float, the chosen index, rect, cells, nav record)."""
    ok = nf.status == 0
    return {"det": det, "chosen": chosen, "rect": tuple(int(v) for v in rect) if chosen >= 0 else None,
            "cells": cells if chosen >= 0 else None,
            "paths": [q["path"] for q in nf.queries] if ok else None,
            "costs": [float(q["cost"]).hex() if q["path"] else None for q in nf.queries] if ok else None}


def compare(got: dict, want: dict, f32: bool) -> dict:
    """Agreement of one device frame with the oracle frame: detections matched, same chosen instance, rect,
    cells, and A* paths -- the last both on identical cells and whenever both sides produced paths (a one-sample
    cell flip can move a path; it is reported, not hidden)."""
    pairs, ug, ur = match(got["det"], want["det"]) if f32 else match(got["det"], want["det"], 2.0, 2e-2)
    nd = max(got["det"].shape[0], want["det"].shape[0])
    c, w = got["chosen"], want["chosen"]
    same_choice = (c < 0 and w < 0) or (c >= 0 and pairs.get(c, -9) == w)
    out = {"ndet": (int(got["det"].shape[0]), int(want["det"].shape[0])), "matched": len(pairs),
           "matched_frac": len(pairs) / nd if nd else 1.0, "det_same": not ug and not ur, "chosen": same_choice,
           "has_mask": w >= 0}
    if w < 0 or c < 0:
        out.update(rect=c == w, cells_mismatch=0 if c == w else -1, cells=c == w, paths=got["paths"] == want["paths"],
                   paths_on_same_cells=None)
        return out
    nmis = int((got["cells"] != want["cells"]).sum())
    same_cells = nmis == 0 and got["rect"] == want["rect"]
    same_paths = got["paths"] == want["paths"] and got["costs"] == want["costs"]
    out.update(rect=got["rect"] == want["rect"], cells_mismatch=nmis, cells=nmis == 0, paths=same_paths,
               paths_on_same_cells=same_paths if same_cells else None)
    return out


def rates(cmps: list[dict]) -> dict:
    n = len(cmps)
    r = {k: round(sum(bool(c[k]) for c in cmps) / n, 3) for k in ("det_same", "chosen", "rect", "cells", "paths")}
    r["frames"] = n
    r["frames_with_mask"] = sum(c["has_mask"] for c in cmps)
    r["matched_frac_min"] = round(min(c["matched_frac"] for c in cmps), 4)
    same = [c["paths_on_same_cells"] for c in cmps if c["paths_on_same_cells"] is not None]
    r["paths_on_same_cells"] = f"{sum(same)}/{len(same)}"
    r["cells_mismatch"] = [c["cells_mismatch"] for c in cmps]
    r["ndet"] = [c["ndet"] for c in cmps]
    return r


FIXTURE = __file__.rsplit("/", 1)[0] + "/golden/chain_oracle.json.gz"


@functools.lru_cache(maxsize=1)
def _fixture_all() -> dict:
    with gzip.open(FIXTURE, "rt") as f:
        return json.load(f)


def load_fixture(name: str) -> list[dict]:
    """Oracle-chain records of tests/golden/chain_oracle.json.gz[name] (tests/golden/gen_chain_fixtures.py) in
    oracle_frame's form."""
    out = []
    for r in _fixture_all()[name]:
        det = np.frombuffer(base64.b64decode(r["det"]), np.float32).reshape(r["ndet"], 6).copy()
        cells = None
        if r["cells"] is not None:
            shape = tuple(r.get("cells_shape") or (32, 32))
            cells = np.frombuffer(base64.b64decode(r["cells"]), np.uint8).reshape(shape).copy()
        out.append({"det": torch.from_numpy(det), "chosen": r["chosen"],
                    "rect": tuple(r["rect"]) if r["rect"] is not None else None, "cells": cells,
                    "paths": [[tuple(p) for p in q] for q in r["paths"]] if r["paths"] is not None else None,
                    "costs": r["costs"]})
    return out


FRAMES_DIR = __file__.rsplit("/", 1)[0] + "/golden/frames"


def real_frames(n: int = 8) -> np.ndarray:
    """The reference's own validation frames (model/valid/images, 640 x 640 camera frames of paths; copied as data
    into tests/golden/frames) as uint8 BGR [n, 640, 640, 3] -- the channel order cv2 delivers (main.py:62-70)."""
    from PIL import Image
    out = []
    for i in range(n):
        rgb = np.asarray(Image.open(f"{FRAMES_DIR}/valid_{i}.jpg").convert("RGB"))
        out.append(rgb[..., ::-1])
    return np.ascontiguousarray(np.stack(out))


def mosaic_1280(frames: np.ndarray) -> np.ndarray:
    """2 x 2 mosaics of consecutive 640 x 640 frames: real content at C5's 1280 x 1280 network size."""
    n = frames.shape[0] // 4
    out = np.zeros((n, 1280, 1280, 3), np.uint8)
    for k in range(n):
        f = frames[4 * k:4 * k + 4]
        out[k, :640, :640], out[k, :640, 640:], out[k, 640:, :640], out[k, 640:, 640:] = f
    return out


def label_polygons(i: int, H: int = 640, W: int = 640) -> list[np.ndarray]:
    """The segmentation labels of validation frame i (YOLO-seg txt: class x1 y1 x2 y2 ..., normalised) as int32
    pixel polygons -- real path shapes as annotated for the reference's model (model/valid/labels)."""
    polys = []
    with open(f"{FRAMES_DIR}/valid_{i}.txt") as f:
        for line in f:
            v = [float(t) for t in line.split()[1:]]
            if len(v) >= 6:
                p = np.array(v, np.float64).reshape(-1, 2) * (W, H)
                polys.append(np.clip(np.round(p), 0, [W - 1, H - 1]).astype(np.int32))
    return polys

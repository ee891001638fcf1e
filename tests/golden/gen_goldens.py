"""Generate the grid-stage golden vectors by RUNNING THE REFERENCE (this container only).

Recipe = SURVEY.md Appendix C:
  * ``/tmp/va_oracle/vision_assist -> /root/reference`` so the reference's own
    ``from vision_assist.X import ...`` lines resolve (PYTHONDONTWRITEBYTECODE=1,
    the reference is read-only);
  * a throw-away ``cv2`` stub (fillPoly / boundingRect / threshold /
    contourArea) and an ``ultralytics`` stub (``class YOLO``) first on
    sys.path.  cv2 is absent here, so the goldens are defined at the post-cv2
    boundary: the harness hands ``_extract_grid_information`` the filled mask
    and the bounding rect it would have received from OpenCV.
  * per frame: fp._extract_grid_information -> _calculate_penalties ->
    _create_graph -> protrusion_detector -> _find_paths -> path_analyser, all
    REFERENCE code, with the angle-cache key set captured around every
    PathFinder.find_path call and time.time frozen for PathAnalyser.

Only outputs are written (tests/golden/nav_goldens.json.gz); nothing from
/root/reference is copied.  Re-run:  python tests/golden/gen_goldens.py
"""
from __future__ import annotations

import gzip
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from workloads.corridors import corridor_cells, cells_to_mask, cells_rect, fixture_640  # noqa: E402

FIXTURE_DIR = os.path.join(REF, "utilities", "generate_testing_grids", "examples")


# --------------------------------------------------------------------------- stubs
class _Harness:
    mask: np.ndarray | None = None
    rect: tuple | None = None


def _install_stubs(tmp: str) -> None:
    os.makedirs(os.path.join(tmp, "cv2"), exist_ok=True)
    os.makedirs(os.path.join(tmp, "ultralytics"), exist_ok=True)
    with open(os.path.join(tmp, "ultralytics", "__init__.py"), "w") as f:
        f.write("class YOLO:\n    pass\n")
    with open(os.path.join(tmp, "cv2", "__init__.py"), "w") as f:
        f.write("")
    link = os.path.join(tmp, "vision_assist")
    if not os.path.exists(link):
        os.symlink(REF, link)
    sys.path.insert(0, tmp)
    import cv2  # the stub

    def fillPoly(img, pts, color):
        if img.ndim == 2 and color == 1 and _Harness.mask is not None:
            img[:] = _Harness.mask
            return img
        for poly in pts:
            poly = np.asarray(poly).reshape(-1, 2)
            x0, y0 = poly.min(0)
            x1, y1 = poly.max(0)
            img[max(0, y0):y1 + 1, max(0, x0):x1 + 1] = color
        return img

    def boundingRect(points):
        return _Harness.rect

    def threshold(img, thresh, maxval, kind):
        return thresh, np.where(img > thresh, maxval, 0).astype(img.dtype)

    def contourArea(c):
        c = np.asarray(c, dtype=np.float64).reshape(-1, 2)
        x, y = c[:, 0], c[:, 1]
        return 0.5 * abs(np.dot(x, np.roll(y, -1)) - np.dot(y, np.roll(x, -1)))

    cv2.fillPoly = fillPoly
    cv2.boundingRect = boundingRect
    cv2.threshold = threshold
    cv2.contourArea = contourArea
    cv2.THRESH_BINARY = 0
    cv2.Mat = object


class _FakeClock:
    t = 1_000_000.0

    @classmethod
    def time(cls):
        return cls.t


def _hexf(v):
    if v is None:
        return None
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        return "i%d" % int(v)
    return float(v).hex()


def _np_default(o):
    if isinstance(o, np.integer):
        return int(o)
    raise TypeError(type(o))


def _key_list(cache) -> list:
    return sorted([[a[0], a[1], b[0], b[1]] for (a, b) in cache.keys()])


class RefRunner:
    """Drives the reference modules exactly as FrameProcessor.__call__ does."""

    def __init__(self):
        import vision_assist.PathAnalyser as PA
        import vision_assist.PathFinder as PF
        from vision_assist.FrameProcessor import FrameProcessor

        PA.time = _FakeClock
        self.PF = PF
        self.PA = PA
        self.fp = FrameProcessor(model=None, verbose=False, debug=False, imshow=False)
        self.queries = []
        orig = PF.path_finder.find_path

        def wrapped(graph, start, end, lookup):
            before = _key_list(PF.path_finder.angle_cache)
            path, cost = orig(graph, start, end, lookup)
            after = _key_list(PF.path_finder.angle_cache)
            self.queries.append({
                "start": [start.coords.x, start.coords.y],
                "end": [end.coords.x, end.coords.y],
                "path": [[g.coords.x, g.coords.y] for g in path],
                "cost": _hexf(cost) if path else "inf",
                "seen_before": before,
                "seen_after": after,
            })
            return path, cost

        PF.path_finder.find_path = wrapped

    def reset_process_state(self):
        """Equivalent of a fresh process: clear the PathFinder angle cache and
        the PathAnalyser history (both process-global in the reference)."""
        self.PF.path_finder.angle_cache.clear()
        self.PA.path_analyser.previous_instructions = {}
        _FakeClock.t = 1_000_000.0

    def frame(self, g: np.ndarray) -> dict:
        R, C = g.shape
        H, W = 20 * R, 20 * C
        fp = self.fp
        fp.frame = np.zeros((H, W, 3), dtype=np.uint8)
        _Harness.mask = cells_to_mask(g)
        _Harness.rect = cells_rect(g)
        poly = np.array([[0, 0], [1, 0], [1, 1]], dtype=np.float32)
        res = types.SimpleNamespace(masks=types.SimpleNamespace(xy=[poly]))
        rec = {"H": H, "W": W, "rect": list(_Harness.rect),
               "cells": ["".join("1" if v else "0" for v in row) for row in g]}
        self.queries = []
        _FakeClock.t += 0.5
        try:
            fp._extract_grid_information([res])
        except IndexError:
            rec["error"] = "IndexError"
            return rec
        if not fp.grids:
            rec["empty"] = True
            return rec
        fp._calculate_penalties()
        graph = fp._create_graph()
        peaks = fp.protrusion_detector(fp.frame, fp.grids, fp.grid_lookup)
        paths = fp._find_paths(peaks, graph)
        answer = self.PA.path_analyser(H, W, paths)
        in_grids = set()
        rows = []
        for row in fp.grids:
            rows.append({
                "y": row[0].coords.y,
                "row": row[0].row,
                "x0": row[0].coords.x,
                "empty": "".join("1" if c.empty else "0" for c in row),
                "art": "".join("1" if c.artificial else "0" for c in row),
                "pen": [_hexf(c.penalty) for c in row],
            })
            for c in row:
                in_grids.add(id(c))
        orphans = [[k[0], k[1], int(v.empty)] for k, v in fp.grid_lookup.items() if id(v) not in in_grids]
        rec.update({
            "rows": rows,
            "orphans": orphans,
            "n_lookup": len(fp.grid_lookup),
            "peaks": [[p.x, p.y] for p in peaks],
            "queries": self.queries,
            "paths": [dict({"coords": [[q.coords.x, q.coords.y] for q in p.grids],
                            "cost": _hexf(p.total_cost)}, **path_structure(p)) for p in paths],
            "answer": answer,
        })
        return rec


def path_structure(p) -> dict:
    """models.Path post-init results (models.py:96-99, 160-364): sections (type, cells, total_cost) and corners."""
    secs = None if p.sections is None else [
        {"type": q.path_type, "coords": [[g.coords.x, g.coords.y] for g in q.grids], "cost": _hexf(q.total_cost)}
        for q in p.sections]
    corners = None if p.corners is None else [
        {"direction": c.direction, "sharpness": c.sharpness, "shape": c.shape, "start": [c.start.x, c.start.y],
         "end": [c.end.x, c.end.y], "angle_change": _hexf(c.angle_change), "length": _hexf(c.length)}
        for c in p.corners]
    return {"sections": secs, "corners": corners, "angle": _hexf(p.angle), "length": _hexf(p.length)}


def path_model_fixtures() -> list:
    """The 12 hand-captured paths of testing/path_model/grids.py (570 Grid literals, frame 720 x 1280) through the
    reference's models.Path as testing/path_model/test.py:35-39 builds them (total_cost=100): the cells and the
    sections / corners the reference computes.  grids.py imports its Grid / Coordinate from `other_models`,
    aliased here to the reference's own models module."""
    import importlib.util
    import vision_assist.models as M
    sys.modules.setdefault("other_models", M)
    spec = importlib.util.spec_from_file_location("va_path_model_grids", os.path.join(REF, "testing", "path_model",
                                                                                     "grids.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = []
    for path in mod.grids:
        p = M.Path(grids=path, total_cost=100, path_type="path")
        out.append(dict({"cells": [{"coords": [g.coords.x, g.coords.y], "centre": [g.centre.x, g.centre.y],
                                    "penalty": _hexf(g.penalty), "row": g.row, "col": g.col, "empty": g.empty,
                                    "artificial": g.artificial} for g in path],
                         "total_cost": "i100"}, **path_structure(p)))
    return out


def load_fixtures() -> dict:
    out = {}
    for fn in sorted(os.listdir(FIXTURE_DIR)):
        if fn.endswith("_grids.npy"):
            out[fn[:-len("_grids.npy")]] = np.load(os.path.join(FIXTURE_DIR, fn))
    return out


def bottom_case(rows_on: list[int], R=32, C=32) -> np.ndarray:
    g = np.zeros((R, C), dtype=bool)
    for r in rows_on:
        g[r, 10:22] = True
    return g


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    tmp = tempfile.mkdtemp(prefix="va_oracle_")
    _install_stubs(tmp)
    import contextlib
    import io
    runner = RefRunner()
    quiet = contextlib.redirect_stdout(io.StringIO())
    quiet.__enter__()
    fixtures = load_fixtures()
    out = {
        "generator": "tests/golden/gen_goldens.py (reference run, SURVEY.md Appendix C)",
        "fixtures": {k: ["".join("1" if v else "0" for v in row) for row in g] for k, g in fixtures.items()},
        "sequences": [],
    }
    names = sorted(fixtures)
    # 1) 640-scale fixture sequence, 3 reps, ONE process state (warm cache)
    runner.reset_process_state()
    seq = {"name": "fixtures640_x3", "frames": []}
    for rep in range(3):
        for n in names:
            rec = runner.frame(fixture_640(fixtures[n]))
            rec["source"] = f"{n}@640"
            seq["frames"].append(rec)
    out["sequences"].append(seq)
    # 2) native 720x1280 fixtures, 2 reps
    runner.reset_process_state()
    seq = {"name": "fixtures_native_x2", "frames": []}
    for rep in range(2):
        for n in names:
            rec = runner.frame(fixtures[n])
            rec["source"] = f"{n}@native"
            seq["frames"].append(rec)
    out["sequences"].append(seq)
    # 3) random corridors, cold cache per mask (independent sequences of 1)
    for s in range(200):
        runner.reset_process_state()
        rec = runner.frame(corridor_cells(s))
        rec["source"] = f"corridor:{s}"
        out["sequences"].append({"name": f"corridor_cold_{s}", "frames": [rec]})
    # 4) random corridors, one warm sequence
    runner.reset_process_state()
    seq = {"name": "corridor_warm_1000_1099", "frames": []}
    for s in range(1000, 1100):
        rec = runner.frame(corridor_cells(s))
        rec["source"] = f"corridor:{s}"
        seq["frames"].append(rec)
    out["sequences"].append(seq)
    # 5) Q10 edge cases: masks confined to the bottom rows (640x640)
    runner.reset_process_state()
    seq = {"name": "bottom_rows_q10", "frames": []}
    for rows_on in ([30, 31], [29, 30, 31], [31], [28], [27, 28], [0, 1], [5]):
        rec = runner.frame(bottom_case(rows_on))
        rec["source"] = f"bottom:{rows_on}"
        seq["frames"].append(rec)
    out["sequences"].append(seq)
    # 6) 128-entry angle table computed by the reference's own _angle_between_grids
    out["angle_table"] = angle_table(runner)
    # 7) models.Path sectioning / corners of the reference's hand-captured paths
    out["path_model"] = path_model_fixtures()
    quiet.__exit__(None, None, None)
    path = os.path.join(HERE, "nav_goldens.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(out, f, separators=(",", ":"), default=_np_default)
    nq = sum(len(fr.get("queries", [])) for s in out["sequences"] for fr in s["frames"])
    nf = sum(len(s["frames"]) for s in out["sequences"])
    print(f"wrote {path}: {nf} frames, {nq} A* queries")


def angle_table(runner) -> list:
    """For all 16 x 8 (prev, next) vectors: the degrees the reference appends on a
    cache miss, via a 7-point path fed to the reference's _angle_between_grids."""
    pf = runner.PF.path_finder
    steps = {(20, 0), (-20, 0), (0, 20), (0, -20)}
    prevs, nexts = set(), set()
    import itertools
    for a, b, c in itertools.product(steps, repeat=3):
        # simple paths only: no immediate reversal
        if (a[0] + b[0], a[1] + b[1]) == (0, 0) or (b[0] + c[0], b[1] + c[1]) == (0, 0):
            continue
        prevs.add((a[0] + b[0] + c[0], a[1] + b[1] + c[1]))
    for a, b in itertools.product(steps, repeat=2):
        if (a[0] + b[0], a[1] + b[1]) == (0, 0):
            continue
        nexts.add((a[0] + b[0], a[1] + b[1]))
    table = []
    saved = dict(pf.angle_cache)
    for p in sorted(prevs):
        for n in sorted(nexts):
            # 8-point path (the 8th = the neighbour, never inside a window) whose only
            # window i=3 has prev = P3 - P0 = p and next = P6 - P4 = n
            q = (p[0] + 20, p[1])
            path = [(0, 0), (0, 0), (0, 0), p, q, q, (q[0] + n[0], q[1] + n[1]), (0, 0)]
            pf.angle_cache.clear()
            deg = pf._angle_between_grids(path, 7)
            pen = 0 if deg <= 30 else (deg / 90) ** 1.5
            table.append([p[0], p[1], n[0], n[1], float(deg).hex(), _hexf(pen)])
    pf.angle_cache.clear()
    pf.angle_cache.update(saved)
    return table


if __name__ == "__main__":
    main()

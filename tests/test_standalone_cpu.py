"""The standalone PenaltyCalculator / ProtrusionDetector surfaces on grids built outside this package's FrameProcessor
(/root/reference PenaltyCalculator.py:112-142, ProtrusionDetector.py:419-535): the host half.

FrameProcessor.implied_grid_inputs reads back from a grid list what the reference's grid builder was given (rounded
rect, mask samples at the cell centres); the device then rebuilds the list from those (tests/test_gpu_nav.py checks
the penalties and peaks it serves).  Here, on every golden frame (the reference's 13 fixtures, the seeded corridors
and the Q9 / Q10 edge cases, tests/golden/nav_goldens.json.gz), the oracle's builder (oracle/nav.build_grids, pinned
to the reference's grids by tests/test_oracle_golden.py) run on one of the candidates must reproduce the list and
the lookup exactly, and a list no mask produces (a flipped artificial flag) must match no candidate."""
import numpy as np
import pytest

from oracle import nav
from tests.golden_io import cells_of, load_goldens
from workloads.corridors import cells_to_mask


def _as_grids(st):
    from vision_assist_amd.models import Grid
    objs = {}

    def conv(c):
        if id(c) not in objs:
            objs[id(c)] = Grid(**c.model_dump())
        return objs[id(c)]
    grids = [[conv(c) for c in row] for row in st.grids]
    lookup = {k: conv(c) for k, c in st.lookup.items()}
    return grids, lookup


def _key(c):
    return (c.coords.x, c.coords.y, c.centre.x, c.centre.y, c.row, c.col, c.empty, c.artificial)


def _same(st, grids, lookup):
    return [[_key(c) for c in r] for r in st.grids] == [[_key(c) for c in r] for r in grids] and \
        list(st.lookup) == list(lookup) and all(_key(st.lookup[k]) == _key(lookup[k]) for k in lookup)


def _frames():
    """The golden frames once each (sequences repeat them), non-corridor ones all, corridors every tenth."""
    out, seen = [], set()
    for seq in load_goldens()["sequences"]:
        name = seq["name"]
        for i, fr in enumerate(seq["frames"]):
            key = ("".join(fr["cells"]), tuple(fr["rect"]), fr["H"], fr["W"])
            if fr.get("error") or fr.get("empty") or key in seen:
                continue
            seen.add(key)
            if "corridor" not in name or len(seen) % 10 == 0:
                out.append((f"{name}/{i}", fr))
    return out


def _rebuilds(grids, lookup, H, W):
    from vision_assist_amd.FrameProcessor import implied_grid_inputs
    x0, y0, w, cands = implied_grid_inputs(grids, lookup, H, W)
    hits = []
    for h, cells in cands:
        try:
            st = nav.build_grids(cells_to_mask(cells.astype(bool)), (x0, y0, w, h), H, W)
        except IndexError:
            continue
        if _same(st, grids, lookup):
            hits.append(h)
            break
    return hits


def test_implied_inputs_rebuild_every_golden_frame():
    frames = _frames()
    assert len(frames) > 60
    for name, fr in frames:
        H, W = fr["H"], fr["W"]
        st = nav.build_grids(cells_to_mask(cells_of(fr)), tuple(fr["rect"]), H, W)
        grids, lookup = _as_grids(st)
        assert _rebuilds(grids, lookup, H, W), name


def test_a_list_no_mask_makes_matches_no_candidate():
    name, fr = _frames()[0]
    H, W = fr["H"], fr["W"]
    st = nav.build_grids(cells_to_mask(cells_of(fr)), tuple(fr["rect"]), H, W)
    grids, lookup = _as_grids(st)
    # an artificial flag on a cell of a column outside the artificial band: no mask gives that
    g = next(c for row in grids for c in row if c.empty and not c.artificial and abs(c.coords.x - W // 2) > 200)
    g.artificial = True
    g.empty = False
    assert _rebuilds(grids, lookup, H, W) == []

"""CPU test of the host decision layer (vision_assist_amd.models.Path sections / corners and
vision_assist_amd.PathAnalyser) against the reference's answers.

The golden frames hold the reference's returned paths (cells + total_cost) and its answer string
(PathAnalyser with a frozen clock); feeding the same paths to the restated Path/PathAnalyser must
give the same answer for every frame of every sequence (history carried within a sequence).
"""
from tests.golden_io import load_goldens, unhex


def _grid(x, y, pen_by_xy):
    from vision_assist_amd.models import Coordinate, Grid
    return Grid(coords=Coordinate(x=x, y=y), centre=Coordinate(x=x + 10, y=y + 10), penalty=pen_by_xy.get((x, y)),
                row=0, col=0, empty=False, artificial=False)


def test_answers_match_reference():
    from vision_assist_amd.models import Path
    from vision_assist_amd.PathAnalyser import PathAnalyser
    pa = PathAnalyser()
    clock = {"t": 0.0}
    pa.clock = lambda: clock["t"]
    n = 0
    for seq in load_goldens()["sequences"]:
        pa.previous_instructions = {}
        clock["t"] = 1_000_000.0
        for fr in seq["frames"]:
            clock["t"] += 0.5
            if fr.get("error") or fr.get("empty"):
                continue
            pens = {}
            for row in fr["rows"]:
                for c, p in enumerate(row["pen"]):
                    pens[(row["x0"] + 20 * c, row["y"])] = unhex(p)
            paths = [Path(grids=[_grid(x, y, pens) for x, y in gp["coords"]], total_cost=unhex(gp["cost"]),
                          path_type="path") for gp in fr["paths"]]
            ans = pa(fr["H"], fr["W"], paths)
            assert ans == fr["answer"], (fr["source"], ans, fr["answer"])
            n += 1
    assert n > 300


def test_path_sections_cover_path():
    """Sections are contiguous slices that share their joint cell and cover the whole path."""
    from vision_assist_amd.models import Path
    for seq in load_goldens()["sequences"][:3]:
        for fr in seq["frames"]:
            for gp in fr.get("paths", []):
                p = Path(grids=[_grid(x, y, {}) for x, y in gp["coords"]], total_cost=1.0, path_type="path")
                if not p.sections:
                    continue
                cells = [(g.coords.x, g.coords.y) for g in p.grids]
                joined = [(g.coords.x, g.coords.y) for g in p.sections[0].grids]
                for sec in p.sections[1:]:
                    sc = [(g.coords.x, g.coords.y) for g in sec.grids]
                    assert sc[0] == joined[-1]
                    joined += sc[1:]
                assert joined == cells


def _hx(v):
    return None if v is None else (("i", int(v)) if isinstance(v, int) else ("f", float(v).hex()))


def _structure(p):
    """Sections and corners of a vision_assist_amd.models.Path in the golden record's form."""
    secs = None if p.sections is None else [
        {"type": q.path_type, "coords": [[g.coords.x, g.coords.y] for g in q.grids], "cost": _hx(q.total_cost)}
        for q in p.sections]
    corners = None if p.corners is None else [
        {"direction": c.direction, "sharpness": c.sharpness, "shape": c.shape, "start": [c.start.x, c.start.y],
         "end": [c.end.x, c.end.y], "angle_change": _hx(c.angle_change), "length": _hx(c.length)}
        for c in p.corners]
    return secs, corners


def _golden_structure(gp):
    secs = None if gp["sections"] is None else [dict(s, cost=_hx(unhex(s["cost"]))) for s in gp["sections"]]
    corners = None if gp["corners"] is None else [
        dict(c, angle_change=_hx(unhex(c["angle_change"])), length=_hx(unhex(c["length"]))) for c in gp["corners"]]
    return secs, corners


def test_path_sections_and_corners_match_reference_runs():
    """models.Path post-init (models.py:96-99 sections :160-270, corners :300-364) on every path the reference
    returned for the golden frames: section types, cells and total_cost (float64 hex) and every corner field
    (direction, sharpness, shape, start, end, angle_change and length as float64 hex) equal the reference's."""
    from vision_assist_amd.models import Path
    n = ncorner = 0
    for seq in load_goldens()["sequences"]:
        for fr in seq["frames"]:
            for gp in fr.get("paths", []):
                p = Path(grids=[_grid(x, y, {}) for x, y in gp["coords"]], total_cost=unhex(gp["cost"]),
                         path_type="path")
                assert _structure(p) == _golden_structure(gp), fr["source"]
                assert _hx(p.angle) == _hx(unhex(gp["angle"])) and _hx(p.length) == _hx(unhex(gp["length"]))
                n += 1
                ncorner += len(gp["corners"] or [])
    assert n > 300 and ncorner > 300  # 317 paths, every one compared


def test_path_model_fixtures_match_reference():
    """The reference's 12 hand-captured paths (testing/path_model/grids.py, 570 Grid literals, 720 x 1280 frame),
    built as testing/path_model/test.py:35-39 builds them (total_cost=100): sections and corners equal the
    reference's models.Path results recorded by tests/golden/gen_goldens.py."""
    from vision_assist_amd.models import Coordinate, Grid, Path
    fx = load_goldens()["path_model"]
    assert len(fx) == 12
    for k, f in enumerate(fx):
        cells = [Grid(coords=Coordinate(x=c["coords"][0], y=c["coords"][1]),
                      centre=Coordinate(x=c["centre"][0], y=c["centre"][1]), penalty=unhex(c["penalty"]),
                      row=c["row"], col=c["col"], empty=c["empty"], artificial=c["artificial"]) for c in f["cells"]]
        p = Path(grids=cells, total_cost=100, path_type="path")
        assert _structure(p) == _golden_structure(f), k
        assert _hx(p.angle) == _hx(unhex(f["angle"])) and _hx(p.length) == _hx(unhex(f["length"])), k


def _naive_analyser(clock):
    """A PathAnalyser whose history handling is the reference's literal form: every entry scanned for pairs and
    the dict rebuilt per call (PathAnalyser.py:185-230, :375-382)."""
    from vision_assist_amd.PathAnalyser import _HISTORY_MS, _PAIR_WINDOW_MS, PathAnalyser
    pa = object.__new__(PathAnalyser)
    pa.paths, pa.previous_instructions, pa.instructions, pa.clock, pa._rows = [], {}, [], clock, None
    pa._upgrade_fast = lambda previous, current, now: False
    pa._recent = lambda previous, now: [(ts, v) for ts, v in previous.items() if now - ts < _PAIR_WINDOW_MS]

    def remember(now, ins):
        pa.previous_instructions[now] = ins
        pa.previous_instructions = {ts: v for ts, v in pa.previous_instructions.items() if now - ts <= _HISTORY_MS}
    pa._remember = remember
    return pa


def test_history_window_equals_full_scan():
    """PathAnalyser's history handling (pairs from the suffix inside the pair window, expired entries deleted from
    the front while the keys arrive in order; the full scan otherwise) against the literal full-scan form, on the
    golden frames' paths at drop-in call rates (2-3 ms apart: thousands of history entries), with repeated
    timestamps, clock steps backwards and outside resets of the history: the same answers, history keys and
    history dangers at every frame."""
    import random

    from vision_assist_amd.models import Path
    from vision_assist_amd.PathAnalyser import path_analyser
    rnd = random.Random(5)
    frames = []
    for seq in load_goldens()["sequences"]:
        for fr in seq["frames"]:
            if fr.get("error") or fr.get("empty") or not fr["paths"]:
                continue
            pens = {}
            for row in fr["rows"]:
                for c, p in enumerate(row["pen"]):
                    pens[(row["x0"] + 20 * c, row["y"])] = unhex(p)
            frames.append((fr["H"], fr["W"], [([(x, y) for x, y in gp["coords"]], unhex(gp["cost"]), pens)
                                               for gp in fr["paths"]]))
    clock = {"t": 2_000_000.0}
    naive = _naive_analyser(lambda: clock["t"])
    fast = path_analyser
    saved = (fast.clock, fast.previous_instructions, fast._rows)
    fast.clock, fast.previous_instructions = (lambda: clock["t"]), {}
    try:
        for k in range(4000):
            H, W, gps = frames[k % len(frames)]
            r = rnd.random()
            clock["t"] += 0.0 if r < 0.05 else -0.4 if r < 0.055 else 0.3 if r < 0.06 else rnd.uniform(0.001, 0.003)
            if k in (1500, 2600):
                fast.previous_instructions, naive.previous_instructions = {}, {}
            mk = lambda: [Path(grids=[_grid(x, y, pens) for x, y in cs], total_cost=cost, path_type="path")
                          for cs, cost, pens in gps]
            assert fast(H, W, mk()) == naive(H, W, mk()), k
            assert list(fast.previous_instructions) == list(naive.previous_instructions), k
            if k % 97 == 0:
                assert [[i.danger for i in v] for v in fast.previous_instructions.values()] == \
                       [[i.danger for i in v] for v in naive.previous_instructions.values()], k
        assert len(naive.previous_instructions) > 1000
    finally:
        fast.clock, fast.previous_instructions, fast._rows = saved

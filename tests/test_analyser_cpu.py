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

"""Pin the CPU oracle (oracle/nav.py) against the reference's own outputs.

The goldens were produced by running the reference code itself
(tests/golden/gen_goldens.py); every value is compared bit-exactly (penalties
and A* costs as float64 hex, path coordinates, peaks, angle-cache key sets
before/after every query, including the int/float type of the penalty).
"""
import numpy as np
import pytest

from oracle import nav
from workloads.corridors import cells_to_mask
from tests.golden_io import cells_of, load_goldens, unhex, key_tuple


def _ptype(v):
    return ("int", v) if isinstance(v, int) else ("float", float(v).hex())


def _run_sequence(seq):
    pf = nav.PathFinderOracle()
    for fr in seq["frames"]:
        g = cells_of(fr)
        H, W = fr["H"], fr["W"]
        mask = cells_to_mask(g)
        if fr.get("error"):
            with pytest.raises(IndexError):
                nav.frame_nav(mask, tuple(fr["rect"]), H, W, pf)
            continue
        out = nav.frame_nav(mask, tuple(fr["rect"]), H, W, pf)
        st = out["state"]
        if fr.get("empty"):
            assert not st.grids
            continue
        # grids list (rows, row attrs, flags, penalties with python type)
        assert len(st.grids) == len(fr["rows"]), fr["source"]
        for row, grow in zip(st.grids, fr["rows"]):
            assert row[0].coords.y == grow["y"] and row[0].row == grow["row"] and row[0].coords.x == grow["x0"]
            assert "".join("1" if c.empty else "0" for c in row) == grow["empty"]
            assert "".join("1" if c.artificial else "0" for c in row) == grow["art"]
            for c, gp in zip(row, grow["pen"]):
                want = unhex(gp)
                if want is None:
                    assert c.penalty is None
                else:
                    assert _ptype(c.penalty) == _ptype(want), (fr["source"], c.coords)
        assert len(st.lookup) == fr["n_lookup"]
        assert [list(p) for p in out["peaks"]] == fr["peaks"], fr["source"]
        assert len(out["queries"]) == len(fr["queries"])
        for (start, end, path, cost, seen), gq in zip(out["queries"], fr["queries"]):
            assert [start.coords.x, start.coords.y] == gq["start"]
            assert [end.coords.x, end.coords.y] == gq["end"]
            assert [[c.coords.x, c.coords.y] for c in path] == gq["path"], fr["source"]
            if path:
                assert float(cost).hex() == float(unhex(gq["cost"])).hex()
            # angle cache after the query
            assert set(seen) == {key_tuple(k) for k in gq["seen_after"]}
        assert len(out["paths"]) == len(fr["paths"])
        for (path, cost), gp in zip(out["paths"], fr["paths"]):
            assert [[c.coords.x, c.coords.y] for c in path] == gp["coords"]


def _seq_ids():
    d = load_goldens()
    return [s["name"] for s in d["sequences"]]


@pytest.mark.parametrize("name", [n for n in _seq_ids() if not n.startswith("corridor_cold_")])
def test_oracle_sequence(name):
    seq = next(s for s in load_goldens()["sequences"] if s["name"] == name)
    _run_sequence(seq)


def test_oracle_cold_corridors():
    for seq in load_goldens()["sequences"]:
        if seq["name"].startswith("corridor_cold_"):
            _run_sequence(seq)


def test_angle_table_matches_reference():
    """The 128-entry (prev, next) -> degrees table the HIP A* uses, against the
    reference's own _angle_between_grids outputs."""
    from oracle.angle_table import angle_table_entries
    want = {(a, b, c, d): (deg, pen) for a, b, c, d, deg, pen in load_goldens()["angle_table"]}
    got = angle_table_entries()
    assert len(got) == 128 == len(want)
    for k, (deg, pen) in got.items():
        wdeg, wpen = want[k]
        assert float(deg).hex() == wdeg
        assert _ptype(pen) == _ptype(unhex(wpen))

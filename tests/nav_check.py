"""Shared comparison helpers: device NavFrame vs reference goldens / oracle."""
from __future__ import annotations

from oracle.angle_table import key_vectors
from tests.golden_io import unhex

_PREVS, _NEXTS = key_vectors()


def key_index(k) -> int:
    """golden key [pdx, pdy, ndx, ndy] (pixels) -> device key prev*8+next."""
    return _PREVS.index((k[0], k[1])) * 8 + _NEXTS.index((k[2], k[3]))


def key_tuple_of_index(i: int):
    p, n = _PREVS[i // 8], _NEXTS[i % 8]
    return (p, n)


def bits_to_keys(w0: int, w1: int) -> set[int]:
    return {k for k in range(128) if ((w0 if k < 64 else w1) >> (k & 63)) & 1}


def pen_value(flags: int, pen: float):
    """Device cell penalty -> the python value the reference stores (None / int 0 / int 1 / float)."""
    if flags & 1:  # VA_CELL_EMPTY
        return None
    if pen == 0.0:
        return 0
    if pen == 1.0:
        return 1
    return pen


def _ptype(v):
    if v is None:
        return None
    return ("int", v) if isinstance(v, int) else ("float", float(v).hex())


def compare_golden_frame(nf, fr: dict, seen_before: set[int]) -> set[int]:
    """Assert NavFrame == golden frame record; returns the seen set after the frame."""
    src = fr.get("source")
    if fr.get("error"):
        assert nf.status == 2, (src, nf.status)  # VA_FRAME_INDEX_ERROR
        return seen_before
    if fr.get("empty"):
        assert nf.status == 1, (src, nf.status)
        return seen_before
    assert nf.status == 0, (src, nf.status)
    assert nf.P == len(fr["rows"]), src
    for p, grow in enumerate(fr["rows"]):
        assert int(nf.pos_y[p]) == grow["y"], (src, p)
        assert int(nf.pos_attr[p]) == grow["row"], (src, p)
        assert nf.x0 == grow["x0"], src
        fl = nf.cell_flags[p]
        assert "".join("1" if v & 1 else "0" for v in fl) == grow["empty"], (src, p)
        assert "".join("1" if v & 2 else "0" for v in fl) == grow["art"], (src, p)
        for c, gp in enumerate(grow["pen"]):
            got = pen_value(int(fl[c]), float(nf.cell_pen[p, c]))
            assert _ptype(got) == _ptype(unhex(gp)), (src, p, c, got, gp)
    nodes = nf.node_flags
    assert int((nodes & 1).sum()) == fr["n_lookup"], src
    orph = sorted((int(20 * xi), int(20 * yi)) for yi, xi in zip(*((nodes & 5) == 1).nonzero()))
    assert orph == sorted((o[0], o[1]) for o in fr["orphans"]), src
    assert [list(p) for p in nf.peaks] == fr["peaks"], src
    seen = set(seen_before)
    assert len(nf.queries) == len(fr["queries"]), src
    C = nf.C
    sp, sc = nf.start
    for k, (q, gq) in enumerate(zip(nf.queries, fr["queries"])):
        assert [nf.x0 + 20 * sc, int(nf.pos_y[sp])] == gq["start"], src
        ep, ec = nf.ends[k]
        assert [nf.x0 + 20 * ec, int(nf.pos_y[ep])] == gq["end"], src
        assert [list(p) for p in q["path"]] == gq["path"], (src, k)
        if gq["path"]:
            assert q["status"] == 1
            want = unhex(gq["cost"])
            assert float(q["cost"]).hex() == float(want).hex(), (src, k, q["cost"], want)
        else:
            assert q["status"] == 2
        assert {key_index(kk) for kk in gq["seen_before"]} == seen, (src, k)
        seen |= bits_to_keys(*q["miss"])
        assert {key_index(kk) for kk in gq["seen_after"]} == seen, (src, k)
    del C
    uniq = sorted((q["order"], q["path"]) for q in nf.queries if q["unique"])
    assert [[list(p) for p in path] for _, path in uniq] == [gp["coords"] for gp in fr["paths"]], src
    return seen

"""The 16 x 8 (prev-window, next-window) angle table, restated (TEST INFRASTRUCTURE).

PathFinder._angle_between_grids (PathFinder.py:51-101) only ever sees window
vectors that are sums of 3 (prev) / 2 (next) unit moves of a simple 4-neighbour
path at grid 20, i.e. 16 x 8 = 128 keys.  This module
computes, for every key, the degrees a cache miss appends and the resulting
``anglePenalty`` (PathFinder.py:168), by feeding a one-window path through the
oracle's restated ``_angle``.  Pinned against the reference-generated
``angle_table`` section of tests/golden/nav_goldens.json.gz.
"""
from __future__ import annotations

import itertools

from oracle.nav import PathFinderOracle

STEPS = ((20, 0), (-20, 0), (0, 20), (0, -20))


def key_vectors():
    prevs, nexts = set(), set()
    for a, b, c in itertools.product(STEPS, repeat=3):
        if (a[0] + b[0], a[1] + b[1]) == (0, 0) or (b[0] + c[0], b[1] + c[1]) == (0, 0):
            continue
        prevs.add((a[0] + b[0] + c[0], a[1] + b[1] + c[1]))
    for a, b in itertools.product(STEPS, repeat=2):
        if (a[0] + b[0], a[1] + b[1]) != (0, 0):
            nexts.add((a[0] + b[0], a[1] + b[1]))
    return sorted(prevs), sorted(nexts)


def angle_table_entries() -> dict:
    prevs, nexts = key_vectors()
    pf = PathFinderOracle()
    out = {}
    for p in prevs:
        for n in nexts:
            q = (p[0] + 20, p[1])
            path = [(0, 0), (0, 0), (0, 0), p, q, q, (q[0] + n[0], q[1] + n[1]), (0, 0)]
            pf.angle_cache.clear()
            deg = pf._angle(path, 7)
            pen = 0 if deg <= 30 else (deg / 90) ** 1.5
            out[(p[0], p[1], n[0], n[1])] = (deg, pen)
    return out

"""Seeded procedural walkable-surface masks (synthetic workload, not product code).

Used by the golden generator (tests/golden/gen_goldens.py), the parity tests
and bench.py's planted-mask regime (SURVEY.md §8d "procedural corridor masks
from the same seed").  A mask is a boolean cell grid ``g[R, C]`` (one entry per
20-px cell, row = y index); the pixel mask handed to the grid builder is
``kron(g, ones(20, 20))`` exactly as in SURVEY.md Appendix C step 5.

Nothing here is on the product path: the product consumes masks, it never
generates them.
"""
from __future__ import annotations

import numpy as np

GRID = 20


def corridor_cells(seed: int, rows: int = 32, cols: int = 32) -> np.ndarray:
    """One seeded corridor-like cell mask of shape (rows, cols), dtype bool.

    The shape mimics a pavement seen from a walking user: a trapezoid rising
    from the bottom edge that narrows with height, drifts left/right, may fork
    into a side branch and may contain obstacles (holes).
    """
    rng = np.random.default_rng(seed)
    g = np.zeros((rows, cols), dtype=bool)
    top = int(rng.integers(0, rows // 2))
    bottom_gap = int(rng.integers(0, 3)) if rng.random() < 0.2 else 0
    centre = cols / 2 + rng.normal(0, cols / 10)
    width0 = rng.uniform(0.3, 0.7) * cols
    drift = rng.normal(0, 0.6)
    turn_at = int(rng.integers(top, rows)) if rng.random() < 0.5 else -1
    turn_drift = rng.choice([-1.5, 1.5]) if turn_at >= 0 else 0.0
    for r in range(rows - 1 - bottom_gap, top - 1, -1):
        frac = (rows - 1 - r) / max(1, rows - 1)
        width = max(1.0, width0 * (1.0 - 0.7 * frac))
        lo = int(round(centre - width / 2))
        hi = int(round(centre + width / 2))
        lo, hi = max(0, lo), min(cols - 1, hi)
        if lo <= hi:
            g[r, lo:hi + 1] = True
        centre += drift + (turn_drift if 0 <= turn_at and r < turn_at else 0.0)
        centre = float(np.clip(centre, 0, cols - 1))
    # side branch
    if rng.random() < 0.4:
        br = int(rng.integers(top, rows))
        direction = 1 if rng.random() < 0.5 else -1
        start = cols // 2
        length = int(rng.integers(3, cols // 2))
        thick = int(rng.integers(1, 4))
        for c in range(start, start + direction * length, direction):
            if 0 <= c < cols:
                g[max(0, br - thick):br + 1, c] = True
        # branch rises
        end_c = int(np.clip(start + direction * length, 0, cols - 1))
        rise = int(rng.integers(0, max(1, br)))
        g[max(0, br - rise):br + 1, max(0, end_c - 1):end_c + 1] = True
    # obstacles
    for _ in range(int(rng.integers(0, 3))):
        orow = int(rng.integers(0, rows))
        ocol = int(rng.integers(0, cols))
        oh, ow = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        g[orow:orow + oh, ocol:ocol + ow] = False
    # speckle
    if rng.random() < 0.3:
        n = int(rng.integers(1, 6))
        g[rng.integers(0, rows, n), rng.integers(0, cols, n)] ^= True
    if not g.any():
        g[rows - 1, cols // 2] = True
    return g


def cells_to_mask(g: np.ndarray) -> np.ndarray:
    """Pixel mask (uint8 0/1) for a cell grid: kron(g, ones(20, 20))."""
    return np.kron(g.astype(np.uint8), np.ones((GRID, GRID), dtype=np.uint8))


def cells_rect(g: np.ndarray) -> tuple[int, int, int, int]:
    """cv2.boundingRect of the filled cell mask: (x, y, w, h) in pixels."""
    rows = np.where(g.any(axis=1))[0]
    cols = np.where(g.any(axis=0))[0]
    r0, r1, c0, c1 = int(rows[0]), int(rows[-1]), int(cols[0]), int(cols[-1])
    return (GRID * c0, GRID * r0, GRID * (c1 - c0 + 1), GRID * (r1 - r0 + 1))


def fixture_640(g_native: np.ndarray) -> np.ndarray:
    """Resample a 64x36 reference fixture to the 640x640 frame: g[::2, 2:34]
    (fixture goldens item 1)."""
    return np.ascontiguousarray(g_native[::2, 2:34])

"""Helpers of the reference's utils.py (utils.py:6-58) for the Python surface.

``get_closest_grid_to_point`` is what FrameProcessor._find_paths uses to pick the
start / end cells; in this package the hot path does that selection on the GPU
(nav_grid_kernel) and this function serves callers that hold Grid objects.
"""
from __future__ import annotations

import numpy as np

from .models import Coordinate, Grid


def get_closest_grid_to_point(point: Coordinate, grids: list[list[Grid]]):
    """Nearest non-empty cell centre (Euclidean), rows in list order, first one wins (utils.py:6-32)."""
    best, best_d = None, np.inf
    for row in grids:
        for g in row:
            if g.empty:
                continue
            d = np.sqrt((point.x - g.centre.x) ** 2 + (point.y - g.centre.y) ** 2)
            if d < best_d:
                best, best_d = g, d
    return best


def point_to_line_distance(point: Coordinate, line_start: Coordinate, line_end: Coordinate) -> float:
    """Perpendicular distance from a point to the line through two points (utils.py:35-58)."""
    x, y = point.to_tuple()
    x1, y1 = line_start.to_tuple()
    x2, y2 = line_end.to_tuple()
    den = np.sqrt((y2 - y1) ** 2 + (x2 - x1) ** 2)
    if den == 0:
        return np.sqrt((x - x1) ** 2 + (y - y1) ** 2)
    return abs((y2 - y1) * x - (x2 - x1) * y + x2 * y1 - y2 * x1) / den

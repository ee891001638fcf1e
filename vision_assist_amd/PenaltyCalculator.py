"""PenaltyCalculator surface (reference: PenaltyCalculator.py).

The per-cell penalties (PenaltyCalculator.py:26-142) are computed for a whole
frame at once on the GPU by ``nav_grid_kernel`` (va_nav_run) -- bit-identical
float64 values, including the int 0 / int 1 clamp branches and the stale-row
easy-segment lookup.  This singleton keeps the
reference's method names for callers that drive FrameProcessor step by step:
``_pre_compute_easy_segments`` records the frame's grids, ``calculate_penalty``
returns the device value for one of that frame's Grid objects.  It does not
evaluate penalties for hand-built grid lists (there is no CPU path).
"""
from __future__ import annotations

from typing import ClassVar, Optional

from .config import penalty_colour_gradient
from .models import Grid


class PenaltyCalculator:
    _instance: ClassVar[Optional["PenaltyCalculator"]] = None
    _initialized: bool = False

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self):
        if not self._initialized:
            self._initialized = True
            self._grids = None
            self._table: dict[int, float] = {}  # id(Grid) -> device penalty, filled by FrameProcessor

    def _pre_compute_easy_segments(self, np_grids, grids) -> None:
        self._grids = grids

    def calculate_penalty(self, grid: Grid, grid_lookup: dict) -> float:
        if grid.empty:
            return 0
        pen = self._table.get(id(grid))
        if pen is None:
            raise ValueError("calculate_penalty: this Grid was not produced by vision_assist_amd.FrameProcessor "
                             "(penalties are computed for whole frames on the GPU)")
        return pen

    def get_penalty_colour(self, penalty: float) -> tuple[int, int, int]:
        """Nearest gradient colour (PenaltyCalculator.py:144-153; debug drawing only)."""
        key = min(penalty_colour_gradient.keys(), key=lambda k: abs(k - penalty))
        return penalty_colour_gradient[key]


penalty_calculator = PenaltyCalculator()

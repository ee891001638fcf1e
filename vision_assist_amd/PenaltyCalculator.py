"""PenaltyCalculator surface (reference: PenaltyCalculator.py).

The per-cell penalties (PenaltyCalculator.py:26-142) are computed for a whole
frame at once on the GPU by ``nav_grid_kernel`` (va_nav_run) -- bit-identical
float64 values, including the int 0 / int 1 clamp branches and the stale-row
easy-segment lookup.  This singleton keeps the
reference's method names for callers that drive FrameProcessor step by step:
``_pre_compute_easy_segments`` records the frame's grids, ``calculate_penalty``
returns the device value for one of that frame's Grid objects.  For grids built
elsewhere (the reference's own builder, e.g. a harness) the device grid stage is
run once on the frame those grids imply (FrameProcessor.device_frame_for: the
rounded rect and mask samples read back from the grids, checked by rebuilding
them on the device) and its values are served; a grid list no mask produces
raises.  The frame size is FrameProcessor's current frame's (as in the
reference, where only FrameProcessor._calculate_penalties calls it).
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
            self._standalone = None  # (grids, lookup, {id(Grid): penalty}) of the last caller-built grid list

    def _pre_compute_easy_segments(self, np_grids, grids) -> None:
        self._grids = grids

    def calculate_penalty(self, grid: Grid, grid_lookup: dict) -> float:
        if grid.empty:
            return 0
        pen = self._table.get(id(grid))
        if pen is None:
            pen = self._standalone_table(grid_lookup).get(id(grid))
            if pen is None:
                raise ValueError("calculate_penalty: this Grid is not in the grids given to _pre_compute_easy_segments "
                                 "or in grid_lookup")
        return pen

    def _standalone_table(self, grid_lookup: dict) -> dict[int, float]:
        """Penalties of a grid list built outside FrameProcessor, from the device grid stage on the frame it implies
        (FrameProcessor.device_frame_for), by list position and by lookup key; computed once per (grids, lookup)."""
        sa = self._standalone
        if sa is not None and sa[0] is self._grids and sa[1] is grid_lookup:
            return sa[2]
        from .FrameProcessor import FrameProcessor, device_frame_for
        fp = FrameProcessor._instance
        if self._grids is None or fp is None or getattr(fp, "frame", None) is None:
            raise ValueError("calculate_penalty on grids built outside FrameProcessor needs _pre_compute_easy_segments("
                             "np_grids, grids) first and FrameProcessor's frame (its size) set")
        H, W = int(fp.frame.shape[0]), int(fp.frame.shape[1])
        st = device_frame_for(self._grids, grid_lookup, H, W)
        table = {}
        for mine, dev in zip(self._grids, st.grids):
            for a, b in zip(mine, dev):
                table[id(a)] = b.penalty
        for k, g in grid_lookup.items():
            d = st.grid_lookup.get(k)
            if g is not None and d is not None and id(g) not in table:
                table[id(g)] = d.penalty
        self._standalone = (self._grids, grid_lookup, table)
        return table

    def get_penalty_colour(self, penalty: float) -> tuple[int, int, int]:
        """Nearest gradient colour (PenaltyCalculator.py:144-153; debug drawing only)."""
        key = min(penalty_colour_gradient.keys(), key=lambda k: abs(k - penalty))
        return penalty_colour_gradient[key]


penalty_calculator = PenaltyCalculator()

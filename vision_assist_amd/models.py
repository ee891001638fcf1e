"""Value types of the Python surface (reference: models.py).

Same class names, fields and computed properties as the reference so code that
consumes FrameProcessor results (PathAnalyser, harness scripts) works unchanged:

  Coordinate  models.py:17-27      Grid     models.py:29-36     Peak  models.py:38-42
  Corner      models.py:58-65      Instruction models.py:67-76  Path  models.py:83-364
  FinalAnswer models.py:11-14

``Path`` splits itself into straight / curved sections and detects corners on
construction (models.py:96-99, 160-364); that host-side logic is restated here
step for step (it feeds PathAnalyser's decision) and is
checked against the reference's own answers in tests/test_surface.py.
"""
from __future__ import annotations

import math

from enum import Enum
from typing import Any, Literal

import numpy as np
from pydantic import BaseModel, computed_field

from .config import grid_size


class FinalAnswer(Enum):
    MOVE_LEFT = "move_left"
    MOVE_RIGHT = "move_right"
    CONTINUE_FORWARD = "continue_forward"


class Coordinate(BaseModel):
    x: int
    y: int

    @computed_field
    @property
    def midpoint(self) -> tuple[int, int]:
        half = grid_size // 2
        return (self.x + half, self.y + half)

    def to_tuple(self) -> tuple[int, int]:
        return (self.x, self.y)


class Grid(BaseModel):
    coords: Coordinate
    centre: Coordinate
    penalty: float | None  # None for empty cells
    row: int
    col: int
    empty: bool
    artificial: bool


class Peak(BaseModel):
    centre: Coordinate
    left: Coordinate | None = None
    right: Coordinate | None = None
    orientation: Literal["left", "right", "up"]


class Corner(BaseModel):
    direction: Literal["left", "right"]
    sharpness: Literal["sharp", "sweeping"]
    shape: Literal["inner", "outer", "optimal"]
    start: Coordinate
    end: Coordinate
    angle_change: float
    length: float


class Instruction(BaseModel):
    direction: Literal["left", "right", "straight"]
    danger: Literal["immediate", "high", "medium", "low"]
    start: Coordinate
    end: Coordinate
    distance: float
    angle_change: float
    length: float
    instruction_type: Literal["turn", "curve", "bearing"]


class PathColours(BaseModel):
    close: tuple[int, int, int]
    mid: tuple[int, int, int]
    far: tuple[int, int, int]


def signed_angle_from_vertical(a: Coordinate, b: Coordinate) -> float:
    """Angle (degrees) between a->b and the vertical through a; negative when b is left of a
    (models.py:101-131)."""
    vx, vy = b.x - a.x, b.y - a.y
    ux, uy = 0, b.y - a.y  # (a.x, b.y) - a
    n1 = np.sqrt(vx ** 2 + vy ** 2)
    n2 = np.sqrt(ux ** 2 + uy ** 2)
    if n1 == 0 or n2 == 0:
        return 0
    deg = np.degrees(np.arccos((vx * ux + vy * uy) / (n1 * n2)))
    return -deg if b.x < a.x else deg


def _first_nearest(point: Coordinate, cells: list[Grid]):
    """Nearest non-empty cell centre, first one wins on ties (models.py:272-298).  math.sqrt, not the
    reference's np.sqrt: both are the correctly rounded square root of the same float64, so every comparison
    (and the cell returned) is the same, without numpy's per-scalar call overhead."""
    best, best_d = None, np.inf
    px, py = point.x, point.y
    sqrt = math.sqrt
    for c in cells:
        if c.empty:
            continue
        ce = c.centre
        d = sqrt((px - ce.x) ** 2 + (py - ce.y) ** 2)
        if d < best_d:
            best, best_d = c, d
    return best


def _vertical_runs(cells: list[Grid]) -> list[tuple[int, int]]:
    """First pass of Path._calculate_sections (models.py:172-198): index ranges of >= 5 cells
    linked by purely vertical moves."""
    runs = []
    run_start, run_len, prev_dir = 0, 1, None
    n = len(cells)
    xy = [(c.coords.x, c.coords.y) for c in cells]
    for i in range(1, n):
        dx = xy[i][0] - xy[i - 1][0]
        dy = xy[i][1] - xy[i - 1][1]
        d = "vertical" if (dx == 0 and dy != 0) else None
        if i == 1:
            prev_dir = d
        if d == prev_dir == "vertical":
            run_len += 1
            if run_len >= 5 and i == n - 1:
                runs.append((run_start, i))
        else:
            if run_len >= 5:
                runs.append((run_start, i - 1))
            run_start, run_len = i, 1
        prev_dir = d
    return runs


class Path(BaseModel):
    """A path of grid cells; a main path ("path") splits itself into sections and corners."""

    grids: list[Grid]
    total_cost: float
    path_type: Literal["path", "section-straight", "section-curved"]
    sections: list[Path] | None = None
    corners: list[Corner] | None = None
    points: list[tuple[Coordinate, Coordinate]] | None = None

    def model_post_init(self, __context: Any) -> None:
        if self.path_type == "path" and self.grids:
            self._calculate_sections()
            self._detect_corners()

    @staticmethod
    def _angle_from_vertical(start: Coordinate, end: Coordinate) -> float:
        return signed_angle_from_vertical(start, end)

    @computed_field
    @property
    def start(self) -> Coordinate:
        return self.grids[0].coords if self.grids else Coordinate(x=0, y=0)

    @computed_field
    @property
    def end(self) -> Coordinate:
        return self.grids[-1].coords if self.grids else Coordinate(x=0, y=0)

    @computed_field
    @property
    def length(self) -> float:
        return np.hypot(self.end.x - self.start.x, self.end.y - self.start.y)

    @property
    def angle(self) -> float:
        return signed_angle_from_vertical(self.start, self.end)

    @property
    def has_a_corner(self) -> bool:
        return self.corners is not None

    # -- sections (models.py:160-270) --------------------------------------------------
    def _share(self, cells: list[Grid]) -> float:
        return self.total_cost * (len(cells) / len(self.grids))

    def _grow(self, section: "Path", cells: list[Grid]) -> None:
        section.grids.extend(cells)
        section.total_cost = self._share(section.grids)

    def _calculate_sections(self) -> None:
        if not self.grids:
            return
        g = self.grids
        self.sections = []
        done = 0  # index of the last cell already covered by a section
        for s, e in _vertical_runs(g):
            if s > done:
                gap = g[done:s + 1]  # joins the previous section at its last cell
                if len(gap) <= 4:
                    if self.sections:
                        self._grow(self.sections[-1], gap[1:])
                    else:
                        merged = gap + g[s:e + 1]
                        self.sections.append(Path(grids=merged, total_cost=self._share(merged),
                                                  path_type="section-straight"))
                        done = e
                        continue
                else:
                    self.sections.append(Path(grids=gap, total_cost=self._share(gap), path_type="section-curved"))
            run = g[s:e + 1]
            if self.sections and self.sections[-1].path_type == "section-straight":
                self._grow(self.sections[-1], run[1:])
            else:
                self.sections.append(Path(grids=run, total_cost=self._share(run), path_type="section-straight"))
            done = e
        if done < len(g) - 1:
            tail = g[done:]
            if len(tail) < 4 and self.sections:
                self._grow(self.sections[-1], tail[1:])
            else:
                self.sections.append(Path(grids=tail, total_cost=self._share(tail), path_type="section-curved"))

    @staticmethod
    def _get_closest_grid_to_point(point: Coordinate, grids: list[Grid]):
        return _first_nearest(point, grids)

    # -- corners (models.py:300-364) ---------------------------------------------------
    def _detect_corners(self) -> None:
        if not self.sections:
            return
        self.corners = []
        self.points = []
        for sec in self.sections:
            for p in (sec.start, sec.end):
                if p not in self.points:
                    self.points.append(p)
        for sec in self.sections:
            if sec.path_type == "section-straight":
                continue
            a, b = sec.grids[0], sec.grids[-1]
            turn = signed_angle_from_vertical(a.centre, b.centre)
            dx, dy = b.centre.x - a.centre.x, b.centre.y - a.centre.y
            side = "right" if a.centre.x - b.centre.x < 0 else "left"
            mid = Coordinate(x=a.centre.x + dx // 2, y=a.centre.y + dy // 2)
            near = _first_nearest(mid, sec.grids)
            off = np.hypot(abs(near.centre.x - mid.x), abs(near.centre.y - mid.y))
            limit = (np.hypot(dx, dy)) ** 2 / (off + 1) ** 2
            if off < limit:
                shape = "optimal"
            else:
                shape = "inner" if (near.centre.y - mid.y) < 0 else "outer"
            while turn > 90:
                turn -= 90
            self.corners.append(Corner(direction=side, sharpness="sharp" if turn > 30 else "sweeping", shape=shape,
                                       start=a.coords, end=b.coords, angle_change=turn, length=sec.length))

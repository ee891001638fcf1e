"""PathVisualiser: the debug drawing of FrameProcessor(debug=True) (PathVisualiser.py:1-123,
FrameProcessor.py:273-299), on the host frame as the reference draws it with OpenCV.

What is drawn, in the reference's order:
  * FrameProcessor._draw_non_path_grids (FrameProcessor.py:287-299): every non-empty grid of ``self.grids``
    (row by row) as cv2.fillPoly of its square (x, y) .. (x + 20, y + 20) in the penalty colour
    (PenaltyCalculator.get_penalty_colour);
  * path_visualiser(frame, paths) (PathVisualiser.py:54-121): per path, its sections' grids in the section's
    colour (PATH_COLORS alternate per section, far / mid / close by the section's position), then a white
    2-pixel line from each section's first to last grid centre, then per corner two white dots of radius 5 at
    (start + 10) and (end + 10).

The squares are cv2.fillPoly of an axis-aligned integer square, which is exactly the inclusive pixel range
[x, x + 20] x [y, y + 20] (clipped to the frame).  OpenCV is absent here, so the thick line (cv2.line, thickness 2)
and the filled circle (cv2.circle, thickness -1) are restated as a 2-pixel-wide Bresenham line and the disc
dx^2 + dy^2 <= r^2 + r, and the corner labels (cv2.putText, Hershey simplex, scale 0.5, thickness 2) are drawn
with strokefont.put_text: the same text, origin, scale and thickness in this module's own stroke glyphs.  This
rendering's pixel parity with cv2 is unpinned (debug output only)."""
from __future__ import annotations

from typing import ClassVar, Optional

import numpy as np

from .config import grid_size
from .models import Corner, Path, PathColours
from .strokefont import put_text


def corner_label(section_idx: int, corner: Corner) -> str:
    """The corner marker's text (PathVisualiser.py:50)."""
    return f"{section_idx + 1} {corner.direction} {corner.shape} {corner.sharpness}"


def fill_square(frame: np.ndarray, x: int, y: int, color) -> None:
    """cv2.fillPoly of the square (x, y), (x + g, y), (x + g, y + g), (x, y + g): the inclusive pixel range."""
    H, W = frame.shape[:2]
    x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + grid_size, W - 1), min(y + grid_size, H - 1)
    if x0 <= x1 and y0 <= y1:
        frame[y0:y1 + 1, x0:x1 + 1] = color


def draw_line2(frame: np.ndarray, x0: int, y0: int, x1: int, y1: int, color) -> None:
    """A 2-pixel-wide line: the 8-connected Bresenham line and its neighbour across the minor axis."""
    H, W = frame.shape[:2]
    dx, dy = abs(x1 - x0), abs(y1 - y0)
    sx, sy = (1 if x1 >= x0 else -1), (1 if y1 >= y0 else -1)
    steep = dy > dx
    err = (dx if not steep else dy) // 2
    x, y = x0, y0
    for _ in range(max(dx, dy) + 1):
        for px, py in ((x, y), (x + 1, y) if steep else (x, y + 1)):
            if 0 <= px < W and 0 <= py < H:
                frame[py, px] = color
        if steep:
            y += sy
            err -= dx
            if err < 0:
                x += sx
                err += dy
        else:
            x += sx
            err -= dy
            if err < 0:
                y += sy
                err += dx


def fill_circle(frame: np.ndarray, cx: int, cy: int, r: int, color) -> None:
    """A filled disc of radius r: pixels with dx^2 + dy^2 <= r^2 + r."""
    H, W = frame.shape[:2]
    ys, xs = np.ogrid[max(cy - r, 0):min(cy + r, H - 1) + 1, max(cx - r, 0):min(cx + r, W - 1) + 1]
    m = (xs - cx) ** 2 + (ys - cy) ** 2 <= r * r + r
    frame[max(cy - r, 0):min(cy + r, H - 1) + 1, max(cx - r, 0):min(cx + r, W - 1) + 1][m] = color


class PathVisualiser:
    _instance: ClassVar[Optional["PathVisualiser"]] = None
    _initialized: bool = False

    PATH_COLORS = [
        PathColours(close=(0, 0, 255), mid=(0, 0, 200), far=(0, 0, 150)),  # blue variants (PathVisualiser.py:13)
        PathColours(close=(255, 0, 0), mid=(200, 0, 0), far=(150, 0, 0)),  # red variants (PathVisualiser.py:14)
    ]

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self):
        if not self._initialized:
            self._initialized = True
            self.frame: np.ndarray | None = None
            self.paths: list[Path] = []

    def _draw_path_grid(self, grid, color) -> None:
        fill_square(self.frame, grid.coords.x, grid.coords.y, color)

    def _draw_corner_marker(self, section_idx: int, corner: Corner, path: Path) -> None:
        fill_circle(self.frame, corner.start.x + 10, corner.start.y + 10, 5, (255, 255, 255))
        fill_circle(self.frame, corner.end.x + 10, corner.end.y + 10, 5, (255, 255, 255))
        put_text(self.frame, corner_label(section_idx, corner), (corner.end.x - 100, corner.end.y - 5), 0.5,
                 (255, 255, 255), 2)

    def _draw_path_sections(self, path: Path, path_idx: int) -> None:
        if not path.sections:
            return
        for i, section in enumerate(path.sections):
            colors = self.PATH_COLORS[i % 2]
            progress = i / len(path.sections)
            color = colors.far if progress < 0.33 else (colors.mid if progress < 0.66 else colors.close)
            for grid in section.grids:
                self._draw_path_grid(grid, color)
        h = grid_size // 2
        for section in path.sections:
            draw_line2(self.frame, section.start.x + h, section.start.y + h, section.end.x + h, section.end.y + h,
                       (255, 255, 255))
        if path.corners:
            for idx, corner in enumerate(path.corners):
                self._draw_corner_marker(idx, corner, path)

    def __call__(self, frame: np.ndarray, paths: list[Path]) -> np.ndarray:
        self.frame = frame
        self.paths = paths
        for idx, path in enumerate(self.paths):
            self._draw_path_sections(path, idx)
        return self.frame


path_visualiser = PathVisualiser()

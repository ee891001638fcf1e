"""A small stroke font for the debug rendering's corner labels (PathVisualiser.py:48-56 draws them with
cv2.putText(frame, f"{idx + 1} {direction} {shape} {sharpness}", (end.x - 100, end.y - 5),
FONT_HERSHEY_SIMPLEX, 0.5, white, 2)).

OpenCV and its Hershey glyph tables are absent from this image, so the glyphs here are this module's own
polylines on the Hershey simplex grid (baseline y = 0, lowercase x-height 14 units, caps / ascenders 21, descenders
7, y grows downward as in image rows; one unit = fontScale pixels), covering the label vocabulary: the digits, the
space and the lowercase letters of left / right / inner / outer / optimal / sharp / sweeping (+ '-' and '.').
An unknown character advances like a space.  What follows cv2.putText: the text string, the origin at the
baseline's left end, the scale and the stroke thickness; the glyph outlines themselves are unpinned
(debug output only)."""
from __future__ import annotations

import math

import numpy as np


def _arc(cx, cy, rx, ry, a0, a1, n=10):
    """Points of an elliptical arc, angles in degrees (0 = +x, 90 = up, i.e. -y)."""
    return [(cx + rx * math.cos(math.radians(a0 + (a1 - a0) * i / n)),
             cy - ry * math.sin(math.radians(a0 + (a1 - a0) * i / n))) for i in range(n + 1)]


# glyph: (advance, [polyline, ...]); polyline = [(x, y), ...] in font units
GLYPHS: dict[str, tuple[float, list[list[tuple[float, float]]]]] = {
    " ": (16, []),
    "-": (18, [[(3, -7), (13, -7)]]),
    ".": (8, [[(3, -1), (3, 0)]]),
    "0": (18, [_arc(6.5, -10.5, 5.5, 10.5, 0, 360, 20)]),
    "1": (18, [[(3, -17), (7, -21), (7, 0)]]),
    "2": (18, [_arc(6.5, -16, 5.5, 5, 165, -30, 8) + [(1, 0), (12, 0)]]),
    "3": (18, [[(1, -21), (12, -21), (6, -13)] + _arc(6.5, -6.5, 5.5, 6.5, 100, -150, 10)]),
    "4": (18, [[(10, 0), (10, -21), (0, -7), (13, -7)]]),
    "5": (18, [[(11, -21), (2, -21), (1, -12)] + _arc(6.5, -6.5, 5.5, 6.5, 130, -150, 10)]),
    "6": (18, [[(11, -19), (8, -21), (5, -21)] + _arc(6.5, -10.5, 5.5, 10.5, 105, 200, 6)
               + _arc(6.5, -6.5, 5.5, 6.5, 180, -180, 16)]),
    "7": (18, [[(1, -21), (12, -21), (4, 0)]]),
    "8": (18, [_arc(6.5, -16, 4.5, 5, -90, 270, 14), _arc(6.5, -5.5, 5.5, 5.5, 90, 450, 16)]),
    "9": (18, [_arc(6.5, -14.5, 5.5, 6.5, 0, 360, 16) + _arc(6.5, -10.5, 5.5, 10.5, 0, -75, 6) + [(2, -2)]]),
    "a": (18, [[(12, -14), (12, 0)], _arc(6.5, -7, 5.5, 7, 45, 315, 12)]),
    "e": (18, [[(1, -7), (12, -7)] + _arc(6.5, -7, 5.5, 7, 0, 315, 14)]),
    "f": (11, [[(9, -21), (7, -21), (5, -19), (4, -16), (4, 0)], [(1, -14), (8, -14)]]),
    "g": (18, [[(12, -14), (12, 3), (11, 6), (9, 7), (5, 7), (2, 6)], _arc(6.5, -7, 5.5, 7, 45, 315, 12)]),
    "h": (18, [[(1, -21), (1, 0)], [(1, -10), (4, -13), (6, -14), (9, -14), (11, -13), (12, -10), (12, 0)]]),
    "i": (8, [[(3, -14), (3, 0)], [(3, -20), (3, -19)]]),
    "l": (8, [[(3, -21), (3, 0)]]),
    "m": (24, [[(1, -14), (1, 0)], [(1, -10), (4, -13), (6, -14), (8, -13), (10, -10), (10, 0)],
               [(10, -10), (13, -13), (15, -14), (17, -13), (19, -10), (19, 0)]]),
    "n": (18, [[(1, -14), (1, 0)], [(1, -10), (4, -13), (6, -14), (9, -14), (11, -13), (12, -10), (12, 0)]]),
    "o": (18, [_arc(6.5, -7, 5.5, 7, 0, 360, 16)]),
    "p": (18, [[(1, -14), (1, 7)], _arc(6.5, -7, 5.5, 7, 135, -135, 12)]),
    "r": (12, [[(1, -14), (1, 0)], [(1, -8), (2, -11), (4, -13), (6, -14), (9, -14)]]),
    "s": (16, [[(11, -11), (10, -13), (7, -14), (4, -14), (1, -13), (0, -11), (1, -9), (3, -8), (8, -7),
                (10, -6), (11, -4), (11, -3), (10, -1), (7, 0), (4, 0), (1, -1), (0, -3)]]),
    "t": (11, [[(4, -21), (4, -4), (5, -1), (7, 0), (9, 0)], [(1, -14), (8, -14)]]),
    "u": (18, [[(1, -14), (1, -4), (2, -1), (4, 0), (7, 0), (9, -1), (12, -4)], [(12, -14), (12, 0)]]),
    "w": (20, [[(1, -14), (4.5, 0), (8, -14), (11.5, 0), (15, -14)]]),
}


def _blit_segment(frame: np.ndarray, x0: float, y0: float, x1: float, y1: float, color, thickness: int) -> None:
    """A segment of the given thickness: discs of diameter `thickness` stamped along it (cv2's thick lines are
    round-capped polygons; this is its stamped counterpart)."""
    H, W = frame.shape[:2]
    r = max(thickness, 1) / 2.0
    n = int(math.ceil(max(abs(x1 - x0), abs(y1 - y0)))) + 1
    for k in range(n + 1):
        cx = x0 + (x1 - x0) * k / n
        cy = y0 + (y1 - y0) * k / n
        for py in range(int(math.floor(cy - r)), int(math.floor(cy + r)) + 1):
            for px in range(int(math.floor(cx - r)), int(math.floor(cx + r)) + 1):
                if 0 <= px < W and 0 <= py < H and (px + 0.5 - cx) ** 2 + (py + 0.5 - cy) ** 2 <= r * r + 0.25:
                    frame[py, px] = color


def text_size(text: str, scale: float, thickness: int) -> tuple[tuple[int, int], int]:
    """((width, height), baseline) like cv2.getTextSize: height = the cap height, baseline = the descender."""
    w = sum(GLYPHS.get(ch, GLYPHS[" "])[0] for ch in text) * scale
    return (int(round(w + thickness)), int(round(21 * scale + thickness))), int(round(7 * scale + thickness))


def put_text(frame: np.ndarray, text: str, org: tuple[int, int], scale: float, color, thickness: int) -> None:
    """cv2.putText(frame, text, org, <this stroke font>, scale, color, thickness): org = the left end of the
    baseline; glyphs clipped to the frame; drawn in place."""
    x = float(org[0])
    y = float(org[1])
    for ch in text:
        adv, strokes = GLYPHS.get(ch, GLYPHS[" "])
        for line in strokes:
            for (ax, ay), (bx, by) in zip(line, line[1:]):
                _blit_segment(frame, x + ax * scale, y + ay * scale, x + bx * scale, y + by * scale, color, thickness)
        x += adv * scale

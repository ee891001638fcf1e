"""CPU restatement of the mask -> polygon -> cells boundary (TEST INFRASTRUCTURE: the checker of the device
kernels in vision_assist_amd/csrc/va_post.hip; never imported by the product).

The reference reduces the chosen YOLO mask to grid cells with OpenCV (FrameProcessor.py:67-97), via
Ultralytics' Results.masks.xy (results.py Masks.xy -> ops.masks2segments, ops.scale_coords; vendored spec copy
testing/old/segmenting_using_tflite/ops.py:784-816, 837-859):

  masks2segments   cv2.findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE), keep the contour with the most
                   points ('largest', first on ties), float32                           (ops.py:850-855)
  scale_coords     (xy - pad) / gain in float32, clipped to [0, W] x [0, H]             (ops.py:784-816)
  choice           max(xy, key=cv2.contourArea) when more than one mask (first maximum) (FrameProcessor.py:72-73)
  np.int32         truncation of the float32 polygon                                    (FrameProcessor.py:75)
  boundingRect     of the int32 points                                                  (FrameProcessor.py:76)
  fillPoly         cv2.fillPoly(zeros(H, W), [points], 1), sampled at the cell centres  (FrameProcessor.py:85-97)

OpenCV (opencv-python 4.x) is not installed here and is third-party to the reference, so its published
algorithms are restated:
  * findContours: Suzuki & Abe border following as in OpenCV's contours.cpp (cvStartFindContours /
    cvFindNextContour / icvFetchContour, the legacy implementation the 4.x rewrite reproduces): the image is
    thresholded to 0/1 and framed by one zero pixel (cv::findContours' copyMakeBorder); a raster scan starts an
    outer border at a 0 -> 1 transition; RETR_EXTERNAL skips it when the last border pixel met on that row
    (lnbd) carries a positive mark, i.e. the scan is inside a traced outer border; the border is followed with
    the 8-neighbour chain code (directions 0 = +x, then counter-clockwise with y down), pixels marked 2 or
    -126 (a "right" border pixel, whose east neighbour was passed as 0); CHAIN_APPROX_SIMPLE keeps the points
    where the chain code changes.
  * contourArea: shoelace in double over float32 points, starting from the last point, |a| / 2.
  * fillPoly (lineType 8, shift 0): CollectPolyEdges (every edge drawn as an 8-connected Bresenham line,
    LineIterator with clipLine; non-horizontal edges kept as 16.16 fixed-point with x at the upper end + 0.5 and
    dx = ((x1 - x0) << 16) / (y1 - y0) truncated; edges leaving the image rebuilt from the clipped line) and
    FillEdgeCollection (per row y0 <= y < y1 the active edges sorted by x are paired, pixels x_left >> 16 ..
    x_right >> 16 filled).

PARITY WITH cv2 ITSELF IS UNPINNED: no reference output or fixture holds OpenCV's result for a mask; the
device kernels are checked bit-exactly against this restatement.
"""
from __future__ import annotations

import numpy as np

XY_SHIFT = 16
XY_ONE = 1 << XY_SHIFT
# chain code directions (icvCodeDeltas): 0 = +x, 1 = (+1, -1), 2 = -y, ... counter-clockwise with y pointing down
CODE_DX = (1, 1, 0, -1, -1, -1, 0, 1)
CODE_DY = (0, -1, -1, -1, 0, 1, 1, 1)
NBD = 2            # icvFetchContour's mark for a traced border pixel
NEG = 2 | -128     # (schar)(nbd | -128) = -126: a border pixel whose east neighbour was passed as 0


# ------------------------------------------------------------------------------------------ findContours
def _fetch_contour(img: np.ndarray, y0: int, x0: int, is_hole: bool) -> list[tuple[int, int]]:
    """icvFetchContour with CHAIN_APPROX_SIMPLE on the framed int image (coordinates of the framed image)."""
    pts = []
    s_end = s = 0 if is_hole else 4
    # the first neighbour clockwise from s: s = (s - 1) & 7 until non-zero or back at s_end
    while True:
        s = (s - 1) & 7
        if img[y0 + CODE_DY[s], x0 + CODE_DX[s]] != 0 or s == s_end:
            break
    if s == s_end:  # single pixel domain
        img[y0, x0] = NEG
        pts.append((x0, y0))
        return pts
    y1, x1 = y0 + CODE_DY[s], x0 + CODE_DX[s]  # i1
    y3, x3 = y0, x0                             # i3
    prev_s = s ^ 4
    px, py = x0, y0
    while True:
        s_end = s
        # counter-clockwise from s_end + 1 to the first non-zero neighbour (deltas repeat past 7)
        while True:
            s += 1
            d = s & 7
            y4, x4 = y3 + CODE_DY[d], x3 + CODE_DX[d]
            if img[y4, x4] != 0:
                break
        s &= 7
        if 0 <= s - 1 < s_end:          # (unsigned)(s - 1) < (unsigned)s_end: passed the east neighbour
            img[y3, x3] = NEG
        elif img[y3, x3] == 1:
            img[y3, x3] = NBD
        if s != prev_s:
            pts.append((px, py))
            prev_s = s
        px += CODE_DX[s]
        py += CODE_DY[s]
        if (y4, x4) == (y0, x0) and (y3, x3) == (y1, x1):
            break
        y3, x3 = y4, x4
        s = (s + 4) & 7
    return pts


def find_contours_external(mask: np.ndarray) -> list[np.ndarray]:
    """cv2.findContours(mask, cv2.RETR_EXTERNAL, cv2.CHAIN_APPROX_SIMPLE)[0]: outer borders in scan order, each an
    int [k, 2] (x, y) array in the mask's coordinates.

    The raster scan of cvFindNextContour, row by row on the live (marked) image: it stops where a pixel differs
    from the last value passed (prev); a 0 -> 1 stop is an outer-border start, traced unless the pixel at lnbd
    carries a positive mark (RETR_EXTERNAL: inside a traced outer border).  lnbd (reset to the frame at each
    row) moves only at stops whose new value is a mark, and at a hole start (p == 0 after a marked prev) to the
    previous pixel; a traced start is passed with prev = its new mark, without moving lnbd."""
    H, W = mask.shape
    img = np.zeros((H + 2, W + 2), dtype=np.int16)
    img[1:H + 1, 1:W + 1] = mask != 0
    width = W + 2
    out = []
    # rows holding a 0 -> 1 transition of the original image: no other row can start a border (traces only turn
    # 1 into a mark, zeros never change)
    rows = np.nonzero(((img[:, 1:] == 1) & (img[:, :-1] == 0)).any(1))[0]
    for y in rows.tolist():
        row = img[y]
        x, prev, lnbd = 1, 0, 0
        while True:
            while x < width and row[x] == prev:
                x += 1
            if x >= width:
                break
            p = int(row[x])
            if prev == 0 and p == 1:  # outer border start
                if row[lnbd] <= 0:
                    pts = _fetch_contour(img, y, x, is_hole=False)
                    out.append(np.array([(px - 1, py - 1) for px, py in pts], dtype=np.int32))
                    prev = int(row[x])  # the scan resumes after the start with prev = its mark; lnbd unchanged
                    x += 1
                    continue
            elif p == 0 and prev >= 1:  # hole start (not traced in RETR_EXTERNAL)
                if prev & -2:
                    lnbd = x - 1
            prev = p  # resume_scan
            if p & -2:
                lnbd = x
            x += 1
    return out


def largest_segment(mask: np.ndarray) -> np.ndarray:
    """masks2segments(strategy='largest') for one mask (ops.py:850-855): float32 [k, 2]."""
    c = find_contours_external(mask.astype(np.uint8))
    if not c:
        return np.zeros((0, 2), dtype=np.float32)
    return c[int(np.argmax([len(x) for x in c]))].astype(np.float32)


def scale_coords(seg: np.ndarray, net_hw: tuple[int, int], frame_hw: tuple[int, int]) -> np.ndarray:
    """ops.scale_coords(img1_shape=net, coords, img0_shape=frame) in float32 (ops.py:784-816)."""
    gain = min(net_hw[0] / frame_hw[0], net_hw[1] / frame_hw[1])
    pad = (net_hw[1] - frame_hw[1] * gain) / 2, (net_hw[0] - frame_hw[0] * gain) / 2
    c = seg.astype(np.float32).copy()
    c[:, 0] -= np.float32(pad[0])
    c[:, 1] -= np.float32(pad[1])
    c[:, 0] /= np.float32(gain)
    c[:, 1] /= np.float32(gain)
    c[:, 0] = np.clip(c[:, 0], np.float32(0), np.float32(frame_hw[1]))
    c[:, 1] = np.clip(c[:, 1], np.float32(0), np.float32(frame_hw[0]))
    return c


def contour_area(poly: np.ndarray) -> float:
    """cv2.contourArea (oriented=False) of a float32 polygon: double shoelace starting from the last point."""
    n = poly.shape[0]
    if n == 0:
        return 0.0
    a = 0.0
    px, py = float(poly[n - 1, 0]), float(poly[n - 1, 1])
    for i in range(n):
        x, y = float(poly[i, 0]), float(poly[i, 1])
        a += px * y - py * x
        px, py = x, y
    return abs(a * 0.5)


def bounding_rect(pts: np.ndarray) -> tuple[int, int, int, int]:
    """cv2.boundingRect of int32 points (x, y, w, h); (0, 0, 0, 0) for none."""
    if pts.shape[0] == 0:
        return (0, 0, 0, 0)
    x0, y0 = int(pts[:, 0].min()), int(pts[:, 1].min())
    return (x0, y0, int(pts[:, 0].max()) - x0 + 1, int(pts[:, 1].max()) - y0 + 1)


# ------------------------------------------------------------------------------------------ fillPoly
def _clip_line(W: int, H: int, x1: int, y1: int, x2: int, y2: int):
    """cv::clipLine(Size2l(W, H), pt1, pt2) -> (inside, x1, y1, x2, y2)."""
    right, bottom = W - 1, H - 1
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8
    if (c1 & c2) == 0 and (c1 | c2) != 0:
        if c1 & 12:
            a = 0 if c1 < 8 else bottom
            x1 += int(float(a - y1) * (x2 - x1) / (y2 - y1))
            y1 = a
            c1 = (x1 < 0) + (x1 > right) * 2
        if c2 & 12:
            a = 0 if c2 < 8 else bottom
            x2 += int(float(a - y2) * (x2 - x1) / (y2 - y1))
            y2 = a
            c2 = (x2 < 0) + (x2 > right) * 2
        if (c1 & c2) == 0 and (c1 | c2) != 0:
            if c1:
                a = 0 if c1 == 1 else right
                y1 += int(float(a - x1) * (y2 - y1) / (x2 - x1))
                x1 = a
                c1 = 0
            if c2:
                a = 0 if c2 == 1 else right
                y2 += int(float(a - x2) * (y2 - y1) / (x2 - x1))
                x2 = a
                c2 = 0
    return (c1 | c2) == 0, x1, y1, x2, y2


def line8_pixels(W: int, H: int, x1: int, y1: int, x2: int, y2: int) -> list[tuple[int, int]]:
    """The pixels cv::Line(img, pt1, pt2, color, 8) sets: LineIterator(connectivity 8, leftToRight) after clipLine."""
    if not (0 <= x1 < W and 0 <= x2 < W and 0 <= y1 < H and 0 <= y2 < H):
        ok, x1, y1, x2, y2 = _clip_line(W, H, x1, y1, x2, y2)
        if not ok:
            return []
    dx, dy = x2 - x1, y2 - y1
    sx = sy = 1
    if dx < 0:  # leftToRight: swap the end points
        dx, dy = -dx, -dy
        x1, y1, x2, y2 = x2, y2, x1, y1
    if dy < 0:
        dy, sy = -dy, -1
    vert = dy > dx
    if vert:
        dx, dy = dy, dx
    err = dx - (dy + dy)
    plus_delta, minus_delta = dx + dx, -(dy + dy)
    # minor step when err < 0 (before the update); major step always
    out = []
    x, y = x1, y1
    for _ in range(dx + 1):
        out.append((x, y))
        minor = err < 0
        err += minus_delta + (plus_delta if minor else 0)
        if vert:
            y += sy
            x += sx if minor else 0
        else:
            x += sx
            y += sy if minor else 0
    return out


def poly_edges(pts: np.ndarray, W: int, H: int):
    """CollectPolyEdges(shift 0, LINE_8): (lines drawn [(x, y) pixels], edges [(y0, y1, x, dx)] in 16.16)."""
    n = pts.shape[0]
    drawn, edges = [], []
    if n == 0:
        return drawn, edges
    v = [(int(p[0]), int(p[1])) for p in pts]
    x0, y0 = v[n - 1]
    p0 = (x0 << XY_SHIFT, y0)
    for i in range(n):
        x1, y1 = v[i]
        p1 = (x1 << XY_SHIFT, y1)
        t0 = ((p0[0] + (XY_ONE >> 1)) >> XY_SHIFT, p0[1])
        t1 = ((p1[0] + (XY_ONE >> 1)) >> XY_SHIFT, p1[1])
        drawn.extend(line8_pixels(W, H, t0[0], t0[1], t1[0], t1[1]))
        p0c, p1c = list(p0), list(p1)
        if not (0 <= t0[0] < W and 0 <= t1[0] < W and 0 <= t0[1] < H and 0 <= t1[1] < H):
            ok, cx0, cy0, cx1, cy1 = _clip_line(W, H, t0[0], t0[1], t1[0], t1[1])
            if cy0 != cy1:
                p0c = [cx0 << XY_SHIFT, cy0]
                p1c = [cx1 << XY_SHIFT, cy1]
        else:
            p0c[0] += XY_ONE >> 1
            p1c[0] += XY_ONE >> 1
        if p0[1] != p1[1]:
            num, den = p1c[0] - p0c[0], p1c[1] - p0c[1]
            dxe = abs(num) // abs(den) * (1 if (num >= 0) == (den > 0) else -1)  # C++ truncating division
            if p0[1] < p1[1]:
                ey0, ey1, ex = p0[1], p1[1], p0c[0] + (p0[1] - p0c[1]) * dxe
            else:
                ey0, ey1, ex = p1[1], p0[1], p1c[0] + (p1[1] - p1c[1]) * dxe
            edges.append((ey0, ey1, ex, dxe))
        p0 = p1
    return drawn, edges


def fill_poly_samples(pts: np.ndarray, H: int, W: int, xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
    """cv2.fillPoly(zeros(H, W), [pts], 1) read at the pixels (ys[r], xs[c]): uint8 [len(ys), len(xs)]."""
    out = np.zeros((len(ys), len(xs)), dtype=np.uint8)
    drawn, edges = poly_edges(pts, W, H)
    col = {int(x): c for c, x in enumerate(xs)}
    row = {int(y): r for r, y in enumerate(ys)}
    for x, y in drawn:
        if x in col and y in row:
            out[row[y], col[x]] = 1
    if len(edges) < 2:
        return out
    ymin = min(e[0] for e in edges)
    ymax = max(e[1] for e in edges)
    xmin = min(min(e[2], e[2] + (e[1] - e[0]) * e[3]) for e in edges)
    xmax = max(max(e[2], e[2] + (e[1] - e[0]) * e[3]) for e in edges)
    if ymax < 0 or ymin >= H or xmax < 0 or xmin >= (W << XY_SHIFT):
        return out
    for r, y in enumerate(ys.tolist()):
        xe = sorted(e[2] + (y - e[0]) * e[3] for e in edges if e[0] <= y < e[1])
        for k in range(0, len(xe) - 1, 2):
            x1, x2 = xe[k] >> XY_SHIFT, xe[k + 1] >> XY_SHIFT
            if x1 < W and x2 >= 0:
                x1, x2 = max(x1, 0), min(x2, W - 1)
                for c, x in enumerate(xs.tolist()):
                    if x1 <= x <= x2:
                        out[r, c] = 1
    return out


def fill_poly(pts: np.ndarray, H: int, W: int) -> np.ndarray:
    """cv2.fillPoly(zeros(H, W), [pts], 1) as a full image (test helper)."""
    return fill_poly_samples(pts, H, W, np.arange(W), np.arange(H))


# ------------------------------------------------------------------------------------------ the choice
def masks_xy(masks: np.ndarray, frame_hw: tuple[int, int]) -> list[np.ndarray]:
    """Results.masks.xy: per mask its largest external contour scaled to the frame (float32 [k, 2])."""
    net_hw = masks.shape[1:]
    return [scale_coords(largest_segment(m), net_hw, frame_hw) for m in masks]


def select_cells(masks: np.ndarray, frame_hw: tuple[int, int], grid: int = 20):
    """FrameProcessor._extract_grid_information's use of the masks (FrameProcessor.py:67-97): -> (chosen index or
    -1, int32 polygon, boundingRect, cell samples uint8 [H0 / grid, W0 / grid] of the filled polygon)."""
    H0, W0 = frame_hw
    cells = np.zeros((H0 // grid, W0 // grid), dtype=np.uint8)
    if masks.shape[0] == 0:
        return -1, np.zeros((0, 2), dtype=np.int32), (0, 0, 0, 0), cells
    xy = masks_xy(masks, frame_hw)
    if len(xy) > 1:
        areas = [contour_area(p) for p in xy]
        k = int(np.argmax(areas))  # max(..., key=contourArea): the first maximum
    else:
        k = 0
    pts = xy[k].astype(np.int32)  # np.int32: truncation
    rect = bounding_rect(pts)
    xs = np.arange(W0 // grid) * grid + grid // 2
    ys = np.arange(H0 // grid) * grid + grid // 2
    cells = fill_poly_samples(pts, H0, W0, xs, ys)
    return k, pts, rect, cells

"""CPU restatement of vision-assist's per-frame grid/navigation path.

TEST INFRASTRUCTURE ONLY (the parity oracle and bench.py's ``cpu_baseline``
leg).  The product path (``vision_assist_amd``) never imports this module; it
runs the HIP kernels in ``vision_assist_amd/csrc`` and fails loudly when they
are missing.

Pinned by ``tests/golden/nav_goldens.json.gz`` (outputs of the reference
itself, run in the build container by ``tests/golden/gen_goldens.py``):
see ``tests/test_oracle_golden.py``.

The restatement deliberately keeps the reference's algorithmic structure
(python per-cell loops, pydantic cell objects, heap A* with the per-relaxation
root-path walk and the linear open-set scan) so that timing it is a fair
stand-in for the reference on the same cores.

Reference anchors (all under /root/reference):
  grid build      FrameProcessor.py:50-171
  penalties       PenaltyCalculator.py:26-142, driver FrameProcessor.py:173-182
  graph           FrameProcessor.py:184-207
  protrusion      ProtrusionDetector.py:38-158, 419-535
  start/end       utils.py:6-32, FrameProcessor.py:237,240
  A*              PathFinder.py:7-189
  path dedupe     FrameProcessor.py:209-271
"""
from __future__ import annotations

import heapq
from collections import defaultdict

import numpy as np
from pydantic import BaseModel

GRID = 20  # config.py:1


class Coordinate(BaseModel):  # models.py:17-27 (fields only)
    x: int
    y: int


class Cell(BaseModel):  # models.py:29-36 ("Grid")
    coords: Coordinate
    centre: Coordinate
    penalty: float | None
    row: int
    col: int
    empty: bool
    artificial: bool


# ----------------------------------------------------------------------------- grid build
class GridState:
    """``self.grids`` / ``self.grid_lookup`` / ``self.np_grids`` of FrameProcessor."""

    def __init__(self):
        self.grids: list[list[Cell]] = []
        self.lookup: dict[tuple[int, int], Cell] = {}
        self.np_grids = np.empty((0, 0), dtype=np.uint8)
        self.H = 0
        self.W = 0


def build_grids(mask_img: np.ndarray, rect: tuple[int, int, int, int], H: int, W: int) -> GridState:
    """FrameProcessor._extract_grid_information (FrameProcessor.py:50-171) for ONE
    mask, starting from what cv2 would have produced: the filled mask image
    (``cv2.fillPoly`` result, :85-86) and the bounding rect (:76).

    Raises IndexError exactly where the reference does (Q10)."""
    st = GridState()
    st.H, st.W = H, W
    art_cols = list(range(W // 2 - GRID * 8, W // 2 + GRID * 9, GRID))  # :60-65
    x, y, w, h = (int(v) for v in rect)
    x -= x % GRID  # :79-83
    y -= y % GRID
    w = w + (GRID - w % GRID) if w % GRID != 0 else w
    w = W if w > W else w
    h = h + (GRID - h % GRID) if h % GRID != 0 else h
    # the reference's own structure from here (:85-97): the filled frame-size mask image, numpy coordinate
    # vectors, the centre grid and one numpy lookup per centre (timed as the CPU baseline)
    mask = np.zeros((H, W), dtype=np.uint8)
    mask[:] = mask_img
    j_np = np.arange(x, x + w, GRID)  # :88-89
    i_np = np.arange(y, y + h, GRID)
    half = GRID // 2
    J, I = np.meshgrid(j_np + half, i_np + half)
    centers = np.stack((J, I), axis=-1).reshape(-1, 2)
    in_np = np.array([mask[pt[1], pt[0]] > 0 for pt in centers]).reshape(len(i_np), len(j_np))  # :94-97
    if not np.any(in_np):  # :99-101
        return st
    for r, i in enumerate(i_np):  # :104-124 (numpy coordinates, as the reference iterates them)
        row = []
        for c, j in enumerate(j_np):
            centre = Coordinate(x=(j + half), y=(i + half))
            cell = Cell(coords=Coordinate(x=j, y=i), centre=centre, penalty=None, row=r, col=c,
                        empty=not in_np[r, c], artificial=False)
            row.append(cell)
            st.lookup[(int(j), int(i))] = cell
        st.grids.append(row)
    j_vals = [int(v) for v in j_np]
    start_y = int(H * 0.875)  # :126-127
    start_y = start_y + (GRID - start_y % GRID) % GRID
    for i in range(start_y, H, GRID):  # :130-165
        row_idx = (i - y) // GRID
        row = []
        for c, j in enumerate(j_vals):
            prev = st.lookup.get((j, i))
            previously_empty = prev.empty if prev else True
            is_art_col = j in art_cols
            if previously_empty:
                empty, artificial = (not is_art_col), is_art_col
            else:
                empty, artificial = False, False
            cell = Cell(coords=Coordinate(x=j, y=i), centre=Coordinate(x=j + half, y=i + half),
                        penalty=None, row=row_idx, col=c, empty=empty, artificial=artificial)
            st.lookup[(j, i)] = cell
            row.append(cell)
        if row_idx < len(st.grids) - 1:
            st.grids[row_idx] = row  # python list semantics: negative index / IndexError (Q10)
        else:
            st.grids.append(row)
    st.np_grids = np.array([[0 if c.empty else 1 for c in row] for row in st.grids], dtype=np.uint8)  # :168-171
    return st


# ----------------------------------------------------------------------------- penalties
def _easy_segments(st: GridState):
    """PenaltyCalculator._pre_compute_easy_segments (PenaltyCalculator.py:26-55)."""
    easy_rows, easy_cols = {}, {}
    g = st.np_grids
    for r in range(g.shape[0]):
        idx = np.where(g[r, :] == 1)[0]
        if len(idx) > 0 and idx[-1] - idx[0] == len(idx) - 1:
            easy_rows[r] = (st.grids[r][idx[0]].coords, st.grids[r][idx[-1]].coords)
    for c in range(g.shape[1]):
        idx = np.where(g[:, c] == 1)[0]
        if len(idx) > 0 and idx[-1] - idx[0] == len(idx) - 1:
            easy_cols[c] = (st.grids[idx[0]][c].coords, st.grids[idx[-1]][c].coords)
    return easy_rows, easy_cols


def _segment_penalty(cell: Cell, lookup, easy, direction: str) -> float:
    """PenaltyCalculator._calculate_segment_penalty (PenaltyCalculator.py:57-110)."""
    s = cell.coords
    x, y = s.x, s.y
    key = cell.row if direction == "row" else cell.col  # Q11: attribute, not list index
    if key in easy:
        left, right = easy[key]
    else:  # the walks build a Coordinate per step, as the reference does (:76-97)
        while True:
            nxt = (x - GRID, y) if direction == "row" else (x, y - GRID)
            if nxt not in lookup or lookup[nxt].empty:
                left = Coordinate(x=x, y=y)
                break
            left = Coordinate(x=nxt[0], y=nxt[1])
            x, y = nxt
        x, y = s.x, s.y
        while True:
            nxt = (x + GRID, y) if direction == "row" else (x, y + GRID)
            if nxt not in lookup or lookup[nxt].empty:
                right = Coordinate(x=x, y=y)
                break
            right = Coordinate(x=nxt[0], y=nxt[1])
            x, y = nxt
    den = right.x - left.x if direction == "row" else right.y - left.y
    if den == 0:
        ratio = 0.5
    else:
        ratio = (s.x - left.x) / den if direction == "row" else (s.y - left.y) / den
    return 2 * abs(ratio - 0.5)


def cell_penalty(cell: Cell, lookup, easy_rows, easy_cols):
    """PenaltyCalculator.calculate_penalty (PenaltyCalculator.py:112-142).
    Returns int 0 / int 1 / float exactly like the reference (Q8)."""
    if cell.empty:
        return 0
    rp = _segment_penalty(cell, lookup, easy_rows, "row")
    cp = _segment_penalty(cell, lookup, easy_cols, "col")
    if rp > 0.99 or cp > 0.99:
        return 1
    total = rp + cp
    if total == 0:
        return 0
    dom = abs(rp - cp) / total
    rw = 0.5 + (0.25 * dom if rp > cp else -0.25 * dom)
    cw = 1 - rw
    return (rp * rw) + (cp * cw)


def compute_penalties(st: GridState) -> None:
    """FrameProcessor._calculate_penalties (FrameProcessor.py:173-182)."""
    er, ec = _easy_segments(st)
    for row in st.grids:
        for cell in row:
            if cell.empty:
                continue
            cell.penalty = cell_penalty(cell, st.lookup, er, ec)


# ----------------------------------------------------------------------------- graph
def create_graph(st: GridState):
    """FrameProcessor._create_graph (FrameProcessor.py:184-207)."""
    graph = defaultdict(list)
    for row in st.grids:
        for cell in row:
            if cell.empty:
                continue
            x, y = cell.coords.x, cell.coords.y
            for nx, ny in ((x + GRID, y), (x - GRID, y), (x, y + GRID), (x, y - GRID)):
                if st.lookup.get((nx, ny)):
                    graph[(x, y)].append(((nx, ny), np.sqrt((x - nx) ** 2 + (y - ny) ** 2)))
    return graph


# ----------------------------------------------------------------------------- protrusions
class Peak(BaseModel):  # models.py:38-42
    centre: Coordinate
    left: Coordinate | None = None
    right: Coordinate | None = None
    orientation: str


def _fill_square(binary: np.ndarray, corners: np.ndarray) -> None:
    """cv2.fillPoly(binary, [corners], 255) for the 4 corners of an axis-aligned square (inclusive edges,
    clipped to the image) -- what the reference's per-cell fillPoly produces (:53)."""
    x0, y0 = corners.min(0)
    x1, y1 = corners.max(0)
    binary[max(0, y0):y1 + 1, max(0, x0):x1 + 1] = 255


def protrusion_peaks(st: GridState) -> list[tuple[int, int]]:
    """ProtrusionDetector.__call__ live path (ProtrusionDetector.py:419-439,535) with the reference's structure:
    _create_binary_image (:38-57: per non-empty cell a 4-corner int32 array and a fill of that square, then the
    binary threshold over the frame), _find_peak on the whole frame (:59-158: np.where of the binary image, the
    top-most row's sorted xs split at gaps > grid_size//4, per group its middle x, the vertical slice below it,
    height / width / upward test and orientation, a Peak object), the global peaks' centres returned (:535)."""
    binary = np.zeros((st.H, st.W), dtype=np.uint8)
    for row in st.grids:
        for cell in row:
            if cell.empty:
                continue
            x, y = cell.coords.x, cell.coords.y
            corners = np.array([[x, y], [x + GRID, y], [x + GRID, y + GRID], [x, y + GRID]], np.int32)
            _fill_square(binary, corners)
    binary = np.where(binary > 127, 255, 0).astype(np.uint8)  # cv2.threshold(binary, 127, 255, THRESH_BINARY)
    ys, xs = np.where(binary == 255)
    if not ys.size:
        return []
    min_y = np.min(ys)
    px = np.sort(xs[ys == min_y])
    gaps = np.diff(px)
    groups = np.split(px, np.where(gaps > (GRID // 4))[0] + 1)
    peaks = []
    for g in groups:
        cx = int(g[len(g) // 2])
        sel = (xs >= cx - GRID // 2) & (xs <= cx + GRID // 2)
        vy = ys[sel]
        if len(vy) == 0:
            continue
        height = np.max(vy) - min_y
        width = np.max(xs) - np.min(xs)
        upward = height > width * 0.5 and len(vy) > height * 0.5
        orientation = "up" if upward else "right" if cx > np.mean(xs) else "left"
        peaks.append(Peak(centre=Coordinate(x=cx, y=int(min_y)), left=Coordinate(x=int(g[0]), y=int(min_y)),
                          right=Coordinate(x=int(g[-1]), y=int(min_y)), orientation=orientation))
    return [(p.centre.x, p.centre.y) for p in peaks]


# ----------------------------------------------------------------------------- start / end
def closest_cell(point: tuple[int, int], st: GridState):
    """utils.get_closest_grid_to_point (utils.py:6-32): row-major over
    ``self.grids`` (stale rows included), strict '<' so the first wins (Q12)."""
    best, best_d = None, np.inf
    px, py = point
    for row in st.grids:
        for cell in row:
            if cell.empty:
                continue
            d = np.sqrt((px - cell.centre.x) ** 2 + (py - cell.centre.y) ** 2)
            if d < best_d:
                best_d, best = d, cell
    return best


# ----------------------------------------------------------------------------- A*
class PathFinderOracle:
    """PathFinder (PathFinder.py:7-189) restated with the same data structures;
    ``angle_cache`` is the process-global, never-cleared cache (:32, Q1/Q2)."""

    def __init__(self):
        self.angle_cache: dict = {}

    @staticmethod
    def _h(a: Cell, b: Cell):  # :44-49
        return abs(a.coords.x - b.coords.x) + abs(a.coords.y - b.coords.y)

    def _angle(self, path, seg: int):  # :51-101 (radians cached, degrees appended: Q1)
        if len(path) < seg:
            return 0
        angles = []
        half = seg // 2
        for i in range(half, len(path) - half - 1):
            pp = path[i - half:i + 1]
            nn = path[i + 1:i + half + 1]
            pv = (pp[-1][0] - pp[0][0], pp[-1][1] - pp[0][1])
            nv = (nn[-1][0] - nn[0][0], nn[-1][1] - nn[0][1])
            key = (pv, nv)
            if key in self.angle_cache:
                angles.append(self.angle_cache[key])
                continue
            dot = pv[0] * nv[0] + pv[1] * nv[1]
            mp = (pv[0] ** 2 + pv[1] ** 2) ** 0.5
            mn = (nv[0] ** 2 + nv[1] ** 2) ** 0.5
            if mp == 0 or mn == 0:
                continue
            ang = np.arccos(np.clip(dot / (mp * mn), -1.0, 1.0))
            angles.append(np.degrees(ang))
            self.angle_cache[key] = ang
        return max(angles) if angles else 0

    def find_path(self, graph, start: Cell, end: Cell, lookup):  # :119-186
        open_set: list = []
        closed: set = set()
        came: dict = {}
        g: dict = {}
        f: dict = {}
        s = (start.coords.x, start.coords.y)
        e = (end.coords.x, end.coords.y)
        g[s] = 0
        f[s] = self._h(start, end)
        heapq.heappush(open_set, (f[s], s))
        while open_set:
            cur = heapq.heappop(open_set)[1]
            if cur == e:
                path, cur2 = [], e
                cost = g[cur2]
                while cur2 in came:
                    path.append(lookup[cur2])
                    cur2 = came[cur2]
                path.append(start)
                path.reverse()
                return path, cost
            closed.add(cur)
            for nb, dist in graph[cur]:
                if nb in closed:
                    continue
                nbc = lookup[nb]
                psf = [cur]
                prev = cur
                while prev in came:
                    prev = came[prev]
                    psf.append(prev)
                psf.reverse()
                a = self._angle(psf + [nb], 7)
                ap = 0 if a <= 30 else (a / 90) ** 1.5
                pm = 1 + (0.5 * (nbc.penalty or 0)) + ap * 1.5
                t = g[cur] + (dist * pm)
                if nb not in g or t < g[nb]:
                    came[nb] = cur
                    g[nb] = t
                    f[nb] = t + self._h(nbc, end)
                    if not any(c == nb for _, c in open_set):
                        heapq.heappush(open_set, (f[nb], nb))
        return [], float("inf")


def path_similarity(p1: list, p2: list) -> float:
    """FrameProcessor._calculate_path_similarity (FrameProcessor.py:209-228)."""
    a = {(c.coords.x, c.coords.y) for c in p1}
    b = {(c.coords.x, c.coords.y) for c in p2}
    if not a or not b:
        return 0.0
    inter = len(a & b)
    if inter == len(a) or inter == len(b):
        return 1.0
    union = len(a | b)
    return inter / union if union > 0 else 0.0


def find_paths(st: GridState, peaks, graph, pf: PathFinderOracle):
    """FrameProcessor._find_paths (FrameProcessor.py:230-271) minus the pydantic
    Path construction: returns (queries, unique) where queries is the list of
    (start_cell, end_cell, path_cells, cost, angle-cache keys after the query)
    per peak in order and unique the surviving
    (path_cells, cost) after the Jaccard / subset filter."""
    if not st.grids:
        return [], []
    start = closest_cell((st.W // 2, st.H), st)
    queries, found = [], []
    for pk in peaks:
        end = closest_cell(pk, st)
        path, cost = pf.find_path(graph, start, end, st.lookup)
        queries.append((start, end, path, cost, frozenset(pf.angle_cache)))
        if path:
            found.append((path, cost))
    found.sort(key=lambda pc: len(pc[0]), reverse=True)
    unique = []
    for p in found:
        if all(path_similarity(p[0], u[0]) < 0.90 for u in unique):
            unique.append(p)
    return queries, unique


def frame_nav(mask_img: np.ndarray, rect, H: int, W: int, pf: PathFinderOracle, timings: dict | None = None) -> dict:
    """Grid-level part of FrameProcessor.__call__ (FrameProcessor.py:325-347).  ``timings``: if given,
    per-stage seconds are added to it (grid / penalty / graph / protrusion / astar+paths, the split of
    SURVEY.md §6 S1)."""
    import time
    clk = time.perf_counter
    t = [clk()]

    def lap(name):
        if timings is not None:
            now = clk()
            timings[name] = timings.get(name, 0.0) + now - t[0]
            t[0] = now

    st = build_grids(mask_img, rect, H, W)
    lap("grid")
    if not st.grids:
        return {"state": st, "peaks": [], "queries": [], "paths": []}
    compute_penalties(st)
    lap("penalty")
    graph = create_graph(st)
    lap("graph")
    peaks = protrusion_peaks(st)
    lap("protrusion")
    queries, unique = find_paths(st, peaks, graph, pf)
    lap("astar+paths")
    return {"state": st, "peaks": peaks, "queries": queries, "paths": unique}

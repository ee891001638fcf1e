"""PathFinder: grid A* on the GPU (reference: PathFinder.py).

Same surface as the reference singleton ``path_finder`` (PathFinder.py:7-189):
``find_path(graph, start_grid, end_grid, grid_lookup) -> (list[Grid], total_cost)``
with ``([], inf)`` when the goal is unreachable.  The search runs in
``nav_astar_kernel`` (va_astar_run) over the cell lattice; results are
bit-identical to the reference, including its process-global angle cache
(``angle_cache``, PathFinder.py:32, never cleared), which lives on the device as a
128-bit seen-key set shared with FrameProcessor's batched path.

The graph must be the 4-neighbour cell graph FrameProcessor._create_graph builds
(FrameProcessor.py:184-207: neighbours right, left, down, up that exist in
grid_lookup, distance 20, the list repeated once per duplicate grid object);
anything else raises ValueError -- there is no CPU A* in this package.
"""
from __future__ import annotations

import ctypes
from typing import ClassVar, Optional

import numpy as np
import torch

from . import _lib
from .config import grid_size
from .models import Grid

_STEPS = ((grid_size, 0), (-grid_size, 0), (0, grid_size), (0, -grid_size))


def _key_vectors():
    import itertools
    prevs, nexts = set(), set()
    for a, b, c in itertools.product(_STEPS, repeat=3):
        if (a[0] + b[0], a[1] + b[1]) == (0, 0) or (b[0] + c[0], b[1] + c[1]) == (0, 0):
            continue
        prevs.add((a[0] + b[0] + c[0], a[1] + b[1] + c[1]))
    for a, b in itertools.product(_STEPS, repeat=2):
        if (a[0] + b[0], a[1] + b[1]) != (0, 0):
            nexts.add((a[0] + b[0], a[1] + b[1]))
    return sorted(prevs), sorted(nexts)


_PREVS, _NEXTS = _key_vectors()  # key index = prev * 8 + next (va_angle_table.h enumeration)


class PathFinder:
    _instance: ClassVar[Optional["PathFinder"]] = None
    _initialized: bool = False

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self):
        if not self._initialized:
            self._initialized = True
            self._seen = None  # AngleSeen, created on first use (needs the GPU)
            self._work = None
            self._work_key = None

    # ---------------------------------------------------------------- shared device state
    @property
    def seen(self):
        """The device-resident angle-cache key set (vision_assist_amd.nav.AngleSeen)."""
        if self._seen is None:
            from .nav import AngleSeen
            _lib.require_gpu()
            self._seen = AngleSeen(torch.device("cuda", torch.cuda.current_device()))
        return self._seen

    @property
    def angle_cache(self) -> dict:
        """Read-only view with the reference's contents: {(prev_vec, next_vec): radians}."""
        out = {}
        for k in sorted(self.seen.keys()):
            p, n = _PREVS[k // 8], _NEXTS[k % 8]
            dot = p[0] * n[0] + p[1] * n[1]
            out[(p, n)] = np.arccos(np.clip(dot / ((p[0] ** 2 + p[1] ** 2) ** 0.5 * (n[0] ** 2 + n[1] ** 2) ** 0.5),
                                            -1.0, 1.0))
        return out

    def reset_angle_cache(self) -> None:
        """A fresh process's state (the reference never clears it; tests use this)."""
        self.seen.clear()

    # ---------------------------------------------------------------- find_path
    def find_path(self, graph: dict, start_grid: Grid, end_grid: Grid,
                  grid_lookup: dict[tuple[int, int], Grid]) -> tuple[list[Grid], float]:
        lib = _lib.load()
        coords = list(grid_lookup.keys())
        if not coords:
            raise ValueError("empty grid_lookup")
        xs = [c[0] for c in coords]
        ys = [c[1] for c in coords]
        if any(v % grid_size for v in xs + ys) or min(xs) < 0 or min(ys) < 0:
            raise ValueError("grid_lookup coordinates must be non-negative multiples of grid_size")
        LC, LR = max(xs) // grid_size + 1, max(ys) // grid_size + 1
        flags = np.zeros((LR, LC), dtype=np.uint8)
        pen = np.zeros((LR, LC), dtype=np.float64)
        for (x, y), g in grid_lookup.items():
            flags[y // grid_size, x // grid_size] = 1  # VA_NODE_EXISTS
            pen[y // grid_size, x // grid_size] = g.penalty or 0
        for (x, y), nbrs in graph.items():
            canon = [((x + dx, y + dy), float(grid_size)) for dx, dy in _STEPS if (x + dx, y + dy) in grid_lookup]
            m = len(nbrs) // len(canon) if canon else 0
            if not canon or m * len(canon) != len(nbrs) or m > 3 or \
                    [(tuple(n), float(d)) for n, d in nbrs] != canon * m:
                if nbrs:
                    raise ValueError(f"graph[{(x, y)}] is not the 4-neighbour grid graph of FrameProcessor._create_graph")
            flags[y // grid_size, x // grid_size] |= (m & 3) << 3
        s = (start_grid.coords.y // grid_size) * LC + start_grid.coords.x // grid_size
        e = (end_grid.coords.y // grid_size) * LC + end_grid.coords.x // grid_size
        dev = self.seen.t.device
        fl_t = torch.from_numpy(flags.reshape(-1)).to(dev)
        pen_t = torch.from_numpy(pen.reshape(-1)).to(dev)
        se = torch.tensor([s, e], dtype=torch.int32, device=dev)
        nbytes = int(lib.va_astar_workspace_bytes(1, LR * LC))
        if self._work is None or self._work.numel() < nbytes:
            self._work = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        rounds = ctypes.c_int32(0)
        _lib.check(lib.va_astar_run(_lib.stream_ptr(), fl_t.data_ptr(), pen_t.data_ptr(), LR, LC,
                                    se[0:1].data_ptr(), se[1:2].data_ptr(), 1, self.seen.t.data_ptr(),
                                    self._work.data_ptr(), ctypes.byref(rounds)), "va_astar_run")
        qbytes = int(lib.va_nav_query_bytes(LR * LC))
        rec = self._work[:qbytes].cpu().numpy()
        status, length = (int(v) for v in rec[:8].view("<i4"))
        if status != 1:  # VA_QUERY_FOUND
            return [], float("inf")
        cost = float(rec[8:16].view("<f8")[0])
        off = 64  # align16(sizeof(va_query_hdr))
        nodes = rec[off:off + 2 * length].view("<u2")
        path = [start_grid]
        for v in nodes[1:]:
            path.append(grid_lookup[(int(v % LC) * grid_size, int(v // LC) * grid_size)])
        return path, (0 if length == 1 else cost)


path_finder = PathFinder()

"""FrameProcessor: the per-frame hot path with the reference's class surface (FrameProcessor.py).

    from vision_assist_amd.yolo import YOLO
    from vision_assist_amd.FrameProcessor import FrameProcessor
    model = YOLO("yolov8s-seg.pt").to("cuda")                      # main.py:43
    processor = FrameProcessor(model=model, verbose=False, debug=False)  # main.py:44 (imshow defaults to False)
    instructions = processor(frame)                                   # main.py:82

``__call__`` (FrameProcessor.py:301-360) runs segmentation, post-processing,
grid build, penalties, protrusions, start/end selection and A* as one device
pipeline (vision_assist_amd.pipeline), copies one frame record back and hands
the unique paths to PathAnalyser.  Same return values: the answer string, ``[]``
when no grid was built (:328-332), ``(frame, answer)`` in debug mode (the frame drawn as the reference draws it:
penalty-coloured grids, then the paths -- vision_assist_amd.PathVisualiser).  The
reference's IndexError on masks confined to the last rows is
raised the same way.

The step-by-step methods harness scripts call (``_extract_grid_information``,
``_calculate_penalties``, ``_create_graph``, ``_find_paths``;
utilities/generate_testing_grids/run_on_main.py:181-193) work too; ``grids``,
``grid_lookup`` and ``np_grids`` are materialised as pydantic objects only when
read (building ~1 K Grid objects per frame would cost more than the whole GPU
pipeline, SURVEY.md §7 hard part 4).
"""
from __future__ import annotations

from collections import defaultdict
from typing import ClassVar, Optional

import numpy as np
import torch

from . import _lib
from .config import grid_size
from .models import Coordinate, Grid, Path
from .PathAnalyser import path_analyser
from .PathFinder import path_finder
from .PathVisualiser import fill_square, path_visualiser
from .PenaltyCalculator import penalty_calculator
from .ProtrusionDetector import ProtrusionDetector
from .utils import get_closest_grid_to_point

G = grid_size


def _pen_value(flags: int, pen: float):
    """Device float64 penalty -> the python value the reference stores: None / int 0 / int 1 / float."""
    if flags & _lib.VA_CELL_EMPTY:
        return None
    if pen == 0.0:
        return 0
    if pen == 1.0:
        return 1
    return float(pen)


class _FrameState:
    """Lazy pydantic view of one device frame record (vision_assist_amd.nav.NavFrame)."""

    def __init__(self, nf, dims):
        self.nf = nf
        self.dims = dims
        self._objs: dict[tuple[int, int], Grid] = {}
        self._grids = None
        self._lookup = None
        self._np = None
        self._pos = None  # object id -> list position (nf.pos_obj is fixed for the frame)
        self.penalties_assigned = False

    # object id: main row r -> r, artificial row a -> LR + a (va_nav.hip nav_grid_kernel)
    def _obj_y(self, o: int) -> int:
        nf, d = self.nf, self.dims
        return nf.y0 + G * o if o < d.LR else d.start_y + G * (o - d.LR)

    def _obj_attr(self, o: int) -> int:
        return o if o < self.dims.LR else (self._obj_y(o) - self.nf.y0) // G

    def _pos_of_obj(self) -> dict[int, int]:
        if self._pos is None:
            self._pos = {int(o): p for p, o in enumerate(self.nf.pos_obj)}
        return self._pos

    def obj(self, o: int, c: int, flags: int | None = None) -> Grid:
        key = (o, c)
        g = self._objs.get(key)
        if g is None:
            nf = self.nf
            x, y = nf.x0 + G * c, self._obj_y(o)
            if flags is None:
                p = self._pos_of_obj()[o]
                flags = int(nf.cell_flags[p, c])
            g = Grid(coords=Coordinate(x=x, y=y), centre=Coordinate(x=x + G // 2, y=y + G // 2), penalty=None,
                     row=self._obj_attr(o), col=c, empty=bool(flags & _lib.VA_CELL_EMPTY),
                     artificial=bool(flags & _lib.VA_CELL_ARTIFICIAL))
            self._objs[key] = g
            if self.penalties_assigned and not g.empty:
                p = self._pos_of_obj().get(o)
                if p is not None:
                    g.penalty = _pen_value(flags, float(nf.cell_pen[p, c]))
        return g

    def lookup_obj(self, x: int, y: int) -> Grid | None:
        nf, d = self.nf, self.dims
        yi, xi = y // G, x // G
        if not (0 <= yi < d.LR and 0 <= xi < d.LC):
            return None
        fl = int(nf.node_flags[yi, xi])
        if not fl & _lib.VA_NODE_EXISTS:
            return None
        c = xi - nf.x0 // G
        ay = d.start_y // G
        o = d.LR + (yi - ay) if 0 <= yi - ay < d.NART else yi - nf.y0 // G
        cell_flags = (0 if fl & _lib.VA_NODE_NONEMPTY else _lib.VA_CELL_EMPTY) | \
                     (_lib.VA_CELL_ARTIFICIAL if fl & _lib.VA_NODE_ARTIFICIAL else 0)
        return self.obj(o, c, cell_flags)

    @property
    def grids(self) -> list[list[Grid]]:
        if self._grids is None:
            nf = self.nf
            self._grids = [[self.obj(int(o), c, int(nf.cell_flags[p, c])) for c in range(nf.C)]
                           for p, o in enumerate(nf.pos_obj)]
        return self._grids

    @property
    def grid_lookup(self) -> dict:
        if self._lookup is None:
            nf, d = self.nf, self.dims
            out = {}
            # insertion order of the reference: main rows first, artificial rows override in place / append
            ys = [nf.y0 + G * r for r in range(nf.Rm)] + [d.start_y + G * a for a in range(d.NART)]
            for y in ys:
                for c in range(nf.C):
                    x = nf.x0 + G * c
                    if (x, y) not in out:
                        out[(x, y)] = None
            for (x, y) in out:
                out[(x, y)] = self.lookup_obj(x, y)
            self._lookup = out
        return self._lookup

    @property
    def np_grids(self) -> np.ndarray:
        if self._np is None:
            self._np = (~self.nf.cell_flags & _lib.VA_CELL_EMPTY).astype(np.uint8) & 1
        return self._np

    def assign_penalties(self) -> None:
        """FrameProcessor._calculate_penalties: the device values onto every non-empty Grid."""
        nf = self.nf
        self.penalties_assigned = True
        table = penalty_calculator._table
        table.clear()
        for p, o in enumerate(nf.pos_obj):
            for c in range(nf.C):
                fl = int(nf.cell_flags[p, c])
                if fl & _lib.VA_CELL_EMPTY:
                    continue
                g = self.obj(int(o), c, fl)
                g.penalty = _pen_value(fl, float(nf.cell_pen[p, c]))
                table[id(g)] = g.penalty

    def graph(self):
        """FrameProcessor._create_graph from the device lattice (neighbours right, left, down, up)."""
        nf = self.nf
        graph = _DeviceGraph(list)
        graph._state = self
        for p, o in enumerate(nf.pos_obj):
            y = self._obj_y(int(o))
            for c in range(nf.C):
                if nf.cell_flags[p, c] & _lib.VA_CELL_EMPTY:
                    continue
                x = nf.x0 + G * c
                for nx, ny in ((x + G, y), (x - G, y), (x, y + G), (x, y - G)):
                    if self.lookup_obj(nx, ny) is not None:
                        graph[(x, y)].append(((nx, ny), np.float64(20.0)))
        return graph

    def peaks(self) -> list[Coordinate]:
        return [Coordinate(x=x, y=y) for x, y in self.nf.peaks]

    def device_paths(self) -> list[Path]:
        """The unique paths of the device run, in FrameProcessor._find_paths order."""
        nf = self.nf
        sp, sc = nf.start
        start = self.obj(int(nf.pos_obj[sp]), sc, int(nf.cell_flags[sp, sc]))
        kept = sorted((q for q in nf.queries if q["unique"]), key=lambda q: q["order"])
        out = []
        for q in kept:
            cells = [start] + [self.lookup_obj(x, y) for x, y in q["path"][1:]]
            cost = 0 if len(q["path"]) == 1 else q["cost"]
            out.append(Path(grids=cells, total_cost=cost, path_type="path"))
        return out


def _same_grid(a: Grid | None, b: Grid | None) -> bool:
    if a is None or b is None:
        return a is b
    return (a.coords.x, a.coords.y, a.centre.x, a.centre.y, a.row, a.col, a.empty, a.artificial) == \
        (b.coords.x, b.coords.y, b.centre.x, b.centre.y, b.row, b.col, b.empty, b.artificial)


def implied_grid_inputs(grids: list, grid_lookup: dict, H: int, W: int):
    """What the reference's grid builder (FrameProcessor.py:50-171) must have been given to make ``grids`` /
    ``grid_lookup`` in an H x W frame: the rect rounded to the 20-px lattice and the mask samples at the cell centres.
    The rect's origin comes from any grid (x - 20 col, y - 20 row: both the main and the artificial rows set row =
    (y - rect y) / 20), its width from the columns; a main-row cell was in the mask iff its FINAL grid in the lookup
    is non-empty and not artificial (an artificial row keeps a non-empty cell non-empty and marks a formerly empty
    one artificial, :138-151).  The rect's height is ambiguous where the main rows run under the artificial ones:
    -> (x0, y0, w, [(h, cells uint8 [H/20, W/20]) for every candidate height, shortest first])."""
    rows = [r for r in grids if r]
    if not rows or not grid_lookup:
        raise ValueError("no grids")
    g0 = rows[0][0]
    x0, y0 = g0.coords.x - G * g0.col, g0.coords.y - G * g0.row
    xs = sorted({x for x, _ in grid_lookup})
    ys = sorted({y for _, y in grid_lookup})
    w = xs[-1] - x0 + G
    if H % G or W % G or x0 % G or y0 % G or x0 < 0 or y0 < 0 or w <= 0:
        raise ValueError("grids not on the 20-px lattice of an H x W frame")
    LR, LC = H // G, W // G
    out = []
    for h in range(G, ys[-1] - y0 + 2 * G, G):
        cells = np.zeros((LR, LC), dtype=np.uint8)
        for r in range(h // G):
            for c in range(w // G):
                x, y = x0 + G * c, y0 + G * r
                g = grid_lookup.get((x, y))
                if g is not None and not g.empty and not g.artificial and y // G < LR and x // G < LC:
                    cells[y // G, x // G] = 1
        if cells.any():
            out.append((h, cells))
    return x0, y0, w, out


def device_frame_for(grids: list, grid_lookup: dict, H: int, W: int) -> "_FrameState":
    """The device grid stage for a grid list built outside this package's FrameProcessor (the standalone
    PenaltyCalculator / ProtrusionDetector surfaces, PenaltyCalculator.py:112-142, ProtrusionDetector.py:419-535).

    The reference's penalties and peaks depend only on what its grid builder was given (the frame size, the rounded
    rect and the mask samples; implied_grid_inputs reads them back from the grids), so the device stage
    (va_nav_run) run on those gives the reference's values.  Of the candidate rect heights the one whose device grid
    list and lookup equal the caller's in every Grid field, in order, is taken; any other list (not one the
    reference's builder makes of some mask) raises ValueError.  A* runs against a scratch copy of the angle cache
    (the process cache is left as it was)."""
    from .nav import AngleSeen, NavEngine
    x0, y0, w, cands = implied_grid_inputs(grids, grid_lookup, H, W)
    LR, LC = H // G, W // G
    dev = torch.device("cuda", torch.cuda.current_device())
    navs = device_frame_for.__dict__.setdefault("_navs", {})
    if (H, W) not in navs:
        navs[(H, W)] = NavEngine(H, W, max_batch=1)
    nav = navs[(H, W)]
    for h, cells in cands:
        scratch = AngleSeen(dev)
        scratch.t.copy_(path_finder.seen.t)
        res = nav.run(torch.from_numpy(cells).to(dev).reshape(1, LR, LC).contiguous(),
                      torch.tensor([[x0, y0, w, h]], dtype=torch.int32, device=dev), scratch, readback=True)
        nf = res.frame(0)
        if nf.status != _lib.VA_FRAME_OK:
            continue
        st = _FrameState(nf, nav.dims)
        st.penalties_assigned = True
        dg, dl = st.grids, st.grid_lookup
        if len(dg) == len(grids) and all(len(a) == len(b) and all(_same_grid(u, v) for u, v in zip(a, b))
                                         for a, b in zip(dg, grids)) and \
                list(dl) == list(grid_lookup) and all(_same_grid(dl[k], grid_lookup[k]) for k in dl):
            return st
    raise ValueError(f"these grids are not what the reference's grid builder makes of any mask in a {H} x {W} frame "
                     f"(rect origin ({x0}, {y0}), width {w}, heights tried {[h for h, _ in cands]})")


class _DeviceGraph(defaultdict):
    """The graph dict of _create_graph, tagged with the frame it was built from."""
    _state = None


class FrameProcessor:
    _instance: ClassVar[Optional["FrameProcessor"]] = None
    _initialized: bool = False

    def __new__(cls, model=None, verbose: bool = False, debug: bool = False, imshow: bool = False):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self, model=None, verbose: bool = False, debug: bool = False, imshow: bool = False):
        if not self._initialized:
            self._initialized = True
            self.model = model
            self.verbose = verbose
            self.debug = debug
            self.imshow = imshow
            self.frame = None
            self._state: _FrameState | None = None
            self._pending_seen = None  # angle-cache state after the device run, committed by _find_paths
            self.protrusion_detector = ProtrusionDetector(debug=debug, imshow=imshow)

    # ---------------------------------------------------------------- lazy reference attributes
    @property
    def grids(self) -> list[list[Grid]]:
        return self._state.grids if self._state is not None else []

    @property
    def grid_lookup(self) -> dict:
        return self._state.grid_lookup if self._state is not None else {}

    @property
    def np_grids(self) -> np.ndarray:
        return self._state.np_grids if self._state is not None else np.empty((0, 0), dtype=np.uint8)

    def _has_grids(self) -> bool:
        return self._state is not None and self._state.nf.status == _lib.VA_FRAME_OK

    # ---------------------------------------------------------------- device run
    def _pipe(self, H: int, W: int):
        if self.model is None or not hasattr(self.model, "pipeline"):
            raise TypeError("FrameProcessor needs a vision_assist_amd.yolo.YOLO model (the device pipeline)")
        return self.model.pipeline(H, W, seen=path_finder.seen)

    def _nav(self, H: int, W: int):
        """Grid-stage engine alone (the step-by-step methods start from a mask, not a frame)."""
        from .nav import NavEngine
        cache = self.__dict__.setdefault("_navs", {})
        if (H, W) not in cache:
            cache[(H, W)] = NavEngine(H, W, max_batch=1)
        return cache[(H, W)]

    def _adopt(self, nav, batch, seen_after=None):
        self._adopt_frame(nav.dims, batch.frame(0), seen_after)

    def _adopt_frame(self, dims, nf, seen_after=None):
        self._state = _FrameState(nf, dims)
        self._pending_seen = seen_after
        if nf.status == _lib.VA_FRAME_INDEX_ERROR:
            self._state = None
            raise IndexError("list assignment index out of range")  # FrameProcessor.py:163

    def _run_nav(self, nav, cells: torch.Tensor, rect, commit: bool):
        """Grid stage for one frame.  commit=False runs A* against a scratch copy of the angle cache
        (the step-by-step harness commits it in _find_paths, where the reference runs A*)."""
        from .nav import AngleSeen
        rects = torch.tensor([list(rect)], dtype=torch.int32, device=cells.device)
        if commit:
            return nav.run(cells.reshape(1, *cells.shape[-2:]).contiguous(), rects, path_finder.seen), None
        scratch = AngleSeen(cells.device)
        scratch.t.copy_(path_finder.seen.t)
        return nav.run(cells.reshape(1, *cells.shape[-2:]).contiguous(), rects, scratch), scratch

    # ---------------------------------------------------------------- reference methods
    def _extract_grid_information(self, results) -> None:
        """FrameProcessor.py:50-171 on the device, from YOLO.predict results (or any object with
        ``.masks.cells`` / ``.masks.rect``: the filled mask sampled at the cell centres + boundingRect)."""
        self._state = None
        self._pending_seen = None
        if self.frame is None:
            raise ValueError("set self.frame first (FrameProcessor.__call__ does)")
        H, W = self.frame.shape[0], self.frame.shape[1]
        for res in results:
            if res.masks is None:
                continue
            nav = self._nav(H, W)
            batch, scratch = self._run_nav(nav, res.masks.cells, res.masks.rect, commit=False)
            self._adopt(nav, batch, scratch)
            if not self._has_grids():
                self._state = None
            return

    def _calculate_penalties(self) -> None:
        if self._has_grids():
            self._state.assign_penalties()

    def _create_graph(self) -> defaultdict:
        return self._state.graph() if self._has_grids() else defaultdict(list)

    def _calculate_path_similarity(self, path1: Path, path2: Path) -> float:
        a = {(g.coords.x, g.coords.y) for g in path1.grids}
        b = {(g.coords.x, g.coords.y) for g in path2.grids}
        if not a or not b:
            return 0.0
        inter = len(a & b)
        if inter == len(a) or inter == len(b):
            return 1.0
        union = len(a | b)
        return inter / union if union > 0 else 0.0

    def _find_paths(self, protrusion_peaks: list[Coordinate], graph) -> list[Path]:
        """FrameProcessor.py:230-271.  For this frame's own peaks and graph the device A* results
        (already computed, bit-identical) are used; anything else runs path_finder.find_path."""
        if not self._has_grids():
            return []
        st = self._state
        if isinstance(graph, _DeviceGraph) and graph._state is st and \
                [(p.x, p.y) for p in protrusion_peaks] == [tuple(p) for p in st.nf.peaks]:
            if self._pending_seen is not None:
                path_finder.seen.t.copy_(self._pending_seen.t)
                self._pending_seen = None
            for q in st.nf.queries:
                if q["status"] != _lib.VA_QUERY_FOUND:
                    print("No path found.")
            return st.device_paths()
        self._pending_seen = None
        H, W = self.frame.shape[0], self.frame.shape[1]
        start = get_closest_grid_to_point(Coordinate(x=W // 2, y=H), self.grids)
        found = []
        for peak in protrusion_peaks:
            end = get_closest_grid_to_point(peak, self.grids)
            cells, cost = path_finder.find_path(graph, start, end, self.grid_lookup)
            if cells:
                found.append(Path(grids=cells, total_cost=cost, path_type="path"))
            else:
                print("No path found.")
        found.sort(key=lambda p: len(p.grids), reverse=True)
        unique: list[Path] = []
        for p in found:
            if all(self._calculate_path_similarity(p, u) < 0.90 for u in unique):
                unique.append(p)
        return unique

    # ---------------------------------------------------------------- the hot path
    def __call__(self, frame) -> tuple[np.ndarray, str] | str:
        """FrameProcessor.py:301-360 as one device pipeline per frame."""
        self.frame = frame
        t = torch.as_tensor(frame) if not isinstance(frame, torch.Tensor) else frame
        H, W = int(t.shape[0]), int(t.shape[1])
        pipe = self._pipe(H, W)
        from .post import PLANT_NEVER
        batch = pipe.run(t.reshape(1, H, W, 3), plant_mode=PLANT_NEVER)
        return self._answer(pipe.nav.dims, batch.frame(0), H, W)

    def _answer(self, dims, nf, H: int, W: int):
        """FrameProcessor.py:325-360 for one frame's device record: adopt it, then paths and the answer."""
        self._adopt_frame(dims, nf)
        if not self._has_grids():
            self._state = None
            return (self.frame, []) if self.debug else []
        st = self._state
        st.penalties_assigned = True
        if not st.nf.peaks:
            print("No protrusions detected.")
        for q in st.nf.queries:
            if q["status"] != _lib.VA_QUERY_FOUND:
                print("No path found.")
        paths = st.device_paths()
        self.protrusion_detector.frames_processed += 1
        final_answer = path_analyser(H, W, paths)
        if self.debug:
            if isinstance(self.frame, torch.Tensor):
                self.frame = self.frame.cpu().numpy()
            self._draw_non_path_grids()
            self.frame = path_visualiser(self.frame, paths)
            return self.frame, final_answer
        return final_answer

    # ------- debug drawing (FrameProcessor.py:273-299; PathVisualiser.py) -------
    def _draw_grid(self, grid, color) -> None:
        fill_square(self.frame, grid.coords.x, grid.coords.y, color)

    def _draw_non_path_grids(self) -> None:
        """Every non-empty grid of self.grids in its penalty colour (the reference's path-grid set is empty)."""
        for grid_row in self.grids:
            for grid in grid_row:
                if grid.empty:
                    continue
                self._draw_grid(grid, penalty_calculator.get_penalty_colour(grid.penalty or 0))

    process = __call__  # the name BASELINE.json's north_star uses

    # ------- a frame stream in device batches (the FrameDealer worker's form) -------
    def _begin_batch(self, frames, max_batch: int):
        """Enqueue up to max_batch host frames (uint8 [H, W, 3] each, one size) as one device batch
        (YOLO.stream_batches: two batches in flight); the frames are copied out before this returns."""
        if self.debug:
            raise ValueError("debug frames are drawn per call: use __call__")
        if self.model is None or not hasattr(self.model, "stream_batches"):
            raise TypeError("FrameProcessor needs a vision_assist_amd.yolo.YOLO model (the device pipeline)")
        H, W = int(frames[0].shape[0]), int(frames[0].shape[1])
        sb = self.model.stream_batches(H, W, max_batch, seen=path_finder.seen)
        # the token keeps the batch's size, not the frames: they are views of ring slots that the dealer reuses as
        # soon as begin returns, so a later read of their pixels would see another frame's
        return sb, sb.begin(frames), len(frames), H, W

    def _end_batch(self, token) -> list:
        """The answers of a begun batch, frame by frame in stream order -- __call__'s on each frame (the grid
        stage ran the frames in order against the one angle cache); an IndexError object in the place of a frame
        whose __call__ would raise it."""
        sb, tok, n, H, W = token
        res = sb.end(tok)
        dims = sb.pipes[0].nav.dims
        out = []
        # debug drawing is per call (_begin_batch refuses debug), so no pixels are read here; self.frame keeps only
        # the frame's shape for the reference methods that read it (a zero-stride read-only array, no memory)
        blank = np.broadcast_to(np.zeros((), np.uint8), (H, W, 3))
        for i in range(n):
            self.frame = blank
            try:
                out.append(self._answer(dims, res.frame(i), H, W))
            except IndexError as e:
                out.append(e)
        return out

    # ------- multi-GPU stream -------
    def map(self, frames, devices=None, slots: int | None = None, batch: int = 16, workers_per_gpu: int = 2,
            readers: int = 0):
        """Answers of a frame stream in frame order, the frames dealt round-robin to worker processes on the GPUs
        (vision_assist_amd.shard.FrameDealer): frame i goes to worker i % G on devices[i % G], each worker running
        this model in its own FrameProcessor with its own PathFinder angle cache -- per shard the answers of
        __call__ over that shard's frames in order.  devices: one GPU index per worker (default: every visible GPU,
        ``workers_per_gpu`` workers on each -- two keep a GPU busy while the other builds its answers on the host:
        3,858-4,031 frames/s per GPU against 2,670 with one); batch: frames a worker runs as one
        device batch (up to; what is waiting in its ring of ``slots`` frames, default 4 x batch: the ring lives in
        /dev/shm, G x slots frames, and the dealer refuses a ring larger than the free space there; the bench's 128
        slots measured 1-3 % above 64).  readers: reader threads that copy frames into the rings (FrameDealer; 0 = the
        calling thread, whose copies cap a node near one GPU's rate; with readers a frame must stay unmodified until its
        answer is back).  The first frame fixes the
        frame size; the dealer is kept for later calls with the same devices, size and model settings (close_map
        ends it); a consumer that stops early leaves nothing behind for the next call (FrameDealer.map), and a
        dealer whose worker died is dropped."""
        from .shard import FrameDealer, dropin_worker
        it = iter(frames)
        try:
            first = next(it)
        except StopIteration:
            return
        H, W = int(first.shape[0]), int(first.shape[1])
        if devices is None:
            devices = [g for _ in range(workers_per_gpu) for g in range(torch.cuda.device_count())]
        devices = list(devices)
        if not hasattr(self.model, "spec"):
            raise TypeError("FrameProcessor.map needs a vision_assist_amd.yolo.YOLO model")
        calib = getattr(self.model, "fp8_calib", None)  # set after construction: travels with the worker spec
        if slots is None:
            slots = 4 * batch
        key = (tuple(devices), H, W, slots, batch, readers, id(calib))
        dealers = self.__dict__.setdefault("_dealers", {})
        if key not in dealers:
            model, kw = self.model.spec
            dealers[key] = FrameDealer(dropin_worker(model, batch=batch, fp8_calib=calib, **kw), devices, H, W,
                                       slots=slots, readers=readers)
        d = dealers[key]

        def chain():
            yield first
            yield from it

        try:
            yield from d.map(chain())
        finally:
            if d.broken:
                dealers.pop(key, None)
                d.close()

    def close_map(self) -> None:
        for d in self.__dict__.pop("_dealers", {}).values():
            d.close()

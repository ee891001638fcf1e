"""Host driver of the grid-level hot path (libva355.so ``va_nav_*``).

``NavEngine`` owns the device workspace for one frame size and batch capacity
and runs, for B frames at once, everything FrameProcessor.__call__ does after
the mask is known (FrameProcessor.py:325-347): grid build, penalties, graph,
protrusion peaks, start/end selection, A* (bit-exact, including the
process-global angle cache) and the path de-duplication.

``NavBatch.frame(i)`` decodes one frame's device record (after a single D2H
copy of the batch) into plain python values the FrameProcessor surface turns
into pydantic objects lazily.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .config import grid_size

GRID = grid_size

FRAME_HDR = np.dtype([(n, "<i4") for n in ("status", "x0", "y0", "C", "Rm", "P", "npeaks", "start_p", "start_c",
                                          "min_y", "rounds", "p0", "p1", "p2", "p3", "p4")])
QUERY_HDR = np.dtype([("status", "<i4"), ("len", "<i4"), ("cost", "<f8"), ("miss", "<u8", (2,)),
                      ("frame", "<i4"), ("k", "<i4"), ("expansions", "<i4"), ("unique", "<i4"),
                      ("order", "<i4"), ("pad", "<i4")])
assert FRAME_HDR.itemsize == 64 and QUERY_HDR.itemsize == 56


class AngleSeen:
    """The PathFinder angle-cache key set (PathFinder.py:32) as 128 bits on the
    device.  Owned by the PathFinder singleton; one per process (per GPU)."""

    def __init__(self, device):
        self.t = torch.zeros(2, dtype=torch.int64, device=device)

    def keys(self) -> set[int]:
        w = self.t.cpu().numpy().view(np.uint64)
        return {k for k in range(128) if (int(w[k >> 6]) >> (k & 63)) & 1}

    def clear(self) -> None:
        self.t.zero_()


@dataclass
class NavFrame:
    """Decoded per-frame result (one entry of a NavBatch)."""
    status: int
    H: int
    W: int
    x0: int = 0
    y0: int = 0
    C: int = 0
    Rm: int = 0
    P: int = 0
    pos_y: np.ndarray | None = None      # [P] pixel y of each list position
    pos_attr: np.ndarray | None = None   # [P] Grid.row attribute
    pos_obj: np.ndarray | None = None    # [P] object id
    cell_flags: np.ndarray | None = None  # [P, C] uint8
    cell_pen: np.ndarray | None = None   # [P, C] float64
    node_flags: np.ndarray | None = None  # [LR, LC]
    node_pen: np.ndarray | None = None
    peaks: list = field(default_factory=list)
    start: tuple | None = None           # (p, c)
    ends: list = field(default_factory=list)  # [(p, c)] per peak
    queries: list = field(default_factory=list)  # dicts: status, path [(x,y)], cost, miss, unique, order


class NavBatch:
    """The records of one va_nav_run.  They are copied to pinned host memory on the stream the run was
    enqueued on, right behind it (so a later run on the same engine cannot overwrite them first and the host
    never reads them before the last kernel of the run has finished); ``host()`` waits for that copy."""

    def __init__(self, engine: "NavEngine", B: int, rounds: int, queries_off: int, stream=None,
                 records: torch.Tensor | None = None):
        """records: the run's records already on the host (pinned uint8, va_nav_run_rb / va_frame_rb filled them
        before returning): read in place, no copy and no wait."""
        self.engine = engine
        self.B = B
        self.rounds = rounds
        self.queries_off = queries_off
        e = engine
        nq = B * e.dims.MAXPK * e.dims.query_bytes
        if records is not None:
            r = records.numpy()
            self._pinned = (records,)
            self._host = (r[: B * e.dims.frame_bytes], r[queries_off: queries_off + nq])
            return
        st = stream if stream is not None else torch.cuda.current_stream(e.device)
        fr = torch.empty(B * e.dims.frame_bytes, dtype=torch.uint8, pin_memory=True)
        qs = torch.empty(nq, dtype=torch.uint8, pin_memory=True)
        with torch.cuda.stream(st):
            # frames then queries: two contiguous ranges of the workspace
            fr.copy_(e.work[: B * e.dims.frame_bytes], non_blocking=True)
            qs.copy_(e.work[queries_off: queries_off + nq], non_blocking=True)
            self._done = torch.cuda.Event()
            self._done.record(st)
        self._pinned = (fr, qs)
        self._host = None

    def host(self) -> np.ndarray:
        if self._host is None:
            self._done.synchronize()
            self._host = (self._pinned[0].numpy(), self._pinned[1].numpy())
        return self._host

    def frame(self, i: int) -> NavFrame:
        d = self.engine.dims
        fr_all, qs_all = self.host()
        rec = fr_all[i * d.frame_bytes:(i + 1) * d.frame_bytes]
        hdr = rec[d.off_hdr:d.off_hdr + 64].view(FRAME_HDR)[0]
        out = NavFrame(status=int(hdr["status"]), H=d.H, W=d.W, x0=int(hdr["x0"]), y0=int(hdr["y0"]),
                       C=int(hdr["C"]), Rm=int(hdr["Rm"]), P=int(hdr["P"]))
        if out.status != _lib.VA_FRAME_OK:
            return out
        P, C, LC = out.P, out.C, d.LC
        out.pos_obj = rec[d.off_pos_obj:d.off_pos_obj + 2 * d.PMAX].view("<i2")[:P].astype(np.int64)
        out.pos_y = GRID * rec[d.off_pos_y:d.off_pos_y + 2 * d.PMAX].view("<i2")[:P].astype(np.int64)
        out.pos_attr = rec[d.off_pos_attr:d.off_pos_attr + 2 * d.PMAX].view("<i2")[:P].astype(np.int64)
        out.cell_flags = rec[d.off_cell_flags:d.off_cell_flags + d.PMAX * LC].reshape(d.PMAX, LC)[:P, :C].copy()
        out.cell_pen = rec[d.off_cell_pen:d.off_cell_pen + 8 * d.PMAX * LC].view("<f8").reshape(d.PMAX, LC)[:P, :C].copy()
        out.node_flags = rec[d.off_node_flags:d.off_node_flags + d.NODES].reshape(d.LR, LC).copy()
        out.node_pen = rec[d.off_node_pen:d.off_node_pen + 8 * d.NODES].view("<f8").reshape(d.LR, LC).copy()
        pk = rec[d.off_peaks:d.off_peaks + 16 * d.MAXPK].view("<i4").reshape(4, d.MAXPK)
        npk = int(hdr["npeaks"])
        out.peaks = [(int(pk[0, k]), int(pk[1, k])) for k in range(npk)]
        out.ends = [(int(pk[2, k]), int(pk[3, k])) for k in range(npk)]
        out.start = (int(hdr["start_p"]), int(hdr["start_c"]))
        for k in range(npk):
            off = (i * d.MAXPK + k) * d.query_bytes
            qrec = qs_all[off:off + d.query_bytes]
            qh = qrec[:56].view(QUERY_HDR)[0]
            n = int(qh["len"])
            nodes = qrec[d.off_q_path:d.off_q_path + 2 * n].view("<u2").astype(np.int64)
            out.queries.append({
                "status": int(qh["status"]),
                "path": [(int(GRID * (v % LC)), int(GRID * (v // LC))) for v in nodes],
                "cost": float(qh["cost"]),
                "miss": (int(qh["miss"][0]), int(qh["miss"][1])),
                "unique": int(qh["unique"]),
                "order": int(qh["order"]),
                "expansions": int(qh["expansions"]),
            })
        return out


class NavEngine:
    """Device workspace + launcher for B frames of one size."""

    def __init__(self, H: int, W: int, max_batch: int = 1, device=None):
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.dims = _lib.nav_dims(H, W)
        self.max_batch = max_batch
        nbytes = int(self.lib.va_nav_workspace_bytes(max_batch, H, W))
        if nbytes <= 0:
            raise _lib.VaError(f"va_nav_workspace_bytes({max_batch}, {H}, {W}) = {nbytes}")
        self.work = torch.empty(nbytes, dtype=torch.uint8, device=self.device)

    @property
    def LR(self):
        return self.dims.LR

    @property
    def LC(self):
        return self.dims.LC

    def check_inputs(self, cells: torch.Tensor, rects: torch.Tensor) -> int:
        """Validates cells uint8 [B, H/20, W/20] / rects int32 [B, 4]; -> B."""
        B = cells.shape[0]
        d = self.dims
        if B > self.max_batch:
            raise _lib.VaError(f"batch {B} > engine capacity {self.max_batch}")
        if tuple(cells.shape[1:]) != (d.LR, d.LC) or cells.dtype != torch.uint8 or not cells.is_contiguous():
            raise _lib.VaError(f"cells must be contiguous uint8 [B, {d.LR}, {d.LC}], got {tuple(cells.shape)}")
        if tuple(rects.shape) != (B, 4) or rects.dtype != torch.int32 or not rects.is_contiguous():
            raise _lib.VaError("rects must be contiguous int32 [B, 4]")
        return B

    def batch(self, B: int, rounds: int, stream=None, records: torch.Tensor | None = None) -> NavBatch:
        """The records of the va_nav_run just enqueued on `stream` (frame records, then query records), or of a
        va_nav_run_rb / va_frame_rb call that left them in `records` (host_records)."""
        d = self.dims
        return NavBatch(self, B, rounds, (B * d.frame_bytes + 15) & ~15, stream, records)

    def host_records(self, B: int) -> torch.Tensor:
        """A pinned host buffer for va_nav_run_rb / va_frame_rb's records of B frames (fresh per call: a
        NavBatch keeps reading its own)."""
        n = int(self.lib.va_nav_records_bytes(B, self.dims.H, self.dims.W))
        if n <= 0:
            raise _lib.VaError(f"va_nav_records_bytes({B}) = {n}")
        return torch.empty(n, dtype=torch.uint8, pin_memory=True)

    def run(self, cells: torch.Tensor, rects: torch.Tensor, seen: AngleSeen, stream=None,
            readback: bool = False) -> NavBatch:
        """cells: uint8 [B, H/20, W/20] (device), rects: int32 [B, 4] (device).  readback: va_nav_run_rb (the
        records copied to the host inside the call, ahead of the A* verdict wait) instead of va_nav_run + an
        asynchronous copy NavBatch.host() waits for."""
        B = self.check_inputs(cells, rects)
        d = self.dims
        rounds = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            if readback:
                rec = self.host_records(B)
                _lib.check(self.lib.va_nav_run_rb(_lib.stream_ptr(stream, self.device), cells.data_ptr(),
                                                  rects.data_ptr(), B, d.H, d.W, seen.t.data_ptr(),
                                                  self.work.data_ptr(), ctypes.byref(rounds), rec.data_ptr(),
                                                  rec.numel()), "va_nav_run_rb")
                return self.batch(B, rounds.value, stream, records=rec)
            _lib.check(self.lib.va_nav_run(_lib.stream_ptr(stream, self.device), cells.data_ptr(), rects.data_ptr(),
                                           B, d.H, d.W, seen.t.data_ptr(), self.work.data_ptr(), ctypes.byref(rounds)),
                       "va_nav_run")
            # frame records then query records (16-byte aligned): va_nav.hip work_bytes()
            return self.batch(B, rounds.value, stream)

    def sample_cells(self, masks: torch.Tensor, stream=None) -> torch.Tensor:
        """Lattice samples of filled masks uint8 [B, H, W] (FrameProcessor.py:88-97)."""
        B, H, W = masks.shape
        d = self.dims
        cells = torch.empty((B, d.LR, d.LC), dtype=torch.uint8, device=masks.device)
        with torch.cuda.device(masks.device):
            _lib.check(self.lib.va_nav_sample_cells(_lib.stream_ptr(stream, masks.device), masks.data_ptr(),
                                                    masks.stride(1), B, H, W, cells.data_ptr()), "va_nav_sample_cells")
        return cells

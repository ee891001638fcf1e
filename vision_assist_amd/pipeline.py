"""The fused per-frame hot path for a batch of frames, device-resident end to end.

    frames (uint8 BGR, HBM) -> va_seg_run  (preprocess + YOLOv8-seg forward, MFMA)
                            -> va_post_run (decode, NMS, process_mask, mask choice -> cells, rect)
                            -> va_nav_run  (grid, penalties, protrusions, start/end, A*, dedupe)

This is FrameProcessor.__call__ (FrameProcessor.py:301-347) for B frames at
once; PathAnalyser (:349) runs on the host per frame in the FrameProcessor
surface.  Frames of one batch are processed in order for the PathFinder angle
cache (the batch gives exactly the sequential result, see va_nav.hip).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .nav import AngleSeen, NavBatch, NavEngine
from .post import PLANT_IF_NONE, PLANT_NEVER, PostEngine, letterbox_geometry
from .seg import SegNet


class FramePipeline:
    def __init__(self, arch, folded, B: int, H: int, W: int, dtype: str = "bf16", conf: float = 0.5,
                 iou: float = 0.7, max_det: int = 300, device=None, seen: AngleSeen | None = None,
                 seg: SegNet | None = None, tag: int = 0, imgsz: int | None = None, fp8_calib=None,
                 lanes: bool | None = None):
        """H x W: the frame size.  ``imgsz`` = YOLO.predict's imgsz: frames are letterboxed to it on the device
        (va_letterbox; LetterBox(imgsz, auto=True, scaleup=True)) whenever that changes them -- the 640
        default of the reference's model.predict call -- and the mask choice maps back to frame coordinates,
        so cells / rects / the nav stage stay at H x W.  ``imgsz=None``: the network runs at the frame's own
        size when its sides are multiples of 32 (the C5 shape, m-seg at 1280x1280, BASELINE.json configs[4];
        640x640 is the same either way), else at the 640 letterbox.  ``lanes``: SegNet.plan's branch-parallel
        list (default: on for small batches)."""
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.B, self.H, self.W = B, H, W
        self.lb = None
        Hn, Wn, frame = H, W, None
        geo = None
        if imgsz is not None:
            geo = letterbox_geometry(H, W, imgsz)
            if geo[:2] == (H, W) and geo[4:6] == (H, W):
                geo = None  # LetterBox is the identity
        elif H % 32 or W % 32:
            geo = letterbox_geometry(H, W, 640)
        if geo is not None:
            Hn, Wn, top, left, newh, neww, gain, pad_x, pad_y = geo
            self.lb = (Hn, Wn, top, left, newh, neww)
            frame = (H, W, gain, pad_x, pad_y)
        self.Hn, self.Wn = Hn, Wn
        self.seg = seg if seg is not None else SegNet(arch, folded, dtype=dtype, device=self.device)
        if fp8_calib is not None:  # fp8: representative frames (uint8 [n, Hn, Wn, 3]) for the activation scales
            self.seg.fp8_calib_frames = torch.as_tensor(fp8_calib)
        self.plan = self.seg.plan(B, Hn, Wn, tag, lanes=lanes)
        self.post = PostEngine(B, Hn, Wn, arch.nc, conf, iou, max_det, device=self.device, frame=frame)
        self.nav = NavEngine(H, W, max_batch=B, device=self.device)
        self.seen = seen if seen is not None else AngleSeen(self.device)
        self.lib = _lib.load()

    @property
    def frames(self) -> torch.Tensor:
        """The device buffer (uint8 [B, Hn, Wn, 3]) the forward reads (the letterboxed frames, if any)."""
        return self.plan["frames"]

    def _pinned(self, frames: torch.Tensor) -> torch.Tensor:
        """Host frames (a camera's numpy frame, main.py:62-82) copied into a pinned staging buffer, so that the H2D
        copy that follows is asynchronous on the launch stream (a pageable source makes it synchronous and staged
        by the runtime).  The buffer is reused only after the previous copy out of it has completed (_pin_ev).
        The copy is numpy's (one thread): torch's CPU copy of a frame this size wakes the OpenMP pool, whose
        workers then spin between calls -- at a call every ~2 ms that kept 15 threads busy, and under the box's
        16-CPU quota the whole process was throttled ~8 ms in every 100 ms period (tools/dropin_split.py)."""
        frames = [frames] if isinstance(frames, torch.Tensor) else frames
        n = sum(int(f.shape[0]) if f.ndim == 4 else 1 for f in frames)
        if getattr(self, "_pin", None) is None:
            self._pin = torch.empty((self.B, self.H, self.W, 3), dtype=torch.uint8, pin_memory=True)
            self._pin_np = self._pin.numpy()
            self._pin_ev = None
        if n > self.B:
            raise _lib.VaError(f"{n} frames for a pipeline of batch {self.B}")
        if self._pin_ev is not None:
            self._pin_ev.synchronize()
        i = 0
        for f in frames:
            a = f.numpy() if isinstance(f, torch.Tensor) else f
            k = a.shape[0] if a.ndim == 4 else 1
            np.copyto(self._pin_np[i:i + k], a.reshape(k, self.H, self.W, 3))
            i += k
        return self._pin[:n]

    def load(self, frames, stream=None) -> None:
        """Frames (uint8 BGR [n, H, W, 3] with n <= B, on the device or the host; or a list of host frames, each
        [H, W, 3]) into the first n entries of the network's input buffer, letterboxed if needed, on ``stream``
        (default: the current stream) -- the H2D copy, the letterbox and the pinned buffer's release event all on
        that one stream; host frames go through a pinned staging buffer (_pinned).  The network always runs B
        frames: entries past n keep what they held (their results are simply not read, see nav_run)."""
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        if isinstance(frames, (list, tuple)):
            for f in frames:
                if tuple(f.shape) != (self.H, self.W, 3) or f.dtype != np.uint8:
                    raise _lib.VaError(f"frames must be uint8 [{self.H}, {self.W}, 3], got {tuple(f.shape)}")
            staged = True
        else:
            if frames.ndim != 4 or tuple(frames.shape[1:]) != (self.H, self.W, 3) or frames.dtype != torch.uint8 \
                    or frames.shape[0] > self.B:
                raise _lib.VaError(f"frames must be uint8 [n <= {self.B}, {self.H}, {self.W}, 3], "
                                   f"got {tuple(frames.shape)} {frames.dtype}")
            staged = frames.device.type == "cpu" and not frames.is_pinned()
        if staged:
            frames = self._pinned(frames)
        n = int(frames.shape[0])
        with torch.cuda.stream(st):
            if self.lb is None:
                self.plan["frames"][:n].copy_(frames, non_blocking=True)
            else:
                frames = frames.to(self.device, non_blocking=True).contiguous()
                Hn, Wn, top, left, newh, neww = self.lb
                with torch.cuda.device(self.device):
                    _lib.check(self.lib.va_letterbox(_lib.stream_ptr(st, self.device), frames.data_ptr(), n,
                                                     self.H, self.W, self.plan["frames"].data_ptr(), Hn, Wn, top,
                                                     left, newh, neww), "va_letterbox")
            if staged:
                self._pin_ev = torch.cuda.Event()
                self._pin_ev.record(st)

    def run(self, frames: torch.Tensor | None = None, plant_cells=None, plant_rects=None,
            plant_mode: int = PLANT_NEVER, stream=None) -> NavBatch:
        """One batch through the whole path: frames in, then ONE va_frame_rb call on the device's handle (forward,
        post-processing and mask choice, grid / penalty / protrusion / A*), which returns with the grid stage's
        records in host memory (copied ahead of the A* verdict wait: one synchronisation per call)."""
        if frames is not None:
            self.load(frames, stream)
        out = self.plan["out"]
        if plant_mode != PLANT_NEVER and plant_cells is None:
            raise ValueError("plant_mode needs plant_cells / plant_rects")
        a = self.post.args(out.levels, out.proto, plant_cells, plant_rects, plant_mode, select=True)
        B = self.nav.check_inputs(self.post.cells, self.post.rects)
        rounds = ctypes.c_int32(0)
        h = _lib.Handle.for_device(self.device)
        rec = self.nav.host_records(B)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.va_frame_rb(h.ptr, _lib.stream_ptr(stream, self.device), self.plan["ops"],
                                            self.plan["n"], ctypes.byref(a), self.H, self.W, self.seen.t.data_ptr(),
                                            self.nav.work.data_ptr(), ctypes.byref(rounds), rec.data_ptr(),
                                            rec.numel()), "va_frame_rb")
        return self.nav.batch(B, rounds.value, stream, records=rec)

    def run_seg_only(self, stream=None) -> None:
        self.seg.run_plan(self.plan, stream)

    # -- split form, for overlapping the grid stage of batch k with the network of batch k+1 ----
    def seg_post(self, plant_cells=None, plant_rects=None, plant_mode: int = PLANT_NEVER, stream=None):
        """Network + post-processing of the frames already in ``self.frames`` (enqueued only)."""
        self.seg.run_plan(self.plan, stream)
        out = self.plan["out"]
        self.post.run(out.levels, out.proto, plant_cells, plant_rects, plant_mode, select=True, stream=stream)

    def nav_run(self, stream=None, n: int | None = None, readback: bool = False) -> NavBatch:
        """Grid stage of the batch whose seg_post was enqueued (synchronises `stream`): its first ``n`` frames
        (default all B; frames past n never reach A*, so the angle cache advances over the n real frames only).
        readback: the records land in host memory inside the call (va_nav_run_rb, one synchronisation)."""
        n = self.B if n is None else n
        return self.nav.run(self.post.cells[:n], self.post.rects[:n], self.seen, stream, readback=readback)


class OverlappedPipelines:
    """`depth` FramePipelines sharing weights and the angle cache, fed round-robin.  Consecutive batches'
    networks alternate between two network streams, so two forwards run concurrently and fill each other's
    kernel tails and launch gaps; the grid stage (a few hundred waves: A* is a chain of dependent pops) runs
    on its own stream, in submission order, so batches leave in order and the angle cache advances in
    order.  A pipeline's buffers are reused only after its previous batch has left the grid stage; with
    depth 3 the host can enqueue batch k+2's network before it blocks in batch k's grid stage (whose A*
    rounds read a device flag), so the GPU always holds two networks."""

    def __init__(self, arch, folded, B: int, H: int, W: int, dtype: str = "bf16", device=None,
                 seg_streams: int = 2, depth: int = 2, **kw):
        if depth < 2:
            raise ValueError("depth >= 2")
        # whole forwards already overlap here: the laned list's extra streams would only contend with them for
        # the hardware queues (C4 shape: 904 -> 506 frames/s with lanes)
        kw.setdefault("lanes", False)
        first = FramePipeline(arch, folded, B, H, W, dtype=dtype, device=device, tag=0, **kw)
        self.pipes = [first] + [FramePipeline(arch, folded, B, H, W, dtype=dtype, device=first.device,
                                              seen=first.seen, seg=first.seg, tag=i, **kw) for i in range(1, depth)]
        self.a, self.b = self.pipes[0], self.pipes[1]
        self.depth = depth
        if seg_streams < 1:
            raise ValueError("seg_streams >= 1")
        self.s_segs = tuple(torch.cuda.Stream(device=first.device) for _ in range(seg_streams))
        self.s_nav = torch.cuda.Stream(device=first.device)
        self.ev = [torch.cuda.Event() for _ in range(depth)]        # network + post of the pipeline's batch
        self.nav_done = [torch.cuda.Event() for _ in range(depth)]  # its grid stage
        self.k = 0

    def submit(self, frames: torch.Tensor, plant_cells=None, plant_rects=None, plant_mode: int = PLANT_NEVER):
        """Enqueue copy + network + post-processing of the next batch on its network stream."""
        i = self.k % self.depth
        p = self.pipes[i]
        s_seg = self.s_segs[self.k % len(self.s_segs)]
        s_seg.wait_stream(torch.cuda.current_stream())
        s_seg.wait_event(self.nav_done[i])  # the pipeline's previous batch has left its grid stage
        with torch.cuda.stream(s_seg):
            p.load(frames, stream=s_seg)
            p.seg_post(plant_cells, plant_rects, plant_mode, stream=s_seg)
            self.ev[i].record(s_seg)
        self.k += 1

    def finish(self, j: int) -> NavBatch:
        """Run the grid stage of submitted batch j (in submission order) on the nav stream."""
        i = j % self.depth
        p = self.pipes[i]
        self.s_nav.wait_event(self.ev[i])
        with torch.cuda.stream(self.s_nav):
            res = p.nav_run(stream=self.s_nav)
            self.nav_done[i].record(self.s_nav)
        return res


class StreamBatches:
    """A frame stream in batches of up to B host frames with two batches in flight: ``begin(frames)`` stages the
    frames in pinned memory and enqueues copy + network + post-processing on one of two network streams (it
    returns as soon as the frames are copied out of the caller's memory), ``end(token)`` runs that batch's grid
    stage on the grid stream -- in begin order, so the angle cache advances frame by frame in stream order -- and
    returns its records on the host.  A caller that begins batch j + 1 before it ends batch j keeps the GPU on
    batch j + 1's network while the host builds batch j's answers.  Two FramePipelines share one SegNet (the
    weights) and the angle cache; a batch of n < B frames runs the network on B entries but only its n frames
    reach the grid stage (FramePipeline.nav_run)."""

    def __init__(self, arch, folded, B: int, H: int, W: int, dtype: str = "f32", device=None, seen=None,
                 seg=None, **kw):
        kw.setdefault("lanes", False)  # two whole forwards overlap already (as OverlappedPipelines)
        first = FramePipeline(arch, folded, B, H, W, dtype=dtype, device=device, seen=seen, seg=seg, tag=0, **kw)
        self.pipes = [first, FramePipeline(arch, folded, B, H, W, dtype=dtype, device=first.device, seen=first.seen,
                                           seg=first.seg, tag=1, **kw)]
        self.device, self.B = first.device, B
        self.s_segs = tuple(torch.cuda.Stream(device=self.device) for _ in self.pipes)
        self.s_nav = torch.cuda.Stream(device=self.device)
        self.ready = [torch.cuda.Event() for _ in self.pipes]
        self.k = 0      # batches begun
        self.done = 0   # batches ended

    def begin(self, frames) -> tuple[int, int]:
        """Host frames (a list of uint8 [H, W, 3], at most B) -> a token for end().  At most two batches may be
        begun and not ended."""
        if not 0 < len(frames) <= self.B:
            raise ValueError(f"1..{self.B} frames per batch, got {len(frames)}")
        if self.k - self.done >= len(self.pipes):
            raise RuntimeError("two batches are in flight: end() the older one first")
        i = self.k % len(self.pipes)
        p, st = self.pipes[i], self.s_segs[i]
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            p.load(list(frames), stream=st)
            p.seg_post(stream=st)
            self.ready[i].record(st)
        tok = (self.k, len(frames))
        self.k += 1
        return tok

    def end(self, token) -> NavBatch:
        """The grid stage of a begun batch (tokens in begin order); returns with the records on the host."""
        j, n = token
        if j != self.done:
            raise RuntimeError(f"batches end in begin order: expected {self.done}, got {j}")
        i = j % len(self.pipes)
        try:
            self.s_nav.wait_event(self.ready[i])
            with torch.cuda.stream(self.s_nav):
                res = self.pipes[i].nav_run(stream=self.s_nav, n=n, readback=True)
        finally:
            # a grid stage that raised loses its own batch only: the token is spent either way, so the next end()
            # and begin() go on in order.  The next begin() on this pipeline rewrites cells / rects the
            # grid stage just read: order it after it
            self.s_segs[i].wait_stream(self.s_nav)
            self.done += 1
        return res


__all__ = ["FramePipeline", "OverlappedPipelines", "StreamBatches", "PLANT_IF_NONE", "PLANT_NEVER"]


class SegPostGraph:
    """The frame copy + network + post-processing of a FramePipeline (``load`` + ``seg_post``) captured once as a
    HIP graph, for the batch-1 latency form (tools/latency.py --graph).

    hipGraphLaunch is only ever issued on a private stream of this object: ``replay(stream)`` makes the private
    stream wait for ``stream``'s prior work (an event), launches the graph there and makes ``stream`` wait for the
    graph's end (another event), so work the caller queues next on ``stream`` -- the grid stage, a copy out --
    is ordered after the graph by an explicit dependency, whatever ``stream`` is.  A graph launched directly on
    the legacy default stream (handle 0) and followed there by the grid stage faulted the GPU (round 2 and
    profiles/r03/graph_fault/: the same sequence on a private stream, and eagerly on the default stream, runs
    clean), so the legacy stream never sees a graph launch."""

    def __init__(self, pipe: FramePipeline, frames: torch.Tensor | None = None, plant_cells=None, plant_rects=None,
                 plant_mode: int = PLANT_NEVER, warmup: int = 2):
        self.pipe = pipe
        if frames is not None and frames.device.type != "cuda":
            # a host frame would be staged by a host-side copy into the pinned buffer, which the graph does not
            # capture: every replay would read whatever that buffer last held
            raise ValueError("SegPostGraph captures device frames only (copy host frames to the device first)")
        dev = pipe.device
        self.stream = torch.cuda.Stream(device=dev)
        s = self.stream
        cur = torch.cuda.current_stream(dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(warmup):  # plans, attributes, lazily allocated buffers: before the capture
                if frames is not None:
                    pipe.load(frames, stream=s)
                pipe.seg_post(plant_cells, plant_rects, plant_mode, stream=s)
        s.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            if frames is not None:
                pipe.load(frames, stream=s)
            pipe.seg_post(plant_cells, plant_rects, plant_mode, stream=s)
        s.synchronize()

    def replay(self, stream=None) -> None:
        """One replay, ordered after ``stream``'s (default: the current stream's) queued work and before
        anything queued on it afterwards."""
        dev = self.pipe.device
        cur = stream if stream is not None else torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.graph.replay()
        cur.wait_stream(self.stream)

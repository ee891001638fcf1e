"""Multi-GPU sharding of the per-frame hot path.

Frames are independent: one process per GPU, frame i goes to rank i % world
(round-robin, like a video read by one reader and dealt to workers), and there
is NO collective on the data path.  torch.distributed is used only around the
timed region (barrier, max of the elapsed times over ranks) and to gather small
per-frame results on rank 0.

Each process has its own PathFinder angle cache (PathFinder.py:32 is
process-global), so a shard's A* results equal the reference run over that
shard's frames in order -- tests/test_shard.py checks exactly that with
world_size 2 over gloo.
"""
from __future__ import annotations

import os
import time
from typing import Callable

import numpy as np
import torch


def dist_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_indices(n_frames: int, world: int, rank: int) -> list[int]:
    """Frames of `rank`: i % world == rank, in stream order."""
    return list(range(rank, n_frames, world))


def timed(fn: Callable[[], object], world: int, sync: Callable[[], None] | None = None) -> tuple[object, float]:
    """Run fn between barriers (+ device sync) and return (result, max elapsed seconds over ranks)."""
    import torch.distributed as dist
    on = world > 1 and dist.is_available() and dist.is_initialized()
    if sync:
        sync()
    if on:
        dist.barrier()
    t0 = time.perf_counter()
    out = fn()
    if sync:
        sync()
    if on:
        dist.barrier()
    el = time.perf_counter() - t0
    if on:
        backend = dist.get_backend()
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return out, el


def gather_by_frame(local: dict[int, object], world: int) -> dict[int, object] | None:
    """Gather {frame index: small result} from every rank onto rank 0 (None elsewhere)."""
    import torch.distributed as dist
    if world == 1 or not (dist.is_available() and dist.is_initialized()):
        return dict(local)
    parts = [None] * world if dist.get_rank() == 0 else None
    dist.gather_object(local, parts, dst=0)
    if dist.get_rank() != 0:
        return None
    out = {}
    for p in parts:
        out.update(p)
    return out


# ------------------------------------------------------------------------------------------------ frame dealer
class FrameDealer:
    """SURVEY.md §8e's reader / worker split for one frame stream on a node: the caller (one reader, e.g. main.py's
    camera loop) deals frame i to worker process i % G, each worker owns one GPU and its own FrameProcessor /
    PathFinder singletons (the reference's process-global state, PathFinder.py:32: a shard's answers equal the
    reference run over that shard's frames in order), and results come back in frame order.  No collective and no
    torch.distributed: pixels travel through a shared-memory ring of ``slots`` frames per worker (a memcpy, no
    pickling), the small results through one queue.

    worker_factory: a picklable callable run once inside each worker, ``worker_factory(device_index) -> fn`` with
    ``fn(frame: np.ndarray uint8 [H, W, 3]) -> picklable result`` (default: dropin_worker -- YOLO + FrameProcessor
    on that GPU, returning FrameProcessor.__call__'s answer).  devices: one entry per worker (GPU indices; several
    workers may share a GPU).  Frames of one dealer share one size (H, W)."""

    def __init__(self, worker_factory, devices, H: int, W: int, slots: int = 4, start_timeout: float = 600.0):
        import torch.multiprocessing as tmp
        self.G = len(devices)
        if self.G < 1:
            raise ValueError("FrameDealer needs at least one worker")
        self.H, self.W, self.slots = H, W, slots
        ctx = tmp.get_context("spawn")
        self.ring = torch.zeros((self.G, slots, H, W, 3), dtype=torch.uint8).share_memory_()
        self._ring_np = self.ring.numpy()  # frames are copied in by numpy (one thread; see submit)
        self.inq = [ctx.Queue() for _ in range(self.G)]
        self.free = [ctx.Queue() for _ in range(self.G)]
        self.outq = ctx.Queue()
        for w in range(self.G):
            for s in range(slots):
                self.free[w].put(s)
        self.procs = [ctx.Process(target=_dealer_worker, daemon=True,
                                  args=(w, devices[w], worker_factory, self.ring, self.inq[w], self.free[w], self.outq))
                      for w in range(self.G)]
        for p in self.procs:
            p.start()
        ready = 0
        while ready < self.G:
            tag, w, payload = self.outq.get(timeout=start_timeout)
            if tag == "error":
                self.close()
                raise RuntimeError(f"dealer worker {w} failed to start: {payload}")
            ready += tag == "ready"
        self.n = 0          # frames submitted
        self.next = 0       # next frame index to hand back
        self._done = {}     # results that arrived ahead of their turn

    def submit(self, frame) -> int:
        """Deal one frame (np.ndarray / tensor uint8 [H, W, 3]) to worker n % G; blocks while that worker's ring is
        full.  -> the frame's index in the stream."""
        idx, w = self.n, self.n % self.G
        t = torch.as_tensor(frame)
        if tuple(t.shape) != (self.H, self.W, 3) or t.dtype != torch.uint8:
            raise ValueError(f"frame must be uint8 [{self.H}, {self.W}, 3], got {tuple(t.shape)} {t.dtype}")
        slot = self.free[w].get()
        # numpy's copy, not torch's: torch's CPU copy of a frame wakes its OpenMP pool, whose workers then spin
        # between frames and exhaust the box's CPU quota for every process of it (pipeline.FramePipeline._pinned)
        np.copyto(self._ring_np[w, slot], t.numpy() if t.device.type == "cpu" else t.cpu().numpy())
        self.inq[w].put((idx, slot))
        self.n += 1
        return idx

    def get(self):
        """The next result in frame order (blocks until it is in)."""
        if self.next >= self.n:
            raise IndexError("no frame in flight")
        while self.next not in self._done:
            tag, idx, payload = self.outq.get()
            if tag == "error":
                raise RuntimeError(f"dealer worker failed on frame {idx}: {payload}")
            self._done[idx] = payload
        out = self._done.pop(self.next)
        self.next += 1
        return out

    def in_flight(self) -> int:
        return self.n - self.next

    def map(self, frames):
        """Results of a frame iterable, in order, with up to G x slots frames in flight."""
        limit = self.G * self.slots
        for fr in frames:
            self.submit(fr)
            while self.in_flight() >= limit:
                yield self.get()
        while self.in_flight():
            yield self.get()

    def close(self) -> None:
        for q in self.inq:
            q.put(None)
        for p in self.procs:
            p.join(timeout=60)
            if p.is_alive():
                p.terminate()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _dealer_worker(w, device, factory, ring, inq, free, outq):
    import traceback
    try:
        if device is not None and torch.cuda.is_available():
            torch.cuda.set_device(device)
        fn = factory(device)
    except Exception:
        outq.put(("error", w, traceback.format_exc()))
        return
    outq.put(("ready", w, None))
    while True:
        item = inq.get()
        if item is None:
            return
        idx, slot = item
        frame = ring[w, slot].numpy().copy()
        free.put(slot)  # the slot is reusable as soon as the pixels are copied out
        try:
            outq.put(("ok", idx, fn(frame)))
        except Exception:
            outq.put(("error", idx, traceback.format_exc()))


class dropin_worker:
    """The default FrameDealer worker: YOLO(model, **kw) + FrameProcessor on the worker's GPU (main.py:43-44);
    each frame -> FrameProcessor.__call__'s answer (main.py:82).  Picklable (a plain object holding the YOLO
    constructor's arguments; the weights are built inside the worker)."""

    def __init__(self, model: str = "yolov8s-seg.pt", **yolo_kw):
        self.model, self.kw = model, yolo_kw

    def __call__(self, device):
        import warnings

        from .FrameProcessor import FrameProcessor
        from .yolo import YOLO
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            yolo = YOLO(self.model, **self.kw).to(torch.device("cuda", device))
        fp = FrameProcessor(model=yolo, verbose=False, debug=False)
        fp.model = yolo
        return fp

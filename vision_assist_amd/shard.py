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
    pickling) whose head / tail counters sit in shared memory too (the reader publishes a frame by bumping the head
    after its copy, the worker frees slots by bumping the tail once it has copied frames out; frame i is worker
    i % G's (i // G)-th frame, so no index travels), the small results through one queue, one message per batch.

    worker_factory: a picklable callable run once inside each worker, ``worker_factory(device_index) -> fn`` with
    ``fn(frame: np.ndarray uint8 [H, W, 3]) -> picklable result`` (default: dropin_worker -- YOLO + FrameProcessor
    on that GPU, returning FrameProcessor.__call__'s answer).  A worker ``fn`` may also process frames in batches:
    with ``fn.max_batch = k``, ``fn.begin(frames) -> token`` (at most k frames, which it must have copied out of
    the list's arrays -- views of ring slots, reused as soon as begin returns -- before it returns) and
    ``fn.end(token) -> results`` (one per frame, in order; an exception object in a frame's place fails that frame
    alone), the worker drains up to k waiting frames into one batch and begins the next batch before it ends the
    previous one, so two batches are in flight.  devices: one entry per worker (GPU indices; several workers may
    share a GPU).  Frames of one dealer share one size (H, W).

    A frame whose worker raised is handed back by get() as a RuntimeError for that frame and the stream moves on;
    a worker process that dies makes the dealer ``broken`` (every later call raises instead of waiting).

    readers: 0 (default) copies each frame into its ring on the calling thread inside submit(); R > 0 hands the copies
    to R reader threads (thread r fills the rings of workers w with w % R == r, in submission order), so submit()
    returns at once and the rings fill in parallel -- one thread's copies cap the whole node's frame rate near one GPU's
    worth.  With readers, a submitted frame must stay unmodified until its result has been returned
    (map() over fresh frames, as a camera or a decoder yields them, is safe)."""

    def __init__(self, worker_factory, devices, H: int, W: int, slots: int = 4, start_timeout: float = 600.0,
                 poll: float = 1.0, readers: int = 0):
        import platform

        import torch.multiprocessing as tmp
        self.G = len(devices)
        if self.G < 1:
            raise ValueError("FrameDealer needs at least one worker")
        if platform.machine() not in ("x86_64", "AMD64"):
            # the ring's head / tail handshake is plain aligned int64 stores: correct under x86's store order only
            raise RuntimeError(f"FrameDealer's ring handshake assumes x86 store ordering, not {platform.machine()}")
        self.H, self.W, self.slots, self.poll = H, W, slots, poll
        need = self.G * slots * H * W * 3
        if os.path.isdir("/dev/shm"):
            st = os.statvfs("/dev/shm")
            free = st.f_bavail * st.f_frsize
            if need > free:
                raise ValueError(f"the frame ring needs {need / 2**20:.0f} MiB of /dev/shm ({self.G} workers x {slots} "
                                 f"slots x {H}x{W}x3), {free / 2**20:.0f} MiB are free: pass fewer slots or workers")
        self.broken: str | None = None
        ctx = tmp.get_context("spawn")
        self.ring = torch.zeros((self.G, slots, H, W, 3), dtype=torch.uint8).share_memory_()
        self._ring_np = self.ring.numpy()  # frames are copied in by numpy (one thread; see submit)
        # per worker: [head = frames published, tail = frames copied out of the ring, stop]; head is written by the
        # reader only, tail by the worker only (aligned int64 stores; x86 keeps the frame's stores ahead of the head's)
        self.ctl = torch.zeros((self.G, 3), dtype=torch.int64).share_memory_()
        self._ctl = self.ctl.numpy()
        self.outq = ctx.Queue()
        self.procs = [ctx.Process(target=_dealer_worker, daemon=True,
                                  args=(w, self.G, devices[w], worker_factory, self.ring, self.ctl, self.outq))
                      for w in range(self.G)]
        for p in self.procs:
            p.start()
        ready, t0 = 0, time.monotonic()
        while ready < self.G:
            try:
                tag, w, payload = self._pull(timeout=start_timeout - (time.monotonic() - t0))
            except RuntimeError:
                self.close()
                raise
            if tag == "start_error":
                self.close()
                raise RuntimeError(f"dealer worker {w} failed to start: {payload}")
            ready += tag == "ready"
        self.n = 0          # frames submitted
        self.next = 0       # next frame index to hand back
        self._done = {}     # results that arrived ahead of their turn (_Failed for a frame whose worker raised)
        self._readers = []
        if readers > 0:
            import queue
            import threading
            self._rq = [queue.SimpleQueue() for _ in range(min(readers, self.G))]
            self._readers = [threading.Thread(target=self._reader, args=(q,), daemon=True) for q in self._rq]
            for t in self._readers:
                t.start()

    def _check_workers(self) -> None:
        for w, p in enumerate(self.procs):
            if not p.is_alive():
                self.broken = f"dealer worker {w} (pid {p.pid}) exited with status {p.exitcode}"
                raise RuntimeError(self.broken)

    def _pull(self, timeout: float | None = None):
        """One message from the workers, checking every `poll` seconds that they are all alive."""
        import queue
        t0 = time.monotonic()
        while True:
            try:
                return self.outq.get(timeout=self.poll)
            except queue.Empty:
                self._check_workers()
                if timeout is not None and time.monotonic() - t0 > timeout:
                    raise RuntimeError(f"no word from the dealer workers in {timeout:.0f} s")

    def submit(self, frame) -> int:
        """Deal one frame (np.ndarray / tensor uint8 [H, W, 3]) to worker n % G; blocks while that worker's ring is
        full.  -> the frame's index in the stream."""
        if self.broken:
            raise RuntimeError(self.broken)
        idx, w = self.n, self.n % self.G
        t = torch.as_tensor(frame)
        if tuple(t.shape) != (self.H, self.W, 3) or t.dtype != torch.uint8:
            raise ValueError(f"frame must be uint8 [{self.H}, {self.W}, 3], got {tuple(t.shape)} {t.dtype}")
        src = t.numpy() if t.device.type == "cpu" else t.cpu().numpy()
        if self._readers:
            self._rq[w % len(self._rq)].put((w, src))
        else:
            self._put(w, src)
        self.n += 1
        return idx

    def _put(self, w: int, src: np.ndarray) -> None:
        """Copy one frame into worker w's ring (waiting for a free slot) and publish it."""
        ctl = self._ctl[w]
        head = int(ctl[0])
        if head - int(ctl[1]) >= self.slots:  # the ring is full: wait for the worker to copy frames out
            nap, t0 = 2e-5, time.monotonic()
            while head - int(ctl[1]) >= self.slots:
                time.sleep(nap)
                nap = min(nap * 2, 1e-3)
                if time.monotonic() - t0 > self.poll:
                    self._check_workers()
                    t0 = time.monotonic()
        # numpy's copy, not torch's: torch's CPU copy of a frame wakes its OpenMP pool, whose workers then spin
        # between frames and exhaust the box's CPU quota for every process of it (pipeline.FramePipeline._pinned);
        # numpy releases the GIL for the copy, so reader threads copy in parallel
        np.copyto(self._ring_np[w, head % self.slots], src)
        ctl[0] = head + 1  # publish: the worker may read the slot from now on

    def _reader(self, q) -> None:
        """Reader thread: copies its workers' frames into their rings in submission order; None ends it."""
        while True:
            item = q.get()
            if item is None:
                return
            try:
                self._put(*item)
            except RuntimeError as e:  # a dead worker: the main thread's next wait sees it too (broken)
                self.broken = self.broken or str(e)

    def get(self):
        """The next result in frame order (blocks until it is in); a RuntimeError for a frame whose worker raised
        (the stream then continues with the next frame)."""
        if self.broken:
            raise RuntimeError(self.broken)
        if self.next >= self.n:
            raise IndexError("no frame in flight")
        while self.next not in self._done:
            tag, idxs, payload = self._pull()
            if tag == "ok":
                self._done.update(zip(idxs, payload))
            else:  # "error": the frames of a batch that failed as a whole, or one frame's exception
                for i in idxs:
                    self._done[i] = _Failed(payload)
        idx = self.next
        out = self._done.pop(idx)
        self.next += 1
        if isinstance(out, _Failed):
            raise RuntimeError(f"dealer worker failed on frame {idx}: {out.tb}")
        return out

    def in_flight(self) -> int:
        return self.n - self.next

    def discard(self) -> None:
        """Drop the results of every frame still in flight (their workers still process them, in order)."""
        while self.in_flight():
            try:
                self.get()
            except RuntimeError:
                if self.broken:
                    raise

    def map(self, frames):
        """Results of a frame iterable, in order, with up to G x slots frames in flight.  A consumer that stops
        early (break, an exception, islice) leaves no result behind: the frames still in flight are drained and
        dropped when the generator is closed, so the next map() starts with its own frames' results."""
        limit = self.G * self.slots
        try:
            for fr in frames:
                self.submit(fr)
                while self.in_flight() >= limit:
                    yield self.get()
            while self.in_flight():
                yield self.get()
        finally:
            if self.in_flight() and not self.broken:
                self.discard()

    def close(self) -> None:
        """The workers finish the frames already dealt, then exit."""
        for q in getattr(self, "_rq", []):
            q.put(None)
        for t in self._readers:
            t.join(timeout=60)
        self._readers = []
        self._ctl[:, 2] = 1
        for p in self.procs:
            p.join(timeout=60)
            if p.is_alive():
                p.terminate()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _Failed:
    """A frame whose worker raised (its traceback): FrameDealer.get() raises it in that frame's turn."""

    def __init__(self, tb: str):
        self.tb = tb


def _dealer_worker(w, G, device, factory, ring, ctl, outq):
    """Worker process: frames from its ring slots, in submission order (its j-th frame is the stream's w + j G).  A
    plain ``fn`` runs frame by frame; a batching one (``max_batch`` / ``begin`` / ``end``, see FrameDealer) gets every
    published frame not yet taken, up to max_batch, as one batch, with the next batch begun before the previous one
    is ended.  Idle, it polls the ring's head with a backoff (20 us doubling to 1 ms); it exits once the reader has
    set stop and every published frame is done."""
    import traceback
    try:
        if device is not None and torch.cuda.is_available():
            torch.cuda.set_device(device)
        fn = factory(device)
    except Exception:
        outq.put(("start_error", w, traceback.format_exc()))
        return
    outq.put(("ready", w, None))
    begin = getattr(fn, "begin", None)
    k = max(1, int(getattr(fn, "max_batch", 1))) if begin is not None else 1
    c = ctl.numpy()[w]
    S = ring.shape[1]
    pend, taken, nap = None, 0, 2e-5

    def emit(idxs, tok):
        if tok[0] == "error":
            outq.put(("error", idxs, tok[1]))
            return
        try:
            res = list(fn.end(tok[1])) if begin is not None else tok[1]
            if len(res) != len(idxs):
                raise RuntimeError(f"{len(res)} results for {len(idxs)} frames")
        except Exception:
            outq.put(("error", idxs, traceback.format_exc()))
            return
        ok = [(i, r) for i, r in zip(idxs, res) if not isinstance(r, BaseException)]
        if ok:
            outq.put(("ok", [i for i, _ in ok], [r for _, r in ok]))
        for i, r in zip(idxs, res):
            if isinstance(r, BaseException):
                outq.put(("error", [i], "".join(traceback.format_exception(type(r), r, r.__traceback__))))

    while True:
        n = min(int(c[0]) - taken, k)
        if n == 0:
            if pend is not None:  # nothing new to overlap with: finish the batch in flight
                emit(*pend)
                pend = None
                continue
            if c[2] and int(c[0]) == taken:
                return
            time.sleep(nap)
            nap = min(nap * 2, 1e-3)
            continue
        nap = 2e-5
        idxs = [w + (taken + j) * G for j in range(n)]
        views = [ring[w, (taken + j) % S].numpy() for j in range(n)]
        frames = None
        try:
            if begin is not None:
                tok = ("ok", begin(views))
            else:
                frames = [v.copy() for v in views]
        except Exception:
            tok = ("error", traceback.format_exc())
        taken += n
        c[1] = taken  # the slots are reusable as soon as the pixels are copied out
        if frames is not None:  # frame by frame: run them once their slots are free
            try:
                tok = ("ok", [fn(f) for f in frames])
            except Exception:
                tok = ("error", traceback.format_exc())
        if pend is not None:
            emit(*pend)
        pend = (idxs, tok)


class dropin_worker:
    """The default FrameDealer worker: YOLO(model, **kw) + FrameProcessor on the worker's GPU (main.py:43-44); each
    frame -> FrameProcessor.__call__'s answer (main.py:82).  With ``batch`` > 1 (the default 8) the worker runs up
    to that many waiting frames as one device batch (vision_assist_amd.pipeline.StreamBatches, two batches in
    flight) and builds their answers frame by frame in order -- the same A* order and angle cache as calling the
    frames one by one.  Picklable (the YOLO constructor's arguments plus post-construction settings such as
    ``fp8_calib``; the weights are built inside the worker)."""

    def __init__(self, model: str = "yolov8s-seg.pt", batch: int = 8, fp8_calib=None, quiet: bool = False,
                 **yolo_kw):
        """quiet: the worker's stdout to /dev/null (FrameProcessor prints "No path found." as the reference does)."""
        self.model, self.kw, self.batch, self.quiet = model, yolo_kw, batch, quiet
        self.fp8_calib = None if fp8_calib is None else np.asarray(torch.as_tensor(fp8_calib).cpu())

    def __call__(self, device):
        import os
        import sys
        import warnings

        from .FrameProcessor import FrameProcessor
        from .yolo import YOLO
        if self.quiet:
            sys.stdout = open(os.devnull, "w")
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            yolo = YOLO(self.model, **self.kw).to(torch.device("cuda", device))
        if self.fp8_calib is not None:
            yolo.fp8_calib = torch.from_numpy(self.fp8_calib)
        fp = FrameProcessor(model=yolo, verbose=False, debug=False)
        fp.model = yolo
        return _BatchedFrameProcessor(fp, self.batch) if self.batch > 1 else fp


class _BatchedFrameProcessor:
    """FrameDealer's batching protocol over the worker's FrameProcessor (FrameProcessor._begin_batch / _end_batch)."""

    def __init__(self, fp, max_batch: int):
        self.fp, self.max_batch = fp, max_batch

    def __call__(self, frame):
        return self.fp(frame)

    def begin(self, frames):
        return self.fp._begin_batch(frames, self.max_batch)

    def end(self, token):
        return self.fp._end_batch(token)

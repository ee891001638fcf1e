"""The frame dealer's transport alone (vision_assist_amd.shard.FrameDealer): one frame source dealt to G worker
processes whose batching workers do no work ("triv") or copy the frames out ("copy"), with the frame copies into the
rings on the calling thread (readers 0) or on R reader threads -- the host-side ceiling of the dealer, CPU only:
python tools/dealer_ceiling.py [G ...]  (DESIGN.md §5-6)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_assist_amd.shard import FrameDealer  # noqa: E402


class Triv:
    max_batch = 32

    def begin(self, frames):
        return [int(f[0, 0, 0]) for f in frames]  # touches the frames; copies nothing big

    def end(self, tok):
        return ["ok"] * len(tok)


class TrivCopy(Triv):
    def begin(self, frames):
        out = np.empty((len(frames), 640, 640, 3), np.uint8)
        for i, f in enumerate(frames):
            np.copyto(out[i], f)
        return [0] * len(frames)


def factory_triv(dev):
    return Triv()


def factory_copy(dev):
    return TrivCopy()


def ceiling(fac, G: int, readers: int, n: int = 2048, slots: int = 32, frames=None) -> float:
    """frames/s through a dealer of G workers built by fac, n frames after a warm-up."""
    if frames is None:
        rng = np.random.default_rng(0)
        frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    with FrameDealer(fac, [None] * G, 640, 640, slots=slots, readers=readers) as d:
        for _ in d.map(frames[i % 16] for i in range(128)):
            pass
        t0 = time.perf_counter()
        for _ in d.map(frames[i % 16] for i in range(n)):
            pass
        return n / (time.perf_counter() - t0)


if __name__ == "__main__":
    Gs = [int(a) for a in sys.argv[1:]] or [1, 2, 4]
    for name, fac in (("triv", factory_triv), ("copy", factory_copy)):
        for G in Gs:
            for readers in sorted({0, 1, G}):
                print(name, "workers", G, "readers", readers, round(ceiling(fac, G, readers), 1), "frames/s", flush=True)

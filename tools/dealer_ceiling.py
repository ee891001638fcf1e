"""The frame dealer's transport alone (vision_assist_amd.shard.FrameDealer): one reader dealing 640x640 frames to 1 or 2
worker processes whose batching workers do no work ("triv") or copy the frames out ("copy") -- the host-side ceiling
of the dealer extra, CPU only:  python tools/dealer_ceiling.py  (DESIGN.md §5)."""
import sys, time
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from vision_assist_amd.shard import FrameDealer


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


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    for name, fac in (("triv", factory_triv), ("copy", factory_copy)):
        for G in (1, 2):
            with FrameDealer(fac, [None] * G, 640, 640, slots=64) as d:
                for _ in d.map(frames[i % 16] for i in range(256)):
                    pass
                t0 = time.perf_counter()
                n = 2048
                for _ in d.map(frames[i % 16] for i in range(n)):
                    pass
                dt = time.perf_counter() - t0
            print(name, G, round(n / dt, 1), "frames/s", flush=True)

"""Bounds-checked run of the contour kernels (libva355_ctcheck.so, `make ctcheck`): the post-processing chain of
tests/test_gpu_post.py's mid / dense regimes and va_post_select_masks on small (LDS-resident) masks; prints the
first out-of-range access each records (code, v0, v1) -- 0 = none.  Debug tool."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_assist_amd import _lib  # noqa: E402

LIB = os.path.join(os.path.dirname(_lib.LIB_PATH), "libva355_ctcheck.so")
lib = _lib.load(LIB)
lib.va_contour_debug.restype = ctypes.c_int
lib.va_contour_debug.argtypes = [ctypes.c_void_p, ctypes.c_int]


def err(tag):
    w = (ctypes.c_uint * 4)()
    _lib.check(lib.va_contour_debug(w, 1), "va_contour_debug")
    print(tag, list(w), flush=True)


def main():
    from tests.contour_cases import blob
    from vision_assist_amd.post import select_masks
    rng = np.random.default_rng(3)
    for hw in (80, 160):
        m = np.stack([np.stack([blob(rng, hw, hw, sigma=3.0) for _ in range(3)]) for _ in range(4)])
        n = np.full(4, 3, np.int32)
        select_masks(torch.from_numpy(m).cuda(), torch.from_numpy(n), hw, hw)
        err(f"select_masks {hw}")
    from vision_assist_amd.post import PostEngine
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    for bias in (0.0, 4.0):
        arch = Arch("s")
        fw = fold(arch, synthetic_state_dict(arch, seed=0, cls_bias=bias))
        net = SegNet(arch, fw, dtype="f32")
        frames = torch.randint(0, 256, (2, 640, 640, 3), generator=torch.Generator().manual_seed(11),
                               dtype=torch.uint8)
        out = net.forward(frames.cuda())
        post = PostEngine(2, 640, 640, arch.nc)
        post.run(out.levels, out.proto, select=False)
        err(f"post no-select bias {bias} ndet {post.ndet.cpu().tolist()}")
        post.polygons(0)
        err(f"polygons bias {bias}")
        post.run(out.levels, out.proto)
        err(f"post select bias {bias} chosen {post.chosen.cpu().tolist()}")
        st = post.contour_stats(0)
        print("npts", st["npts"][:10].tolist(), "ncont", st["ncont"][:10].tolist(), "status", np.unique(st["status"]))


if __name__ == "__main__":
    main()

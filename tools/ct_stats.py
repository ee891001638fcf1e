"""Contour statistics of a dense-regime batch (synthetic weights, cls bias +4): per frame the chosen instance's
point count and contour count, the largest point count of any instance, and the post-processing time with and
without the fill (events).  Debug tool."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

from vision_assist_amd import _lib  # noqa: E402

lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), "libva355_ctcheck.so"))
lib.va_contour_fill_prof.restype = ctypes.c_int
lib.va_contour_fill_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]


def main():
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    scale = sys.argv[1] if len(sys.argv) > 1 else "s"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    arch = Arch(scale)
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, cls_bias=4.0)), B, 640, 640,
                         dtype=dtype)
    frames = torch.randint(0, 256, (B, 640, 640, 3), generator=torch.Generator().manual_seed(1), dtype=torch.uint8)
    pipe.load(frames.cuda())
    for _ in range(2):
        pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.synchronize()
    ch = pipe.post.chosen.cpu().numpy()
    fp = np.zeros((1024, 8), np.uint64)
    _lib.check(lib.va_contour_fill_prof(fp.ctypes.data, 1024), "va_contour_fill_prof")
    out = {"frames": []}
    for b in range(B):
        cs = pipe.post.contour_stats(b)
        k = int(ch[b])
        out["frames"].append({"chosen": k, "npts": int(cs["npts"][k]) if k >= 0 else None,
                              "ncont": int(cs["ncont"][k]) if k >= 0 else None,
                              "max_npts": int(cs["npts"].max()), "sum_ncont": int(cs["ncont"].sum()),
                              "over_1024": int((cs["npts"] > 1024).sum()),
                              "fill_cycles(choose+pts, edges, fill)": [int(v) for v in fp[b, :3]],
                              "fill_n": int(fp[b, 3]), "fallback": int(fp[b, 4])})
    fr = out["frames"]
    tot = [sum(f["fill_cycles(choose+pts, edges, fill)"]) for f in fr]
    order = np.argsort(tot)[::-1]
    print(json.dumps({"n_frames": B, "fallbacks": sum(f["fallback"] for f in fr),
                      "fill_cycles_max": int(max(tot)), "fill_cycles_median": float(np.median(tot)),
                      "slowest": [fr[i] for i in order[:6]]}, indent=1))


if __name__ == "__main__":
    main()

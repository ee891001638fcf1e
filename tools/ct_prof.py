"""Per-detection phase clocks of the contour kernel (libva355_ctcheck.so, `make ctcheck`): YOLOv8n-seg synthetic
weights, one 640 x 640 frame, 300 detections; prints the slowest detections' build / scan / area cycles, contour
and row / position counts.  Debug tool."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_assist_amd import _lib  # noqa: E402

lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), "libva355_ctcheck.so"))
lib.va_contour_prof.restype = ctypes.c_int
lib.va_contour_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]


def main():
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(sys.argv[1] if len(sys.argv) > 1 else "n")
    if len(sys.argv) > 2 and sys.argv[2] == "sparse":  # the bench's headline regime (bench.regime_kwargs)
        from bench import regime_kwargs
        kw = regime_kwargs("sparse", 640)
    else:
        bias = float(sys.argv[2]) if len(sys.argv) > 2 else None  # e.g. 4.0: the bench's dense regime
        solid = len(sys.argv) > 3 and sys.argv[3] == "box"         # the dense_box regime's solid box masks
        kw = dict(cls_bias=bias, solid_masks=solid)
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, **kw)), 1, 640, 640, dtype="bf16")
    frame = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(1), dtype=torch.uint8)
    pipe.load(frame.cuda())
    for _ in range(2):
        pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.synchronize()
    n = int(pipe.post.ndet[0])
    buf = np.zeros((4096, 8), np.uint64)
    _lib.check(lib.va_contour_prof(buf.ctypes.data, 4096), "va_contour_prof")
    p = buf[:n].astype(np.int64)
    order = np.argsort(-(p[:, 0] + p[:, 1] + p[:, 2]))
    cols = ["build", "scan", "area", "ncont", "rows", "positions", "steps", "trace_cycles"]
    cs = pipe.post.contour_stats(0)
    st = pipe.post.stats[0, :n].cpu().numpy()
    out = {"ndet": n, "sum_cycles": [int(v) for v in p[:, :3].sum(0)], "slowest": [],
           "mask_pixels_median": float(np.median(st[:, 0])), "npts_median": float(np.median(cs["npts"])),
           "bbox_w_median": float(np.median(st[:, 3] - st[:, 1] + 1)), "bbox_h_median": float(np.median(st[:, 4] - st[:, 2] + 1))}
    for i in order[:12]:
        out["slowest"].append({c: int(p[i, j]) for j, c in enumerate(cols)})
    out["median"] = {c: float(np.median(p[:, j])) for j, c in enumerate(cols)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

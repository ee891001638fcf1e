"""Calibrates the 'sparse' synthetic regime (seg_arch.SPARSE_THRESHOLDS): per head level, the class-0 logit
(bias 0, solid masks) exceeded on average by one anchor per frame of seeded uniform-noise frames, so that with
the class-0 weights scaled by SPARSE_GAIN and bias -gain * threshold a frame keeps ~1-5 detections (one live
class, compact box masks) -- what a trained model's few-object frames feed FrameProcessor.py:67-97.
Run on the CPU with the oracle forward; prints the table entries.  Usage: python tools/sparse_calib.py s 640"""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle import yolo_ref as Y  # noqa: E402
from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict  # noqa: E402


def calibrate(scale: str, res: int, seed: int = 0, nframes: int = 16, per_level: float = 1.0):
    arch = Arch(scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=seed, cls_bias=0.0, solid_masks=True))
    # calibration frames of their own seed (not any test's or bench's frames: a threshold equal to a test frame's
    # logit would put that anchor exactly at the conf threshold)
    fr = torch.randint(0, 256, (nframes, res, res, 3), generator=torch.Generator().manual_seed(99991), dtype=torch.uint8)
    c0 = []
    with torch.no_grad():
        for i in range(0, nframes, 4):
            c0.append(Y.forward(arch, fw, Y.preprocess(fr[i:i + 4]))[1][:, 0, :].numpy())
    c0 = np.concatenate(c0)
    out, lo = [], 0
    for s in (8, 16, 32):
        n = (res // s) ** 2
        v = np.sort(c0[:, lo:lo + n].ravel())[::-1]
        k = int(per_level * nframes)
        out.append(round(float(v[k - 1] + v[k]) / 2, 6))  # between two calibration logits
        lo += n
    return tuple(out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    sc, rs = sys.argv[1], int(sys.argv[2])
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    print(f'("{sc}", {rs}, 0): {calibrate(sc, rs, nframes=nf)},')

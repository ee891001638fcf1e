"""Conditioning of a synthetic YOLOv8-seg network on the CPU oracle forward: per conv, the output's RMS and the
share of it that varies across positions (per channel, the std over batch x H x W, RMS over channels, divided by
the output RMS).  A deep random network whose ratio decays toward 0 has collapsed: every anchor sees nearly the
same features, so its head outputs differ between anchors by far less than a low-precision forward's error.
    python tools/m_condition.py m 1280 [--frames 1] [--seed 0] [--real]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scale")
    ap.add_argument("res", type=int)
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--real", action="store_true", help="2 x 2 mosaics of the reference's validation frames")
    ap.add_argument("--kw", default="{}", help="synthetic_state_dict keywords (JSON)")
    a = ap.parse_args()
    from oracle import yolo_ref as Y
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    torch.set_num_threads(8)
    arch = Arch(a.scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=a.seed, **json.loads(a.kw)))
    if a.real:
        import numpy as np

        from tests.chain_util import mosaic_1280, real_frames
        fr = torch.from_numpy(mosaic_1280(real_frames(4 * a.frames)) if a.res == 1280 else real_frames(a.frames))
    else:
        fr = torch.randint(0, 256, (a.frames, a.res, a.res, 3), generator=torch.Generator().manual_seed(5),
                           dtype=torch.uint8)
    names = {id(v[0]): k for k, v in fw.items()}
    rows = []
    real_conv = F.conv2d

    def conv2d(x, w, b=None, stride=1, padding=0, *args):
        y = real_conv(x, w, b, stride, padding, *args)
        rms = float(y.pow(2).mean().sqrt())
        sp = float(y.std(dim=(0, 2, 3)).pow(2).mean().sqrt())
        rows.append({"name": names.get(id(w), "?"), "rms": round(rms, 4), "spatial": round(sp / max(rms, 1e-30), 6),
                     "mean": round(float(y.mean()), 4), "amax": round(float(y.abs().max()), 4)})
        return y

    F.conv2d = conv2d
    try:
        with torch.no_grad():
            box, cls, coef, proto = Y.forward(arch, fw, Y.preprocess(fr))
    finally:
        F.conv2d = real_conv
    for r in rows:
        print(json.dumps(r))
    c0 = cls[:, 0]
    print(json.dumps({"cls0": {"mean": round(float(c0.mean()), 4), "std": round(float(c0.std()), 6),
                               "max": round(float(c0.max()), 4)}}))


if __name__ == "__main__":
    main()

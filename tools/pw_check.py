"""Same-box check of the streaming 1x1 kernel (va_pw.hip) inside whole forwards at bench batch sizes:
repeated forwards must be bit-identical and finite, and the forward with VA_PW=0 (those layers on conv2)
must agree within bf16 rounding; prints the count of anchors whose best class logit passes conf 0.5.
    python tools/pw_check.py [--batch 64,256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vision_assist_amd import _lib  # noqa: E402
from vision_assist_amd.seg import SegNet  # noqa: E402
from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict  # noqa: E402


def heads(net, frames):
    out = net.forward(frames)
    torch.cuda.synchronize()
    lv = torch.cat([t.float().flatten(1, 2) for t in out.levels], 1)
    return lv, out.proto.float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="64,256")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    arch = Arch("s")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    net = SegNet(arch, fw, dtype="bf16")
    for B in [int(b) for b in args.batch.split(",")]:
        frames = torch.randint(0, 256, (B, 640, 640, 3), generator=torch.Generator().manual_seed(B),
                               dtype=torch.uint8).cuda()
        os.environ["VA_PW"] = "1"
        _lib.reload_switches()
        first = heads(net, frames)
        bad = 0
        for _ in range(args.reps):
            again = heads(net, frames)
            for g, r in zip(again, first):
                if not torch.equal(g, r):
                    bad += 1
        nonfin = [int((~torch.isfinite(t)).sum()) for t in first]
        os.environ["VA_PW"] = "0"
        _lib.reload_switches()
        ref = heads(net, frames)
        os.environ["VA_PW"] = "1"
        _lib.reload_switches()
        d = [((g - r).abs().max() / r.abs().max()).item() for g, r in zip(first, ref)]
        cls = lambda lv: int((lv[..., 64:64 + arch.nc].amax(-1) > 0).sum())  # noqa: E731
        print(f"B={B}: run-to-run mismatches {bad}, non-finite {nonfin}, pw vs conv2 rel max diff {d}, "
              f"anchors conf>0.5: pw {cls(first[0])} conv2 {cls(ref[0])}", flush=True)


if __name__ == "__main__":
    main()

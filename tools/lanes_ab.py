"""A/B of the laned small-batch list (va355.h VA_OP_FORK): seg forward time per batch, lanes on / off.
python tools/lanes_ab.py [--scale s] [--dtypes f32,bf16] [--batches 1,2,4,8,16] -> one JSON line per row."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--batches", default="1,2,4,8,16")
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    s = torch.cuda.Stream()
    for dtype in a.dtypes.split(","):
        net = SegNet(arch, fw, dtype=dtype)
        net.lanes_max_b = 1 << 20
        for B in [int(x) for x in a.batches.split(",")]:
            frames = torch.randint(0, 256, (B, a.res, a.res, 3), dtype=torch.uint8, device="cuda")
            row = {"dtype": dtype, "scale": a.scale, "B": B}
            for lanes in (False, True):
                net.lanes = lanes
                net._plans.clear()
                p = net.plan(B, a.res, a.res)
                p["frames"].copy_(frames)
                with torch.cuda.stream(s):
                    for _ in range(5):
                        net.run_plan(p, s)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(a.iters):
                        net.run_plan(p, s)
                    e1.record(s)
                e1.synchronize()
                row["lanes" if lanes else "serial"] = round(e0.elapsed_time(e1) * 1000 / a.iters, 1)
            row["saving_us"] = round(row["serial"] - row["lanes"], 1)
            print(json.dumps(row), flush=True)
            net._plans.clear()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Which batch-1 f32 C2f blocks pay as one va_seg_c2fb launch, block by block: the s-seg f32 batch-1 forward (lanes as
the drop-in plans them) with the planner's fused blocks against the same plan with one block (or several) left as its
layers (SegNet.c2fb_tile[i] = 0), forwards interleaved round by round, HIP events per forward.  Diagnostic only.
    python tools/c2fb_b1_blocks.py [--variants "4;12;15;18;12,18;4,12,15,18"]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="4;12;15;18;12,18;4,15;4,12,15,18")
    a = ap.parse_args()
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    frames = torch.randint(0, 256, (1, 640, 640, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(3))
    nets, plans = {}, {}
    for v in ["default"] + a.variants.split(";"):
        net = SegNet(arch, fw, dtype="f32")
        if v != "default":
            net.c2fb_tile = {int(i): 0 for i in v.split(",")}
        p = net.plan(1, 640, 640)
        p["frames"].copy_(frames)
        nets[v], plans[v] = net, p
        print(v, [m["name"] for m in p["meta"] if "fused C2f" in m["name"]], flush=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: [] for v in nets}
    for r in range(a.rounds + 1):
        for v, net in nets.items():
            for _ in range(2):
                net.run_plan(plans[v])
            torch.cuda.synchronize()
            for _ in range(a.iters):
                ev0.record()
                net.run_plan(plans[v])
                ev1.record()
                ev1.synchronize()
                if r:
                    times[v].append(ev0.elapsed_time(ev1) * 1e3)
    for v, t in times.items():
        print(json.dumps({"unfused": v, "median_us": round(float(np.median(t)), 1),
                          "p10_us": round(float(np.percentile(t, 10)), 1), "n": len(t)}), flush=True)


if __name__ == "__main__":
    main()

"""Batch-1 forward latency across split-K settings (the library's VA_SPLITK / VA_SPLITK_KS switches, re-read in
process): the same plan (lanes as the drop-in call plans them) run eagerly, synchronised per forward, settings
interleaved round by round; one JSON line per setting with the median and p10 in us.  Diagnostic only.
    python tools/splitk_sweep.py --scale s --dtype f32 [--settings "default,ticket,0,ks:4,ks:8,ks:16,ks:32"]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply(setting: str) -> None:
    for k in ("VA_SPLITK", "VA_SPLITK_KS", "VA_CONV3T"):
        os.environ.pop(k, None)
    if setting.startswith("env:"):  # env:NAME=VALUE (a library switch)
        k, v = setting[4:].split("=", 1)
        os.environ[k] = v
    elif setting == "ticket":
        os.environ["VA_SPLITK"] = "ticket"
    elif setting == "0":
        os.environ["VA_SPLITK"] = "0"
    elif setting.startswith("ks:"):
        os.environ["VA_SPLITK_KS"] = setting[3:]
    elif setting.startswith("ticket:"):
        os.environ["VA_SPLITK"] = "ticket"
        os.environ["VA_SPLITK_KS"] = setting[7:]
    from vision_assist_amd import _lib
    _lib.reload_switches()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=25)
    ap.add_argument("--settings", default="default,ticket,0,ks:4,ks:8,ks:12,ks:16,ks:24,ks:32")
    a = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype=a.dtype)
    plan = net.plan(1, a.res, a.res)
    plan["frames"].copy_(torch.randint(0, 256, plan["frames"].shape, dtype=torch.uint8))
    _lib.load()
    settings = a.settings.split(",")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {s: [] for s in settings}
    for _ in range(a.rounds):
        for s in settings:
            apply(s)
            for _ in range(3):
                net.run_plan(plan)
            torch.cuda.synchronize()
            for _ in range(a.iters):
                ev0.record()
                net.run_plan(plan)
                ev1.record()
                ev1.synchronize()
                times[s].append(ev0.elapsed_time(ev1) * 1e3)
    apply("default")
    for s in settings:
        t = np.array(times[s])
        print(json.dumps({"scale": a.scale, "dtype": a.dtype, "setting": s, "median_us": round(float(np.median(t)), 1),
                          "p10_us": round(float(np.percentile(t, 10)), 1), "n": len(t)}), flush=True)


if __name__ == "__main__":
    main()

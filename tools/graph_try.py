"""Experiment: HIP-graph capture of the batch-1 network alone (torch.cuda.CUDAGraph around va_seg_run),
replayed and checked bit-for-bit against the eager forward, then timed.  python tools/graph_try.py [--scale n]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="n")
    args = ap.parse_args()
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(args.scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype="bf16")
    plan = net.plan(1, 640, 640)
    plan["frames"].copy_(torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(2),
                                       dtype=torch.uint8).cuda())
    net.run_plan(plan)
    torch.cuda.synchronize()
    ref = [t.clone() for t in plan["out"].levels] + [plan["out"].proto.clone()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            net.run_plan(plan)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        net.run_plan(plan)
    torch.cuda.synchronize()
    print("captured", flush=True)
    for t in plan["out"].levels:
        t.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in plan["out"].levels] + [plan["out"].proto.clone()]
    same = all(torch.equal(a, b) for a, b in zip(got, ref))
    out = {"graph_equals_eager": same}
    for name, fn in (("eager", lambda: net.run_plan(plan)), ("graph", g.replay)):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_median_ms"] = round(float(np.median(np.array(ts) * 1e3)), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

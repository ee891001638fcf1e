"""Diagnosis: HIP-graph capture of network + post-processing (seg_post of one FramePipeline), replayed once and
compared bit-for-bit with the eager run.  Prints a JSON line.  Run alone under a time limit:
    timeout -k 10 120 python tools/graph_post.py [--scale n] [--dtype bf16] [--batch 1] [--regime dense]"""
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
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--regime", default="dense")
    ap.add_argument("--time", action="store_true")
    args = ap.parse_args()
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(args.scale)
    bias = {"natural": None, "mid": 0.0, "dense": 4.0}[args.regime]
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, cls_bias=bias)), args.batch, 640, 640,
                         dtype=args.dtype)
    pipe.frames.copy_(torch.randint(0, 256, pipe.frames.shape, generator=torch.Generator().manual_seed(2),
                                    dtype=torch.uint8).cuda())
    outs = lambda: [pipe.post.ndet, pipe.post.dets, pipe.post.stats, pipe.post.cells, pipe.post.rects,  # noqa: E731
                    pipe.post.chosen, pipe.plan["out"].proto] + list(pipe.plan["out"].levels)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = [t.clone() for t in outs()]
    print(json.dumps({"eager_ndet": pipe.post.ndet.tolist()}), flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.synchronize()
    print("captured", flush=True)
    for t in outs():
        t.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("replayed", flush=True)
    same = [bool(torch.equal(a, b)) for a, b in zip(outs(), ref)]
    res = {"graph_equals_eager": all(same), "per_output": same}
    if args.time:
        for name, fn in (("eager", lambda: pipe.seg_post(plant_mode=PLANT_NEVER)), ("graph", g.replay)):
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(200):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            res[name + "_median_ms"] = round(float(np.median(np.array(ts) * 1e3)), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

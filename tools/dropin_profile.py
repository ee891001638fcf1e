#!/usr/bin/env python
"""Where FrameProcessor.__call__'s time goes (bench.py's dropin extra): cProfile of N calls on the sparse regime
(host side: H2D staging, the va_frame call, result read-back, Path construction, PathAnalyser), plus the same
calls with the device pipeline alone (pipe.run + read-back) for the split.  Prints the top functions by
cumulative time and one JSON line.   python tools/dropin_profile.py [--calls 200]"""
import argparse
import contextlib
import cProfile
import io
import json
import os
import pstats
import sys
import time
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--dtype", default="f32")
    args = ap.parse_args()
    from bench import regime_kwargs
    from vision_assist_amd.FrameProcessor import FrameProcessor
    from vision_assist_amd.yolo import YOLO
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = YOLO("yolov8s-seg.pt", dtype=args.dtype, **regime_kwargs("sparse", 640)).to("cuda")
    fp = FrameProcessor(model=model, verbose=False, debug=False)
    fp.model = model
    rng = np.random.default_rng(77)
    frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    out = {}
    with contextlib.redirect_stdout(io.StringIO()):
        for i in range(10):
            fp(frames[i % 16])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.calls):
            fp(frames[i % 16])
        out["call_ms"] = round(1e3 * (time.perf_counter() - t0) / args.calls, 4)
        pipe = fp._pipe(640, 640)
        t0 = time.perf_counter()
        for i in range(args.calls):
            t = torch.as_tensor(frames[i % 16])
            b = pipe.run(t.reshape(1, 640, 640, 3))
            b.frame(0)
        out["pipe_run_ms"] = round(1e3 * (time.perf_counter() - t0) / args.calls, 4)
        pr = cProfile.Profile()
        pr.enable()
        for i in range(args.calls):
            fp(frames[i % 16])
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
    print(s.getvalue())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

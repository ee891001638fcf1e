#!/usr/bin/env python
"""Stage clocks of every va_seg_c2fb op of a batch-1 plan (va_c2fb_trace: thread 0's s_memtime at the start and after
each stage's barrier), one op at a time after a full forward has filled its inputs: per stage the median over
workgroups of its cycles, the slowest workgroup's total, and the op's event time.  Run on the GPU box:
    python tools/c2fb_stages.py --scale n --dtype bf16        (C2's plan)
    python tools/c2fb_stages.py --scale s --dtype f32         (the opt-in f32 form)"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGES = ["stage-in", "prologue", "cv1", "m0.cv1", "m0.cv2", "m1.cv1", "m1.cv2", "-", "cv2(end)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="n")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    net = S.SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype=a.dtype, c2fb_f32=True)
    net.c2fb_max_b = max(net.c2fb_max_b, a.batch)
    plan = net.plan(a.batch, 640, 640, lanes=False)
    plan["frames"].copy_(torch.randint(0, 256, plan["frames"].shape, dtype=torch.uint8))
    net.run_plan(plan)
    torch.cuda.synchronize()
    lib = _lib.load()
    st = torch.cuda.current_stream()
    out = []
    for i in range(plan["n"]):
        op = plan["ops"][i]
        if op.kind != S.VA_OP_C2F or op.a.mode != 3:
            continue
        ar = op.a
        T = ar.stride
        grid = ar.N * -(-ar.H // T) * -(-ar.W // T)
        buf = torch.zeros(grid * 10, dtype=torch.int64, device="cuda")
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):  # warm
            _lib.check(lib.va_seg_c2fb(_lib.stream_ptr(), ctypes.byref(ar)), "va_seg_c2fb")
        ev0.record()
        for _ in range(10):
            _lib.check(lib.va_seg_c2fb(_lib.stream_ptr(), ctypes.byref(ar)), "va_seg_c2fb")
        ev1.record()
        torch.cuda.synchronize()
        us = ev0.elapsed_time(ev1) * 100.0
        _lib.check(lib.va_c2fb_trace(ctypes.c_void_p(buf.data_ptr())), "va_c2fb_trace")
        _lib.check(lib.va_seg_c2fb(_lib.stream_ptr(), ctypes.byref(ar)), "va_seg_c2fb")
        torch.cuda.synchronize()
        _lib.check(lib.va_c2fb_trace(None), "va_c2fb_trace")
        t = buf.view(grid, 10).cpu().numpy().astype(np.int64)
        pts = [p for p in range(10) if (t[:, p] != 0).all()]
        rows = {}
        for p0, p1 in zip(pts, pts[1:]):
            d = t[:, p1] - t[:, p0]
            rows[f"{p0}->{p1}"] = int(np.median(d))
        tot = t[:, pts[-1]] - t[:, pts[0]]
        start_spread = int(t[:, 0].max() - t[:, 0].min())
        name = plan["meta"][i]["name"]
        rec = {"op": name, "grid": grid, "event_us": round(us, 2), "stage_median_cycles": rows,
               "wg_total_median": int(np.median(tot)), "wg_total_max": int(tot.max()),
               "start_spread_cycles": start_spread}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""Where a batch-1 conv2_kernel launch spends its time: every conv op of one forward's plan run ALONE (its
args from the plan, split-K workspace included) on the phase-clock build (`make -C vision_assist_amd/csrc
stamps` -> libva355_stamps.so, -DVA_CONV2_STAMPS), and per workgroup the shader-clock spans
  prologue (start -> first stage landed), K-loop, split-K slab + arrival, combine (last slice), epilogue,
plus the clock (cycles / real time).  One JSON line per conv2 op: medians over workgroups and the slowest one;
ops on other kernels are listed without phases.  Diagnostic only.
    VA355_LIB=vision_assist_amd/libva355_stamps.so python tools/conv2_phases.py --scale s --dtype f32 --batch 1"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("VA355_LIB", os.path.join(REPO, "vision_assist_amd", "libva355_stamps.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="s")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--plan-ab", default="", help="planner switch NAME: each op also run from the NAME=0 plan (same "
                                                 "op index), e.g. VA_W8 for w8a16's e4m3 bytes vs bf16 weights")
    ap.add_argument("--only", default="", help="comma list of op-name prefixes to run (default: every conv op)")
    a = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import VA_OP_CONV, SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype=a.dtype)
    plan = net.plan(a.batch, a.res, a.res)
    plan["frames"].copy_(torch.randint(0, 256, plan["frames"].shape, dtype=torch.uint8))
    plans = [("default", plan)]
    if a.plan_ab:
        os.environ[a.plan_ab] = "0"
        p0 = net.plan(a.batch, a.res, a.res, tag=7)
        del os.environ[a.plan_ab]
        p0["frames"].copy_(plan["frames"])
        net.run_plan(p0)
        plans.append((f"{a.plan_ab}=0", p0))
    for _ in range(3):
        net.run_plan(plan)
    torch.cuda.synchronize()
    lib = _lib.load()
    lib.va_conv2_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.va_conv2_stamps.restype = ctypes.c_int
    nb, npt = 4096, 8
    buf = (ctypes.c_ulonglong * (nb * npt))()
    st = _lib.stream_ptr()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    only = [x for x in a.only.split(",") if x]
    todo = [(tag, i, op, m) for i in range(plan["n"]) for tag, p_ in plans
            for op, m in [(p_["ops"][i], p_["meta"][i])]]
    for tag, i, op, m in todo:
        if op.kind != VA_OP_CONV or (only and not any(m["name"].startswith(o) for o in only)):
            continue
        spans, us = [], []
        for _ in range(a.reps):
            _lib.check(lib.va_conv2_stamps(None, 1), "va_conv2_stamps")
            ev0.record()
            _lib.check(lib.va_seg_conv(st, ctypes.byref(op.a)), "va_seg_conv")
            ev1.record()
            torch.cuda.synchronize()
            us.append(ev0.elapsed_time(ev1) * 1e3)
            _lib.check(lib.va_conv2_stamps(buf, 0), "va_conv2_stamps")
            s = np.frombuffer(buf, dtype=np.uint64).reshape(nb, npt).astype(np.int64)
            s = s[s[:, 0] != 0]
            if len(s):
                spans.append(s)
        row = {"i": i, "plan": tag, "name": m["name"], "event_us": round(float(np.median(us)), 2)}
        if spans:
            s = spans[-1]
            t0 = s[:, 0]
            clk = np.median((s[:, 5] - s[:, 0]) / np.maximum(s[:, 7] - s[:, 6], 1) / 10.0)  # GHz
            last = s[:, 4] != 0

            def med(x):
                return round(float(np.median(x)) / clk / 1e3, 2) if len(x) else None
            row.update({"blocks": int(len(s)), "clock_ghz": round(float(clk), 3),
                        "prologue_us": med(s[:, 1] - t0), "kloop_us": med(s[:, 2] - s[:, 1]),
                        "slab_arrive_us": med(s[~last, 3] - s[~last, 2]) if (~last).any() else None,
                        "combine_us": med(s[last, 4] - s[last, 3]) if last.any() and (s[last, 3] != 0).any() else None,
                        "epilogue_us": med(s[last, 5] - s[last, 4]) if last.any() else None,
                        "block_us_med": med(s[:, 5] - t0), "block_us_max": round(float((s[:, 5] - t0).max()) / clk / 1e3, 2),
                        "start_spread_us": round(float(t0.max() - t0.min()) / clk / 1e3, 2)})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

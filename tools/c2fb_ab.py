#!/usr/bin/env python
"""Batch-1 n-seg bf16 forward (C2's seg kernels) with the C2f blocks fused (va_seg_c2fb) or not, and with tile-side
choices, timed the way bench.c2_latency times its seg_only leg (one plan per frame on a stream of its own, synchronised
per frame, median over iters), the variants interleaved in rounds in one process; then per-op event times of the
fused blocks (va_prof, ops serialised).  Run on the GPU box:  python tools/c2fb_ab.py [--batch 1] [--rounds 5]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--scale", default="n")
    ap.add_argument("--dtype", default="bf16", help="bf16 (C2) or f32 (the drop-in call's network)")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-tiles", default="32,96,256", help="C2FB_MIN_TILES values to compare")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(a.scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B = a.batch
    frames = torch.randint(0, 256, (B, 640, 640, 3), generator=torch.Generator().manual_seed(1),
                           dtype=torch.uint8).cuda()
    variants = {}
    off = S.SegNet(arch, fw, dtype=a.dtype)
    off.c2fb_max_b = 0
    variants["unfused"] = off
    for mt in [int(v) for v in a.min_tiles.split(",") if v]:
        S.C2FB_MIN_TILES = mt
        net = S.SegNet(arch, fw, dtype=a.dtype, c2fb_f32=True)
        net.c2fb_max_b = B
        plan = net.plan(B, 640, 640)  # tile sides are chosen at planning time
        variants[f"c2fb_min{mt}"] = net
        print(mt, [m["name"] for m in plan["meta"] if "fused C2f" in m["name"]], flush=True)
    st = torch.cuda.Stream()
    plans = {}
    for k, net in variants.items():
        p = net.plan(B, 640, 640)
        p["frames"].copy_(frames)
        plans[k] = p
        with torch.cuda.stream(st):
            for _ in range(20):
                net.run_plan(p, stream=st)
        st.synchronize()
    res = {k: [] for k in variants}
    for r in range(a.rounds):
        for k, net in variants.items():
            p = plans[k]
            ts = []
            with torch.cuda.stream(st):
                for _ in range(a.iters):
                    t0 = time.perf_counter()
                    net.run_plan(p, stream=st)
                    st.synchronize()
                    ts.append(time.perf_counter() - t0)
            res[k].append(float(np.median(ts) * 1e3))
        print(f"round {r}: " + ", ".join(f"{k} {v[-1]:.4f} ms" for k, v in res.items()), flush=True)
    summary = {k: {"median_ms": round(float(np.median(v)), 4), "rounds": [round(x, 4) for x in v]} for k, v in res.items()}
    # per-op event times (ops serialised: va_prof ignores lanes)
    lib = _lib.load()
    ops = {}
    for k in variants:
        p, net = plans[k], variants[k]
        n = p["n"]
        _lib.check(lib.va_prof_start(n * 10 + 8), "va_prof_start")
        for _ in range(10):
            net.run_plan(p)
        ms = (ctypes.c_double * n)()
        lib.va_prof_stop_ops(ms, n)
        kinds = (ctypes.c_double * 8)()
        cnt = (ctypes.c_int64 * 8)()
        lib.va_prof_stop(kinds, cnt, 8)
        ops[k] = [(m["name"], round(ms[i] * 1e3 / 10, 2)) for i, m in enumerate(p["meta"]) if m["kind"] != "sync"]
        tot = sum(v for _, v in ops[k])
        print(f"{k}: {len(ops[k])} ops, serial sum {tot:.1f} us", flush=True)
        for nm, us in ops[k]:
            if "C2f" in nm or k == "unfused":
                print(f"   {nm:50s} {us:8.2f}")
    out = {"batch": B, "scale": a.scale, "dtype": a.dtype, "seg_only": summary, "ops_us": ops}
    print(json.dumps(summary))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""va_seg_c2fb at large batches: the f32 (or bf16) forward with chosen C2f blocks as one launch each (tile sides given
per block) against the default plan, rounds interleaved in one process (HIP events around whole forwards), then
per-op event times of the fused blocks.  The fused variants run with the stem's cv1 tail off (VA_STEM_TAIL=0: the
block's cv1 is part of the fused launch; --rest planner: the unlisted blocks as the planner takes them).  Run on
the GPU box:
    python tools/c2fb_big.py --batch 64 --blocks 2:8 --blocks 2:4"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BLOCKS = (2, 4, 6, 8, 12, 15, 18, 21)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--scale", default="s")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--blocks", action="append", default=[], help="variant: i:T[,i:T..] (fused blocks, tile sides)")
    ap.add_argument("--rest", default="off", choices=["off", "planner"],
                    help="blocks a variant does not list: unfused (off) or the planner's choice")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
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
    nets = {"default": S.SegNet(arch, fw, dtype=a.dtype)}
    for v in a.blocks:
        tiles = {int(p.split(":")[0]): int(p.split(":")[1]) for p in v.split(",")}
        os.environ["VA_STEM_TAIL"] = "0"
        net = S.SegNet(arch, fw, dtype=a.dtype, c2fb_f32=True)
        del os.environ["VA_STEM_TAIL"]
        net.c2fb_max_b = B
        net.c2fb_tile = dict(tiles) if a.rest == "planner" else {i: tiles.get(i, 0) for i in BLOCKS}
        nets["fused " + v] = net
    plans = {}
    for k, net in nets.items():
        p = net.plan(B, 640, 640)
        p["frames"].copy_(frames)
        plans[k] = p
        print(k, [m["name"] for m in p["meta"] if "fused C2f" in m["name"]], flush=True)
        for _ in range(2):
            net.run_plan(p)
    torch.cuda.synchronize()
    res = {k: [] for k in nets}
    for r in range(a.rounds):
        for k, net in nets.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                net.run_plan(plans[k])
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / a.iters)
        print(f"round {r}: " + ", ".join(f"{k} {v[-1]:.3f} ms" for k, v in res.items()), flush=True)
    summary = {k: round(float(np.median(v)), 4) for k, v in res.items()}
    # the fused plans' outputs against the default plan's (same weights, same frames)
    outs = {}
    for k, net in nets.items():
        o = net.forward(frames)
        torch.cuda.synchronize()
        outs[k] = [t.float().cpu() for t in o.levels] + [o.proto.float().cpu()]
    diff = {k: max((x - y).abs().max().item() for x, y in zip(outs[k], outs["default"])) for k in nets}
    lib = _lib.load()
    ops = {}
    for k, net in nets.items():
        p = plans[k]
        n = p["n"]
        _lib.check(lib.va_prof_start(n * 3 + 8), "va_prof_start")
        for _ in range(3):
            net.run_plan(p)
        ms = (ctypes.c_double * n)()
        lib.va_prof_stop_ops(ms, n)
        kinds = (ctypes.c_double * 8)()
        cnt = (ctypes.c_int64 * 8)()
        lib.va_prof_stop(kinds, cnt, 8)
        ops[k] = [(m["name"], round(ms[i] * 1e3 / 3, 1)) for i, m in enumerate(p["meta"]) if m["kind"] != "sync"]
        print(f"{k}: {len(ops[k])} ops, serial sum {sum(v for _, v in ops[k]):.1f} us", flush=True)
        for nm, us in ops[k]:
            if "model.2" in nm or "model.1" in nm or "fused" in nm or "stem" in nm:
                print(f"   {nm:50s} {us:9.1f}")
    out = {"batch": B, "scale": a.scale, "dtype": a.dtype, "forward_ms": summary, "max_abs_diff_vs_default": diff,
           "ops_us": ops}
    print(json.dumps({"forward_ms": summary, "max_abs_diff_vs_default": diff}))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

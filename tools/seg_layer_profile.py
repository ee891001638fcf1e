#!/usr/bin/env python
"""Per-layer timing of the YOLOv8-seg forward (HIP events around every op of va_seg_run).

Prints one line per op: name, GEMM shape, us, TFLOP/s, GB/s (algorithmic bytes: input
activations + weights + output), and a JSON summary at the end.  Used to pick what to
optimise in the conv kernel; run on the GPU box:
    python tools/seg_layer_profile.py --batch 64 --iters 10
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--scale", default="s")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--ab", default="", help="env switch NAME (or NAME:V0:V1): interleave rounds with NAME=0 and "
                                            "NAME=1 (or V0 / V1) (one process, cdna_hip_programming.md §5.4 rule 24)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VAL set before planning")
    ap.add_argument("--plan-ab", default="", help="planner switch NAME (NAME=0 vs unset): two plans (e.g. fusions "
                                                 "that change the op list), rounds interleaved, totals and per-op rows")
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(args.scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype=args.dtype)
    B, H = args.batch, args.res
    plan = net.plan(B, H, H)
    plan["frames"].copy_(torch.randint(0, 256, plan["frames"].shape, dtype=torch.uint8))
    for _ in range(3):
        net.run_plan(plan)
    torch.cuda.synchronize()
    lib = _lib.load()
    n = plan["n"]

    def timed(iters):
        _lib.check(lib.va_prof_start(n * iters + 8), "va_prof_start")
        for _ in range(iters):
            net.run_plan(plan)
        ms = (ctypes.c_double * n)()
        lib.va_prof_stop_ops(ms, n)
        kinds = (ctypes.c_double * 8)()
        cnt = (ctypes.c_int64 * 8)()
        lib.va_prof_stop(kinds, cnt, 8)
        return list(ms)

    if args.plan_ab:
        name = args.plan_ab
        os.environ[name] = "0"
        plan0 = net.plan(B, H, H, tag=7)
        del os.environ[name]
        plans = {f"{name}=0": plan0, "default": plan}
        for p_ in plans.values():
            p_["frames"].copy_(plan["frames"])
            net.run_plan(p_)
        tot = {k: [0.0] * p_["n"] for k, p_ in plans.items()}
        for rnd in range(args.iters):
            for k, p_ in plans.items():
                net.run_plan(p_)
                _lib.check(lib.va_prof_start(p_["n"] + 8), "va_prof_start")
                net.run_plan(p_)
                ms = (ctypes.c_double * p_["n"])()
                lib.va_prof_stop_ops(ms, p_["n"])
                kinds, cnt = (ctypes.c_double * 8)(), (ctypes.c_int64 * 8)()
                lib.va_prof_stop(kinds, cnt, 8)
                tot[k] = [a + b for a, b in zip(tot[k], ms)]
        for k, p_ in plans.items():
            for i, m in enumerate(p_["meta"]):
                print(json.dumps({"plan": k, "i": i, "name": m["name"], "us": round(1000 * tot[k][i] / args.iters, 2)}))
        print(json.dumps({"total_us": {k: round(1000 * sum(v) / args.iters, 1) for k, v in tot.items()}}))
        return
    if args.ab:
        name, v0, v1 = (args.ab.split(":") + ["0", "1"])[:3] if ":" in args.ab else (args.ab, "0", "1")
        tot = {v0: [0.0] * n, v1: [0.0] * n}
        for rnd in range(args.iters):
            for v in (v0, v1):
                os.environ[name] = v
                _lib.reload_switches()  # the library reads its switches once per process otherwise
                net.run_plan(plan)  # one untimed forward after the switch
                t = timed(1)
                tot[v] = [a + b for a, b in zip(tot[v], t)]
        for i, m in enumerate(plan["meta"]):
            a0, a1 = 1000 * tot[v0][i] / args.iters, 1000 * tot[v1][i] / args.iters
            print(json.dumps({"i": i, "name": m["name"], f"{name}={v0}": round(a0, 2), f"{name}={v1}": round(a1, 2),
                              "ratio": round(a1 / a0, 3) if a0 else None}))
        s0, s1 = 1000 * sum(tot[v0]) / args.iters, 1000 * sum(tot[v1]) / args.iters
        print(json.dumps({"total_us": {f"{name}={v0}": round(s0, 1), f"{name}={v1}": round(s1, 1)}}))
        return
    ms = timed(args.iters)
    rows = []
    tot = 0.0
    for i, m in enumerate(plan["meta"]):
        us = 1000.0 * ms[i] / args.iters
        tot += us
        r = {"i": i, "name": m["name"], "kind": m["kind"], "us": round(us, 2)}
        if m["kind"] == "conv":
            fl = m.get("flops", 2.0 * m["M"] * m["N"] * m["K"])
            r.update({"M": m["M"], "N": m["N"], "K": m["K"], "k": m["k"], "s": m["stride"],
                      "tflops": round(fl / (us * 1e-6) / 1e12, 1), "gbps": round(m["bytes"] / (us * 1e-6) / 1e9, 1)})
        rows.append(r)
        print(json.dumps(r))
    conv_us = sum(r["us"] for r in rows if r["kind"] == "conv")
    fl = sum(m.get("flops", 2.0 * m["M"] * m["N"] * m["K"]) for m in plan["meta"] if m["kind"] == "conv")
    summ = {"total_us": round(tot, 1), "conv_us": round(conv_us, 1), "conv_tflops": round(fl / (conv_us * 1e-6) / 1e12, 1),
            "batch": B, "res": H, "scale": args.scale}
    print(json.dumps(summ))
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"rows": rows, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()

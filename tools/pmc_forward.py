#!/usr/bin/env python
"""Forwards of the YOLOv8-seg plan for rocprofv3 PMC passes: writes the op names of the plan (one kernel
dispatch per op, in order) to <out>.json, then runs --fwd forwards.  tools/pmc_summary.py maps the dispatches
of the last forward back to these names.
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES ... -d gpurun_out/x -o run -- python3 tools/pmc_forward.py --dtype f32
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--scale", default="s")
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--fwd", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/pmc_plan")
    args = ap.parse_args()
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(args.scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype=args.dtype)
    plan = net.plan(args.batch, args.res, args.res)
    plan["frames"].copy_(torch.randint(0, 256, plan["frames"].shape, dtype=torch.uint8))
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out + ".json", "w") as f:
        json.dump({"dtype": args.dtype, "scale": args.scale, "res": args.res, "batch": args.batch, "fwd": args.fwd,
                   "ops": [{k: m.get(k) for k in ("name", "kind", "M", "N", "K", "flops", "bytes")}
                           for m in plan["meta"]]}, f, indent=1)
    for _ in range(args.fwd):
        net.run_plan(plan)
    torch.cuda.synchronize()
    print("forwards done", flush=True)


if __name__ == "__main__":
    main()

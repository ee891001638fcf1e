"""Interleaved A/B of two segmentation plans that differ by a plan-time environment switch (e.g. VA_FUSE_UP,
VA_STEM, VA_C2F): both plans are built in one process and their forwards alternate, timed with events.
python tools/plan_ab.py NAME [--batch 64] [--rounds 20] [--dtype bf16|f32]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s", 80)
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    nets, plans = {}, {}
    for v in ("0", "1"):
        os.environ[args.name] = v
        nets[v] = SegNet(arch, fw, dtype=args.dtype)
        plans[v] = nets[v].plan(args.batch, 640, 640)
        plans[v]["frames"].copy_(torch.randint(0, 256, plans[v]["frames"].shape, dtype=torch.uint8, device="cuda"))
    times = {"0": [], "1": []}
    for r in range(args.rounds + 2):
        for v in ("0", "1") if r % 2 == 0 else ("1", "0"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            nets[v].run_plan(plans[v])
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                times[v].append(e0.elapsed_time(e1) * 1e3)
    for v in ("0", "1"):
        t = sorted(times[v])
        print(f"{args.name}={v}: median {t[len(t) // 2]:.1f} us  min {t[0]:.1f} us  ({len(t)} forwards of {args.batch})")


if __name__ == "__main__":
    main()

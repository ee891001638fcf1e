"""Time va_seg_stem alone (preprocess + model.0 + model.1 of YOLOv8s-seg for B frames of 640 x 640).
python tools/stem_micro.py [--batch 64] [--iters 20]  (run under rocprofv3 for counters)"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s", 80)
    net = S.SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype="bf16")
    blob, bias = net.stem
    B, H = args.batch, 640
    fr = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device="cuda")
    y = torch.empty(B, H // 4, H // 4, 64, device="cuda", dtype=torch.bfloat16)
    a = S.ConvArgs(x=fr.data_ptr(), N=B, H=H, W=H, Cin=32, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                   y=y.data_ptr(), ldy=64, dtype=S.VA_DTYPE_BF16)
    lib = _lib.load()
    st = _lib.stream_ptr()
    for _ in range(3):
        _lib.check(lib.va_seg_stem(st, ctypes.byref(a)), "stem")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        lib.va_seg_stem(st, ctypes.byref(a))
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    byt = B * H * H * 3 + 2 * B * (H // 4) ** 2 * 64
    print(f"stem B={B}: {us:.1f} us/launch, {byt / us / 1e3:.0f} GB/s (in+out)")


if __name__ == "__main__":
    main()

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
    ap.add_argument("--trace", action="store_true", help="stage stamps of one launch (va_stem_trace)")
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
    if args.trace:
        G = 256
        tr = torch.zeros(G * 8 * 32 * 5, dtype=torch.int64, device="cuda")
        lib.va_stem_trace(ctypes.c_void_p(tr.data_ptr()))
        lib.va_seg_stem(st, ctypes.byref(a))
        torch.cuda.synchronize()
        lib.va_stem_trace(None)
        t = tr.view(G, 8, 32, 5).cpu().double() * 10.0  # ns
        ok = (t > 0).all(-1)
        d = t[..., 1:] - t[..., :-1]
        for j, nm in enumerate(["model.0", "barrier1", "model.1", "store+bar2"]):
            v = d[..., j][ok]
            print(f"{nm:10s} mean {v.mean():7.0f} ns  p50 {v.median():7.0f}  p90 {v.quantile(0.9):7.0f}")
        st0 = t[:, 0, 0, 0]
        nk = ok[:, 0, :].sum(1)
        en = t[torch.arange(G), 0, nk - 1, 4]
        base = st0.min()
        print(f"start skew ns: p50 {(st0 - base).median():.0f} max {(st0 - base).max():.0f}; "
              f"end ns: min {(en - base).min():.0f} p50 {(en - base).median():.0f} max {(en - base).max():.0f}; "
              f"tiles/wg {nk.float().mean():.1f}")
        print("model.0 by wave:", [round(d[:, w, :, 0][ok[:, w]].mean().item()) for w in range(8)])
        print("model.1 by wave:", [round(d[:, w, :, 2][ok[:, w]].mean().item()) for w in range(8)])
    byt = B * H * H * 3 + 2 * B * (H // 4) ** 2 * 64
    print(f"stem B={B}: {us:.1f} us/launch, {byt / us / 1e3:.0f} GB/s (in+out)")


if __name__ == "__main__":
    main()

"""Time va_seg_c2f alone (model.2 of YOLOv8s-seg at B frames of 640 x 640: 160 x 160 x 64 in/out).
python tools/c2f_micro.py [--batch 64] [--iters 20]  (run under rocprofv3 for counters)"""
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
    ap.add_argument("--hw", type=int, default=160)
    ap.add_argument("--trace", action="store_true", help="stage clocks of one launch (va_c2f_trace)")
    args = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s", 80)
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    net = S.SegNet(arch, fw, dtype="bf16")
    blob, bias = net.c2f_fused[2]
    B, H = args.batch, args.hw
    x = torch.randn(B, H, H, 64, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, H, H, 64, device="cuda", dtype=torch.bfloat16)
    a = S.ConvArgs(x=x.data_ptr(), N=B, H=H, W=H, Cin=64, ldx=64, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                   y=y.data_ptr(), ldy=64, dtype=S.VA_DTYPE_BF16)
    lib = _lib.load()
    st = _lib.stream_ptr()
    for _ in range(3):
        _lib.check(lib.va_seg_c2f(st, ctypes.byref(a)), "c2f")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        lib.va_seg_c2f(st, ctypes.byref(a))
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    if args.trace:
        cfg = int(os.environ.get("VA_C2F_CFG", "2"))
        NW, G = {0: (8, 256), 1: (16, 256), 2: (4, 512)}[cfg]
        tr = torch.zeros(G * NW * 32 * 6, dtype=torch.int64, device="cuda")
        lib.va_c2f_trace(ctypes.c_void_p(tr.data_ptr()))
        lib.va_seg_c2f(st, ctypes.byref(a))
        torch.cuda.synchronize()
        lib.va_c2f_trace(None)
        t = tr.view(G, NW, 32, 6).cpu().double()
        ok = (t > 0).all(-1)
        d = t[..., 1:] - t[..., :-1]  # stage 1, prefetch+barrier1, stage 2, barrier 2, stages 3-4
        names = ["stage1", "pf+bar1", "stage2", "bar2", "stage3+4"]
        for j, nm in enumerate(names):
            v = d[..., j][ok]
            print(f"{nm:10s} mean {v.mean():8.0f}  p50 {v.median():8.0f}  p90 {v.quantile(0.9):8.0f} clk")
        loop = (t[:, :, 1:, 0] - t[:, :, :-1, 0])[ok[:, :, 1:] & ok[:, :, :-1]]
        print(f"tile loop  mean {loop.mean():8.0f}  p50 {loop.median():8.0f} clk")
        # per wave id means of stage 2 (imbalance)
        # per workgroup: first stamp, last stamp (wave 0), skew across the grid
        st0 = t[:, 0, 0, 0]
        lastk = ok[:, 0, :].sum(1) - 1
        en = t[torch.arange(G), 0, lastk, 5]
        base = st0.min()
        dur = en - st0
        print(f"start skew: min 0 p50 {(st0 - base).median():.0f} p90 {(st0 - base).quantile(0.9):.0f} max {(st0 - base).max():.0f}")
        print(f"end: p10 {(en - base).quantile(0.1):.0f} p50 {(en - base).median():.0f} max {(en - base).max():.0f}")
        print(f"wg duration: p10 {dur.quantile(0.1):.0f} p50 {dur.median():.0f} max {dur.max():.0f}; tiles/wg {(lastk + 1).float().mean():.1f}")
        xcd = torch.arange(G) % 8
        print("wg duration by XCD:", [round(dur[xcd == x].mean().item()) for x in range(8)])
        print("wg duration max by XCD:", [round(dur[xcd == x].max().item()) for x in range(8)])
        slow = dur.argsort(descending=True)[:12].tolist()
        print("slowest wgs:", [(b, round(dur[b].item())) for b in slow])
        print("stage2 by wave:", [round(d[:, w, :, 2][ok[:, w]].mean().item()) for w in range(NW)])
        print("stage1 by wave:", [round(d[:, w, :, 0][ok[:, w]].mean().item()) for w in range(NW)])
        print("stage3+4 by wave:", [round(d[:, w, :, 4][ok[:, w]].mean().item()) for w in range(NW)])
    byt = 2 * B * H * H * 128
    print(f"c2f B={B} {H}x{H}: {us:.1f} us/launch, {byt / us / 1e3:.0f} GB/s (in+out)")


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""One conv layer shape, launched back to back through va_seg_conv: the unit under test for PMC passes
(every conv dispatch of the process is this layer) and for quick kernel A/B timing.

    python tools/conv_micro.py --cin 128 --cout 224 --k 3 --hw 80 --batch 64 --iters 50 [--env VA_CONV3=0]
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
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=224)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--hw", type=int, default=80)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--env", action="append", default=[])
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    lib = _lib.load()
    net = S.SegNet.__new__(S.SegNet)
    net.dtype, net.tdtype, net.va_dtype, net.vec = "bf16", torch.bfloat16, S.VA_DTYPE_BF16, 8
    net.device = torch.device("cuda")
    g = torch.Generator().manual_seed(1)
    w = torch.randn(args.cout, args.cin, args.k, args.k, generator=g) * (2.0 / (args.cin * args.k * args.k)) ** 0.5
    p = net._pack(w, torch.randn(args.cout, generator=g) * 0.1)
    B, H = args.batch, args.hw
    pad = args.k // 2
    Ho = (H + 2 * pad - args.k) // args.stride + 1
    x = (torch.rand(B, H, H, p.cin, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = torch.empty(B, Ho, Ho, args.cout, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=x.data_ptr(), N=B, H=H, W=H, Cin=p.cin, ldx=p.cin, kh=args.k, kw=args.k, stride=args.stride,
                   pad=pad, Ho=Ho, Wo=Ho, w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=args.cout, Npad=p.Npad, K=p.K,
                   Kpad=p.Kpad, y=y.data_ptr(), ldy=args.cout, act=1, mode=0, M=B * Ho * Ho, dtype=S.VA_DTYPE_BF16)
    st = _lib.stream_ptr()
    for _ in range(3):
        _lib.check(lib.va_seg_conv(st, ctypes.byref(a)), "va_seg_conv")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        lib.va_seg_conv(st, ctypes.byref(a))
    e1.record()
    torch.cuda.synchronize()
    us = 1000 * e0.elapsed_time(e1) / args.iters
    fl = 2.0 * B * Ho * Ho * args.cout * args.k * args.k * args.cin
    print(json.dumps({"shape": vars(args), "us": round(us, 2), "tflops": round(fl / us / 1e6, 1)}))


if __name__ == "__main__":
    main()

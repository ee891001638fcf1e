"""Debug helper: run one conv through va_seg.conv with structured weights/inputs and report where the output
differs from torch (channel / pixel mapping).  python tools/conv4_debug.py"""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    lib = _lib.load()
    net = S.SegNet.__new__(S.SegNet)
    net.dtype, net.tdtype, net.va_dtype, net.vec = "bf16", torch.bfloat16, S.VA_DTYPE_BF16, 8
    net.device = torch.device("cuda")
    cin, cout, k, B, H = 128, 256, 3, 1, 16
    w = torch.zeros(cout, cin, k, k)
    for co in range(cout):
        w[co, co % cin, 1, 1] = 1.0 + (co // cin)  # output co = input channel co % cin (x1 or x2)
    b = torch.zeros(cout)
    p = net._pack(w, b)
    x = torch.zeros(B, H, H, cin)
    for c in range(cin):
        x[..., c] = c / 8.0
    x[0, :, :, 0] = torch.arange(H * H).view(H, H).float() / 64.0  # channel 0 encodes the pixel
    xd = x.to(torch.bfloat16).cuda()
    y = torch.zeros(B, H, H, cout, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=xd.data_ptr(), N=B, H=H, W=H, Cin=cin, ldx=cin, kh=k, kw=k, stride=1, pad=1, Ho=H, Wo=H,
                   w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad,
                   y=y.data_ptr(), ldy=cout, act=0, mode=0, M=B * H * H, dtype=S.VA_DTYPE_BF16)
    _lib.check(lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)), "conv")
    torch.cuda.synchronize()
    ref = F.conv2d(xd.float().cpu().permute(0, 3, 1, 2), w, b, 1, 1).permute(0, 2, 3, 1)
    got = y.float().cpu()
    bad = (got - ref).abs() > 0.05 * (ref.abs() + 0.1)
    print("bad fraction", bad.float().mean().item())
    # channel mapping at pixel (0, 5, 7) (channel 0 there = pixel code)
    g, r = got[0, 5, 7], ref[0, 5, 7]
    print("got ch0..40:", [round(v, 3) for v in g[:40].tolist()])
    print("ref ch0..40:", [round(v, 3) for v in r[:40].tolist()])
    print("got ch0 over row 5:", [round(v, 2) for v in got[0, 5, :, 0].tolist()])
    print("ref ch0 over row 5:", [round(v, 2) for v in ref[0, 5, :, 0].tolist()])
    bc = bad[0].float().mean((0, 1))
    print("bad channels:", [i for i in range(cout) if bc[i] > 0][:80])
    bp = bad[0].float().mean(2)
    print("bad pixels (rows x cols):")
    for yy in range(H):
        print("".join("#" if bp[yy, xx] > 0 else "." for xx in range(H)))
    ch = [i for i in range(cout) if bc[i] > 0]
    if ch:
        c = ch[0]
        print("channel", c, "got row 0:", [round(v, 2) for v in got[0, 0, :, c].tolist()])
        print("channel", c, "ref row 0:", [round(v, 2) for v in ref[0, 0, :, c].tolist()])


if __name__ == "__main__":
    main()

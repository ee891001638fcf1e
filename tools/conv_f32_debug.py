"""Debug: a 1x1 f32 conv through va_seg_conv with one-hot inputs (pixel p has channel p % Cin set) and weights
W[c][k] = 1000 c + k, no bias / activation: out[p][c] should be 1000 c + p % Cin.  Prints the first mismatches."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    cin, cout, M = int(sys.argv[1]) if len(sys.argv) > 1 else 32, 64, 256
    x = torch.zeros(M, cin)
    x[torch.arange(M), torch.arange(M) % cin] = 1.0
    Kpad = (cin + 31) // 32 * 32
    w = torch.zeros(128, Kpad)
    for c in range(cout):
        w[c, :cin] = 1000.0 * c + torch.arange(cin)
    xd, wd = x.cuda().contiguous(), w.cuda().contiguous()
    bd = torch.zeros(128, device="cuda")
    y = torch.zeros(M, cout, device="cuda")
    a = S.ConvArgs(x=xd.data_ptr(), N=1, H=1, W=M, Cin=cin, ldx=cin, kh=1, kw=1, stride=1, pad=0, Ho=1, Wo=M,
                   w=wd.data_ptr(), bias=bd.data_ptr(), Cout=cout, Npad=128, K=cin, Kpad=Kpad, y=y.data_ptr(), ldy=cout,
                   act=0, mode=0, M=M, dtype=S.VA_DTYPE_F32)
    _lib.check(_lib.load().va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)), "conv")
    torch.cuda.synchronize()
    got = y.cpu()
    want = 1000.0 * torch.arange(cout)[None, :] + (torch.arange(M) % cin)[:, None]
    bad = (got != want).nonzero()
    print("mismatches", bad.shape[0], "of", M * cout)
    for p, c in bad[:24].tolist():
        print(p, c, float(got[p, c]), float(want[p, c]))


if __name__ == "__main__":
    main()

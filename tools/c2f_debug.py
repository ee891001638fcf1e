"""Debug helper for va_seg_c2f: error of the fused block vs the bf16-rounded fp32 reference, broken
down by pixel position inside the 16 x 16 tile and by channel.  python tools/c2f_debug.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_gpu_seg import _c2f_reference, _net
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    arch, fw, net = _net("bf16", "s")
    blob, bias = net.c2f_fused[2]
    B, H, W = [int(v) for v in os.environ.get('C2F_DBG_SHAPE', '2,64,64').split(',')]
    T = 8 if os.environ.get('VA_C2F_CFG', '2') == '2' else 16
    g = torch.Generator().manual_seed(1)
    xin = (torch.randn(B, H, W, 64, generator=g) * 1.5).to(torch.bfloat16)
    xd = xin.cuda()
    y = torch.zeros(B, H, W, 64, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=xd.data_ptr(), N=B, H=H, W=W, Cin=64, ldx=64, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                   y=y.data_ptr(), ldy=64, dtype=S.VA_DTYPE_BF16)
    _lib.check(_lib.load().va_seg_c2f(_lib.stream_ptr(), ctypes.byref(a)), "c2f")
    torch.cuda.synchronize()
    got = y.float().cpu()
    ref = _c2f_reference(xin.float().permute(0, 3, 1, 2), fw, 2).permute(0, 2, 3, 1)
    d = (got - ref).abs()
    print("rel", ((got - ref).norm() / ref.norm()).item(), "frac exact", (d == 0).float().mean().item())
    e = d.mean(-1)  # [B,H,W]
    yy = torch.arange(H) % T
    xx = torch.arange(W) % 16
    tab = torch.zeros(T, 16)
    for i in range(T):
        for j in range(16):
            tab[i, j] = e[:, yy == i][:, :, xx == j].mean()
    torch.set_printoptions(precision=4, linewidth=200)
    print("mean abs err by (y%16, x%16):\n", tab)
    print("by channel:", d.mean((0, 1, 2)))
    print("image border rows/cols:", e[:, 0].mean().item(), e[:, -1].mean().item(), e[:, :, 0].mean().item(),
          e[:, :, -1].mean().item(), "interior", e[:, 2:-2, 2:-2].mean().item())
    print("ref mean abs", ref.abs().mean().item())
    # per tile (tile index order of va_c2f: frame, tile row, tile column)
    th = T
    et = e.view(B, H // th, th, W // 16, 16).mean((2, 4)).reshape(-1)
    bad = (et > 0.05).nonzero().flatten().tolist()
    print("tiles", et.numel(), "bad tiles:", len(bad), bad[:40])


if __name__ == "__main__":
    main()

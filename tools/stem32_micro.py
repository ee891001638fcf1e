"""Time va_seg_stem_f32 alone (model.0 + model.1 of YOLOv8s-seg in f32 for B frames of 640 x 640), and the two
unfused launches it replaces (va_seg_conv0_f32m + model.1 on va_seg_conv) on the same frames.  With VA355_LIB set
to an ablation build (tools/build_variant.sh) the fused kernel's phases can be timed apart.
python tools/stem32_micro.py [--batch 64] [--iters 20]"""
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
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s", 80)
    net = S.SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=0)), dtype="f32")
    B, H = args.batch, 640
    fr = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device="cuda")
    y = torch.empty(B, H // 4, H // 4, 64, device="cuda")
    y0 = torch.empty(B, H // 2, H // 2, 32, device="cuda")
    p1 = net.w["model.1"]
    a = S.ConvArgs(x=fr.data_ptr(), N=B, H=H, W=H, Cin=32, Cout=64, w3=net.w0_3.data_ptr(), bias=net.w0[1].data_ptr(),
                   w=p1.w.data_ptr(), b2=p1.b.data_ptr(), Npad=p1.Npad, K=p1.K, Kpad=p1.Kpad, y=y.data_ptr(), ldy=64,
                   dtype=S.VA_DTYPE_F32)
    lib = _lib.load()
    st = _lib.stream_ptr()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return 1e3 * e0.elapsed_time(e1) / args.iters

    fused = timed(lambda: _lib.check(lib.va_seg_stem_f32(st, ctypes.byref(a)), "stem_f32"))
    conv0 = timed(lambda: _lib.check(lib.va_seg_conv0_f32m(st, ctypes.c_void_p(fr.data_ptr()), B, H, H,
                                                           ctypes.c_void_p(net.w0_3.data_ptr()),
                                                           ctypes.c_void_p(net.w0[1].data_ptr()), 32,
                                                           ctypes.c_void_p(y0.data_ptr()), 32), "conv0_f32m"))
    c = S.ConvArgs(x=y0.data_ptr(), N=B, H=H // 2, W=H // 2, Cin=32, ldx=32, kh=3, kw=3, stride=2, pad=1, Ho=H // 4,
                   Wo=H // 4, w=p1.w.data_ptr(), bias=p1.b.data_ptr(), Cout=64, Npad=p1.Npad, K=p1.K, Kpad=p1.Kpad,
                   y=y.data_ptr(), ldy=64, act=1, mode=0, M=B * (H // 4) ** 2, dtype=S.VA_DTYPE_F32,
                   w3=p1.w3.data_ptr() if p1.w3 is not None else None)
    m1 = timed(lambda: _lib.check(lib.va_seg_conv(st, ctypes.byref(c)), "model.1"))
    print(json.dumps({"batch": B, "fused_stem_f32_us": round(fused, 1), "conv0_f32m_us": round(conv0, 1),
                      "model1_us": round(m1, 1), "lib": os.environ.get("VA355_LIB", "libva355.so")}))


if __name__ == "__main__":
    main()

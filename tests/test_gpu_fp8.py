"""The fp8 convolution path (va_fp8.hip, BASELINE.json configs[4] "YOLOv8m-seg 1280x1280 fp8 MFMA weights").

* one conv op against torch on the SAME quantized operands (bf16 or e4m3 input, bf16 / float / e4m3 output, bf16
  or e4m3 residual -- the fp8 mode keeps its activations as e4m3 bytes): e4m3 weights with their per-channel scales as packed,
  the bf16 input scaled by a power of two, saturated to +-448 and rounded to e4m3 (torch.float8_e4m3fn), f32
  accumulation, then the dequant scale, bias, SiLU, residual -- the kernel differs only by summation order, its
  fast SiLU and the bf16 output rounding: within 2e-2 of the output's scale (3x3 / 1x1 / stride 2 / residual / channel slices /
  ConvTranspose / float output), which also pins the MFMA operand lane map;
* the YOLOv8m-seg 1280 x 1280 forward against the fp32 oracle: e4m3 keeps 3 mantissa bits, so the bar is a
  relative L2 error (stated per output below), not the f32 mode's 1e-3;
* the fused batch at 1280 with planted corridor masks: grid / A* bit-exact (the nav stage does not see the
  network's precision).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

FP8_L2 = {"box": 0.25, "cls": 0.25, "coef": 0.25, "proto": 0.25}  # relative L2 vs the fp32 oracle (measured 0.15-0.20)


def _e4m3(t: torch.Tensor, s: float) -> torch.Tensor:
    """sat(t * s) as e4m3 bytes (uint8), round to nearest even."""
    from vision_assist_amd import seg as S
    return (t.float() * s).clamp(-S.F8_MAX, S.F8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)


def _pow2_scale(amax: float) -> float:
    from vision_assist_amd import seg as S
    return 2.0 ** np.floor(np.log2(S.F8_MAX / amax))


def _conv8(cin, cout, k, stride, H, W, residual=False, deconv=False, slice_in=0, out_f32=False, act=True,
           x8=False, y8=False, r8=False):
    """One va_seg_conv fp8 op and its reference.  x8 / y8 / r8: input / output / residual as e4m3 bytes (the fp8
    mode's activation buffers); y8 returns (got, ref) both scaled by the output scale (e4m3 units)."""
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch
    g = torch.Generator().manual_seed(cin * 1000 + cout + k + 7 * stride)
    B = 2
    if deconv:
        w = torch.randn(cin, cout, 2, 2, generator=g) * 0.2
    else:
        w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(B, cin, H, W, generator=g) * 1.7
    net = S.SegNet.__new__(S.SegNet)
    net.arch, net.dtype, net.device = Arch("n"), "fp8", torch.device("cuda")
    net.tdtype, net.va_dtype, net.vec = torch.bfloat16, S.VA_DTYPE_BF16, 8
    net.lib = _lib.load()
    p = net._pack(w, b, deconv=deconv)
    w8, sw, Kp = net._pack_fp8(p)
    ld_in = cin + slice_in + 16
    xb = x.permute(0, 2, 3, 1).to(torch.bfloat16).float()  # NHWC, the bf16 values
    xs = _pow2_scale(float(xb.abs().max()))  # a power of two, as calibrate_fp8 picks
    if x8:  # the e4m3 buffer holds sat(x * xs)
        xin = torch.zeros(B, H, W, ld_in, dtype=torch.uint8, device="cuda")
        xin[..., slice_in:slice_in + cin] = _e4m3(xb, xs).cuda()
    else:
        xin = torch.zeros(B, H, W, ld_in, dtype=torch.bfloat16, device="cuda")
        xin[..., slice_in:slice_in + cin] = xb.to(torch.bfloat16).cuda()
    pad = k // 2 if not deconv else 0
    if deconv:
        Ho, Wo, oh, ow = H, W, 2 * H, 2 * W
    else:
        Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        oh, ow = Ho, Wo
    odt = torch.float32 if out_f32 else (torch.uint8 if y8 else torch.bfloat16)
    ld_out = cout + 16
    y = torch.zeros(B, oh, ow, ld_out, dtype=odt, device="cuda")
    res, rs = None, 0.0
    if residual:
        rf = torch.randn(B, oh, ow, cout, generator=g).to(torch.bfloat16).float()
        if r8:
            rs = _pow2_scale(float(rf.abs().max()))
            res = _e4m3(rf, rs).cuda()
        else:
            res = rf.to(torch.bfloat16).cuda()
    ws = (sw / xs).contiguous()
    args = S.ConvArgs(x=xin.data_ptr() + slice_in * xin.element_size(), N=B, H=H, W=W, Cin=p.cin, ldx=ld_in, kh=p.k,
                      kw=p.k,
                      stride=stride if not deconv else 1, pad=pad, Ho=Ho, Wo=Wo, w=w8.data_ptr(), bias=p.b.data_ptr(),
                      Cout=p.cout, Npad=p.Npad, K=p.K, Kpad=Kp, y=y.data_ptr() + 8 * y.element_size(), ldy=ld_out,
                      res=res.data_ptr() if res is not None else None, ldr=cout, act=1 if act else 0,
                      mode=1 if deconv else 0, M=B * Ho * Wo, dtype=S.VA_DTYPE_FP8, out_f32=1 if out_f32 else 0,
                      wscale=ws.data_ptr(), xscale=xs, x8=1 if x8 else 0, rscale=rs)
    # the reference on the same quantized operands
    xq = _e4m3(xb, xs).view(torch.float8_e4m3fn).float().permute(0, 3, 1, 2)
    wq = w8.cpu().view(torch.float8_e4m3fn).float()[:, :p.K]  # [Npad][K], K = (ky, kx, ci)
    rows = 4 * cout if deconv else cout
    wq = wq[:rows].reshape(rows, p.k, p.k, p.cin).permute(0, 3, 1, 2)
    acc = F.conv2d(xq, wq, None, 1 if deconv else stride, pad)  # [B, rows, Ho, Wo]
    acc = acc * ws.cpu()[:rows].view(1, rows, 1, 1) + p.b.cpu()[:rows].view(1, rows, 1, 1)
    if deconv:  # rows q * cout + co, q = 2 dy + dx -> pixel (2 ho + dy, 2 wo + dx)
        acc = acc.view(B, 2, 2, cout, Ho, Wo).permute(0, 3, 4, 1, 5, 2).reshape(B, cout, 2 * Ho, 2 * Wo)
    if act:
        acc = F.silu(acc)
    ref = acc.permute(0, 2, 3, 1)
    if residual:
        ref = ref + (res.cpu().view(torch.float8_e4m3fn).float() / rs if r8 else res.float().cpu())
    ys = 0.0
    if y8:
        ys = _pow2_scale(float(ref.abs().max()))
        args.yscale = ys
        args.y = y.data_ptr() + 8
    _lib.check(net.lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(args)), "va_seg_conv")
    torch.cuda.synchronize()
    if y8:  # e4m3 units
        return y[..., 8:8 + cout].cpu().view(torch.float8_e4m3fn).float(), ref * ys
    return y[..., 8:8 + cout].float().cpu(), ref


@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,deconv,slice_in,out_f32", [
    (64, 128, 3, 1, 20, 24, False, False, 0, False),
    (96, 192, 3, 2, 33, 40, False, False, 16, False),  # stride 2, ragged M, channel slice
    (128, 64, 1, 1, 17, 19, True, False, 0, False),    # 1x1 + residual
    (48, 96, 3, 1, 40, 40, True, False, 0, False),     # K = 432 (not a multiple of 128), residual
    (192, 256, 3, 1, 10, 10, False, False, 0, False),  # two channel tiles
    (64, 32, 2, 1, 12, 10, False, True, 0, False),     # ConvTranspose2d(2, 2) as mode 1
    (96, 80, 1, 1, 13, 13, False, False, 0, True),     # head-like: float output, no activation
])
def test_fp8_conv_op(cin, cout, k, stride, H, W, residual, deconv, slice_in, out_f32):
    got, ref = _conv8(cin, cout, k, stride, H, W, residual, deconv, slice_in, out_f32,
                      act=not (deconv or out_f32))
    assert got.shape == ref.shape
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,deconv,slice_in,x8,y8,r8", [
    (64, 128, 3, 1, 20, 24, False, False, 0, True, True, False),    # e4m3 in and out
    (96, 192, 3, 2, 33, 40, False, False, 16, True, True, False),   # stride 2, ragged M, 16-channel slice
    (128, 64, 1, 1, 17, 19, True, False, 0, True, True, True),      # 1x1 + e4m3 residual (C2f bottleneck)
    (48, 96, 3, 1, 40, 40, True, False, 0, False, True, True),      # bf16 in (model.1), e4m3 out + residual
    (64, 32, 2, 1, 12, 10, False, True, 0, True, True, False),      # ConvTranspose2d(2, 2) into e4m3
    (96, 80, 1, 1, 13, 13, False, False, 0, True, False, False),    # head-like: e4m3 in, float out
])
def test_fp8_conv_op_e4m3_buffers(cin, cout, k, stride, H, W, residual, deconv, slice_in, x8, y8, r8):
    """The fp8 mode's ops on e4m3 activation buffers: e4m3 output within one e4m3 step of the exact value (the
    kernel rounds its float result) plus 1e-4 of the output's scale (float summation order, where partial sums
    cancel)."""
    out_f32 = not y8 and cout == 80
    got, ref = _conv8(cin, cout, k, stride, H, W, residual, deconv, slice_in, out_f32,
                      act=not (deconv or out_f32), x8=x8, y8=y8, r8=r8)
    assert got.shape == ref.shape
    if y8:
        r = ref.clamp(-448, 448)
        ulp = torch.where(r.abs() >= 2.0 ** -6, 2.0 ** (torch.floor(torch.log2(r.abs().clamp_min(1e-30))) - 3),
                          torch.full_like(r, 2.0 ** -9))
        # one e4m3 step, plus the float sums' own error where large partial sums cancel (1e-4 of the output's
        # scale: the kernel and torch add in different orders)
        badm = (got - r).abs() > ulp * 1.0001 + 1e-4 * r.abs().max()
        bad = int(badm.sum().item())
        assert bad == 0, (bad, (got - r).abs().max().item(), got[badm][:8].tolist(), r[badm][:8].tolist(),
                          badm.nonzero()[:8].tolist())
    else:
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err < 2e-2, err


def test_fp8_sppf_and_upsample_on_e4m3_bytes():
    """SPPF maxima and the FPN upsample copy on e4m3 bytes equal the same ops on the decoded values."""
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    B, H, W, c = 2, 20, 20, 64
    v = torch.randn(B, H, W, c, generator=g) * 30
    buf = torch.zeros(B, H, W, 4 * c, dtype=torch.uint8)
    buf[..., :c] = _e4m3(v, 4.0)
    d = buf.cuda()
    _lib.check(lib.va_seg_sppf_pool(_lib.stream_ptr(), d.data_ptr(), B, H, W, c, 4 * c, S.VA_DTYPE_FP8), "sppf")
    torch.cuda.synchronize()
    got = d.cpu().view(torch.float8_e4m3fn).float()
    x = got[..., :c].permute(0, 3, 1, 2)
    want = []
    for _ in range(3):
        x = F.max_pool2d(x, 5, 1, 2)
        want.append(x.permute(0, 2, 3, 1))
    assert torch.equal(got[..., c:], torch.cat(want, -1))
    up = torch.zeros(B, 2 * H, 2 * W, c + 16, dtype=torch.uint8, device="cuda")
    _lib.check(lib.va_seg_upsample2x(_lib.stream_ptr(), d.data_ptr(), 4 * c, up.data_ptr() + 16, c + 16, B, H, W, c,
                                     S.VA_DTYPE_FP8), "upsample")
    torch.cuda.synchronize()
    assert torch.equal(up[..., 16:].cpu(), d[..., :c].cpu().repeat_interleave(2, 1).repeat_interleave(2, 2))


def test_fp8_conv0_e4m3_output_matches_bf16_kernel():
    """va_seg_conv0_e4m3 (model.0 fused with the preprocess, e4m3 output) = the bf16 kernel's output quantized:
    within one e4m3 step (the e4m3 form rounds the float result directly, the bf16 one after a bf16 rounding)."""
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("m")
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=2)), dtype="bf16")
    B, H, W = 2, 160, 192
    fr = _frames(B, H, W, 9).cuda()
    c = arch.c1
    yb = torch.zeros(B, H // 2, W // 2, c, dtype=torch.bfloat16, device="cuda")
    y8 = torch.zeros(B, H // 2, W // 2, c, dtype=torch.uint8, device="cuda")
    w, b = net.w0
    _lib.check(net.lib.va_seg_conv0(_lib.stream_ptr(), fr.data_ptr(), B, H, W, w.data_ptr(), b.data_ptr(), c,
                                    yb.data_ptr(), c), "conv0")
    torch.cuda.synchronize()
    ys = _pow2_scale(float(yb.float().abs().max()))
    _lib.check(net.lib.va_seg_conv0_e4m3(_lib.stream_ptr(), fr.data_ptr(), B, H, W, w.data_ptr(), b.data_ptr(), c,
                                         y8.data_ptr(), c, ys), "conv0_e4m3")
    torch.cuda.synchronize()
    got = y8.cpu().view(torch.float8_e4m3fn).float()
    r = (yb.float().cpu() * ys).clamp(-448, 448)
    ulp = torch.where(r.abs() >= 2.0 ** -6, 2.0 ** (torch.floor(torch.log2(r.abs().clamp_min(1e-30))) - 3),
                      torch.full_like(r, 2.0 ** -9))
    assert ((got - r).abs() <= ulp * 1.0001 + 1e-3 * r.abs().max()).all()


def _frames(B, H, W, seed):
    return torch.randint(0, 256, (B, H, W, 3), generator=torch.Generator().manual_seed(seed), dtype=torch.uint8)


def test_fp8_forward_medium_1280_vs_fp32_oracle():
    from oracle import yolo_ref as Y
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    torch.set_num_threads(8)
    arch = Arch("m")
    fw = fold(arch, synthetic_state_dict(arch, seed=4))
    frames = _frames(1, 1280, 1280, 6)
    box, cls, coef, proto = Y.forward(arch, fw, Y.preprocess(frames))
    net = SegNet(arch, fw, dtype="fp8")
    out = net.forward(frames.cuda())
    torch.cuda.synchronize()
    n_fp8 = sum(1 for m in net.plan(1, 1280, 1280)["meta"] if m.get("fp8"))
    assert n_fp8 >= 60, n_fp8  # every conv but model.0 (3 input channels) runs on the fp8 kernel
    lv = torch.cat([t.float().cpu().flatten(1, 2) for t in out.levels], 1).permute(0, 2, 1)
    nc = arch.nc
    got = (lv[:, :64], lv[:, 64:64 + nc], lv[:, 64 + nc:], out.proto.float().cpu().permute(0, 3, 1, 2))
    errs = {}
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, (box, cls, coef, proto)):
        assert torch.isfinite(g).all(), name
        errs[name] = ((g - r).norm() / r.norm()).item()
    print("fp8 relative L2 vs fp32:", errs)
    for name, e in errs.items():
        assert e < FP8_L2[name], (name, e)


def test_fp8_pipeline_1280_planted_nav_matches_oracle():
    from oracle import nav as onav
    from workloads.corridors import cells_rect, cells_to_mask, corridor_cells
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("m")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B, H, W = 2, 1280, 1280
    pipe = FramePipeline(arch, fw, B, H, W, dtype="fp8")
    grids = [corridor_cells(7400 + i, H // 20, W // 20) for i in range(B)]
    pc = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    res = pipe.run(_frames(B, H, W, 17).cuda(), pc, pr, PLANT_ALWAYS)
    pf = onav.PathFinderOracle()
    for i, g in enumerate(grids):
        out = onav.frame_nav(cells_to_mask(g), cells_rect(g), H, W, pf)
        nf = res.frame(i)
        assert [q["path"] for q in nf.queries] == [[(c.coords.x, c.coords.y) for c in q[2]] for q in out["queries"]]


# relative L2 bars on real frames, calibrated on noise (the default) and on the real frames themselves: with the
# default headroom of 8 (seg.FP8_HEADROOM) measured 0.148 / 0.153 / 0.160 / 0.153 and 0.151 / 0.154 / 0.163 / 0.154
# (profiles/r04/fp8/); at headroom 2 the noise calibration clipped real frames' activations, which run 2.3-2.8x
# the noise frames' amax from model.3 on (tools/m_condition.py --real), to 0.30-0.33
FP8_REAL_L2 = {"noise": {"box": 0.2, "cls": 0.2, "coef": 0.2, "proto": 0.2},
               "real": {"box": 0.2, "cls": 0.2, "coef": 0.2, "proto": 0.2}}
_FP8_REPORT = {}


def _write_report():
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "fp8_accuracy.json"), "w") as f:
            json.dump(_FP8_REPORT, f, indent=1)


@pytest.mark.parametrize("calib", ["noise", "real"])
def test_fp8_forward_real_frames_vs_fp32_oracle(calib):
    """The m@1280 fp8 forward on inputs OTHER than its calibration distribution: 2 x 2 mosaics of the
    reference's own validation frames (real camera frames of paths), with the activation scales calibrated on
    seeded noise frames (the default) or on the real frames themselves (FramePipeline / YOLO fp8_calib); relative
    L2 per head output against the fp32 oracle."""
    from oracle import yolo_ref as Y
    from tests.chain_util import mosaic_1280, real_frames
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    torch.set_num_threads(16)
    arch = Arch("m")
    fw = fold(arch, synthetic_state_dict(arch, seed=4))
    frames = torch.from_numpy(mosaic_1280(real_frames(8)))
    with torch.no_grad():
        box, cls, coef, proto = Y.forward(arch, fw, Y.preprocess(frames))
    net = SegNet(arch, fw, dtype="fp8")
    if calib == "real":
        net.fp8_calib_frames = frames
    out = net.forward(frames.cuda())
    torch.cuda.synchronize()
    lv = torch.cat([t.float().cpu().flatten(1, 2) for t in out.levels], 1).permute(0, 2, 1)
    nc = arch.nc
    got = (lv[:, :64], lv[:, 64:64 + nc], lv[:, 64 + nc:], out.proto.float().cpu().permute(0, 3, 1, 2))
    errs = {}
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, (box, cls, coef, proto)):
        assert torch.isfinite(g).all(), name
        errs[name] = round(((g - r).norm() / r.norm()).item(), 4)
    _FP8_REPORT[f"forward_real_frames/calib_{calib}"] = errs
    _write_report()
    print(f"fp8 on real frames (calibrated on {calib}) relative L2 vs fp32:", errs)
    for name, e in errs.items():
        assert e < FP8_REAL_L2[calib][name], (name, e)


# fp8 chain agreement over 8 frames (profiles/r04/fp8/fp8_accuracy.json): dense_box chosen 0.25, cells and paths
# 0.75 (6 of 8 frames reach the same navigation mask and paths); floors one frame below.  'sparse' is run and its
# rates recorded, with no floor: its detections are the far tail of a unimodal class-logit distribution (m@1280
# synthetic: cls0 mean 114, std 140, the threshold at the top ~1 anchor per frame, tools/m_condition.py), and the
# e4m3 forward's head error (relative L2 0.15-0.21, i.e. tens of logit units) moves hundreds of anchors across it --
# fp8 keeps 210-287 detections where fp32 keeps 2-7.  A trained head separates objects from background by margins
# far above that error; this synthetic regime has no such margin, so its fp8 agreement is not a kernel property
FP8_CHAIN_FLOOR = {"dense_box": {"chosen": 0.125, "cells": 0.625, "paths": 0.625}, "sparse": {}}


# the weight-only form (SegNet dtype "w8a16": e4m3 weight bytes in HBM, converted to bf16 in the bf16 kernels' A stage,
# the accumulator scaled per output channel; bf16 activations), C5's kept form.  Measured on the GPU (profiles/r06/c5/
# fp8_accuracy.json): dense_box chosen 0.75, rect / cells / paths 0.875; sparse chosen 0.25, rect / cells / paths
# 0.375 (round 5's host-dequantized form: 0.125 / 0.25 / 0.125 -- its weights were rounded twice, to e4m3 and then
# to bf16 with a non-power-of-two scale).  Floors one frame below the measurements.  Sparse stays low for the reason
# FP8_CHAIN_FLOOR's comment gives: its detections are the far tail of the synthetic head's unimodal class-logit
# distribution, which the weights' e4m3 error alone moves across the threshold
W8A16_CHAIN_FLOOR = {"dense_box": {"chosen": 0.625, "cells": 0.75, "paths": 0.75},
                     "sparse": {"chosen": 0.125, "cells": 0.25, "paths": 0.25}}


@pytest.mark.parametrize("regime", ["dense_box", "sparse"])
def test_w8a16_chain_1280_vs_fp32_oracle(regime):
    """C5's weight-only form down the whole chain (m@1280, 8 frames) against the fp32 oracle chain, as
    test_fp8_chain_1280_vs_fp32_oracle does for the e4m3 MFMA form: rates written out, held to measured floors."""
    _chain_1280("w8a16", regime, W8A16_CHAIN_FLOOR[regime])


@pytest.mark.parametrize("regime", ["dense_box", "sparse"])
def test_fp8_chain_1280_vs_fp32_oracle(regime):
    """C5's whole chain at fp8 (BASELINE configs[4]: YOLOv8m-seg 1280 on e4m3 MFMA): the network's own detections
    through NMS, contours, the mask choice and grid / A* on 4 frames, against the fp32 oracle chain
    (tests/golden/chain_oracle.json.gz["c5/*"]): detections matched (boxes within 2 px, scores within 2e-2), the
    same chosen instance, cells and A* paths -- rates written out and held to measured floors."""
    _chain_1280("fp8", regime, FP8_CHAIN_FLOOR[regime])


def _chain_1280(dtype, regime, floors):
    from tests.chain_util import compare, frame_batch, load_fixture, rates, weights
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    arch, fw = weights(regime, scale="m")
    want = load_fixture(f"c5/{regime}")
    B = len(want)
    pipe = FramePipeline(arch, fw, B, 1280, 1280, dtype=dtype)
    res = pipe.run(frame_batch(8000, B, 1280).cuda(), plant_mode=PLANT_NEVER)
    torch.cuda.synchronize()
    cmps = []
    for i, w in enumerate(want):
        det, _ = pipe.post.det_tensor(i)
        nf = res.frame(i)
        chosen = int(pipe.post.chosen[i])
        ok = nf.status == 0
        got = {"det": det, "chosen": chosen,
               "rect": tuple(int(v) for v in pipe.post.rects[i].cpu()) if chosen >= 0 else None,
               "cells": pipe.post.cells[i].cpu().numpy() if chosen >= 0 else None,
               "paths": [q["path"] for q in nf.queries] if ok else None,
               "costs": [float(q["cost"]).hex() if q["path"] else None for q in nf.queries] if ok else None}
        cmps.append(compare(got, w, f32=False))
    rr = rates(cmps)
    _FP8_REPORT[f"chain_1280/{regime}" if dtype == "fp8" else f"{dtype}_chain_1280/{regime}"] = rr
    _write_report()
    print(dtype, "chain", regime, rr)
    for k, floor in floors.items():
        assert rr[k] >= floor, (k, rr[k], floor)

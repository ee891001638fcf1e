"""C5's weight-only fp8 form on the bf16 kernels (va355.h va_conv_args.w8: e4m3 weight BYTES in HBM with one scale per
GEMM row, converted exactly to bf16 in the kernels' A stage, the f32 accumulator times the scale in the epilogue).

Bit-level checks: with power-of-two scales every e4m3 value times its scale is exact in bf16 and the scaling commutes
with the f32 sums, so an op with e4m3 bytes + scales must equal, bit for bit, the same op on the dequantized bf16
weights -- through every kernel form the bf16 dispatcher picks (conv_dn, conv2's three tile shapes with and without
the FK addressing, split-K, the upsampled prefix, mode 1, conv4 at stride 1 and 2, a residual) and through a whole
YOLOv8m-seg forward (the proto's sub-pixel fold as mode 2, the fused tails).  Accuracy of the form itself (production
scales amax / 448) down the whole chain: tests/test_gpu_fp8.py::test_w8a16_chain_1280_vs_fp32_oracle."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

F8_MAX = 448.0


def _q_pow2(rows: torch.Tensor):
    """Per-row e4m3 quantization with power-of-two scales: (bytes uint8, scales f32, dequantized f32)."""
    amax = rows.abs().amax(1)
    sw = torch.where(amax > 0, torch.exp2(torch.ceil(torch.log2(amax / F8_MAX))), torch.ones_like(amax)).float()
    q = (rows / sw[:, None]).clamp(-F8_MAX, F8_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).contiguous(), sw.contiguous(), q.float() * sw[:, None]


def _net(dtype="bf16"):
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch
    net = S.SegNet.__new__(S.SegNet)
    net.arch = Arch("n")
    net.dtype = dtype
    net.form = dtype
    net.tdtype = torch.bfloat16
    net.va_dtype = S.VA_DTYPE_BF16
    net.vec = 8
    net.device = torch.device("cuda")
    net.lib = _lib.load()
    return net


# (cin, cout, k, stride, H, W, B, residual, deconv, up, splitk) -- the dispatcher's bf16 forms for these shapes
CASES = [
    (48, 48, 3, 1, 40, 40, 3, False, False, 0, False),     # conv_dn (Cout <= 64, >= 4096 pixels): m's C2f 3x3
    (48, 48, 3, 1, 40, 40, 3, True, False, 0, False),      # conv_dn + residual (Bottleneck shortcut)
    (64, 32, 3, 1, 20, 20, 2, False, False, 0, False),     # conv2 <4, 1, 2> (800 pixels: not conv_dn), FK
    (96, 48, 1, 1, 20, 24, 2, False, False, 0, False),     # conv2 <4, 1, 4>, general (non-FK) addressing
    (128, 192, 3, 1, 40, 40, 2, False, False, 0, False),   # conv2 <2, 2, 4>, FK (13 256-tiles: not conv4)
    (96, 96, 3, 2, 40, 40, 2, False, False, 0, False),     # conv2 <2, 2, 4>, stride 2, general addressing
    (256, 256, 3, 1, 10, 10, 1, False, False, 0, True),    # conv2 split over K (few tiles, a workspace)
    (128, 64, 2, 1, 20, 20, 2, False, True, 0, False),     # ConvTranspose2d(2, 2) as mode 1 (4 x 64 rows)
    (384, 128, 1, 1, 20, 20, 2, False, False, 192, False),  # conv2 with the FPN's upsampled prefix read in place
    (192, 384, 3, 1, 40, 40, 2, False, False, 0, False),   # conv4 (VA_CONV4=all), stride 1
    (192, 384, 3, 2, 80, 80, 2, False, False, 0, False),   # conv4, stride 2
    (192, 256, 1, 1, 40, 40, 2, True, False, 0, False),    # conv4, 1x1 + residual
    (576, 384, 1, 1, 20, 20, 2, False, False, 576 - 192, False),  # conv4 with the upsampled prefix
]


# the patch kernel (narrow stride-1 3x3, Cin / Cout 32 or 64; m's box branch cv2.l.1 64 -> 64): weights staged once
PATCH_CASES = [(64, 64, 3, 1, 40, 40, 2, False, False, 0, False), (32, 64, 3, 1, 37, 45, 2, True, False, 0, False),
               (64, 32, 3, 1, 20, 20, 3, False, False, 0, False)]


@pytest.mark.parametrize("cin,cout,k,stride,H,W,B,residual,deconv,up,splitk",
                         CASES + [pytest.param(*c, id=f"patch{i}") for i, c in enumerate(PATCH_CASES)])
def test_w8_op_bit_identical_to_dequantized_bf16(cin, cout, k, stride, H, W, B, residual, deconv, up, splitk, switch,
                                                  request):
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    switch("VA_CONV4", "all")  # every conv4-eligible shape on conv4, so its W8 form is reached at small sizes
    # the w8 ops skip the streaming 1x1 kernel (no A stage to convert in): off for the bf16 runs too; the patch
    # kernel only for its own cases
    switch("VA_PW", "0")
    if "patch" not in request.node.callspec.id:
        switch("VA_CONV_PATCH", "0")
    net = _net()
    g = torch.Generator().manual_seed(cin * 31 + cout * 7 + k + stride)
    if deconv:
        w = torch.randn(cin, cout, 2, 2, generator=g) * 0.2
    else:
        w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    w[0] *= 1e-3  # a row of tiny weights: e4m3 subnormals after the row's scale
    b = torch.randn(cout, generator=g) * 0.1
    p = net._pack(w, b, deconv=deconv)
    q8, sw, dq = _q_pow2(net._rows(w, deconv=deconv))
    w16 = dq.to(torch.bfloat16)
    assert torch.equal(w16.float(), dq), "e4m3 x 2^k must be exact in bf16"
    q8, sw, w16 = S.w8_order(q8).cuda(), sw.cuda(), w16.cuda()  # the kernels' K order of the e4m3 rows
    ld_in = cin + 8
    xin = (torch.randn(B, H, W, ld_in, generator=g) * 0.7).to(torch.bfloat16).cuda()
    pad = 0 if deconv else k // 2
    Ho, Wo = (H, W) if deconv else ((H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1)
    oh, ow = (2 * H, 2 * W) if deconv else (Ho, Wo)
    ld_out = cout + 16
    res = (torch.randn(B, oh, ow, cout, generator=g)).to(torch.bfloat16).cuda() if residual else None
    xu = None
    if up:
        xu = (torch.randn(B, H // 2, W // 2, up, generator=g) * 0.7).to(torch.bfloat16).cuda()
    ws = (torch.empty(S.SPLITK_WS_BYTES, dtype=torch.uint8, device="cuda"),
          torch.zeros(S.SPLITK_NCNT, dtype=torch.int32, device="cuda")) if splitk else None
    outs = []
    for w8 in (False, True):
        y = torch.full((B, oh, ow, ld_out), float("nan"), dtype=torch.bfloat16, device="cuda")
        a = S.ConvArgs(x=xin.data_ptr(), N=B, H=H, W=W, Cin=p.cin, ldx=ld_in, kh=p.k, kw=p.k,
                       stride=1 if deconv else stride, pad=pad, Ho=Ho, Wo=Wo,
                       w=(q8 if w8 else w16).data_ptr(), bias=p.b.data_ptr(), Cout=p.cout, Npad=p.Npad, K=p.K,
                       Kpad=p.Kpad, y=y.data_ptr(), ldy=ld_out, res=res.data_ptr() if res is not None else None,
                       ldr=cout, act=1, mode=1 if deconv else 0, M=B * Ho * Wo, dtype=S.VA_DTYPE_BF16)
        if xu is not None:
            a.xu, a.ldu, a.cu = xu.data_ptr(), up, up
        if ws is not None:
            a.ws, a.ws_bytes, a.wcnt, a.ncnt = ws[0].data_ptr(), ws[0].numel(), ws[1].data_ptr(), ws[1].numel()
        if w8:
            a.wscale, a.w8 = sw.data_ptr(), 1
        _lib.check(net.lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_conv")
        torch.cuda.synchronize()
        outs.append(y[..., :cout].float().cpu())
    ref, got = outs
    assert torch.isfinite(ref).all()
    assert torch.equal(got, ref), (got - ref).abs().max().item()


def test_w8_rejects_bad_args():
    """w8 is a bf16 form: an f32 op, a missing or misaligned scale vector is refused (VA_ERR_ARG), not run."""
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    net = _net()
    x = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device="cuda")
    y = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device="cuda")
    w = torch.zeros(128, 64, dtype=torch.uint8, device="cuda")
    b = torch.zeros(128, device="cuda")
    sw = torch.ones(132, device="cuda")
    base = dict(x=x.data_ptr(), N=1, H=8, W=8, Cin=64, ldx=64, kh=1, kw=1, stride=1, pad=0, Ho=8, Wo=8,
                w=w.data_ptr(), bias=b.data_ptr(), Cout=64, Npad=128, K=64, Kpad=64, y=y.data_ptr(), ldy=64, act=1,
                M=64, dtype=S.VA_DTYPE_BF16, w8=1)
    for bad in ({"wscale": None}, {"wscale": sw.data_ptr() + 4}, {"wscale": sw.data_ptr(), "dtype": S.VA_DTYPE_F32}):
        a = S.ConvArgs(**{**base, **bad})
        assert net.lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)) == _lib.VA_ERR_ARG, bad
    a = S.ConvArgs(**{**base, "wscale": sw.data_ptr()})
    assert net.lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)) == 0
    torch.cuda.synchronize()


def test_w8a16_forward_bit_identical_to_dequantized_plan(monkeypatch, switch):
    """A whole YOLOv8m-seg forward (320 x 320, 2 frames) of SegNet(dtype="w8a16") with power-of-two row scales, against
    the SAME op list with every w8 op pointed at its dequantized bf16 rows instead: bit-identical heads and proto.  The
    plan must carry e4m3 bytes on every conv (the proto's sub-pixel fold included); the streaming 1x1 kernel, which
    the w8 ops skip, is off for both runs so the same kernel forms compare."""
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    switch("VA_PW", "0")

    def pack_pow2(self, wm):
        q, sw, _ = _q_pow2(wm.float())
        return S.w8_order(q).to(self.device), sw.to(self.device)
    monkeypatch.setattr(S.SegNet, "_pack_e4m3", pack_pow2)
    arch = Arch("m")
    fw = fold(arch, synthetic_state_dict(arch, seed=3))
    net = S.SegNet(arch, fw, dtype="w8a16")
    plan = net.plan(2, 320, 320)
    frames = torch.randint(0, 256, (2, 320, 320, 3), generator=torch.Generator().manual_seed(9), dtype=torch.uint8)
    plan["frames"].copy_(frames.cuda())
    convs = [plan["ops"][i] for i in range(plan["n"]) if plan["ops"][i].kind == S.VA_OP_CONV]
    w8ops = [op for op in convs if op.a.w8]
    assert len(w8ops) == len(convs) and len(convs) > 60, (len(w8ops), len(convs))
    assert any(op.a.mode == 2 for op in w8ops), "the proto fold carries e4m3 bytes"

    def run():
        net.run_plan(plan)
        torch.cuda.synchronize()
        return [t.clone().cpu() for t in plan["out"].levels] + [plan["out"].proto.clone().cpu()]
    got = run()
    # the SegNet's own e4m3 tensors by device pointer: the per-layer rows and the proto fold's [4][Npad][Kpad]
    by_ptr = {q.data_ptr(): (q, sw) for q, sw in list(net.w8w.values()) + [net.proto_fold8]}
    keep, saved = [], []
    for op in w8ops:
        a = op.a
        q, sw = by_ptr[a.w]
        assert sw.data_ptr() == a.wscale
        n_cls = 4 if a.mode == 2 else 1
        qn = S.w8_order(q, inverse=True)  # natural K order
        dq = qn.view(torch.float8_e4m3fn).float().view(n_cls, a.Npad, a.Kpad) * sw.view(n_cls, a.Npad, 1)
        w16 = dq.to(torch.bfloat16).contiguous()
        assert torch.equal(w16.float(), dq)
        keep.append(w16)
        saved.append((op, a.w, a.wscale))
        a.w, a.w8, a.wscale = w16.data_ptr(), 0, None
    try:
        want = run()
    finally:
        for op, w, s in saved:
            op.a.w, op.a.wscale, op.a.w8 = w, s, 1
    for name, g, r in zip(("level0", "level1", "level2", "proto"), got, want):
        assert torch.isfinite(r).all(), name
        assert torch.equal(g, r), f"{name}: w8 vs dequantized bf16 max diff {(g - r).abs().max().item()}"


"""GPU numerics of the segmentation kernels vs a plain PyTorch fp32 reference.

* single ops (va_seg_conv incl. stride 2, residual, channel slices, ConvTranspose;
  SPPF pool; nearest upsample) against torch.nn.functional on the CPU;
* the whole YOLOv8-seg forward (oracle/yolo_ref.py, seeded synthetic weights):
  f32 mode (exact three-term bf16 products with f32 accumulation, and the f32 MFMA form) within 1e-3 of the
  fp32 reference logits (BASELINE.json north_star tolerance); bf16 mode within a relative bound.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import yolo_ref as Y

pytestmark = pytest.mark.gpu


def _net(dtype, scale="s", nc=80, seed=0, cls_bias=None):
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(scale, nc)
    fw = fold(arch, synthetic_state_dict(arch, seed=seed, cls_bias=cls_bias))
    return arch, fw, SegNet(arch, fw, dtype=dtype)


def _run_single_conv(dtype, cin, cout, k, stride, H, W, residual=False, deconv=False, slice_in=0, act=True, ws=None,
                     B=2, w3=False):
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch
    g = torch.Generator().manual_seed(cin * 1000 + cout + k)
    if deconv:
        w = torch.randn(cin, cout, 2, 2, generator=g) * 0.2
    else:
        w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(B, cin, H, W, generator=g)
    net = S.SegNet.__new__(S.SegNet)
    net.arch = Arch("n")
    net.dtype = dtype
    net.tdtype = torch.bfloat16 if dtype == "bf16" else torch.float32
    net.va_dtype = S.VA_DTYPE_BF16 if dtype == "bf16" else S.VA_DTYPE_F32
    net.vec = 8 if dtype == "bf16" else 4
    net.device = torch.device("cuda")
    from vision_assist_amd import _lib
    net.lib = _lib.load()
    p = net._pack(w, b, deconv=deconv, stride=stride)
    ld_in = cin + slice_in + 8
    xin = torch.zeros(B, H, W, ld_in, dtype=net.tdtype, device="cuda")
    xin[..., slice_in:slice_in + cin] = x.permute(0, 2, 3, 1).to(net.tdtype).cuda()
    xr = xin[..., slice_in:slice_in + cin].float().cpu().permute(0, 3, 1, 2)  # what the kernel sees
    pad = k // 2 if not deconv else 0
    if deconv:
        Ho, Wo, oh, ow = H, W, 2 * H, 2 * W
    else:
        Ho = (H + 2 * pad - k) // stride + 1
        Wo = (W + 2 * pad - k) // stride + 1
        oh, ow = Ho, Wo
    ld_out = cout + 16
    y = torch.zeros(B, oh, ow, ld_out, dtype=net.tdtype, device="cuda")
    res = None
    if residual:
        res = torch.randn(B, oh, ow, cout, generator=g).to(net.tdtype).cuda()
    args = S.ConvArgs(x=xin.data_ptr() + slice_in * xin.element_size(), N=B, H=H, W=W, Cin=p.cin, ldx=ld_in,
                      kh=p.k, kw=p.k, stride=stride if not deconv else 1, pad=pad, Ho=Ho, Wo=Wo,
                      w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=p.cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad,
                      y=y.data_ptr() + 8 * y.element_size(), ldy=ld_out,
                      res=res.data_ptr() if res is not None else None, ldr=cout, act=1 if act else 0,
                      mode=1 if deconv else 0, M=B * Ho * Wo, dtype=net.va_dtype, out_f32=0)
    if w3:  # f32: the pre-split weight planes -> the three-plane kernels (conv3t / conv3h)
        args.w3 = p.w3.data_ptr()
    if ws is not None:  # split-K workspace (va_conv_args.ws): (slabs uint8, counters int32)
        args.ws, args.ws_bytes, args.wcnt, args.ncnt = ws[0].data_ptr(), ws[0].numel(), ws[1].data_ptr(), ws[1].numel()
    _lib.check(net.lib.va_seg_conv(_lib.stream_ptr(), __import__("ctypes").byref(args)), "va_seg_conv")
    torch.cuda.synchronize()
    got = y[..., 8:8 + cout].float().cpu().permute(0, 3, 1, 2)
    wr = w.to(net.tdtype).float() if dtype == "bf16" else w
    if deconv:
        ref = F.conv_transpose2d(xr, wr, b, stride=2)
    else:
        ref = F.conv2d(xr, wr, b, stride, pad)
    if act:
        ref = F.silu(ref)
    if residual:
        ref = ref + res.float().cpu().permute(0, 3, 1, 2)
    return got, ref


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,deconv,slice_in", [
    (8, 32, 3, 2, 34, 30, False, False, 0),
    (32, 64, 3, 1, 20, 20, True, False, 16),
    (64, 96, 1, 1, 24, 17, False, False, 8),
    (96, 80, 1, 1, 13, 13, False, False, 0),
    (16, 256, 3, 2, 40, 40, False, False, 0),
    (64, 32, 2, 1, 10, 12, False, True, 0),
    (64, 32, 3, 1, 23, 41, False, False, 8),   # patch kernel: ragged 16 x 16 tiles, channel slice
    (64, 64, 3, 1, 37, 16, True, False, 0),    # patch kernel: residual
    (128, 256, 3, 1, 19, 23, True, False, 0),  # wide patch kernel: ragged tiles, two channel tiles, residual
    (64, 136, 3, 1, 16, 40, False, False, 64), # wide patch kernel: ragged channel tile, channel slice
    (128, 128, 1, 1, 20, 20, False, False, 0), # streaming 1x1 (va_pw.hip)
    (192, 128, 1, 1, 13, 11, False, False, 8), # streaming 1x1: ragged last tile, channel slice
    (448, 128, 1, 1, 9, 30, False, False, 0),  # streaming 1x1 at its largest K
    (128, 128, 1, 1, 320, 320, False, False, 0),  # streaming 1x1: > 2 tiles per wave (persistent loop)
    (256, 128, 1, 1, 200, 328, False, False, 8),  # streaming 1x1: several tiles per wave, K = 256, slice
])
def test_conv_op(dtype, cin, cout, k, stride, H, W, residual, deconv, slice_in):
    got, ref = _run_single_conv(dtype, cin, cout, k, stride, H, W, residual, deconv, slice_in, act=not deconv)
    if dtype == "f32":
        assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    else:
        err = (got - ref).abs().max() / ref.abs().max()
        assert err < 2e-2, err


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,slice_in", [
    (256, 256, 3, 1, 20, 20, False, 0),   # 4 tiles x 16 slices
    (128, 256, 3, 2, 40, 40, True, 8),    # stride 2, residual, channel slice
    (512, 192, 1, 1, 17, 23, False, 0),   # 1x1, ragged last tile
    (96, 160, 3, 1, 11, 9, False, 0),     # bf16: per-lane im2col (Cin % 64 != 0), ragged channel tile
    (40, 136, 3, 1, 12, 10, False, 0),    # both dtypes per-lane im2col, K padded past 9 Cin
])
def test_conv_split_k(dtype, cin, cout, k, stride, H, W, residual, slice_in):
    """Split-K (va_conv_args.ws, batch-1 shapes): against torch at the unsplit tolerances, bit-identical on a
    second run (the slices are summed in slice order, not arrival order), and the arrival counters back at zero."""
    ws = (torch.empty(32 << 20, dtype=torch.uint8, device="cuda"), torch.zeros(128, dtype=torch.int32, device="cuda"))
    got, ref = _run_single_conv(dtype, cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1)
    again, _ = _run_single_conv(dtype, cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1)
    assert int(ws[1].abs().sum()) == 0
    assert torch.equal(got, again)
    if dtype == "f32":
        assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    else:
        err = (got - ref).abs().max() / ref.abs().max()
        assert err < 2e-2, err


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("ks", ["4", "8", "13"])
@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,slice_in", [
    (256, 256, 3, 1, 20, 20, False, 0),
    (128, 256, 3, 2, 40, 40, True, 8),
    (512, 192, 1, 1, 17, 23, False, 0),
    (40, 136, 3, 1, 12, 10, True, 0),
])
def test_split_k_reduce_form_bit_identical_to_ticket(dtype, ks, cin, cout, k, stride, H, W, residual, slice_in, switch):
    """The reduce form (conv2_reduce_kernel, the default) adds the slabs in slice order and applies the epilogue's
    element work as conv_epilogue does: bit-identical to the ticket combine (VA_SPLITK=ticket) at the same slice
    count (forced, VA_SPLITK_KS), residual and ragged tiles included."""
    ws = (torch.empty(32 << 20, dtype=torch.uint8, device="cuda"), torch.zeros(128, dtype=torch.int32, device="cuda"))
    switch("VA_SPLITK_KS", ks)
    switch("VA_SPLITK", "ticket")
    t, ref = _run_single_conv(dtype, cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1)
    switch("VA_SPLITK", None)
    r, _ = _run_single_conv(dtype, cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1)
    assert int(ws[1].abs().sum()) == 0
    assert torch.equal(t, r)
    if dtype == "f32":
        assert torch.allclose(r, ref, atol=1e-4, rtol=1e-4), (r - ref).abs().max()


@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual,slice_in", [
    (256, 256, 3, 1, 20, 20, False, 0),   # 3x3 stride 1 (conv3h's shape; split, it runs on conv3t)
    (128, 256, 3, 2, 40, 40, True, 8),    # stride 2, residual, channel slice
    (512, 192, 1, 1, 17, 23, False, 0),   # 1x1, ragged pixel and channel tiles
    (256, 512, 1, 1, 20, 20, True, 0),    # 1x1, four channel tiles, residual
])
def test_conv3t_split_k_f32(cin, cout, k, stride, H, W, residual, slice_in, switch):
    """A batch-1 f32 layer conv2 would split over K runs on conv3t split over K (the default), its slabs in the
    32 x 32 fragment layout summed by conv2_reduce_kernel: within the f32 bar of torch and bit-identical run to run."""
    ws = (torch.empty(32 << 20, dtype=torch.uint8, device="cuda"), torch.zeros(128, dtype=torch.int32, device="cuda"))
    switch("VA_CONV3T", None)
    got, ref = _run_single_conv("f32", cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1, w3=True)
    again, _ = _run_single_conv("f32", cin, cout, k, stride, H, W, residual, False, slice_in, ws=ws, B=1, w3=True)
    assert torch.equal(got, again)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()


def test_forward_batch1_conv3t_split_within_f32_bar(switch):
    """The s-seg f32 batch-1 forward with the split layers on conv3t (default) against conv2's split-K
    (VA_CONV3T=nosplit): every head output within the f32 rounding of reordered sums (the two forms add the same
    exact term products in other orders)."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(1, seed=8)
    switch("VA_CONV3T", "nosplit")
    a = _gpu_heads(net, frames)
    switch("VA_CONV3T", None)
    b = _gpu_heads(net, frames)
    for name, x, y in zip(("box", "cls", "coef", "proto"), a, b):
        err = ((x - y).abs().max() / y.abs().max()).item()
        assert err < 1e-5, f"{name}: {err}"


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_forward_batch1_split_k_matches_unsplit(dtype, monkeypatch, switch):
    """The batch-1 n-seg forward with split-K (the C2 shape) against the same forward with VA_SPLITK=0: f32 to
    f32 rounding of the reordered sums, bf16 to bf16 rounding of the stored activations."""
    arch, fw, net = _net(dtype, "n", seed=5)
    frames = _frames(1, seed=8)
    switch("VA_SPLITK", "1")
    a = _gpu_heads(net, frames)
    switch("VA_SPLITK", "0")
    b = _gpu_heads(net, frames)
    for name, x, y in zip(("box", "cls", "coef", "proto"), a, b):
        err = ((x - y).abs().max() / y.abs().max()).item()
        assert err < (1e-5 if dtype == "f32" else 3e-2), f"{name}: {err}"


def _ref_heads(arch, fw, frames):
    box, cls, coef, proto = Y.forward(arch, fw, Y.preprocess(frames))
    return box, cls, coef, proto


def _gpu_heads(net, frames):
    out = net.forward(frames.cuda())
    torch.cuda.synchronize()
    lv = [t.float().cpu().flatten(1, 2) for t in out.levels]  # [B, hw, no]
    cat = torch.cat(lv, 1).permute(0, 2, 1)  # [B, no, A]
    nc = net.arch.nc
    return cat[:, :64], cat[:, 64:64 + nc], cat[:, 64 + nc:], out.proto.float().cpu().permute(0, 3, 1, 2)


def _frames(B, H=640, W=640, seed=0):
    return torch.randint(0, 256, (B, H, W, 3), generator=torch.Generator().manual_seed(seed), dtype=torch.uint8)


@pytest.mark.parametrize("form", ["6", "0"])  # three-term bf16 products (default) / the f32 MFMA (VA_F32_SPLIT=0)
def test_forward_f32_within_1e3_of_torch_reference(form, monkeypatch, switch):
    switch("VA_F32_SPLIT", form)  # the library re-reads its switches (va_switches_reload)
    torch.set_num_threads(8)
    arch, fw, net = _net("f32", "s")
    frames = _frames(2)
    ref = _ref_heads(arch, fw, frames)
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        err = (g - r).abs().max().item()
        assert err <= 1e-3, f"{name}: max |gpu - torch fp32| = {err}"
        # both forms are f32-accurate: far inside the bar (measured ~1e-5)
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: {err} is not f32-level"


def test_forward_bf16_close_to_torch_reference():
    arch, fw, net = _net("bf16", "s")
    frames = _frames(2, seed=1)
    ref = _ref_heads(arch, fw, frames)
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        rel = ((g - r).norm() / r.norm()).item()
        assert rel < 5e-2, f"{name}: relative L2 error {rel}"


def test_forward_f32_nano_1280():
    arch, fw, net = _net("f32", "n", seed=3)
    frames = _frames(1, 1280, 1280, seed=2)
    ref = _ref_heads(arch, fw, frames)
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        err = (g - r).abs().max().item()
        assert err <= 1e-3, f"{name}: max |gpu - torch fp32| = {err}"


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("H,W,c", [(20, 20, 256), (40, 40, 256), (13, 7, 64)])
def test_sppf_pool_exact(dtype, H, W, c):
    """va_seg_sppf_pool == three chained MaxPool2d(5, 1, 2) (SPPF, ultralytics nn/modules/block.py), bit-exact."""
    import ctypes
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    lib = _lib.load()
    td = torch.bfloat16 if dtype == "bf16" else torch.float32
    B, ld = 3, 4 * c + 8
    g = torch.Generator().manual_seed(H * 100 + W + c)
    x = torch.randn(B, H, W, c, generator=g).to(td)
    buf = torch.zeros(B, H, W, ld, dtype=td, device="cuda")
    buf[..., :c] = x.cuda()
    vd = S.VA_DTYPE_BF16 if dtype == "bf16" else S.VA_DTYPE_F32
    _lib.check(lib.va_seg_sppf_pool(_lib.stream_ptr(), ctypes.c_void_p(buf.data_ptr()), B, H, W, c, ld, vd), "sppf")
    torch.cuda.synchronize()
    y = x.float().permute(0, 3, 1, 2)
    for k in range(1, 4):
        y = F.max_pool2d(y, 5, 1, 2)
        got = buf[..., k * c:(k + 1) * c].float().cpu().permute(0, 3, 1, 2)
        assert torch.equal(got, y), (k, (got - y).abs().max())


def test_fused_tail_matches_unfused(monkeypatch):
    """proto.cv2+proto.cv3 and the head's cv2/cv3/cv4 .l.1+.l.2 pairs run as one op (1x1 tail in the 3x3's epilogue, va_conv_args.w2);
    the tail sees the same bf16-rounded activations the unfused layer stores, so both plans agree to
    fp32 accumulation-order noise."""
    monkeypatch.setenv("VA_FOLD_PROTO", "0")  # keep proto.cv2 -> proto.cv3 as the Cout-128 tail case
    arch, fw, net = _net("bf16", "s")
    frames = _frames(2, seed=5)
    names = [m["name"] for m in net.plan(2, 640, 640)["meta"]]
    assert "model.22.proto.cv2+model.22.proto.cv3" in names
    assert sum("+" in n and "fused" not in n for n in names) == 10  # proto + cv2/cv3/cv4 at 3 levels
    fused = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_FUSE_TAIL", "0")
    from vision_assist_amd.seg import SegNet
    net2 = SegNet(arch, fw, dtype="bf16")
    assert not any("+" in m["name"] and "fused" not in m["name"] for m in net2.plan(2, 640, 640)["meta"])
    plain = _gpu_heads(net2, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), fused, plain):
        err = ((g - r).abs().max() / r.abs().max()).item()
        assert err < 1e-3, f"{name}: fused vs unfused {err}"


@pytest.mark.parametrize("scale,res", [("s", 640), ("m", 320)])
def test_proto_subpixel_fold(monkeypatch, scale, res):
    """bf16 proto via the sub-pixel fold (upsample + cv2 [+ cv3 as its tail] as one mode-2 op; m's 192-channel proto
    folds without the tail, cv3 a 1x1 of its own) vs the unfolded deconv -> 3x3 -> 1x1 chain and vs the fp32 torch
    reference: the fold drops the bf16 rounding of the 4x intermediate (s), so it must be at least about as close to
    fp32 as the unfolded path."""
    arch, fw, net = _net("bf16", scale)
    names = [m["name"] for m in net.plan(2, res, res)["meta"]]
    assert any("sub-pixel fold" in n for n in names)
    frames = _frames(2, res, res, seed=6)
    ref = _ref_heads(arch, fw, frames)[3]
    folded = _gpu_heads(net, frames)[3]
    monkeypatch.setenv("VA_FOLD_PROTO", "0")
    from vision_assist_amd.seg import SegNet
    plain = _gpu_heads(SegNet(arch, fw, dtype="bf16"), frames)[3]
    rel = lambda g, r: ((g - r).norm() / r.norm()).item()
    assert rel(folded, ref) < 2e-2, rel(folded, ref)
    assert rel(folded, ref) < 1.25 * rel(plain, ref) + 1e-3, (rel(folded, ref), rel(plain, ref))
    assert rel(folded, plain) < 3e-2


@pytest.mark.parametrize("cout,H,W", [(32, 64, 64), (48, 34, 48), (64, 40, 80), (16, 16, 16)])
def test_conv0_fused_preprocess(cout, H, W):
    """va_seg_conv0 (uint8 BGR -> RGB/255 -> 3x3 s2 conv + bias + SiLU) vs torch fp32 on the same
    bf16-rounded inputs/weights; covers odd fragment counts (48) and ragged edges (H = 34)."""
    import ctypes
    from vision_assist_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(cout + H + W)
    B = 2
    frames = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8)
    w = torch.randn(cout, 3, 3, 3, generator=g) * 0.3
    b = torch.randn(cout, generator=g) * 0.1
    wp = torch.zeros(cout, 32)
    wp[:, :27] = w.permute(0, 2, 3, 1).reshape(cout, 27)  # k = (ky*3 + kx)*3 + c, c in RGB
    wd = wp.to(torch.bfloat16).cuda()
    bd = b.float().cuda()
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    y = torch.zeros(B, Ho, Wo, cout, dtype=torch.bfloat16, device="cuda")
    fd = frames.cuda()
    rc = lib.va_seg_conv0(_lib.stream_ptr(), ctypes.c_void_p(fd.data_ptr()), B, H, W, ctypes.c_void_p(wd.data_ptr()),
                          ctypes.c_void_p(bd.data_ptr()), cout, ctypes.c_void_p(y.data_ptr()), cout)
    _lib.check(rc, "va_seg_conv0")
    torch.cuda.synchronize()
    x = (frames.flip(-1).float() / 255.0).to(torch.bfloat16).float().permute(0, 3, 1, 2)
    ref = F.silu(F.conv2d(x, w.to(torch.bfloat16).float(), b, 2, 1))
    got = y.float().cpu().permute(0, 3, 1, 2)
    err = ((got - ref).abs() / (ref.abs() + 0.05)).max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("cout,H,W", [(32, 64, 64), (48, 34, 48), (64, 40, 80), (16, 16, 16), (32, 640, 640)])
def test_conv0_f32_mfma_matches_fp32(cout, H, W):
    """va_seg_conv0_f32m (three exact bf16 weight terms x the raw frame bytes on the MFMA, the sum scaled by 1/255)
    against torch fp32 (x / 255 then conv2d, bias, SiLU) and against the VALU kernel va_seg_conv0_f32: f32-level
    agreement (odd fragment count at 48, ragged edges at H = 34, a full 640 frame)."""
    import ctypes
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import split3_bf16
    lib = _lib.load()
    g = torch.Generator().manual_seed(cout + H + W + 7)
    B = 2
    frames = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8)
    w = torch.randn(cout, 3, 3, 3, generator=g) * 0.3
    b = torch.randn(cout, generator=g) * 0.1
    wp = torch.zeros(cout, 32)
    wp[:, :27] = w.permute(0, 2, 3, 1).reshape(cout, 27)
    w3 = split3_bf16(wp).cuda()
    w27 = wp[:, :27].contiguous().cuda()
    bd = b.float().cuda()
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    fd = frames.cuda()
    ym = torch.full((B, Ho, Wo, cout), float("nan"), device="cuda")
    yv = torch.full((B, Ho, Wo, cout), float("nan"), device="cuda")
    _lib.check(lib.va_seg_conv0_f32m(_lib.stream_ptr(), ctypes.c_void_p(fd.data_ptr()), B, H, W,
                                     ctypes.c_void_p(w3.data_ptr()), ctypes.c_void_p(bd.data_ptr()), cout,
                                     ctypes.c_void_p(ym.data_ptr()), cout), "va_seg_conv0_f32m")
    _lib.check(lib.va_seg_conv0_f32(_lib.stream_ptr(), ctypes.c_void_p(fd.data_ptr()), B, H, W,
                                    ctypes.c_void_p(w27.data_ptr()), ctypes.c_void_p(bd.data_ptr()), cout,
                                    ctypes.c_void_p(yv.data_ptr()), cout), "va_seg_conv0_f32")
    torch.cuda.synchronize()
    x = (frames.flip(-1).float() / 255.0).permute(0, 3, 1, 2)
    ref = F.silu(F.conv2d(x.double(), w.double(), b.double(), 2, 1)).float()
    got = ym.cpu().permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 2e-6 * max(1.0, ref.abs().max().item())
    assert (got - yv.cpu().permute(0, 3, 1, 2)).abs().max().item() < 4e-6 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B", [2, 3])
def test_conv3t_matches_conv2_f32(B, monkeypatch, switch):
    """conv3t (pre-split weight planes by LDS-DMA, activations split once per workgroup, 32 x 32 blocks) against
    conv2's three-term form (VA_CONV3T=0) on the f32 forward's wide layers -- 3x3 and 1x1, stride 2, Cout 224 (a
    ragged channel tile), the proto sub-pixel fold (mode 2), ragged pixel tiles at B = 3: the same six exact term
    products per f32 product summed in another order, so f32-rounding close; and within the f32 bar of torch."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(B, seed=11)
    switch("VA_CONV3T", "0")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV3T")
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: conv3t vs conv2 max diff {d}"
    if B == 2:
        torch.set_num_threads(8)
        want = _ref_heads(arch, fw, frames)
        for name, g, r in zip(("box", "cls", "coef", "proto"), got, want):
            assert (g - r).abs().max().item() <= 1e-3, name


@pytest.mark.parametrize("cin,cout,H,W,B,residual", [
    (128, 224, 80, 80, 2, False),  # TW 16 tiles cover the map exactly; Cout 224: a ragged channel tile
    (128, 256, 23, 21, 3, True),   # TW 8, ragged columns, tiles straddling images of the stacked map, residual
    (256, 128, 20, 20, 3, False),  # TW 4 (the P5 map), 32-row tiles spanning two images
    (64, 96, 40, 40, 2, False),    # four 16-channel chunks, TW 8 with 16-row tiles across the image seam
    (64, 64, 80, 80, 2, False),    # the narrow form (64-channel tiles): a C2f bottleneck 3x3 at P3
    (64, 48, 23, 21, 3, True),     # narrow, ragged channels / columns, image seams, residual
    (32, 64, 40, 40, 2, False),    # narrow, two chunks
])
def test_conv3h_op(monkeypatch, cin, cout, H, W, B, residual, switch):
    """conv3h (halo-staged B: the tile's input halo loaded and split once per 16-channel chunk, every 3x3 tap read
    from it; zero rows where a tap leaves the pixel's image) on single f32 ops: within f32 rounding of torch fp32
    and of conv3t (VA_CONV3H=0: per-tap staging, the same six term products summed in another order)."""
    got, ref = _run_single_conv("f32", cin, cout, 3, 1, H, W, residual, w3=True, B=B)
    scale = max(1.0, ref.abs().max().item())
    assert (got - ref).abs().max().item() <= 2e-5 * scale, (got - ref).abs().max().item()
    switch("VA_CONV3H", "0")
    got_t, _ = _run_single_conv("f32", cin, cout, 3, 1, H, W, residual, w3=True, B=B)
    assert (got - got_t).abs().max().item() <= 2e-5 * scale


@pytest.mark.parametrize("cin,cout,c2,act2,H,W,B", [
    (64, 64, 64, False, 40, 40, 2),    # the box branch: narrow main conv (64-channel tile), 64 float outputs
    (128, 128, 80, False, 23, 21, 3),  # the cls branch: 80 outputs (a ragged third 32-row block), image seams
    (128, 128, 32, True, 20, 20, 3),   # proto.cv3's shape: 32 outputs with SiLU
    (32, 32, 32, False, 80, 80, 3),    # the cv4 branch (cv4.l.1 -> cv4.l.2) on conv3q's tail form
    (32, 32, 20, True, 37, 45, 5),     # conv3q's tail: ragged tiles, fewer outputs, SiLU
])
def test_conv3h_fused_tail_op(cin, cout, c2, act2, H, W, B):
    """The f32 fused 1x1 tail (va_seg.hip conv_tail32; 32-channel main convs: conv3q's TAIL form): a stride-1 3x3
    conv whose whole channel set is one tile, + bias + SiLU, contracted in the epilogue with the tail's pre-split
    weights (six exact term products per f32 product) + b2 (+ SiLU): within f32 rounding of torch fp32 of the two
    layers in sequence."""
    import ctypes

    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    from vision_assist_amd.seg_arch import Arch
    g = torch.Generator().manual_seed(cin + 7 * c2 + B)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    w2 = torch.randn(c2, cout, 1, 1, generator=g) * (2.0 / cout) ** 0.5
    b2 = torch.randn(c2, generator=g) * 0.1
    x = torch.randn(B, cin, H, W, generator=g)
    net = S.SegNet.__new__(S.SegNet)
    net.arch, net.dtype, net.tdtype, net.va_dtype, net.vec = Arch("n"), "f32", torch.float32, S.VA_DTYPE_F32, 4
    net.device = torch.device("cuda")
    net.lib = _lib.load()
    p, p2 = net._pack(w, b), net._pack(w2, b2)
    planes = S.split3_bf16(p2.w[:32 * ((c2 + 31) // 32), :cout])
    ld_in = cin + 8
    xin = torch.zeros(B, H, W, ld_in, dtype=torch.float32, device="cuda")
    xin[..., :cin] = x.permute(0, 2, 3, 1).cuda()
    ld_out = c2 + 12
    y = torch.zeros(B, H, W, ld_out, dtype=torch.float32, device="cuda")
    args = S.ConvArgs(x=xin.data_ptr(), N=B, H=H, W=W, Cin=p.cin, ldx=ld_in, kh=3, kw=3, stride=1, pad=1, Ho=H,
                      Wo=W, w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad,
                      y=y.data_ptr() + 4 * 4, ldy=ld_out, act=1, mode=0, M=B * H * W, dtype=S.VA_DTYPE_F32,
                      w3=p.w3.data_ptr() if p.w3 is not None else None, w2=planes.data_ptr(), b2=p2.b.data_ptr(),
                      c2=c2, act2=1 if act2 else 0)
    _lib.check(net.lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(args)), "va_seg_conv")
    torch.cuda.synchronize()
    got = y[..., 4:4 + c2].cpu().permute(0, 3, 1, 2)
    assert int(y[..., :4].abs().sum()) == 0 and int(y[..., 4 + c2:].abs().sum()) == 0  # nothing outside the slice
    ref = F.conv2d(F.silu(F.conv2d(x.double(), w.double(), b.double(), 1, 1)), w2.double(), b2.double())
    if act2:
        ref = F.silu(ref)
    scale = max(1.0, ref.abs().max().item())
    assert (got.double() - ref).abs().max().item() <= 2e-5 * scale, (got.double() - ref).abs().max().item()


def test_conv3q_tail_forward(monkeypatch):
    """B = 44: the head's cv4.0.1 -> cv4.0.2 fused on conv3q (1,100 tiles of the 80 x 80 map: four per CU); heads
    against the same forward with the tails unfused (VA_FUSE_TAIL=0): f32-rounding close."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(44, seed=43)
    names = [m["name"] for m in net.plan(44, 640, 640)["meta"]]
    assert "model.22.cv4.0.1+model.22.cv4.0.2" in names and "model.22.cv4.1.1" in names  # level 1: 275 tiles
    got = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_FUSE_TAIL", "0")
    net._plans.clear()
    assert "model.22.cv4.0.2" in [m["name"] for m in net.plan(44, 640, 640)["meta"]]
    ref = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: fused vs unfused max diff {d}"


def test_fused_tails_f32_forward(monkeypatch):
    """The f32 forward with the head's box / cls 1x1s and proto.cv3 in their 3x3s' epilogues (conv3h + conv_tail32;
    the plan's op names carry the fusion) against the same forward unfused (VA_FUSE_TAIL=0): f32-rounding close,
    and within the f32 bar of torch."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(3, seed=17)
    monkeypatch.setenv("VA_FUSE_TAIL", "0")
    ref = _gpu_heads(net, frames)
    assert not any("+model.22" in m["name"] or "+cv3" in m["name"] for m in net.plan(3, 640, 640)["meta"])
    monkeypatch.delenv("VA_FUSE_TAIL")
    net._plans.clear()
    # fused where the launch has >= 128 tiles (level 0 and the fold at B = 3); level 1's 38 tiles stay on conv2's
    # split-K form, unfused
    names = [m["name"] for m in net.plan(3, 640, 640)["meta"]]
    assert "model.22.cv3.0.1+model.22.cv3.0.2" in names and "model.22.cv2.0.1+model.22.cv2.0.2" in names
    assert "model.22.proto.upsample+cv2+cv3 (sub-pixel fold)" in names and "model.22.cv3.1.1" in names
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: fused vs unfused max diff {d}"
    torch.set_num_threads(8)
    want = _ref_heads(arch, fw, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, want):
        assert (g - r).abs().max().item() <= 1e-3, name


@pytest.mark.parametrize("B", [2, 3])
def test_conv3h_matches_conv3t_forward(B, monkeypatch, switch):
    """The f32 forward with conv3h on its layers (every stride-1 3x3 with Cout > 64: P3-P5 C2f bottlenecks, the
    head's fused first 3x3 (Cout 224) and cls 3x3s, proto.cv1; the proto sub-pixel fold's 2x2 taps in mode 2) against
    the same forward on conv3t (VA_CONV3H=0): f32-rounding close, and within the f32 bar of torch."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(B, seed=13)
    switch("VA_CONV3H", "0")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV3H")
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: conv3h vs conv3t max diff {d}"
    if B == 2:
        torch.set_num_threads(8)
        want = _ref_heads(arch, fw, frames)
        for name, g, r in zip(("box", "cls", "coef", "proto"), got, want):
            assert (g - r).abs().max().item() <= 1e-3, name


def test_patch_conv_matches_dn(monkeypatch, switch):
    """The patch-staged narrow 3x3 kernel (input patch in LDS once per 16 x 16 tile) against the im2col
    narrow-layer kernel on a whole bf16 forward (P2/P3 bottlenecks with residuals, the fused head tails).
    The 3x3 GEMMs use the same fragments and K order (bit-identical: cls and proto, which only see those);
    the fused 1x1 tails (box and coef branches) sum their 64 / 32 channels in a different order (the patch
    kernel's channel-permuted weights make the tail's K order natural), so those agree to f32 rounding."""
    arch, fw, net = _net("bf16", "s", seed=8)
    frames = _frames(2, seed=9)
    switch("VA_CONV_PATCH", "0")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV_PATCH")
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        if name in ("cls", "proto"):
            assert torch.equal(g, r), f"{name}: patch vs dn max diff {(g - r).abs().max().item()}"
        else:
            err = ((g - r).abs().max() / r.abs().max()).item()
            assert err < 1e-5, f"{name}: patch vs dn rel diff {err}"


@pytest.mark.parametrize("cin,cout,k,stride,H,W,residual", [
    (128, 256, 3, 1, 23, 21, False),  # ragged pixel tile
    (128, 224, 3, 2, 40, 38, False),  # stride 2, ragged channel tile (head.l.0 width)
    (256, 384, 1, 1, 17, 30, True),   # 1x1, two channel tiles, residual
])
def test_conv4_op(monkeypatch, cin, cout, k, stride, H, W, residual, switch):
    """conv4 (256 x 256 tiles, four-phase K-tile with counted vmcnt, permuted weight rows, epilogue from the
    accumulators) forced on single ops vs torch fp32 on the same bf16-rounded inputs."""
    switch("VA_CONV4", "all")
    got, ref = _run_single_conv("bf16", cin, cout, k, stride, H, W, residual, False, 0, act=True)
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 2e-2, err


def test_conv4_matches_conv2(monkeypatch, switch):
    """conv4 forced onto every eligible layer of a bf16 forward (Cout > 128, Cin % 64 == 0) against conv2:
    same 32-deep MFMA k-sequence per output, so bit-identical."""
    arch, fw, net = _net("bf16", "s", seed=12)
    frames = _frames(2, seed=13)
    switch("VA_SPLITK", "0")  # conv2 slicing the P5 layers' K loops would sum in another order
    switch("VA_CONV4", "0")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV4", "all")
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        assert torch.equal(g, r), f"{name}: conv4 vs conv2 max diff {(g - r).abs().max().item()}"


def _c2f_reference(x, fw, i):
    """block.py C2f(n=1, shortcut) in fp32 on the CPU with every intermediate rounded to bf16 the way the
    unfused layers store it (x: NCHW float of bf16 values)."""
    bf = lambda t: t.to(torch.bfloat16).float()
    silu = torch.nn.functional.silu
    w1, b1 = fw[f"model.{i}.cv1"]
    wm1, bm1 = fw[f"model.{i}.m.0.cv1"]
    wm2, bm2 = fw[f"model.{i}.m.0.cv2"]
    w2, b2 = fw[f"model.{i}.cv2"]
    t = bf(silu(F.conv2d(x, w1.float(), b1.float())))
    a, b = t[:, :32], t[:, 32:]
    m = bf(silu(F.conv2d(b, wm1.float(), bm1.float(), padding=1)))
    bp = bf(silu(F.conv2d(m, wm2.float(), bm2.float(), padding=1)) + b)
    return bf(silu(F.conv2d(torch.cat([a, b, bp], 1), w2.float(), b2.float())))


@pytest.mark.parametrize("B,H,W,ldx,ldy", [(3, 160, 160, 64, 64), (1, 40, 56, 72, 80), (3, 24, 20, 64, 64),
                                           (1, 7, 33, 64, 72)])
def test_c2f_fused_op(B, H, W, ldx, ldy):
    """va_seg_c2f (model.2 as one kernel: cv1 -> m.0.cv1 -> m.0.cv2 + residual -> cv2) vs the block in
    fp32 with the unfused layers' bf16 rounding; ragged tiles (H, W not multiples of 16), channel slices
    and a persistent grid that walks several tiles per workgroup."""
    import ctypes
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    arch, fw, net = _net("bf16", "s")
    assert 2 in net.c2f_fused
    blob, bias = net.c2f_fused[2]
    g = torch.Generator().manual_seed(B * 1000 + H + W)
    xin = torch.zeros(B, H, W, ldx, dtype=torch.bfloat16)
    xin[..., :64] = (torch.randn(B, H, W, 64, generator=g) * 1.5).to(torch.bfloat16)
    xd = xin.cuda()
    y = torch.full((B, H, W, ldy), 7.0, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=xd.data_ptr(), N=B, H=H, W=W, Cin=64, ldx=ldx, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                   y=y.data_ptr(), ldy=ldy, dtype=S.VA_DTYPE_BF16)
    lib = _lib.load()
    _lib.check(lib.va_seg_c2f(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_c2f")
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert (got[..., 64:] == 7.0).all(), "wrote outside its channel slice"
    ref = _c2f_reference(xin[..., :64].float().permute(0, 3, 1, 2), fw, 2).permute(0, 2, 3, 1)
    got = got[..., :64]
    # the same block as the four unfused layers (va_seg_conv through the 96-channel concat buffer)
    t = torch.zeros(B, H, W, 96, dtype=torch.bfloat16, device="cuda")
    tmp = torch.zeros(B, H, W, 32, dtype=torch.bfloat16, device="cuda")
    y2 = torch.zeros(B, H, W, 64, dtype=torch.bfloat16, device="cuda")
    es = 2

    def conv(prefix, x, ldx_, y_, ldy_, res=None):
        p = net.w[prefix]
        c = S.ConvArgs(x=x, N=B, H=H, W=W, Cin=p.cin, ldx=ldx_, kh=p.k, kw=p.k, stride=1, pad=p.k // 2, Ho=H, Wo=W,
                       w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=p.cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad, y=y_,
                       ldy=ldy_, res=res, ldr=96 if res else 0, act=1, mode=0, M=B * H * W, dtype=S.VA_DTYPE_BF16)
        _lib.check(lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(c)), prefix)

    conv("model.2.cv1", xd.data_ptr(), ldx, t.data_ptr(), 96)
    conv("model.2.m.0.cv1", t.data_ptr() + 32 * es, 96, tmp.data_ptr(), 32)
    conv("model.2.m.0.cv2", tmp.data_ptr(), 32, t.data_ptr() + 64 * es, 96, res=t.data_ptr() + 32 * es)
    conv("model.2.cv2", t.data_ptr(), 96, y2.data_ptr(), 64)
    torch.cuda.synchronize()
    plain = y2.float().cpu()
    rel = lambda u, v: ((u - v).norm() / v.norm()).item()
    # both differ from the reference by bf16 rounding flips (fast SiLU, accumulation order) that the
    # chain of four layers spreads; the fused block must be no further from it than the unfused layers
    assert rel(plain, ref) < 1e-2, rel(plain, ref)
    assert rel(got, ref) < 1.25 * rel(plain, ref) + 5e-4, (rel(got, ref), rel(plain, ref))
    assert ((got - ref).abs() <= 0.03 * ref.abs() + 2e-2).float().mean().item() > 0.999


def test_c2f_fused_in_plan(monkeypatch):
    """The bf16 's' plan runs model.2 as one fused op, and the heads match the plan without it."""
    arch, fw, net = _net("bf16", "s")
    names = [m["name"] for m in net.plan(2, 640, 640)["meta"]]
    assert "model.2 (fused C2f)" in names and "model.2.cv1" not in names
    frames = _frames(2, seed=9)
    fused = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_C2F", "0")
    from vision_assist_amd.seg import SegNet
    net2 = SegNet(arch, fw, dtype="bf16")
    assert "model.2.cv1" in [m["name"] for m in net2.plan(2, 640, 640)["meta"]]
    plain = _gpu_heads(net2, frames)
    for name, g_, r in zip(("box", "cls", "coef", "proto"), fused, plain):
        err = ((g_ - r).norm() / r.norm()).item()
        assert err < 1e-2, f"{name}: fused vs unfused C2f {err}"


def _stem_reference(frames_u8, fw):
    """preprocess + model.0 + SiLU (rounded to bf16 as the stored layer) + model.1 + SiLU in fp32 on the CPU
    (frames: [B, H, W, 3] uint8 BGR)."""
    bf = lambda t: t.to(torch.bfloat16).float()
    silu = torch.nn.functional.silu
    x = bf(frames_u8[..., [2, 1, 0]].float().permute(0, 3, 1, 2) / 255.0)
    w0, b0 = fw["model.0"]
    w1, b1 = fw["model.1"]
    a0 = bf(silu(F.conv2d(x, bf(w0.float()), b0.float(), stride=2, padding=1)))
    return bf(silu(F.conv2d(a0, bf(w1.float()), b1.float(), stride=2, padding=1)))


@pytest.mark.parametrize("B,H,W,ldy", [(3, 640, 640, 64), (1, 96, 160, 72), (2, 64, 48, 64), (1, 40, 80, 64)])
def test_stem_fused_op(B, H, W, ldy):
    """va_seg_stem (uint8 frame -> model.0 -> model.1 as one kernel) vs the fp32 reference with the unfused
    layers' bf16 rounding, and no further from it than the unfused va_seg_conv0 + va_seg_conv pair; ragged
    tiles (output not a multiple of 16) and a persistent grid walking several tiles per workgroup."""
    import ctypes
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    arch, fw, net = _net("bf16", "s")
    assert net.stem is not None
    blob, bias = net.stem
    g = torch.Generator().manual_seed(B * 7 + H + W)
    fr = torch.randint(0, 256, (B, H, W, 3), generator=g, dtype=torch.uint8)
    frd = fr.cuda()
    Ho1, Wo1 = (H + 3) // 4, (W + 3) // 4
    y = torch.full((B, Ho1, Wo1, ldy), 7.0, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=frd.data_ptr(), N=B, H=H, W=W, Cin=32, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                   y=y.data_ptr(), ldy=ldy, dtype=S.VA_DTYPE_BF16)
    lib = _lib.load()
    _lib.check(lib.va_seg_stem(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_stem")
    # unfused: va_seg_conv0 -> [B, H/2, W/2, 32] -> va_seg_conv model.1
    a0 = torch.zeros(B, (H + 1) // 2, (W + 1) // 2, 32, dtype=torch.bfloat16, device="cuda")
    _lib.check(lib.va_seg_conv0(_lib.stream_ptr(), ctypes.c_void_p(frd.data_ptr()), B, H, W,
                                ctypes.c_void_p(net.w0[0].data_ptr()), ctypes.c_void_p(net.w0[1].data_ptr()), 32,
                                ctypes.c_void_p(a0.data_ptr()), 32), "conv0")
    y2 = torch.zeros(B, Ho1, Wo1, 64, dtype=torch.bfloat16, device="cuda")
    p = net.w["model.1"]
    c = S.ConvArgs(x=a0.data_ptr(), N=B, H=a0.shape[1], W=a0.shape[2], Cin=p.cin, ldx=32, kh=3, kw=3, stride=2, pad=1,
                   Ho=Ho1, Wo=Wo1, w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=64, Npad=p.Npad, K=p.K, Kpad=p.Kpad,
                   y=y2.data_ptr(), ldy=64, act=1, mode=0, M=B * Ho1 * Wo1, dtype=S.VA_DTYPE_BF16)
    _lib.check(lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(c)), "model.1")
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert (got[..., 64:] == 7.0).all(), "wrote outside its channel slice"
    got = got[..., :64]
    plain = y2.float().cpu()
    ref = _stem_reference(fr, fw).permute(0, 2, 3, 1)
    rel = lambda u, v: ((u - v).norm() / v.norm()).item()
    assert rel(plain, ref) < 1e-2, rel(plain, ref)
    assert rel(got, ref) < 1.25 * rel(plain, ref) + 5e-4, (rel(got, ref), rel(plain, ref))
    assert ((got - ref).abs() <= 0.03 * ref.abs() + 2e-2).float().mean().item() > 0.999


def test_stem_fused_in_plan(monkeypatch):
    """The bf16 's' plan runs preprocess + model.0 + model.1 as one op; heads match the plan without it."""
    arch, fw, net = _net("bf16", "s")
    names = [m["name"] for m in net.plan(2, 640, 640)["meta"]]
    assert "model.0+model.1 (fused stem)" in names and "model.1" not in names
    frames = _frames(2, seed=11)
    fused = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_STEM", "0")
    from vision_assist_amd.seg import SegNet
    net2 = SegNet(arch, fw, dtype="bf16")
    assert "model.1" in [m["name"] for m in net2.plan(2, 640, 640)["meta"]]
    plain = _gpu_heads(net2, frames)
    for name, g_, r in zip(("box", "cls", "coef", "proto"), fused, plain):
        err = ((g_ - r).norm() / r.norm()).item()
        assert err < 1e-2, f"{name}: fused vs unfused stem {err}"


@pytest.mark.parametrize("B,H,W,cu,cin,cout", [(2, 40, 40, 512, 768, 256),   # model.12.cv1 shape (conv2)
                                                (4, 128, 128, 128, 192, 256),  # conv4 (>= 256 tiles)
                                                (1, 26, 34, 256, 384, 128),    # model.15.cv1 shape, ragged
                                                (2, 16, 20, 64, 128, 64)])     # conv2 4 x 1 waves
def test_conv_upsampled_prefix(B, H, W, cu, cin, cout):
    """va_conv_args.xu: a 1x1 conv whose first cu input channels are the nearest-x2 upsample of a half-
    resolution slice, read in place (the FPN Upsample + Concat never materialised) vs torch fp32 on the
    materialised concat.  The concat buffer's first cu channels hold NaN: any read of them shows."""
    import ctypes
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    g = torch.Generator().manual_seed(H * W + cin)
    w = torch.randn(cout, cin, 1, 1, generator=g) * (2.0 / cin) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    net = S.SegNet.__new__(S.SegNet)
    net.dtype, net.tdtype, net.va_dtype, net.vec = "bf16", torch.bfloat16, S.VA_DTYPE_BF16, 8
    net.device = torch.device("cuda")
    p = net._pack(w, b)
    ldu = cu + 64
    xu = torch.zeros(B, H // 2, W // 2, ldu, dtype=torch.bfloat16)
    xu[..., 32:32 + cu] = torch.randn(B, H // 2, W // 2, cu, generator=g).to(torch.bfloat16)
    xc = torch.full((B, H, W, cin), float("nan"), dtype=torch.bfloat16)
    xc[..., cu:] = torch.randn(B, H, W, cin - cu, generator=g).to(torch.bfloat16)
    xud, xcd = xu.cuda(), xc.cuda()
    y = torch.zeros(B, H, W, cout, dtype=torch.bfloat16, device="cuda")
    a = S.ConvArgs(x=xcd.data_ptr(), N=B, H=H, W=W, Cin=cin, ldx=cin, kh=1, kw=1, stride=1, pad=0, Ho=H, Wo=W,
                   w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad, y=y.data_ptr(),
                   ldy=cout, act=1, mode=0, M=B * H * W, dtype=S.VA_DTYPE_BF16,
                   xu=xud.data_ptr() + 32 * 2, ldu=ldu, cu=cu)
    lib = _lib.load()
    _lib.check(lib.va_seg_conv(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_conv xu")
    torch.cuda.synchronize()
    up = xu[..., 32:32 + cu].float().repeat_interleave(2, 1).repeat_interleave(2, 2)
    xin = torch.cat([up, xc[..., cu:].float()], -1).permute(0, 3, 1, 2)
    ref = F.silu(F.conv2d(xin, w.to(torch.bfloat16).float(), b)).permute(0, 2, 3, 1)
    got = y.float().cpu()
    assert torch.isfinite(got).all(), "read the NaN prefix of the concat buffer"
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


def test_fpn_upsample_read_in_place(monkeypatch):
    """The bf16 plan has no upsample ops (model.12 / model.15 cv1 read the upsampled halves in place); the
    heads match the plan that materialises them (same GEMMs, same operand values)."""
    arch, fw, net = _net("bf16", "s")
    kinds = [m["kind"] for m in net.plan(2, 640, 640)["meta"]]
    assert "upsample" not in kinds
    frames = _frames(2, seed=14)
    fused = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_FUSE_UP", "0")
    from vision_assist_amd.seg import SegNet
    net2 = SegNet(arch, fw, dtype="bf16")
    assert [m["kind"] for m in net2.plan(2, 640, 640)["meta"]].count("upsample") == 2
    plain = _gpu_heads(net2, frames)
    for name, g_, r in zip(("box", "cls", "coef", "proto"), fused, plain):
        assert torch.equal(g_, r), f"{name}: in-place upsample vs materialised, max diff {(g_ - r).abs().max().item()}"


def test_forward_large_batch_pw_matches_conv2(monkeypatch, switch):
    """At bench batch sizes the persistent kernels loop over many tiles per wave (the 4-frame tests run one
    tile per wave): a 64-frame forward is finite, repeatable, and the streaming 1x1 layers agree with the same
    layers on conv2 (VA_PW=0) to bf16 rounding."""
    arch, fw, net = _net("bf16", "s")
    frames = _frames(64, seed=3).cuda()

    def run():
        out = net.forward(frames)
        torch.cuda.synchronize()
        return torch.cat([t.float().flatten(1, 2) for t in out.levels], 1), out.proto.float()

    switch("VA_PW", "1")
    a, b = run(), run()
    switch("VA_PW", "0")
    c = run()
    for x, y, z in zip(a, b, c):
        assert torch.isfinite(x).all()
        assert torch.equal(x, y)
        assert ((x - z).abs().max() / z.abs().max()).item() < 2e-2


def test_forward_deterministic():
    """Five bf16 forwards of the same frames are bit-identical (every kernel of the plan: stem, C2f, the
    streaming 1x1, conv2 / conv4 / patch / tails, the proto fold): a scheduling hazard or race shows up as
    run-to-run differences long before it breaks a tolerance."""
    arch, fw, net = _net("bf16", "s")
    frames = _frames(4, seed=21)
    first = _gpu_heads(net, frames)
    for _ in range(4):
        again = _gpu_heads(net, frames)
        for name, g_, r in zip(("box", "cls", "coef", "proto"), again, first):
            assert torch.isfinite(g_).all(), name
            assert torch.equal(g_, r), f"{name}: run-to-run max diff {(g_ - r).abs().max().item()}"


@pytest.mark.parametrize("dtype,scale,B", [("bf16", "s", 1), ("f32", "s", 1), ("bf16", "n", 3), ("f32", "n", 2),
                                            ("fp8", "s", 1)])
def test_lanes_match_serial(dtype, scale, B):
    """The small-batch laned list (head levels 0 / 1 and proto on lanes 1 / 2 beside the neck, head level 2's
    branches on three streams, each lane with its own split-K workspace -- va355.h VA_OP_FORK) gives bit-identical outputs to the same plan run serially,
    run after run."""
    arch, fw, net = _net(dtype, scale)
    frames = _frames(B, seed=31)
    p = net.plan(B, 640, 640)
    kinds = [m["kind"] for m in p["meta"]]
    split = dtype == "f32"  # head level 2's branches on lanes too
    assert kinds.count("sync") == (7 if split else 4)
    assert {op.lane for op in p["ops"]} == ({0, 1, 2, 3} if split else {0, 1, 2})
    assert sorted(m["name"] for m in p["meta"] if m["kind"] != "sync") == \
        sorted(m["name"] for m in net.plan(B, 640, 640, lanes=False)["meta"])
    laned = [_gpu_heads(net, frames) for _ in range(3)]
    net.lanes = False
    net._plans.clear()
    assert "sync" not in [m["kind"] for m in net.plan(B, 640, 640)["meta"]]
    serial = _gpu_heads(net, frames)
    for run in laned:
        for name, g_, r in zip(("box", "cls", "coef", "proto"), run, serial):
            assert torch.isfinite(g_).all(), name
            assert torch.equal(g_, r), f"{name}: laned vs serial max diff {(g_ - r).abs().max().item()}"


def test_lanes_two_streams_concurrently():
    """Two laned batch-1 plans (own buffers, tags 0 / 1) enqueued alternately on two streams, so both forwards and
    their lanes are in flight together: each calling stream gets its own lane set (va_seg.hip lane_set) and each
    plan its own split-K workspaces, so the outputs equal a serial run of the same frames, round after round."""
    arch, fw, net = _net("f32", "n")
    fa, fb = _frames(1, seed=41).cuda(), _frames(1, seed=42).cuda()
    pa, pb = net.plan(1, 640, 640, tag=0), net.plan(1, 640, 640, tag=1)
    assert {op.lane for op in pa["ops"]} >= {1, 2}
    ser = net.plan(1, 640, 640, tag=2, lanes=False)

    def serial(frames):
        ser["frames"].copy_(frames)
        net.run_plan(ser)
        torch.cuda.synchronize()
        return [t.clone() for t in ser["out"].levels] + [ser["out"].proto.clone()]

    want_a, want_b = serial(fa), serial(fb)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(4):
        for p, f, st in ((pa, fa, sa), (pb, fb, sb)):
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                p["frames"].copy_(f, non_blocking=True)
                net.run_plan(p, st)
        torch.cuda.synchronize()
        for p, want in ((pa, want_a), (pb, want_b)):
            got = list(p["out"].levels) + [p["out"].proto]
            for g_, w_ in zip(got, want):
                assert torch.equal(g_, w_)


# ---- BASELINE.json configs[4] shape (C5): YOLOv8m-seg at 1280 x 1280 (bf16 here; fp8 weights are not built)
_M1280 = {}


def _m1280_ref():
    if not _M1280:
        from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
        arch = Arch("m")
        fw = fold(arch, synthetic_state_dict(arch, seed=4))
        frames = _frames(1, 1280, 1280, seed=6)
        torch.set_num_threads(8)
        _M1280.update(arch=arch, fw=fw, frames=frames, ref=_ref_heads(arch, fw, frames))
    return _M1280


def test_forward_f32_medium_1280_within_1e3():
    """m@1280 in exact f32 against the torch fp32 oracle, relative to the logits' scale: max |gpu - r| <= 1e-5 *
    max |r|.  The headline s@640 and n@1280 tests hold 1e-3 absolute; here the synthetic m weights drive logits to
    |r| ~ 290, and at that scale fp32 rounding alone moves results by ~1e-3 absolute in any summation order --
    measured against a float64 forward of the same weights (tools/save_heads.py): torch fp32 CPU differs from it
    by 6.9e-4 (box) / 5.5e-4 (cls) / 6.3e-4 (coef) / 3.8e-4 (proto), the GPU by 1.5e-3 / 1.3e-3 / 1.2e-3 / 8.2e-4
    (5e-6 of the scale), the GPU from fp32 CPU by 1.6e-3."""
    from vision_assist_amd.seg import SegNet
    c = _m1280_ref()
    got = _gpu_heads(SegNet(c["arch"], c["fw"], dtype="f32"), c["frames"])
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, c["ref"]):
        assert g.shape == r.shape, name
        err = ((g - r).abs().max() / r.abs().max()).item()
        assert err <= 1e-5, f"{name}: max |gpu - torch fp32| / max |r| = {err}"


def test_forward_bf16_medium_1280_close():
    from vision_assist_amd.seg import SegNet
    c = _m1280_ref()
    got = _gpu_heads(SegNet(c["arch"], c["fw"], dtype="bf16"), c["frames"])
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, c["ref"]):
        rel = ((g - r).norm() / r.norm()).item()
        assert rel < 5e-2, f"{name}: relative L2 error {rel}"


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_c2_plan_nseg_bf16_batch1_vs_fp32_oracle(seed):
    """C2's own configuration (BASELINE.json configs[1]: YOLOv8n-seg 640x640 bf16, batch 1; the weights of bench.py's
    c2 extra, the sparse regime) through the plan the planner builds for it -- the laned list (head levels 0 / 1 and
    proto on lanes 1 / 2 beside the neck), split-K on the few-tile layers, model.0 fused with the preprocess, the
    patch kernel on the narrow 3x3 layers -- against the plain-PyTorch fp32 oracle (oracle/yolo_ref.py) at the bf16
    bar: relative L2 < 5e-2 per head output (the other batch-1 tests hold this plan only against itself)."""
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("n")
    fw = fold(arch, synthetic_state_dict(arch, seed=0, sparse=640))
    net = SegNet(arch, fw, dtype="bf16")
    p = net.plan(1, 640, 640)
    assert {op.lane for op in p["ops"]} == {0, 1, 2}, "the batch-1 plan is laned"
    assert p["meta"][0]["name"] == "model.0"  # preprocess fused into model.0 (conv0)
    torch.set_num_threads(8)
    frames = _frames(1, seed=seed)
    got = _gpu_heads(net, frames)
    ref = _ref_heads(arch, fw, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        assert torch.isfinite(g).all(), name
        rel = ((g - r).norm() / r.norm()).item()
        assert rel < 5e-2, f"{name}: relative L2 error {rel}"


@pytest.mark.parametrize("H,W,B,residual,slice_in", [
    (160, 160, 11, False, 0),  # model.2's bottleneck map (100 tiles per frame; conv3q from four tiles per CU)
    (160, 160, 11, True, 4),   # + the shortcut, the input a channel slice
    (37, 45, 120, True, 0),    # ragged tiles at the right / bottom edge, many frames
    (20, 20, 260, False, 0),   # head level 2's map
])
def test_conv3q_op(H, W, B, residual, slice_in, switch):
    """conv3q (the 32 -> 32 stride-1 3x3 f32 layers: weights split once into registers, each 18 x 18 input halo split
    once into LDS planes, persistent over the tiles) on single ops: within f32 rounding of torch fp32, and of conv2's
    three-term form (VA_CONV3Q=0) -- the same six term products per f32 product, summed in another order, so equal
    in value but not in every bit (which also shows that the other kernel ran)."""
    got, ref = _run_single_conv("f32", 32, 32, 3, 1, H, W, residual, slice_in=slice_in, B=B)
    scale = max(1.0, ref.abs().max().item())
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() <= 2e-5 * scale, (got - ref).abs().max().item()
    switch("VA_CONV3Q", "0")
    got_c2, _ = _run_single_conv("f32", 32, 32, 3, 1, H, W, residual, slice_in=slice_in, B=B)
    assert (got - got_c2).abs().max().item() <= 2e-5 * scale
    assert not torch.equal(got, got_c2)


def test_conv3q_dynamic_schedule(switch):
    """conv3q with a work counter (va_conv_args.wcnt: tiles claimed by the workgroups as they start, the schedule the
    plans use) against the static schedule: bit-identical (the same per-tile arithmetic), twice in a row (the last
    workgroup out zeroes the counters for the next launch), counters zero afterwards."""
    ws = (torch.empty(1 << 20, dtype=torch.uint8, device="cuda"), torch.zeros(128, dtype=torch.int32, device="cuda"))
    static, ref = _run_single_conv("f32", 32, 32, 3, 1, 160, 160, True, slice_in=4, B=11)
    for _ in range(2):
        dyn, _ = _run_single_conv("f32", 32, 32, 3, 1, 160, 160, True, slice_in=4, B=11, ws=ws)
        assert torch.equal(dyn, static), (dyn - static).abs().max().item()
        assert int(ws[1].abs().sum()) == 0
    switch("VA_CONV3Q", "static")
    st2, _ = _run_single_conv("f32", 32, 32, 3, 1, 160, 160, True, slice_in=4, B=11, ws=ws)
    assert torch.equal(st2, static)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_work_queue_forward_bit_identical(dtype, switch):
    """The persistent kernels' work-queue schedule (the plan's counter: the bf16 stem and C2f, the f32 stem + cv1 tail
    and conv3q) against their static schedule (VA_CONV3Q=static): the whole forward bit-identical, run twice (the
    counters are zeroed by each launch's last workgroup).  B = 12: conv3q on model.2's bottleneck."""
    arch, fw, net = _net(dtype, "s", seed=5)
    frames = _frames(12, seed=37)
    names = [m["name"] for m in net.plan(12, 640, 640)["meta"]]
    assert any("fused" in n and "stem" in n for n in names)
    switch("VA_CONV3Q", "static")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV3Q", None)
    for _ in range(2):
        got = _gpu_heads(net, frames)
        for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
            assert torch.equal(g, r), f"{name}: work queue vs static max diff {(g - r).abs().max().item()}"


def test_conv3q_f32_forward(switch):
    """The f32 forward with model.2's bottleneck convs on conv3q (B = 12: 1,200 tiles of the 160 x 160 map, four per
    CU) against the same forward with them on conv2 (VA_CONV3Q=0): f32-rounding close, and within the f32 bar of
    torch."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(12, seed=29)
    switch("VA_CONV3Q", "0")
    ref = _gpu_heads(net, frames)
    switch("VA_CONV3Q", None)
    got = _gpu_heads(net, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: conv3q vs conv2 max diff {d}"


@pytest.mark.parametrize("H,W,B", [(72, 112, 2), (640, 640, 1)])
@pytest.mark.parametrize("tail", [False, True])
def test_stem_f32_op_vs_fp64(H, W, B, tail):
    """va_seg_stem_f32 (uint8 frame -> model.0 -> model.1 in f32 as one kernel, model.0's map kept in LDS as three
    exact bf16 planes) on single ops against float64 torch of the two layers (x / 255, conv, SiLU, conv s2, SiLU):
    within f32 rounding; ragged model.1 tiles at 72 x 112 (18 x 28: 4 x 16 tiles), frame edges, a full 640 frame.
    tail: + model.2.cv1 (1x1, 64 -> 64, SiLU) in the epilogue, model.1's map kept in LDS too."""
    import ctypes

    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    arch, fw, net = _net("f32", "s", seed=29)
    lib = _lib.load()
    frames = _frames(B, H, W, seed=H + W)
    Ho1, Wo1 = ((H + 1) // 2 + 1) // 2, ((W + 1) // 2 + 1) // 2
    y = torch.full((B, Ho1, Wo1, 64 + 8), float("nan"), device="cuda")
    p1 = net.w["model.1"]
    a = S.ConvArgs(x=frames.cuda().data_ptr(), N=B, H=H, W=W, Cin=32, Cout=64, w3=net.w0_3.data_ptr(),
                   bias=net.w0[1].data_ptr(), w=p1.w.data_ptr(), b2=p1.b.data_ptr(), Npad=p1.Npad, K=p1.K, Kpad=p1.Kpad,
                   y=y.data_ptr(), ldy=72, dtype=S.VA_DTYPE_F32)
    if tail:
        assert net.stem32_b2 is not None
        a.w2, a.b2, a.c2, a.act2 = net.w["model.2.cv1"].w.data_ptr(), net.stem32_b2.data_ptr(), 64, 1
    fd = frames.cuda()
    a.x = fd.data_ptr()
    _lib.check(lib.va_seg_stem_f32(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_stem_f32")
    torch.cuda.synchronize()
    w0, b0 = fw["model.0"]
    w1, b1 = fw["model.1"]
    x = (frames.flip(-1).double() / 255.0).permute(0, 3, 1, 2)
    ref = F.silu(F.conv2d(F.silu(F.conv2d(x, w0.double(), b0.double(), 2, 1)), w1.double(), b1.double(), 2, 1))
    if tail:
        wc, bc = fw["model.2.cv1"]
        ref = F.silu(F.conv2d(ref, wc.double(), bc.double()))
    got = y[..., :64].cpu().permute(0, 3, 1, 2).double()
    assert torch.isfinite(y[..., :64]).all() and torch.isnan(y[..., 64:]).all()  # nothing past the slice
    scale = max(1.0, ref.abs().max().item())
    assert (got - ref).abs().max().item() <= 2e-5 * scale, (got - ref).abs().max().item()


def test_stem_f32_dynamic_schedule():
    """va_seg_stem_f32 with a work counter (va_conv_args.wcnt: the tiles claimed by the workgroups as they start, two
    ahead; the schedule the plans use) against the static schedule (no counter): bit-identical, with and without the
    cv1 tail, twice in a row (the counters are zeroed by the last workgroup out)."""
    import ctypes

    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    arch, fw, net = _net("f32", "s", seed=29)
    lib = _lib.load()
    B, H, W = 3, 640, 640
    fd = _frames(B, H, W, seed=7).cuda()
    wcnt = torch.zeros(128, dtype=torch.int32, device="cuda")
    p1 = net.w["model.1"]
    for tail in (False, True):
        outs = []
        for dyn in (False, True, True):
            y = torch.full((B, H // 4, W // 4, 64), float("nan"), device="cuda")
            a = S.ConvArgs(x=fd.data_ptr(), N=B, H=H, W=W, Cin=32, Cout=64, w3=net.w0_3.data_ptr(),
                           bias=net.w0[1].data_ptr(), w=p1.w.data_ptr(), b2=p1.b.data_ptr(), Npad=p1.Npad, K=p1.K,
                           Kpad=p1.Kpad, y=y.data_ptr(), ldy=64, dtype=S.VA_DTYPE_F32)
            if tail:
                a.w2, a.b2, a.c2, a.act2 = net.w["model.2.cv1"].w.data_ptr(), net.stem32_b2.data_ptr(), 64, 1
            if dyn:
                a.wcnt, a.ncnt = wcnt.data_ptr(), wcnt.numel()
            _lib.check(lib.va_seg_stem_f32(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_stem_f32")
            torch.cuda.synchronize()
            outs.append(y)
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[1], outs[0]) and torch.equal(outs[2], outs[0]), tail
        assert int(wcnt.abs().sum()) == 0


def test_stem_f32_forward(monkeypatch):
    """The f32 s-seg plan runs model.0 + model.1 as one op (va_seg_stem_f32); heads against the same forward with
    the two layers apart (VA_STEM=0: conv0_f32m, then conv2's three-term form): f32-rounding close, and within the
    f32 bar of torch."""
    arch, fw, net = _net("f32", "s", seed=5)
    frames = _frames(2, seed=31)
    names = [m["name"] for m in net.plan(2, 640, 640)["meta"]]
    assert "model.0+model.1+model.2.cv1 (fused f32 stem)" in names and "model.1" not in names
    assert "model.2.cv1" not in names
    got = _gpu_heads(net, frames)
    monkeypatch.setenv("VA_STEM_TAIL", "0")  # cv1 a launch of its own
    from vision_assist_amd.seg import SegNet
    net1 = SegNet(arch, fw, dtype="f32")
    names1 = [m["name"] for m in net1.plan(2, 640, 640)["meta"]]
    assert "model.0+model.1 (fused f32 stem)" in names1 and "model.2.cv1" in names1
    ref1 = _gpu_heads(net1, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref1):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: stem with / without the cv1 tail max diff {d}"
    monkeypatch.delenv("VA_STEM_TAIL")
    monkeypatch.setenv("VA_STEM", "0")
    net2 = SegNet(arch, fw, dtype="f32")
    assert "model.1" in [m["name"] for m in net2.plan(2, 640, 640)["meta"]]
    ref = _gpu_heads(net2, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, ref):
        d = (g - r).abs().max().item()
        assert d <= 1e-4 * max(1.0, r.abs().max().item()), f"{name}: fused vs unfused stem max diff {d}"
    torch.set_num_threads(8)
    want = _ref_heads(arch, fw, frames)
    for name, g, r in zip(("box", "cls", "coef", "proto"), got, want):
        assert (g - r).abs().max().item() <= 1e-3, name

"""va_seg_c2fb (va_c2fb.hip): a whole C2f block of YOLOv8n/s-seg as one launch for small batches, against the block
in fp32 with every intermediate rounded to bf16 the way the unfused layers store it (block.py C2f / Bottleneck,
the reference's model.predict at FrameProcessor.py:322), and the batch-1 n-seg forward with and without it."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (block, ci, co, n, shortcut, upsampled prefix channels, H, W) of YOLOv8n-seg at 640 x 640
N_BLOCKS = [(2, 32, 32, 1, True, 0, 160, 160), (4, 64, 64, 2, True, 0, 80, 80), (6, 128, 128, 2, True, 0, 40, 40),
            (8, 256, 256, 1, True, 0, 20, 20), (12, 384, 128, 1, False, 256, 40, 40),
            (15, 192, 64, 1, False, 128, 80, 80), (18, 192, 128, 1, False, 0, 40, 40),
            (21, 384, 256, 1, False, 0, 20, 20)]


def _block_ref(x, fw, i, n, shortcut):
    """block.py C2f in fp32 on the CPU, weights as the bf16 values the kernels read, each conv's output rounded to
    bf16 (x: NCHW float of bf16 values)."""
    bf = lambda t: t.to(torch.bfloat16).float()
    silu = F.silu

    def conv(name, t, pad=0):
        w, b = fw[name]
        return silu(F.conv2d(t, bf(w.float()), b.float(), padding=pad))

    t = bf(conv(f"model.{i}.cv1", x))
    c = t.shape[1] // 2
    ys = [t[:, :c], t[:, c:]]
    for j in range(n):
        h = bf(conv(f"model.{i}.m.{j}.cv1", ys[-1], 1))
        o = conv(f"model.{i}.m.{j}.cv2", h, 1)
        ys.append(bf(o + ys[-1] if shortcut else o))
    return bf(conv(f"model.{i}.cv2", torch.cat(ys, 1)))


# the same blocks of YOLOv8s-seg (the f32 form: the drop-in call's batch-1 network)
S_BLOCKS = [(2, 64, 64, 1, True, 0, 160, 160), (4, 128, 128, 2, True, 0, 80, 80), (6, 256, 256, 2, True, 0, 40, 40),
            (8, 512, 512, 1, True, 0, 20, 20), (12, 768, 256, 1, False, 512, 40, 40),
            (15, 384, 128, 1, False, 256, 80, 80), (18, 384, 256, 1, False, 0, 40, 40),
            (21, 768, 512, 1, False, 0, 20, 20)]


def _net(scale="n", dtype="bf16"):
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=3))
    return arch, fw, SegNet(arch, fw, dtype=dtype, c2fb_f32=dtype == "f32")


def _run_block(net, i, ci, co, n, shortcut, cu, B, H, W, T, pad_x=8, pad_y=16, seed=0):
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    f32 = net.store == "f32"
    dt = torch.float32 if f32 else torch.bfloat16
    g = torch.Generator().manual_seed(seed * 7919 + i)
    ldx, ldy = ci + pad_x, co + pad_y
    x = (torch.randn(B, H, W, ci, generator=g) * 1.5).to(dt)
    xin = torch.full((B, H, W, ldx), float("nan"), dtype=dt)  # channels never read stay NaN
    xin[..., cu:ci] = x[..., cu:]
    xu = None
    if cu:
        half = (torch.randn(B, H // 2, W // 2, cu, generator=g) * 1.5).to(dt)
        x[..., :cu] = half.repeat_interleave(2, 1).repeat_interleave(2, 2)
        xu = torch.zeros(B, H // 2, W // 2, cu + 8, dtype=dt)
        xu[..., :cu] = half
        xu = xu.cuda()
    xd = xin.cuda()
    y = torch.full((B, H, W, ldy), 7.0, dtype=dt, device="cuda")
    blob, bias = net._pack_c2fb(i, n)
    a = S.ConvArgs(x=xd.data_ptr(), N=B, H=H, W=W, Cin=ci, ldx=ldx, w=blob.data_ptr(), bias=bias.data_ptr(), Cout=co,
                   y=y.data_ptr(), ldy=ldy, dtype=net.va_dtype, mode=3, kh=n, kw=1 if shortcut else 0, Npad=co // 2,
                   stride=T)
    if cu:
        a.xu, a.ldu, a.cu = xu.data_ptr(), cu + 8, cu
    lib = _lib.load()
    _lib.check(lib.va_seg_c2fb(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_c2fb")
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert (got[..., co:] == 7.0).all(), "wrote outside its channel slice"
    return x, got[..., :co]


def _check(got, ref):
    rel = ((got - ref).norm() / ref.norm()).item()
    # bf16 rounding flips (accumulation order inside each conv, the hardware SiLU) spread by the chain of convs
    assert rel < 1e-2, rel
    assert ((got - ref).abs() <= 0.03 * ref.abs() + 2e-2).float().mean().item() > 0.999
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("blk", N_BLOCKS, ids=[f"model.{b[0]}" for b in N_BLOCKS])
def test_c2fb_block_batch1(blk):
    """Every C2f block of n-seg at its 640 x 640 size, batch 1, with the planner's tile side; channel slices on
    both sides, the FPN upsample read in place (model.12 / .15: x's first cu channels are NaN, never read)."""
    i, ci, co, n, sc, cu, H, W = blk
    arch, fw, net = _net()
    T = net._c2fb_tile(i, 1, H, W, ci, co, n)
    assert T > 0
    x, got = _run_block(net, i, ci, co, n, sc, cu, 1, H, W, T)
    ref = _block_ref(x.float().permute(0, 3, 1, 2), fw, i, n, sc).permute(0, 2, 3, 1)
    _check(got, ref)


@pytest.mark.parametrize("i,T,B,H,W", [(4, 2, 2, 20, 28), (4, 8, 1, 13, 30), (6, 4, 3, 12, 9), (2, 16, 2, 40, 24),
                                       (8, 2, 1, 6, 10), (21, 4, 2, 10, 14)])
def test_c2fb_tiles_ragged(i, T, B, H, W):
    """Tile sides the planner may not pick, ragged maps (H, W not multiples of T), several frames: the halo and
    the frame border (zero padding of the 3x3s) at every tile position."""
    blk = next(b for b in N_BLOCKS if b[0] == i)
    _, ci, co, n, sc, cu, _, _ = blk
    arch, fw, net = _net()
    x, got = _run_block(net, i, ci, co, n, sc, cu, B, H, W, T, seed=B + H)
    ref = _block_ref(x.float().permute(0, 3, 1, 2), fw, i, n, sc).permute(0, 2, 3, 1)
    _check(got, ref)


def test_c2fb_forward_vs_unfused(monkeypatch):
    """The batch-1 n-seg bf16 plan runs its eight C2f blocks as va_seg_c2fb ops; its heads match the plan with the
    blocks' layers unfused (VA_C2FB=0) within bf16 rounding."""
    from vision_assist_amd.seg import SegNet
    arch, fw, net = _net()
    names = [m["name"] for m in net.plan(1, 640, 640)["meta"]]
    assert sum("fused C2f, T=" in nm for nm in names) == 8, names
    # the stride-2 prologues where they leave the block its tile side (all five at the cost model's sides)
    assert [nm.split("+")[0] for nm in names if "+model." in nm and "C2f" in nm] == \
        ["model.3", "model.5", "model.7", "model.16", "model.19"], names
    frames = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(4), dtype=torch.uint8)

    def heads(nt):
        out = nt.forward(frames.cuda())
        torch.cuda.synchronize()
        return [t.float().cpu() for t in out.levels] + [out.proto.float().cpu()]

    fused = heads(net)
    monkeypatch.setenv("VA_C2FB", "0")
    net2 = SegNet(arch, fw, dtype="bf16")
    assert not any("fused C2f, T=" in m["name"] for m in net2.plan(1, 640, 640)["meta"])
    plain = heads(net2)
    for k, (g_, r) in enumerate(zip(fused, plain)):
        err = ((g_ - r).norm() / r.norm()).item()
        assert err < 2e-2, f"output {k}: fused vs unfused C2f blocks {err}"


def _block_ref64(x, fw, i, n, shortcut):
    """block.py C2f in float64 (x: NCHW float64), the f32 weights as given."""
    silu = F.silu

    def conv(name, t, pad=0):
        w, b = fw[name]
        return silu(F.conv2d(t, w.double(), b.double(), padding=pad))

    t = conv(f"model.{i}.cv1", x)
    c = t.shape[1] // 2
    ys = [t[:, :c], t[:, c:]]
    for j in range(n):
        o = conv(f"model.{i}.m.{j}.cv2", conv(f"model.{i}.m.{j}.cv1", ys[-1], 1), 1)
        ys.append(o + ys[-1] if shortcut else o)
    return conv(f"model.{i}.cv2", torch.cat(ys, 1))


@pytest.mark.parametrize("blk", S_BLOCKS, ids=[f"model.{b[0]}" for b in S_BLOCKS])
def test_c2fb_f32_block_batch1(blk):
    """The f32 form on every C2f block of s-seg at its 640 x 640 size, batch 1 (the planner's tile side) against the
    block in float64: every product as six exact bf16 term products, f32 accumulation, so f32 rounding level."""
    i, ci, co, n, sc, cu, H, W = blk
    arch, fw, net = _net("s", "f32")
    # the planner's tile side, or for the blocks it leaves unfused (model.6: no room for the term planes; 8 / 21: 256
    # wide) the largest side whose layout fits -- the kernel covers them all
    T = net._c2fb_tile(i, 1, H, W, ci, co, n) or next(
        t for t in (4, 2) if net.c2fb_layout(co // 2, n, ci, co, t)[0] > 0 and 1 * -(-H // t) * -(-W // t) >= 96)
    assert T > 0
    x, got = _run_block(net, i, ci, co, n, sc, cu, 1, H, W, T)
    ref = _block_ref64(x.double().permute(0, 3, 1, 2), fw, i, n, sc).permute(0, 2, 3, 1)
    err = (got.double() - ref).abs()
    assert err.max().item() <= 2e-5 * max(1.0, ref.abs().max().item()), (err.max().item(), ref.abs().max().item())
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("i,T,B,H,W", [(4, 2, 2, 20, 28), (6, 2, 1, 7, 9), (21, 2, 2, 6, 10), (2, 8, 1, 24, 40)])
def test_c2fb_f32_tiles_ragged(i, T, B, H, W):
    blk = next(b for b in S_BLOCKS if b[0] == i)
    _, ci, co, n, sc, cu, _, _ = blk
    arch, fw, net = _net("s", "f32")
    x, got = _run_block(net, i, ci, co, n, sc, cu, B, H, W, T, seed=B + H)
    ref = _block_ref64(x.double().permute(0, 3, 1, 2), fw, i, n, sc).permute(0, 2, 3, 1)
    err = (got.double() - ref).abs()
    assert err.max().item() <= 2e-5 * max(1.0, ref.abs().max().item()), err.max().item()


@pytest.mark.parametrize("scale,nfused", [("s", 4), ("n", 8)])
def test_c2fb_f32_forward_vs_unfused(scale, nfused):
    """The batch-1 f32 plan (s: the drop-in call's network) with its C2f blocks as va_seg_c2fb ops where the planner
    takes them (term-plane layouts, hidden width <= 128: s's model.4 / 12 / 15 / 18, every block of n): heads equal
    to the unfused plan's at f32 rounding level, and within the 1e-3 bar of the float32 torch reference."""
    from oracle import yolo_ref as Y
    from vision_assist_amd.seg import SegNet
    arch, fw, net = _net(scale, "f32")
    names = [m["name"] for m in net.plan(1, 640, 640)["meta"]]
    assert sum("fused C2f, T=" in nm for nm in names) == nfused, names
    frames = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(4), dtype=torch.uint8)

    def heads(nt):
        out = nt.forward(frames.cuda())
        torch.cuda.synchronize()
        return [t.float().cpu() for t in out.levels] + [out.proto.float().cpu()]

    fused = heads(net)
    plain_net = SegNet(arch, fw, dtype="f32", c2fb_f32=False)
    assert not any("fused C2f, T=" in m["name"] for m in plain_net.plan(1, 640, 640)["meta"])
    plain = heads(plain_net)
    for k, (g_, r) in enumerate(zip(fused, plain)):
        assert (g_ - r).abs().max().item() <= 1e-4, f"output {k}: {(g_ - r).abs().max().item()}"
    box, cls, coef, proto = Y.forward(arch, fw, Y.preprocess(frames))
    lv = torch.cat([t.flatten(1, 2) for t in fused[:3]], 1).permute(0, 2, 1)
    ref = torch.cat([box, cls, coef], 1)
    assert (lv - ref).abs().max().item() <= 1e-3
    assert (fused[3].permute(0, 3, 1, 2) - proto).abs().max().item() <= 1e-3


S2_CASES = [(4, "model.3", 1, 80, 80, 0), (6, "model.5", 1, 40, 40, 0), (8, "model.7", 1, 20, 20, 0),
            (18, "model.16", 1, 40, 40, 0), (21, "model.19", 1, 20, 20, 0), (4, "model.3", 2, 10, 14, 4),
            (21, "model.19", 2, 6, 10, 2)]


@pytest.mark.parametrize("i,s2,B,H,W,T", S2_CASES)
def test_c2fb_stride2_prologue(i, s2, B, H, W, T):
    """The stride-2 conv that feeds a block (model.3 / 5 / 7 / 16 / 19 of n-seg) as va_seg_c2fb's prologue: the block's
    first cs input channels computed per tile from the 2x-resolution source (x's first cs channels are NaN, never
    read; for model.18 / .21 the rest of the concat comes from x), against the conv + block in fp32 with the unfused
    layers' bf16 rounding; T = 0: the planner's tile side."""
    from vision_assist_amd import _lib
    from vision_assist_amd import seg as S
    blk = next(b for b in N_BLOCKS if b[0] == i)
    _, ci, co, n, sc, cu, _, _ = blk
    arch, fw, net = _net()
    ps2 = net.w[s2]
    cs, cis = ps2.cout, ps2.cin
    T = T or net._c2fb_tile(i, B, H, W, ci, co, n, cs, cis)
    assert T > 0
    g = torch.Generator().manual_seed(i * 31 + B)
    xs = (torch.randn(B, 2 * H, 2 * W, cis, generator=g) * 1.5).to(torch.bfloat16)
    xsd = torch.zeros(B, 2 * H, 2 * W, cis + 8, dtype=torch.bfloat16)
    xsd[..., :cis] = xs
    rest = (torch.randn(B, H, W, ci - cs, generator=g) * 1.5).to(torch.bfloat16)
    xin = torch.full((B, H, W, ci + 8), float("nan"), dtype=torch.bfloat16)
    xin[..., cs:ci] = rest
    xd, xsdd = xin.cuda(), xsd.cuda()
    y = torch.full((B, H, W, co + 16), 7.0, dtype=torch.bfloat16, device="cuda")
    blob, bias = net._pack_c2fb(i, n, s2)
    a = S.ConvArgs(x=xd.data_ptr(), N=B, H=H, W=W, Cin=ci, ldx=ci + 8, w=blob.data_ptr(), bias=bias.data_ptr(),
                   Cout=co, y=y.data_ptr(), ldy=co + 16, dtype=S.VA_DTYPE_BF16, mode=3, kh=n, kw=1 if sc else 0,
                   Npad=co // 2, stride=T, res=xsdd.data_ptr(), ldr=cis + 8, c2=cs, K=cis)
    _lib.check(_lib.load().va_seg_c2fb(_lib.stream_ptr(), ctypes.byref(a)), "va_seg_c2fb")
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert (got[..., co:] == 7.0).all(), "wrote outside its channel slice"
    bf = lambda t: t.to(torch.bfloat16).float()
    w2, b2 = fw[s2]
    head = bf(F.silu(F.conv2d(xs.float().permute(0, 3, 1, 2), bf(w2.float()), b2.float(), stride=2, padding=1)))
    x = torch.cat([head, rest.float().permute(0, 3, 1, 2)], 1)
    ref = _block_ref(x, fw, i, n, sc).permute(0, 2, 3, 1)
    _check(got[..., :co], ref)

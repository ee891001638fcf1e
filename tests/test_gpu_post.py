"""GPU post-processing (va_post_run) vs the oracle (oracle/yolo_ref.py) on the SAME head outputs.

The GPU forward runs in exact-f32 mode and its own head tensors are handed to
the oracle's decode / NMS / process_mask / mask choice, so the comparison
isolates the post-processing kernels:
  * kept detections: same count, classes and order; boxes within 1e-3 px, scores within 1e-6;
  * per-instance mask pixel counts within 0.05 % (sign of bilinear values that are zero to
    float32 rounding may differ between summation orders);
  * chosen instance, its boundingRect and the 20-px cell samples.
Regimes: natural (Ultralytics prior cls bias: no detections with these weights),
mid (cls bias 0) and dense (cls bias +4: 300 detections survive NMS).
"""
import numpy as np
import pytest
import torch

from oracle import yolo_ref as Y

pytestmark = pytest.mark.gpu


def _setup(cls_bias, B=2, H=640, W=640, seed=0, scale="s"):
    from vision_assist_amd.post import PostEngine
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(scale)
    fw = fold(arch, synthetic_state_dict(arch, seed=seed, cls_bias=cls_bias))
    net = SegNet(arch, fw, dtype="f32")
    frames = torch.randint(0, 256, (B, H, W, 3), generator=torch.Generator().manual_seed(seed + 11),
                           dtype=torch.uint8)
    out = net.forward(frames.cuda())
    post = PostEngine(B, H, W, arch.nc)
    post.run(out.levels, out.proto)
    torch.cuda.synchronize()
    lv = torch.cat([t.cpu().flatten(1, 2) for t in out.levels], 1).permute(0, 2, 1)
    nc = arch.nc
    box, cls, coef = lv[:, :64], lv[:, 64:64 + nc], lv[:, 64 + nc:]
    proto = out.proto.cpu().permute(0, 3, 1, 2)
    return post, box, cls, coef, proto


@pytest.mark.parametrize("regime,cls_bias", [("natural", None), ("mid", 0.0), ("dense", 4.0)])
def test_post_matches_oracle(regime, cls_bias):
    H = W = 640
    post, box, cls, coef, proto = _setup(cls_bias)
    pred = Y.decode(box, cls, H, W)
    for b in range(box.shape[0]):
        det_ref = Y.nms_image(pred[b], coef[b])
        det_gpu, _anchors = post.det_tensor(b)
        assert det_gpu.shape[0] == det_ref.shape[0], (regime, b)
        if regime == "dense":
            assert det_ref.shape[0] == 300
        if not det_ref.shape[0]:
            continue
        assert torch.equal(det_gpu[:, 5], det_ref[:, 5]), "classes / order differ"
        assert torch.allclose(det_gpu[:, :4], det_ref[:, :4], atol=1e-3, rtol=0), (det_gpu[:, :4] - det_ref[:, :4]).abs().max()
        assert torch.allclose(det_gpu[:, 4], det_ref[:, 4], atol=1e-6, rtol=0)
        masks = Y.process_mask(proto[b], det_ref[:, 6:], det_ref[:, :4], H, W)
        cnt_ref = masks.flatten(1).sum(1).long()
        st = post.stats[b, :det_ref.shape[0]].cpu()
        cnt_gpu = st[:, 0].long()
        tol = torch.clamp((cnt_ref.float() * 5e-4).long(), min=2)
        assert ((cnt_gpu - cnt_ref).abs() <= tol).all(), (cnt_gpu - cnt_ref).abs().max()
        k_ref, _pts, rect, cells_ref = Y.select_cells(masks)
        chosen = int(post.chosen[b])
        assert chosen == k_ref
        if k_ref < 0:
            continue
        got_rect = tuple(int(v) for v in post.rects[b].cpu())
        assert max(abs(g - r) for g, r in zip(got_rect, rect)) <= 1, (got_rect, rect)
        cells_gpu = post.cells[b].cpu().numpy()
        assert (cells_ref != cells_gpu).sum() <= 1

def test_nms_long_candidate_list_matches_oracle():
    """1280 x 1280 dense regime: > 16384 candidates per frame, so the NMS takes its batched path (exact radix
    select of the 16384 largest keys below the previous batch, sorted and scanned per batch); the kept
    detections are the oracle's, in order."""
    H = W = 1280
    post, box, cls, coef, proto = _setup(4.0, B=1, H=H, W=W, seed=2, scale="n")
    pred = Y.decode(box, cls, H, W)
    n_cand = int((pred[0, 4:].amax(0) > 0.5).sum())
    assert n_cand > 16384, n_cand
    det_ref = Y.nms_image(pred[0], coef[0])
    det_gpu, _anchors = post.det_tensor(0)
    assert det_gpu.shape[0] == det_ref.shape[0]
    assert torch.equal(det_gpu[:, 5], det_ref[:, 5]), "classes / order differ"
    assert torch.allclose(det_gpu[:, :4], det_ref[:, :4], atol=1e-3, rtol=0)
    assert torch.allclose(det_gpu[:, 4], det_ref[:, 4], atol=1e-6, rtol=0)


@pytest.mark.parametrize("H,max_nms,max_det", [(1280, 20000, 300), (1280, 200, 300), (640, 150, 300),
                                               (640, 500, 1500)])
def test_nms_max_nms_truncation_matches_oracle(H, max_nms, max_det):
    """non_max_suppression's max_nms cut (ops.py:332-333) on long candidate lists: batched sorted path with the
    cut inside the second batch / inside the first, the cut on a list that fits LDS, and the fallback path
    (max_det > 1024); same kept detections, in order, as the oracle with the same cut."""
    from vision_assist_amd.post import PostEngine
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("n")
    fw = fold(arch, synthetic_state_dict(arch, seed=2, cls_bias=4.0))
    net = SegNet(arch, fw, dtype="f32")
    frames = torch.randint(0, 256, (1, H, H, 3), generator=torch.Generator().manual_seed(13), dtype=torch.uint8)
    out = net.forward(frames.cuda())
    post = PostEngine(1, H, H, arch.nc, max_det=max_det, max_nms=max_nms)
    post.run(out.levels, out.proto, select=False)
    torch.cuda.synchronize()
    lv = torch.cat([t.cpu().flatten(1, 2) for t in out.levels], 1).permute(0, 2, 1)
    box, cls, coef = lv[:, :64], lv[:, 64:64 + arch.nc], lv[:, 64 + arch.nc:]
    pred = Y.decode(box, cls, H, H)
    n_cand = int((pred[0, 4:].amax(0) > 0.5).sum())
    assert n_cand > max_nms, n_cand
    det_ref = Y.nms_image(pred[0], coef[0], max_det=max_det, max_nms=max_nms)
    assert not torch.equal(det_ref, Y.nms_image(pred[0], coef[0], max_det=max_det, max_nms=10 ** 9)) or \
        det_ref.shape[0] == max_det, "the cut changes nothing here: pick a smaller max_nms"
    det_gpu, _ = post.det_tensor(0)
    assert det_gpu.shape[0] == det_ref.shape[0]
    assert torch.equal(det_gpu[:, 5], det_ref[:, 5]), "classes / order differ"
    assert torch.allclose(det_gpu[:, :4], det_ref[:, :4], atol=1e-3, rtol=0)
    assert torch.allclose(det_gpu[:, 4], det_ref[:, 4], atol=1e-6, rtol=0)


def test_pipeline_planted_nav_matches_oracle():
    """Full fused batch (seg + post + nav) with planted corridor masks: the nav outputs are the
    oracle's on the same masks."""
    from oracle import nav as onav
    from workloads.corridors import cells_rect, cells_to_mask, corridor_cells
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B = 8
    pipe = FramePipeline(arch, fw, B, 640, 640, dtype="bf16")
    grids = [corridor_cells(300 + i) for i in range(B)]
    pc = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    frames = torch.randint(0, 256, (B, 640, 640, 3), dtype=torch.uint8).cuda()
    res = pipe.run(frames, pc, pr, PLANT_ALWAYS)
    pf = onav.PathFinderOracle()
    for i, g in enumerate(grids):
        out = onav.frame_nav(cells_to_mask(g), cells_rect(g), 640, 640, pf)
        nf = res.frame(i)
        assert [q["path"] for q in nf.queries] == [[(c.coords.x, c.coords.y) for c in q[2]] for q in out["queries"]]


def test_pipeline_medium_1280_planted_nav_matches_oracle():
    """C5 shape (YOLOv8m-seg, 1280 x 1280, bf16): the fused batch runs and, with planted 64 x 64-cell
    corridor masks, its grid / penalty / protrusion / A* outputs are the oracle's."""
    from oracle import nav as onav
    from workloads.corridors import cells_rect, cells_to_mask, corridor_cells
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("m")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B, H, W = 4, 1280, 1280
    pipe = FramePipeline(arch, fw, B, H, W, dtype="bf16")
    grids = [corridor_cells(7300 + i, H // 20, W // 20) for i in range(B)]
    pc = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    frames = torch.randint(0, 256, (B, H, W, 3), generator=torch.Generator().manual_seed(13), dtype=torch.uint8).cuda()
    res = pipe.run(frames, pc, pr, PLANT_ALWAYS)
    pf = onav.PathFinderOracle()
    for i, g in enumerate(grids):
        out = onav.frame_nav(cells_to_mask(g), cells_rect(g), H, W, pf)
        nf = res.frame(i)
        assert [q["path"] for q in nf.queries] == [[(c.coords.x, c.coords.y) for c in q[2]] for q in out["queries"]]


@pytest.mark.parametrize("depth", [2, 3])
def test_overlapped_pipelines_match_sequential(depth):
    """bench.py's overlapped form (two network streams, `depth` batches in flight, grid stage in submission
    order on its own stream) gives the sequential pipeline's nav answers batch by batch, with the angle
    cache advancing in the same order."""
    from workloads.corridors import cells_rect, corridor_cells
    from vision_assist_amd.pipeline import FramePipeline, OverlappedPipelines
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("n")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B, nb = 4, 5
    batches = []
    for k in range(nb):
        grids = [corridor_cells(900 + 10 * k + i) for i in range(B)]
        batches.append((torch.randint(0, 256, (B, 640, 640, 3), generator=torch.Generator().manual_seed(k),
                                      dtype=torch.uint8).cuda(),
                        torch.tensor(np.stack(grids).astype(np.uint8)).cuda(),
                        torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()))
    seq = FramePipeline(arch, fw, B, 640, 640, dtype="bf16")
    want = []
    for fr, pc, pr in batches:
        res = seq.run(fr, pc, pr, PLANT_ALWAYS)
        want.append([[(q["path"], q["cost"], q["unique"], q["order"]) for q in res.frame(i).queries] for i in range(B)])
    ov = OverlappedPipelines(arch, fw, B, 640, 640, dtype="bf16", depth=depth)
    got, held = [], []
    ahead = depth - 1
    for s in range(min(ahead, nb)):
        ov.submit(*batches[s], PLANT_ALWAYS)
    for s in range(nb):
        if s + ahead < nb:
            ov.submit(*batches[s + ahead], PLANT_ALWAYS)
        res = ov.finish(s)
        held.append(res)  # read back only after later batches reuse the pipelines: the records must not change
    for res in held:
        got.append([[(q["path"], q["cost"], q["unique"], q["order"]) for q in res.frame(i).queries] for i in range(B)])
    assert got == want
    assert ov.a.seen.keys() == seq.seen.keys()


@pytest.mark.parametrize("H0,W0", [(720, 1280), (480, 848)])
def test_letterbox_kernel_matches_restatement(H0, W0):
    import ctypes  # noqa: F401
    from vision_assist_amd import _lib
    from vision_assist_amd.post import letterbox_geometry
    lib = _lib.load()
    Hn, Wn, top, left, newh, neww, _g, _px, _py = letterbox_geometry(H0, W0)
    B = 2
    fr = torch.randint(0, 256, (B, H0, W0, 3), generator=torch.Generator().manual_seed(H0), dtype=torch.uint8)
    out = torch.empty((B, Hn, Wn, 3), dtype=torch.uint8, device="cuda")
    _lib.check(lib.va_letterbox(_lib.stream_ptr(), fr.cuda().data_ptr(), B, H0, W0, out.data_ptr(), Hn, Wn, top, left,
                                newh, neww), "va_letterbox")
    torch.cuda.synchronize()
    for b in range(B):
        want = Y.letterbox_np(fr[b].numpy(), Hn, Wn, top, left, newh, neww)
        assert np.array_equal(out[b].cpu().numpy(), want)


def test_letterboxed_mask_choice_in_frame_coordinates():
    """720 x 1280 frame -> 384 x 640 network input: the chosen mask's cells and boundingRect come back in frame
    coordinates (the chosen polygon scale_coords'd to the frame, np.int32, boundingRect, fillPoly sampled at the
    frame's cell centres), against the oracle on the same head outputs."""
    from vision_assist_amd import _lib
    from vision_assist_amd.post import PostEngine, letterbox_geometry
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    H0, W0 = 720, 1280
    Hn, Wn, top, left, newh, neww, gain, px, py = letterbox_geometry(H0, W0)
    arch = Arch("s")
    fw = fold(arch, synthetic_state_dict(arch, seed=3, cls_bias=0.0))
    net = SegNet(arch, fw, dtype="f32")
    fr = torch.randint(0, 256, (1, H0, W0, 3), generator=torch.Generator().manual_seed(8), dtype=torch.uint8)
    x = torch.empty((1, Hn, Wn, 3), dtype=torch.uint8, device="cuda")
    lib = _lib.load()
    _lib.check(lib.va_letterbox(_lib.stream_ptr(), fr.cuda().data_ptr(), 1, H0, W0, x.data_ptr(), Hn, Wn, top, left,
                                newh, neww), "va_letterbox")
    out = net.forward(x)
    post = PostEngine(1, Hn, Wn, arch.nc, frame=(H0, W0, gain, px, py))
    post.run(out.levels, out.proto)
    torch.cuda.synchronize()
    lv = torch.cat([t.cpu().flatten(1, 2) for t in out.levels], 1).permute(0, 2, 1)
    box, cls, coef = lv[:, :64], lv[:, 64:64 + arch.nc], lv[:, 64 + arch.nc:]
    proto = out.proto.cpu().permute(0, 3, 1, 2)
    pred = Y.decode(box, cls, Hn, Wn)
    det = Y.nms_image(pred[0], coef[0])
    assert det.shape[0] > 0, "regime produced no detection"
    masks = Y.process_mask(proto[0], det[:, 6:], det[:, :4], Hn, Wn)
    k_ref, _pts, rect, cells_ref = Y.select_cells(masks, (H0, W0))
    assert k_ref >= 0
    assert int(post.chosen[0]) == k_ref
    cells_gpu = post.cells[0].cpu().numpy()
    assert cells_gpu.shape == (H0 // 20, W0 // 20)
    assert (cells_ref != cells_gpu).sum() <= 1
    got = tuple(int(v) for v in post.rects[0].cpu())
    assert max(abs(g - w) for g, w in zip(got, rect)) <= 2, (got, rect)


def test_pipeline_720x1280_frames_letterboxed_nav_matches_oracle():
    """Camera-size frames (720 x 1280, not multiples of 32) run through the letterboxed fused batch; with planted
    36 x 64-cell corridors the grid / A* outputs are the oracle's at frame resolution."""
    from oracle import nav as onav
    from workloads.corridors import cells_rect, cells_to_mask, corridor_cells
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s")
    fw = fold(arch, synthetic_state_dict(arch, seed=0))
    B, H, W = 3, 720, 1280
    pipe = FramePipeline(arch, fw, B, H, W, dtype="bf16")
    assert (pipe.Hn, pipe.Wn) == (384, 640)
    grids = [corridor_cells(8100 + i, H // 20, W // 20) for i in range(B)]
    pc = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    frames = torch.randint(0, 256, (B, H, W, 3), generator=torch.Generator().manual_seed(4), dtype=torch.uint8).cuda()
    res = pipe.run(frames, pc, pr, PLANT_ALWAYS)
    pf = onav.PathFinderOracle()
    for i, g in enumerate(grids):
        out = onav.frame_nav(cells_to_mask(g), cells_rect(g), H, W, pf)
        assert [q["path"] for q in res.frame(i).queries] == [[(c.coords.x, c.coords.y) for c in q[2]] for q in out["queries"]]


def test_mask_counts_1280_multi_strip():
    """1280 x 1280 (proto 320 x 320): crop windows up to 320 low-res pixels wide run in several LDS strips of
    the mask kernel; per-instance pixel counts of the first detections match the oracle's process_mask."""
    H = W = 1280
    post, box, cls, coef, proto = _setup(0.0, B=1, H=H, W=W, seed=5, scale="n")
    pred = Y.decode(box, cls, H, W)
    det_ref = Y.nms_image(pred[0], coef[0])
    det_gpu, _anchors = post.det_tensor(0)
    assert det_gpu.shape[0] == det_ref.shape[0] and det_ref.shape[0] > 0
    k = min(12, det_ref.shape[0])
    masks = Y.process_mask(proto[0], det_ref[:k, 6:], det_ref[:k, :4], H, W)
    cnt_ref = masks.flatten(1).sum(1).long()
    cnt_gpu = post.stats[0, :k, 0].cpu().long()
    tol = torch.clamp((cnt_ref.float() * 5e-4).long(), min=2)
    assert ((cnt_gpu - cnt_ref).abs() <= tol).all(), (cnt_gpu - cnt_ref).abs().max()


def test_mask_big_box_many_strips():
    """A synthetic head with one detection whose box spans ~960 px of a 1280 x 1280 frame: its 240 x 240 low-res
    crop window needs ten LDS strips of the mask kernel; pixel count and bbox match the oracle's process_mask."""
    from vision_assist_amd.post import PostEngine
    H = W = 1280
    nc, no = 80, 64 + 80 + 32
    g = torch.Generator().manual_seed(17)
    levels = []
    for s in (8, 16, 32):
        t = torch.zeros(1, H // s, W // s, no)
        t[..., 64:64 + nc] = -10.0
        levels.append(t)
    t = levels[2]
    t[0, 20, 20, 64 + 3] = 5.0              # one candidate (class 3) at the stride-32 anchor (20, 20)
    for side in range(4):
        t[0, 20, 20, side * 16 + 15] = 10.0  # DFL expectation ~15 bins = ~480 px per side
    t[0, 20, 20, 64 + nc:] = torch.randn(32, generator=g)
    proto = torch.randn(1, H // 4, W // 4, 32, generator=g)
    post = PostEngine(1, H, W, nc)
    post.run([x.cuda().contiguous() for x in levels], proto.cuda().contiguous())
    torch.cuda.synchronize()
    lv = torch.cat([x.flatten(1, 2) for x in levels], 1).permute(0, 2, 1)
    box, cls, coef = lv[:, :64], lv[:, 64:64 + nc], lv[:, 64 + nc:]
    pred = Y.decode(box, cls, H, W)
    det_ref = Y.nms_image(pred[0], coef[0])
    assert det_ref.shape[0] == 1 and int(post.ndet[0]) == 1
    assert (det_ref[0, 2] - det_ref[0, 0]) > 900
    m = Y.process_mask(proto[0].permute(2, 0, 1), det_ref[:, 6:], det_ref[:, :4], H, W)[0]
    st = post.stats[0, 0].cpu()
    cnt_ref = int(m.sum())
    assert abs(int(st[0]) - cnt_ref) <= max(2, int(cnt_ref * 5e-4)), (int(st[0]), cnt_ref)
    ys, xs = torch.nonzero(m, as_tuple=True)
    want = [int(xs.min()), int(ys.min()), int(xs.max()), int(ys.max())]
    assert max(abs(int(a) - b) for a, b in zip(st[1:5], want)) <= 1, (st[1:5].tolist(), want)

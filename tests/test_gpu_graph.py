"""HIP-graph capture of the network + post-processing of a FramePipeline (FramePipeline.seg_post: letterbox-free
preprocess, the forward, decode, NMS, masks, contours, the mask choice), replayed once and compared bit for bit
with the eager run -- the round-1 capture faulted on replay (post_nms_kernel's 150 KiB of dynamic LDS was never
set on the function for a graph kernel node; va_post.hip now sets it explicitly, per device)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale,dtype,B,regime", [("n", "bf16", 1, "dense"), ("s", "f32", 2, "mid")])
def test_graph_replay_equals_eager(scale, dtype, B, regime):
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch(scale)
    bias = {"mid": 0.0, "dense": 4.0}[regime]
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, cls_bias=bias)), B, 640, 640,
                         dtype=dtype)
    pipe.frames.copy_(torch.randint(0, 256, pipe.frames.shape, generator=torch.Generator().manual_seed(2),
                                    dtype=torch.uint8).cuda())

    def outs():
        p = pipe.post
        return [p.ndet, p.cells, p.rects, p.chosen, pipe.plan["out"].proto] + list(pipe.plan["out"].levels)

    def per_det():  # rows past a frame's ndet are not written
        p = pipe.post
        n = p.ndet.tolist()
        return [t[b, :n[b]].clone() for t in (p.dets, p.stats, p.cstats) for b in range(B)]

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = [t.clone() for t in outs()]
    ref_det = per_det()
    assert int(ref[0].sum()) > 0, "the regime produced no detection"
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        pipe.seg_post(plant_mode=PLANT_NEVER)
    torch.cuda.synchronize()
    for t in outs() + [pipe.post.dets, pipe.post.stats, pipe.post.cstats]:
        t.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    same = [bool(torch.equal(a, b)) for a, b in zip(outs(), ref)]
    assert all(same), same
    same = [bool(torch.equal(a, b)) for a, b in zip(per_det(), ref_det)]
    assert all(same), same


def test_graph_replay_then_nav_equals_eager():
    """The batch-1 latency form (tools/latency.py --graph, pipeline.SegPostGraph): frame copy + network +
    post-processing replayed from a graph, then the grid / A* stage eagerly on the replayed cells -- the same paths,
    costs and angle-cache keys as the eager pipeline, over several replays, issued from the default stream."""
    import numpy as np
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from workloads.corridors import cells_rect, corridor_cells
    arch = Arch("n")
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0)), 1, 640, 640, dtype="bf16")
    frame = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(1),
                          dtype=torch.uint8).cuda()
    runs = []
    for seed in (11, 12, 13):
        gc_ = corridor_cells(seed, 32, 32)
        runs.append((torch.tensor(gc_[None].astype(np.uint8)).cuda(),
                     torch.tensor(np.array([cells_rect(gc_)], dtype=np.int32)).cuda()))
    pc = torch.zeros_like(runs[0][0])
    pr = torch.zeros_like(runs[0][1])

    def summary(res):
        f = res.frame(0)
        return [(q["path"], float(q["cost"]).hex() if q["path"] else None) for q in f.queries]

    want = []
    for c, r in runs:  # eager
        res = pipe.run(frame, c, r, PLANT_ALWAYS)
        want.append((summary(res), sorted(pipe.seen.keys())))
    pipe.seen.clear()
    from vision_assist_amd.pipeline import SegPostGraph
    g = SegPostGraph(pipe, frame, pc, pr, PLANT_ALWAYS)
    # from the caller's current stream -- the legacy default stream here, where a direct hipGraphLaunch followed
    # by the grid stage faulted (profiles/r03/graph_fault/): the replay runs on the graph's own stream, ordered by
    # events before and after, and the grid stage follows on the default stream
    assert torch.cuda.current_stream().cuda_stream == 0
    got = []
    for c, r in runs:
        pc.copy_(c)
        pr.copy_(r)
        g.replay()
        res = pipe.nav_run()
        got.append((summary(res), sorted(pipe.seen.keys())))
    assert got == want

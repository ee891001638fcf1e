"""The round-2/3 fault form, kept as a regression test (profiles/r03/graph_fault/, profiles/r04/graph_fault/): a seg +
post-processing graph replayed with hipGraphLaunch directly on the LEGACY default stream (handle 0) -- not through
SegPostGraph's private stream -- each replay followed on that stream, with no synchronisation, by the grid / A*
stage (nav_run).  Paths, costs and angle-cache keys must equal the eager pipeline's and no kernel may record a
rejected access (va_diag: the nav kernels check every data-dependent global index, codes 31-36).

Round 3 saw this sequence end in hipErrorIllegalAddress; on the round-4 tree the same script
(tools/graph_order_probe.py) and the localizer (tools/graph_fault_localize.py, synchronised and not) ran clean.
The file sorts last among the GPU tests so that, were the fault to come back, it ends the run after every other
test has reported."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_legacy_stream_graph_replay_then_nav_equals_eager():
    import numpy as np

    from vision_assist_amd import _lib
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
        g_ = corridor_cells(seed, 32, 32)
        runs.append((torch.tensor(g_[None].astype(np.uint8)).cuda(),
                     torch.tensor(np.array([cells_rect(g_)], dtype=np.int32)).cuda()))
    pc, pr = torch.zeros_like(runs[0][0]), torch.zeros_like(runs[0][1])

    def summary(res):
        f = res.frame(0)
        return [(q["path"], float(q["cost"]).hex() if q["path"] else None) for q in f.queries]

    want = []
    for c, r in runs:
        res = pipe.run(frame, c, r, PLANT_ALWAYS)
        want.append((summary(res), sorted(pipe.seen.keys())))
    pipe.seen.clear()
    _lib.diag()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            pipe.load(frame)
            pipe.seg_post(pc, pr, PLANT_ALWAYS)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        pipe.load(frame)
        pipe.seg_post(pc, pr, PLANT_ALWAYS)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    assert st.cuda_stream == 0
    got = []
    for c, r in runs:
        pc.copy_(c)
        pr.copy_(r)
        g.replay()
        res = pipe.nav_run(stream=st)
        got.append((summary(res), sorted(pipe.seen.keys())))
    torch.cuda.synchronize()
    assert _lib.diag() == {}
    assert got == want

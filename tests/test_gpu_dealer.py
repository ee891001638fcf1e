"""The §8e frame dealer on the GPU: one reader deals the C4 frame stream (frames 7000 + i, s-seg 640, the network's
own masks) round-robin to 2 worker processes on the test GPU (on a node each worker takes its own GPU; the code
path is the same), each with a batch-1 f32 FramePipeline and its own PathFinder angle cache.  The in-order
results must equal each shard's frames replayed in order through the oracle chain with a fresh PathFinder per
shard -- tests/golden/chain_oracle.json.gz["c4/<regime>"], the same per-shard replay test_gpu_c4.py checks --
with the f32 bar: every detection matched, the same chosen instance, rect, cells and A* paths and costs.  And
FrameProcessor.map (the drop-in surface's multi-GPU mode) hands back one answer per frame, in order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_FRAMES = 8


class C4RecordWorker:
    """FrameDealer worker factory: a batch-1 f32 FramePipeline of the regime's weights on the worker's GPU; a
    frame -> its detections, chosen instance, rect, cells and A* paths / costs (plain numpy / python)."""

    def __init__(self, regime: str):
        self.regime = regime

    def __call__(self, device):
        import torch

        from tests.chain_util import weights
        from vision_assist_amd.pipeline import FramePipeline
        from vision_assist_amd.post import PLANT_NEVER
        arch, fw = weights(self.regime)
        pipe = FramePipeline(arch, fw, 1, 640, 640, dtype="f32", device=torch.device("cuda", device))

        def run(frame):
            res = pipe.run(torch.from_numpy(frame[None]), plant_mode=PLANT_NEVER)
            nf = res.frame(0)
            det, _ = pipe.post.det_tensor(0)
            return {"det": det.numpy(), "chosen": int(pipe.post.chosen[0]), "rect": pipe.post.rects[0].cpu().tolist(),
                    "cells": pipe.post.cells[0].cpu().numpy(), "status": nf.status,
                    "queries": [(q["path"], float(q["cost"]).hex() if q["path"] else None) for q in nf.queries]}
        return run


class C4BatchRecordWorker(C4RecordWorker):
    """The same records through the batching protocol (FrameDealer: max_batch / begin / end) on
    pipeline.StreamBatches -- up to 4 waiting frames per device batch, two batches in flight."""

    def __call__(self, device):
        import torch

        from tests.chain_util import weights
        from vision_assist_amd.pipeline import StreamBatches
        arch, fw = weights(self.regime)
        sb = StreamBatches(arch, fw, 4, 640, 640, dtype="f32", device=torch.device("cuda", device))

        class Fn:
            max_batch = 4

            def begin(self, frames):
                return sb.begin(frames)

            def end(self, tok):
                res = sb.end(tok)
                post = sb.pipes[tok[0] % 2].post
                out = []
                for i in range(tok[1]):
                    nf = res.frame(i)
                    det, _ = post.det_tensor(i)
                    out.append({"det": det.numpy(), "chosen": int(post.chosen[i]), "rect": post.rects[i].cpu().tolist(),
                                "cells": post.cells[i].cpu().numpy(), "status": nf.status,
                                "queries": [(q["path"], float(q["cost"]).hex() if q["path"] else None)
                                            for q in nf.queries]})
                return out
        return Fn()


@pytest.mark.parametrize("batched,readers", [(False, 0), (True, 0), (True, 2)])
@pytest.mark.parametrize("regime", ["sparse", "dense_box"])
def test_dealer_two_workers_vs_per_shard_oracle_replay(regime, batched, readers):
    import torch

    from tests.chain_util import compare, frame_batch, load_fixture
    from vision_assist_amd.shard import FrameDealer
    frames = [frame_batch(7000 + i, 1)[0].numpy() for i in range(N_FRAMES)]
    want = load_fixture(f"c4/{regime}")
    worker = C4BatchRecordWorker(regime) if batched else C4RecordWorker(regime)
    with FrameDealer(worker, [0, 0], 640, 640, slots=4 if batched else 2, readers=readers) as d:
        got = list(d.map(frames))
    bad = []
    for i, (g, w) in enumerate(zip(got, want)):
        ok = g["status"] == 0
        rec = {"det": torch.from_numpy(g["det"]), "chosen": g["chosen"],
               "rect": tuple(g["rect"]) if g["chosen"] >= 0 else None,
               "cells": g["cells"] if g["chosen"] >= 0 else None,
               "paths": [p for p, _ in g["queries"]] if ok else None,
               "costs": [c for _, c in g["queries"]] if ok else None}
        c = compare(rec, w, f32=True)
        frac = 1.0 if regime == "sparse" else 0.98
        if c["matched"] < frac * max(c["ndet"]) or not c["chosen"] or c["cells_mismatch"] != 0 or not c["paths"]:
            bad.append((i, c))
    assert len(got) == N_FRAMES and not bad, bad


def test_frameprocessor_map_answers_in_order():
    import warnings

    from tests.chain_util import frame_batch
    from vision_assist_amd.FrameProcessor import FrameProcessor
    from vision_assist_amd.yolo import YOLO
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = YOLO("yolov8s-seg.pt", sparse=640, dtype="f32").to("cuda")
    fp = FrameProcessor(model=model, verbose=False, debug=False)
    fp.model = model
    frames = [frame_batch(7100 + i, 1)[0].numpy() for i in range(6)]
    try:
        answers = list(fp.map(frames, devices=[0, 0], slots=2))
    finally:
        fp.close_map()
    assert len(answers) == len(frames)
    assert all(isinstance(a, (str, list)) for a in answers)
    assert any(a != [] for a in answers)


def test_stream_batches_failed_end_loses_only_its_batch():
    """a grid stage that raises in StreamBatches.end spends that batch's token -- the next batches begin
    and end in order, with the answers of the same frames run through a fresh StreamBatches."""
    import torch

    from tests.chain_util import frame_batch, weights
    from vision_assist_amd.pipeline import StreamBatches
    arch, fw = weights("sparse")
    frames = [frame_batch(7200 + i, 1)[0].numpy() for i in range(6)]

    def answers(sb, batches, fail_first=False):
        out = []
        toks = [sb.begin(frames[a:b]) for a, b in batches[:2]]
        if fail_first:
            real = sb.pipes[0].nav_run

            def boom(*a, **k):
                sb.pipes[0].nav_run = real
                raise RuntimeError("injected grid-stage failure")
            sb.pipes[0].nav_run = boom
            with pytest.raises(RuntimeError, match="injected"):
                sb.end(toks[0])
        else:
            res = sb.end(toks[0])
            out += [[q["path"] for q in res.frame(i).queries] for i in range(toks[0][1])]
        for k, (a, b) in enumerate(batches[1:]):
            if k + 2 < len(batches):
                toks.append(sb.begin(frames[batches[k + 2][0]:batches[k + 2][1]]))
            res = sb.end(toks[k + 1])
            out += [[q["path"] for q in res.frame(i).queries] for i in range(toks[k + 1][1])]
        return out

    batches = [(0, 2), (2, 4), (4, 6)]
    sb = StreamBatches(arch, fw, 2, 640, 640, dtype="f32", device=torch.device("cuda", 0))
    got = answers(sb, batches, fail_first=True)
    assert sb.done == sb.k == 3
    # the same later frames through a fresh object whose first batch ends normally: the angle cache then holds that
    # batch's keys, which the failed run never added -- so compare the frames of batches 2 and 3 run alone
    ref = StreamBatches(arch, fw, 2, 640, 640, dtype="f32", device=torch.device("cuda", 0))
    want = answers(ref, [(2, 4), (4, 6)])
    assert got == want

"""GPU parity of the grid-level hot path (libva355.so va_nav_run) -- bit-exact.

* against the reference's own outputs (tests/golden/nav_goldens.json.gz):
  grid list / row attrs / flags / penalties (float64 hex + int type), lookup
  size and orphans, protrusion peaks, start/end cells, every A* path and cost,
  the angle-cache key set before/after every query, the de-duplicated paths;
  each sequence once as ONE batch (speculative parallel A* rounds) and once
  frame-by-frame (B = 1, state carried);
* against the oracle (oracle/nav.py) on seeded procedural corridors at
  640x640, 1280x1280 and 720x1280 (warm, order-dependent sequences).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import nav as onav
from workloads.corridors import cells_rect, cells_to_mask, corridor_cells
from tests.golden_io import cells_of, load_goldens
from tests.nav_check import bits_to_keys, compare_golden_frame, key_index, pen_value, _ptype

pytestmark = pytest.mark.gpu


def _engine(H, W, B):
    from vision_assist_amd.nav import NavEngine
    return NavEngine(H, W, max_batch=B)


def _seen():
    from vision_assist_amd.nav import AngleSeen
    return AngleSeen("cuda")


def _inputs(frames):
    cells = torch.tensor(np.stack([cells_of(f) for f in frames]).astype(np.uint8)).cuda()
    rects = torch.tensor(np.array([f["rect"] for f in frames], dtype=np.int32)).cuda()
    return cells, rects


@pytest.mark.parametrize("mode", ["batch", "batch_rb", "single", "single_rb"])
def test_nav_matches_reference_goldens(mode):
    """batch / single: va_nav_run + NavBatch's asynchronous copy; *_rb: va_nav_run_rb (records copied to the host
    inside the call, re-copied by every re-run round -- a whole sequence as one batch takes several)"""
    d = load_goldens()
    rb = mode.endswith("_rb")
    nframes = nq = rerun = 0
    for seq in d["sequences"]:
        frames = seq["frames"]
        H, W = frames[0]["H"], frames[0]["W"]
        eng = _engine(H, W, len(frames))
        seen_dev = _seen()
        seen = set()
        if mode.startswith("batch"):
            cells, rects = _inputs(frames)
            res = eng.run(cells, rects, seen_dev, readback=rb)
            rerun += res.rounds > 1
            for i, fr in enumerate(frames):
                seen = compare_golden_frame(res.frame(i), fr, seen)
        else:
            for fr in frames:
                cells, rects = _inputs([fr])
                res = eng.run(cells, rects, seen_dev, readback=rb)
                seen = compare_golden_frame(res.frame(0), fr, seen)
        assert seen_dev.keys() == seen
        nframes += len(frames)
        nq += sum(len(f.get("queries", [])) for f in frames)
    assert nframes == 372 and nq == 392
    if mode == "batch_rb":
        assert rerun > 0  # the re-copy behind a re-run round is exercised


def test_nav_run_rb_checks_host_size():
    from vision_assist_amd import _lib
    eng = _engine(640, 640, 2)
    lib = _lib.load()
    n = int(lib.va_nav_records_bytes(2, 640, 640))
    d = eng.dims
    assert n == ((2 * d.frame_bytes + 15) & ~15) + 2 * d.MAXPK * d.query_bytes
    assert lib.va_nav_records_bytes(0, 640, 640) == _lib.VA_ERR_ARG
    cells = torch.zeros((2, d.LR, d.LC), dtype=torch.uint8, device="cuda")
    rects = torch.zeros((2, 4), dtype=torch.int32, device="cuda")
    rec = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    rounds = ctypes.c_int32(0)
    args = (None, cells.data_ptr(), rects.data_ptr(), 2, 640, 640, _seen().t.data_ptr(), eng.work.data_ptr(),
            ctypes.byref(rounds), rec.data_ptr())
    assert lib.va_nav_run_rb(*args, n - 1) == _lib.VA_ERR_ARG
    assert lib.va_nav_run_rb(*args, n) == _lib.VA_OK


def _oracle_compare(nf, out, seen_before: set, pf_keys_after: list, src):
    st = out["state"]
    if not st.grids:
        assert nf.status == 1, src
        return seen_before
    assert nf.status == 0 and nf.P == len(st.grids), src
    for p, row in enumerate(st.grids):
        assert int(nf.pos_y[p]) == row[0].coords.y and int(nf.pos_attr[p]) == row[0].row
        for c, cell in enumerate(row):
            fl = int(nf.cell_flags[p, c])
            assert bool(fl & 1) == cell.empty and bool(fl & 2) == cell.artificial
            assert _ptype(pen_value(fl, float(nf.cell_pen[p, c]))) == _ptype(cell.penalty), (src, p, c)
    assert [tuple(p) for p in nf.peaks] == [tuple(p) for p in out["peaks"]], src
    seen = set(seen_before)
    for q, (s, e, path, cost, keys_after) in zip(nf.queries, out["queries"]):
        assert q["path"] == [(c.coords.x, c.coords.y) for c in path], src
        if path:
            assert float(q["cost"]).hex() == float(cost).hex(), src
        seen |= bits_to_keys(*q["miss"])
        want = {key_index([a[0], a[1], b[0], b[1]]) for (a, b) in keys_after}
        assert seen == want, src
    uniq = [q["path"] for q in sorted(nf.queries, key=lambda q: q["order"]) if q["unique"]]
    assert uniq == [[(c.coords.x, c.coords.y) for c in p] for p, _ in out["paths"]], src
    return seen


@pytest.mark.parametrize("H,W,n,seed0", [(640, 640, 160, 5000), (1280, 1280, 40, 7000), (1280, 720, 40, 9000)])
def test_nav_matches_oracle_corridors(H, W, n, seed0):
    grids = [corridor_cells(seed0 + i, H // 20, W // 20) for i in range(n)]
    eng = _engine(H, W, n)
    seen_dev = _seen()
    cells = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    rects = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    res = eng.run(cells, rects, seen_dev)
    pf = onav.PathFinderOracle()
    seen = set()
    for i, g in enumerate(grids):
        out = onav.frame_nav(cells_to_mask(g), cells_rect(g), H, W, pf)
        seen = _oracle_compare(res.frame(i), out, seen, [q[4] for q in out["queries"]], f"corridor:{seed0 + i}")
    assert seen_dev.keys() == seen


def test_nav_sample_cells_matches_lattice():
    rng = np.random.default_rng(3)
    masks = (rng.random((3, 640, 640)) < 0.5).astype(np.uint8)
    eng = _engine(640, 640, 3)
    got = eng.sample_cells(torch.tensor(masks).cuda()).cpu().numpy()
    assert np.array_equal(got, masks[:, 10::20, 10::20])


@pytest.mark.parametrize("rect,err", [((600, 100, 41, 100), True), ((100, 600, 100, 41), True),
                                      ((0, 40, 641, 200), False), ((20, 0, 600, 640), False)])
def test_nav_rect_past_the_frame(rect, err):
    """FrameProcessor.py:79-97: the snapped rect's cell centres index mask_img; a rect reaching past the frame
    (a polygon clipped onto x = W0 / y = H0, rounded up to whole cells) raises numpy's IndexError there -- the
    device frame status is VA_FRAME_INDEX_ERROR; w alone is clamped to the frame width (no error)."""
    H = W = 640
    g = corridor_cells(4242, H // 20, W // 20)
    eng = _engine(H, W, 1)
    res = eng.run(torch.tensor(g[None].astype(np.uint8)).cuda(), torch.tensor([rect], dtype=torch.int32).cuda(),
                  _seen())
    nf = res.frame(0)
    if err:
        with pytest.raises(IndexError):
            onav.frame_nav(cells_to_mask(g), rect, H, W, onav.PathFinderOracle())
        assert nf.status == 2  # VA_FRAME_INDEX_ERROR
    else:
        out = onav.frame_nav(cells_to_mask(g), rect, H, W, onav.PathFinderOracle())
        _oracle_compare(nf, out, set(), [q[4] for q in out["queries"]], str(rect))


def test_standalone_singletons_on_caller_built_grids():
    """PenaltyCalculator.calculate_penalty and ProtrusionDetector()(frame, grids, lookup) on grids built OUTSIDE this
    package's FrameProcessor -- here by the oracle's builder, pinned to the reference's -- as the reference's
    FrameProcessor._calculate_penalties / __call__ drive them (/root/reference FrameProcessor.py:180-182, :341): the
    device grid stage runs on the frame the grids imply (FrameProcessor.device_frame_for) and serves every penalty
    bit-exact with its python type, and the peaks, against the reference-run goldens (the fixtures, corridors and
    edge cases of tests/test_standalone_cpu.py)."""
    from tests.golden_io import unhex
    from tests.test_standalone_cpu import _as_grids, _frames
    from vision_assist_amd.FrameProcessor import FrameProcessor
    from vision_assist_amd.PenaltyCalculator import penalty_calculator
    from vision_assist_amd.PathFinder import path_finder
    from vision_assist_amd.ProtrusionDetector import ProtrusionDetector
    fp = FrameProcessor(model=None)
    seen_before = path_finder.seen.t.clone()
    for name, fr in _frames()[:40]:
        H, W = fr["H"], fr["W"]
        st = onav.build_grids(cells_to_mask(cells_of(fr)), tuple(fr["rect"]), H, W)
        grids, lookup = _as_grids(st)
        fp.frame = np.zeros((H, W, 3), np.uint8)
        fp._state = None  # not FrameProcessor's own frame
        penalty_calculator._pre_compute_easy_segments(st.np_grids, grids)
        for row, grow in zip(grids, fr["rows"]):
            for g, want in zip(row, grow["pen"]):
                got = penalty_calculator.calculate_penalty(g, lookup)
                w = unhex(want)
                if g.empty:
                    assert got == 0
                else:
                    assert _ptype(got) == _ptype(w), (name, g.coords)
        peaks = ProtrusionDetector()(fp.frame, grids, lookup)
        assert [[p.x, p.y] for p in peaks] == fr["peaks"], name
    assert torch.equal(path_finder.seen.t, seen_before), "the process angle cache is left as it was"

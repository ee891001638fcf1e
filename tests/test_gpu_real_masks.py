"""Real path shapes through the mask -> polygon -> cells -> grid / A* stages: the segmentation labels the
reference's model was trained on (its own validation set, model/valid/labels; tests/golden/frames) rasterised as
instance masks (oracle/contours.fill_poly = cv2.fillPoly restated), then va_post_select_masks (findContours
'largest', contourArea choice, boundingRect, fillPoly at the cell centres) and the nav stage (grid, penalties,
protrusion, A*) on the device, against oracle/contours.select_cells + oracle/nav.frame_nav with one angle cache:
chosen instance, rect and cells bit-exact, A* paths and costs bit-exact.  These are the masks a trained model
produces (corridors, forks, several instances per frame), not synthetic ones."""
import numpy as np
import pytest
import torch

from oracle import contours as C
from oracle import nav as onav
from tests.chain_util import label_polygons

pytestmark = pytest.mark.gpu

N = 8


def test_label_masks_select_and_nav_match_oracle():
    from vision_assist_amd.nav import AngleSeen, NavEngine
    from vision_assist_amd.post import select_masks
    inst = [[C.fill_poly(p, 640, 640) for p in label_polygons(i)] for i in range(N)]
    maxn = max(len(m) for m in inst)
    masks = np.zeros((N, maxn, 640, 640), np.uint8)
    for b, ms in enumerate(inst):
        for k, m in enumerate(ms):
            masks[b, k] = m
    n = np.array([len(m) for m in inst], np.int32)
    got = select_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(n), 640, 640)
    assert (got["status"] == 0).all()
    want = [C.select_cells(masks[b, :n[b]], (640, 640)) for b in range(N)]
    for b, (k, pts, rect, cells) in enumerate(want):
        assert got["chosen"][b] == k, b
        assert tuple(got["rects"][b]) == rect, (b, tuple(got["rects"][b]), rect)
        assert np.array_equal(got["cells"][b], cells), b
    eng = NavEngine(640, 640, max_batch=N)
    seen = AngleSeen(torch.device("cuda"))
    res = eng.run(torch.from_numpy(got["cells"]).cuda().contiguous(),
                  torch.from_numpy(got["rects"].astype(np.int32)).cuda().contiguous(), seen)
    pf = onav.PathFinderOracle()
    found = 0
    for b, (k, pts, rect, cells) in enumerate(want):
        out = onav.frame_nav(np.kron(cells, np.ones((20, 20), np.uint8)), rect, 640, 640, pf)
        nf = res.frame(b)
        want_q = [([(c.coords.x, c.coords.y) for c in q[2]], float(q[3]).hex() if q[2] else None)
                  for q in out["queries"]]
        got_q = [(q["path"], float(q["cost"]).hex() if q["path"] else None) for q in nf.queries]
        assert got_q == want_q, b
        found += sum(1 for p, _ in got_q if p)
    assert found >= N // 2  # real corridors: most frames yield a path

"""The mask -> polygon -> cells boundary on the GPU (va_post_select_masks: post_contour_kernel + post_fill_kernel)
against oracle/contours.py, bit for bit, on the same binary masks (tests/contour_cases.py): holes, several
components, islands behind one- and three-pixel walls, thin lines, single pixels, empty masks, masks at the
network input's edges and seeded random blobs; frames equal to the network input (640 x 640), letterboxed
720 x 1280 camera frames (gain 0.5, pad 12: integer scale_coords) and 500 x 880 frames (gain 0.7272..., pad
10.18: fractional float32 scale_coords).

Per frame: the chosen instance (max contourArea, first maximum), boundingRect, the fillPoly samples at every cell
centre; per instance: the point count of its largest external contour, the number of external contours, its
contourArea (float64, exact) and the Results.masks.xy polygon (float32, exact).  Parity with cv2 itself is
unpinned (OpenCV is absent): the oracle is the restatement.
"""
import numpy as np
import pytest
import torch

from oracle import contours as C
from tests.contour_cases import frames_of

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Hn,Wn,H0,W0", [(640, 640, 640, 640), (384, 640, 720, 1280), (384, 640, 500, 880)])
def test_select_masks_matches_oracle(Hn, Wn, H0, W0):
    from vision_assist_amd.post import select_masks
    masks, n = frames_of(Hn, Wn, seed=Hn + W0)
    got = select_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(n), H0, W0)
    assert (got["status"] == 0).all()
    for b in range(masks.shape[0]):
        ms = masks[b, :n[b]]
        xy = C.masks_xy(ms, (H0, W0))
        for k in range(n[b]):
            segs = C.find_contours_external(ms[k])
            st = got["cstats"][b, k]
            assert st["ncont"] == len(segs), (b, k)
            assert st["npts"] == (max(len(s) for s in segs) if segs else 0), (b, k)
            assert st["area"] == C.contour_area(xy[k]), (b, k, st["area"], C.contour_area(xy[k]))
            assert np.array_equal(got["polys"][b][k], xy[k]), (b, k)
        kk, pts, rect, cells = C.select_cells(ms, (H0, W0))
        assert got["chosen"][b] == kk, (b, got["chosen"][b], kk)
        assert tuple(got["rects"][b]) == rect, (b, tuple(got["rects"][b]), rect)
        assert np.array_equal(got["cells"][b], cells), (b, int((got["cells"][b] != cells).sum()))



def test_select_masks_small_frames_lds_image():
    """80 x 160 masks: the framed image fits the small LDS instantiation (the 640-pixel cases use the large one)."""
    from tests.contour_cases import blob
    from vision_assist_amd.post import select_masks
    rng = np.random.default_rng(11)
    Hn, Wn = 80, 160
    masks = np.stack([np.stack([blob(rng, Hn, Wn, sigma=float(rng.uniform(2, 4)), thr=0.52) for _ in range(3)])
                      for _ in range(6)])
    masks[0, 1] = 0  # an empty mask
    n = np.array([3, 3, 2, 3, 1, 3], np.int32)
    got = select_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(n), Hn, Wn)
    assert (got["status"] == 0).all()
    for b in range(masks.shape[0]):
        ms = masks[b, :n[b]]
        xy = C.masks_xy(ms, (Hn, Wn))
        for k in range(n[b]):
            st = got["cstats"][b, k]
            assert st["area"] == C.contour_area(xy[k]), (b, k)
            assert np.array_equal(got["polys"][b][k], xy[k]), (b, k)
        kk, pts, rect, cells = C.select_cells(ms, (Hn, Wn))
        assert got["chosen"][b] == kk and tuple(got["rects"][b]) == rect
        assert np.array_equal(got["cells"][b], cells)


@pytest.mark.parametrize("cap", [1024, 16384])
def test_select_masks_contours_longer_than_the_point_buffer(cap):
    """Noise masks whose largest external contour has 14k-45k points (more than the contour kernel's kept 1024
    and, at p = 0.42, more than the fill kernel's 16384-point buffer): the fill kernel follows the chosen contour
    again once per chunk of `cap` points (a capped buffer dropped the frame's grid); cells, rect and
    chosen instance equal to the oracle's, status 0."""
    from vision_assist_amd.post import select_masks
    rng = np.random.default_rng(3)
    ms = [(rng.random((640, 640)) < p).astype(np.uint8) for p in (0.42, 0.45)]
    masks = np.stack([np.stack([ms[0], ms[1]]), np.stack([ms[1], np.zeros_like(ms[1])])])
    n = np.array([2, 1], np.int32)
    got = select_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(n), 640, 640, cap=cap)
    assert (got["status"] == 0).all()
    for b in range(2):
        kk, pts, rect, cells = C.select_cells(masks[b, :n[b]], (640, 640))
        assert len(pts) > 14000
        assert got["chosen"][b] == kk
        assert tuple(got["rects"][b]) == rect, (b, tuple(got["rects"][b]), rect)
        assert np.array_equal(got["cells"][b], cells), (b, int((got["cells"][b] != cells).sum()))


def test_select_masks_many_items_persistent_form():
    """12 frames x 88 masks (1056 detections > the 1024 scratch slots): the persistent workgroup form
    (post_contour_wgp_kernel -- claims mapped through the frame prefix of the mask counts, ragged counts and an
    empty frame included) gives the oracle's contours, choice, rect and cells."""
    from tests.contour_cases import blob
    from vision_assist_amd.post import select_masks
    rng = np.random.default_rng(23)
    Hn, Wn, B, maxn = 80, 160, 12, 88
    masks = np.zeros((B, maxn, Hn, Wn), np.uint8)
    n = np.array([88, 3, 0, 88, 17, 88, 1, 60, 88, 88, 5, 88], np.int32)
    for b in range(B):
        for k in range(n[b]):
            masks[b, k] = blob(rng, Hn, Wn, sigma=float(rng.uniform(2, 4)), thr=0.52)
    got = select_masks(torch.from_numpy(masks).cuda(), torch.from_numpy(n), Hn, Wn)
    assert (got["status"] == 0).all()
    for b in range(B):
        ms = masks[b, :n[b]]
        xy = C.masks_xy(ms, (Hn, Wn)) if n[b] else []
        for k in range(n[b]):
            st = got["cstats"][b, k]
            assert st["area"] == C.contour_area(xy[k]), (b, k)
            assert np.array_equal(got["polys"][b][k], xy[k]), (b, k)
        if n[b] == 0:
            assert got["chosen"][b] < 0
            continue
        kk, pts, rect, cells = C.select_cells(ms, (Hn, Wn))
        assert got["chosen"][b] == kk and tuple(got["rects"][b]) == rect
        assert np.array_equal(got["cells"][b], cells)

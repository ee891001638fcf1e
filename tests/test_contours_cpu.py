"""CPU checks of oracle/contours.py (the restatement of OpenCV's findContours / contourArea / boundingRect /
fillPoly the device kernels are checked against).  cv2 itself is absent, so these pin the restatement by
properties OpenCV's algorithms have:
  * an axis-aligned rectangle's CHAIN_APPROX_SIMPLE contour is its four corners, from the top-left corner down
    the left side (counter-clockwise in image coordinates);
  * RETR_EXTERNAL returns one contour per 8-connected component that is not inside another one's hole, holes
    and islands inside holes (behind a wall of >= 2 pixels) excluded;
  * fillPoly of every external contour reproduces the mask with its holes filled (the drawContours(FILLED)
    round trip), on seeded random blobs;
  * a single pixel's contour is that pixel; a one-pixel line's contour goes out and back.
"""
import numpy as np
from scipy import ndimage

from oracle import contours as C
from tests.contour_cases import blob, shapes


def test_rectangle_corners_in_opencv_order():
    m = np.zeros((8, 9), np.uint8)
    m[2:6, 3:8] = 1
    (c,) = C.find_contours_external(m)
    assert c.tolist() == [[3, 2], [3, 5], [7, 5], [7, 2]]
    assert C.contour_area(c.astype(np.float32)) == 12.0
    assert C.bounding_rect(c) == (3, 2, 5, 4)


def test_single_pixel_and_line():
    m = np.zeros((6, 6), np.uint8)
    m[2, 3] = 1
    assert [c.tolist() for c in C.find_contours_external(m)] == [[[3, 2]]]
    m = np.zeros((6, 6), np.uint8)
    for k in range(4):
        m[1 + k, 1 + k] = 1
    assert [c.tolist() for c in C.find_contours_external(m)] == [[[1, 1], [4, 4]]]


def test_external_only_one_contour_per_outer_component():
    m = np.zeros((40, 40), np.uint8)
    m[2:20, 2:20] = 1
    m[6:16, 6:16] = 0         # hole (3+ px wall)
    m[9:12, 9:12] = 1         # island in the hole
    m[25:30, 25:38] = 1       # second component
    cs = C.find_contours_external(m)
    assert len(cs) == 2
    assert C.bounding_rect(cs[0]) == (2, 2, 18, 18) and C.bounding_rect(cs[1]) == (25, 25, 13, 5)


def test_fill_of_external_contours_is_the_hole_filled_mask():
    rng = np.random.default_rng(7)
    for _ in range(60):
        m = blob(rng, 48, 60, sigma=float(rng.uniform(2, 5)), thr=0.52)
        f = np.zeros_like(m)
        for c in C.find_contours_external(m):
            f |= C.fill_poly(c, *m.shape)
        assert np.array_equal(f, ndimage.binary_fill_holes(m).astype(np.uint8))


def test_largest_is_by_point_count_not_area():
    m = shapes(640, 640)[1]  # big rectangle (4 points) + small staircase (many points)
    seg = C.largest_segment(m)
    assert seg.shape[0] > 4 and seg[:, 0].min() >= 300


def test_scale_coords_letterbox_float32():
    seg = np.array([[0, 0], [639, 383], [320, 12]], np.float32)
    out = C.scale_coords(seg, (384, 640), (720, 1280))
    assert out.dtype == np.float32
    assert out.tolist() == [[0.0, 0.0], [1278.0, 720.0], [640.0, 0.0]]  # y: (383 - 12) / 0.5 = 742 -> clipped to H


def test_select_cells_choice_by_area():
    masks = np.stack(shapes(640, 640)[:3])
    k, pts, rect, cells = C.select_cells(masks, (640, 640))
    areas = [C.contour_area(p) for p in C.masks_xy(masks, (640, 640))]
    assert k == int(np.argmax(areas)) and cells.shape == (32, 32) and rect[2] > 0


def test_fill_samples_against_full_fill():
    """The cell-centre evaluation of fillPoly (order-free edge counts + line hits) equals sampling the oracle's
    full fillPoly image, on polygons with clipped edges (points at x = W0 / y = H0 after scale_coords)."""
    rng = np.random.default_rng(3)
    H0, W0 = 720, 1280
    for _ in range(20):
        n = int(rng.integers(3, 40))
        pts = np.stack([rng.integers(0, W0 + 1, n), rng.integers(0, H0 + 1, n)], 1).astype(np.int32)
        full = C.fill_poly(pts, H0, W0)
        xs, ys = np.arange(W0 // 20) * 20 + 10, np.arange(H0 // 20) * 20 + 10
        assert np.array_equal(C.fill_poly_samples(pts, H0, W0, xs, ys), full[ys][:, xs])

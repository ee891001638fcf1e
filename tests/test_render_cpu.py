"""Debug rendering (FrameProcessor(debug=True), PathVisualiser.py / FrameProcessor.py:273-299) on the host frame:
squares are cv2.fillPoly of an axis-aligned integer square = the inclusive pixel range, penalty colours from the
nearest gradient key, section colours by position, white section lines and corner dots; later draws cover earlier
ones.  (cv2 itself is absent: the line / circle rasters and the label glyphs are restated and unpinned; the label text,
origin, scale and thickness follow PathVisualiser.py:48-56.)"""
import numpy as np

from vision_assist_amd.models import Coordinate, Corner, Grid, Path
from vision_assist_amd.PathVisualiser import PathVisualiser, draw_line2, fill_circle, fill_square
from vision_assist_amd.PenaltyCalculator import penalty_calculator


def test_fill_square_is_inclusive_and_clipped():
    f = np.zeros((100, 100, 3), np.uint8)
    fill_square(f, 20, 40, (1, 2, 3))
    ys, xs = np.nonzero(f[..., 0])
    assert (ys.min(), ys.max(), xs.min(), xs.max()) == (40, 60, 20, 40)
    assert (f[40, 20] == (1, 2, 3)).all()
    fill_square(f, 90, 90, (9, 9, 9))  # runs off the frame
    assert (f[99, 99] == 9).all() and (f[90, 90] == 9).all()


def test_penalty_colours_nearest_key():
    assert penalty_calculator.get_penalty_colour(0) == (0, 255, 15)
    assert penalty_calculator.get_penalty_colour(1) == (0, 0, 255)
    assert penalty_calculator.get_penalty_colour(0.55) == (8, 145, 255)   # nearest key 0.5833


def test_line_and_circle():
    f = np.zeros((64, 64, 3), np.uint8)
    draw_line2(f, 10, 10, 10, 40, (255, 255, 255))
    col = np.nonzero(f[:, :, 0].any(0))[0]
    assert set(col.tolist()) == {10, 11} and f[10:41, 10, 0].all()
    g = np.zeros((64, 64, 3), np.uint8)
    fill_circle(g, 30, 30, 5, (255, 255, 255))
    ys, xs = np.nonzero(g[..., 0])
    assert (ys.min(), ys.max(), xs.min(), xs.max()) == (25, 35, 25, 35) and g[30, 30, 0] == 255


def test_path_visualiser_draws_sections_in_order():
    grids = [Grid(coords=Coordinate(x=300 + 20 * (i // 6), y=600 - 20 * i),
                  centre=Coordinate(x=310 + 20 * (i // 6), y=610 - 20 * i), penalty=0.0, row=i, col=15 + i // 6,
                  empty=False, artificial=False) for i in range(12)]
    p = Path(grids=grids, total_cost=1.0, path_type="path")
    f = np.zeros((640, 640, 3), np.uint8)
    out = PathVisualiser()(f, [p])
    assert out is f
    n = len(p.sections)
    assert n >= 1
    # the first section's first grid in that section's colour (far for a section at position 0)
    s0 = p.sections[0]
    g0 = s0.grids[0]
    want = PathVisualiser.PATH_COLORS[0].far
    assert tuple(f[g0.coords.y + 3, g0.coords.x + 3]) == want
    # the white line through the section's cell centres
    assert tuple(f[s0.start.y + 10, s0.start.x + 10]) == (255, 255, 255)


def test_corner_label_text_and_placement():
    from vision_assist_amd.PathVisualiser import corner_label
    from vision_assist_amd.strokefont import GLYPHS, put_text, text_size
    c = Corner(direction="left", sharpness="sharp", shape="inner", start=Coordinate(x=300, y=400),
               end=Coordinate(x=340, y=300), angle_change=40.0, length=80.0)
    assert corner_label(0, c) == "1 left inner sharp"
    words = ["left", "right", "inner", "outer", "optimal", "sharp", "sweeping", "0123456789"]
    assert all(ch in GLYPHS for w in words for ch in w)
    f = np.zeros((640, 640, 3), np.uint8)
    pv = PathVisualiser()
    pv.frame = f
    pv._draw_corner_marker(0, c, None)
    ys, xs = np.nonzero(f[..., 0])
    # the dots at start/end + 10 and the text whose baseline starts at (end.x - 100, end.y - 5)
    text = np.zeros_like(f)
    put_text(text, "1 left inner sharp", (240, 295), 0.5, (255, 255, 255), 2)
    assert ((f == 255) | (text == 0)).all()  # every text pixel is drawn
    (w, h), base = text_size("1 left inner sharp", 0.5, 2)
    ty, tx = np.nonzero(text[..., 0])
    assert tx.min() >= 240 and tx.max() < 240 + w and ty.min() >= 295 - h and ty.max() <= 295 + base
    assert tx.max() - tx.min() > 100 and ty.max() - ty.min() >= 9
    assert f[310, 350, 0] == 255 and f[410, 310, 0] == 255  # the two dots

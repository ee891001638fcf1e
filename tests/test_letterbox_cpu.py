"""Host logic of the LetterBox restatement (no GPU): the geometry YOLO.predict's LetterBox(640, auto=True)
and scale_coords give for the reference's frame sizes, and the numpy resize restatement on known cases."""
import numpy as np

from oracle import yolo_ref as Y
from vision_assist_amd.post import letterbox_geometry


def test_geometry_reference_frame_sizes():
    # 720 x 1280 camera frames (the reference fixtures' native size): 0.5x to 360 x 640, 12 rows of 114 above/below
    assert letterbox_geometry(720, 1280) == (384, 640, 12, 0, 360, 640, 0.5, 0, 12)
    # 640 x 640: identity
    assert letterbox_geometry(640, 640) == (640, 640, 0, 0, 640, 640, 1.0, 0, 0)
    # 480 x 848: r = 640/848, 362 rows + 11 + 11
    Hn, Wn, top, left, newh, neww, gain, px, py = letterbox_geometry(480, 848)
    assert (Hn, Wn, top, left, newh, neww, px, py) == (384, 640, 11, 0, 362, 640, 0, 11)
    assert Hn % 32 == 0 and Wn % 32 == 0


def test_resize_restatement_known_cases():
    rng = np.random.default_rng(0)
    f = rng.integers(0, 256, (8, 12, 3), dtype=np.uint8)
    # identity placement
    out = Y.letterbox_np(f, 10, 12, 1, 0, 8, 12)
    assert (out[1:9] == f).all() and (out[0] == 114).all() and (out[9] == 114).all()
    # exact 2x downscale: rounded mean of each 2x2 block (weights 1/2, 1/2 on both axes)
    out = Y.letterbox_np(f, 4, 6, 0, 0, 4, 6)
    blk = f.astype(np.int64).reshape(4, 2, 6, 2, 3).sum((1, 3))
    assert (out == ((blk * 1024 * 1024 + (1 << 21)) >> 22)).all()
    # a constant frame stays constant under any resize
    c = np.full((37, 53, 3), 77, dtype=np.uint8)
    assert (Y.letterbox_np(c, 64, 96, 5, 7, 41, 83)[5:46, 7:90] == 77).all()

"""CPU check of the chunked raster scan of the device contour kernel (va_contour.hip contour_item): between two
traces it evaluates a chunk of the row at once from the current image -- stops, outer-border candidates (row[x-1]
== 0, row[x] == 1) and lnbd events (a stop on a mark; a hole start after a mark) -- with the sign of row[lnbd]
carried across chunks, takes the first candidate whose last event before it leaves row[lnbd] <= 0, traces it and
restarts from x + 1 with row[lnbd] <= 0.  Restated here position by position inside a chunk (what the kernel's
ballots compute in parallel) and compared with the oracle's cvFindNextContour scan (oracle/contours.py) on the
contour test cases and on noise masks, with small chunks so that the carries are exercised."""
import numpy as np
import pytest

from oracle import contours as C
from tests.contour_cases import blob, shapes


def find_contours_chunked(mask: np.ndarray, chunk: int) -> list[np.ndarray]:
    H, W = mask.shape
    img = np.zeros((H + 2, W + 2), dtype=np.int16)
    img[1:H + 1, 1:W + 1] = mask != 0
    width = W + 2
    out = []
    rows = np.nonzero(((img[:, 1:] == 1) & (img[:, :-1] == 0)).any(1))[0]
    for y in rows.tolist():
        row = img[y]
        lpos = False  # row[lnbd] > 0; lnbd starts on the frame
        for c0 in range(0, width, chunk):
            frm = c0
            while True:
                cur, found = lpos, None
                for x in range(frm, min(c0 + chunk, width)):
                    p, pv = int(row[x]), (int(row[x - 1]) if x > 0 else 0)
                    if p == pv:
                        continue  # not a stop
                    if pv == 0 and p == 1:  # outer-border candidate
                        if not cur:
                            found = x
                            break
                    elif p & -2:  # a stop on a mark: lnbd = x
                        cur = p > 0
                    elif p == 0 and pv & -2:  # hole start after a mark: lnbd = x - 1
                        cur = pv > 0
                if found is None:
                    lpos = cur
                    break
                pts = C._fetch_contour(img, y, found, is_hole=False)
                out.append(np.array([(px - 1, py - 1) for px, py in pts], dtype=np.int32))
                lpos, frm = False, found + 1
    return out


def _masks():
    ms = list(shapes(160, 200, seed=3))
    rng = np.random.default_rng(7)
    for thr in (0.3, 0.5, 0.7):  # salt-and-pepper noise: many contours, holes, one-pixel walls
        ms.append((rng.random((96, 140)) < thr).astype(np.uint8))
    for s in range(3):
        ms.append(blob(np.random.default_rng(11 + s), 96, 130, sigma=3.0, thr=0.5))
    return ms


@pytest.mark.parametrize("chunk", [32, 64, 2048])
def test_chunked_scan_equals_sequential(chunk):
    for i, m in enumerate(_masks()):
        want = C.find_contours_external(m)
        got = find_contours_chunked(m, chunk)
        assert len(got) == len(want), (i, len(got), len(want))
        for a, b in zip(got, want):
            assert np.array_equal(a, b), i

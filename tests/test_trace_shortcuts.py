"""CPU checks of the two shortcuts the contour kernels take (va_contour.hip), restated in Python:

* follow_border's straight-run crossing (border_run): where the follow leaves a pixel in the direction it came
  from, the run ahead -- pixels whose counter-clockwise search from s_end + 1 meets zeros at D + 5, D + 6, D + 7 and a
  non-zero at D -- is crossed in one move, its marks set at once, the stop test (i1 followed by i0) checked inside the
  run.  Same kept points and the same marks as the step-by-step follow, on random / box / ellipse / line masks.
* post_fill_kernel's cv::line cell-centre samples: after t major-axis steps the Bresenham walk (err = dx - 2 dy) has
  taken (2 dy t + dx - 1) // (2 dx) minor steps, so only the steps landing on 10 mod 20 need evaluating."""
import numpy as np

DX = [1, 1, 0, -1, -1, -1, 0, 1]
DY = [0, -1, -1, -1, 0, 1, 1, 1]


def _nbrs(img, x, y):
    return sum(1 << d for d in range(8) if img[y + DY[d], x + DX[d]])


def _follow(img, x0, y0, runs):
    H, W = img.shape
    nb = _nbrs(img, x0, y0)
    s = 4
    while True:
        s = (s - 1) & 7
        if (nb >> s) & 1 or s == 4:
            break
    if s == 4:
        return {(x0, y0, True)}, [(x0, y0)]
    marks, pts = set(), []
    x1, y1 = x0 + DX[s], y0 + DY[s]
    x3, y3, prev, nb3, cont1 = x0, y0, s ^ 4, nb, False
    while True:
        se = s
        rot = ((nb3 | (nb3 << 8)) >> ((se + 1) & 7)) & 0xFF
        s = (se + 1 + ((rot & -rot).bit_length() - 1)) & 7
        cont = s == prev
        k = 0
        if runs and cont and cont1:
            for j in range(63):
                px, py = x3 + j * DX[s], y3 + j * DY[s]
                if not (px >= 1 and py >= 1 and py < H - 1 and px + 1 < W):
                    break
                n = _nbrs(img, px, py)
                if (n >> s) & 1 and not any((n >> ((s + e) & 7)) & 1 for e in (5, 6, 7)):
                    k += 1
                else:
                    break
        cont1 = cont
        right = ((s - 1) & 0xFFFFFFFF) < se
        if k > 0:
            dx, dy = DX[s], DY[s]
            j1 = (x1 - x3) * dx if dx else (y1 - y3) * dy
            if 0 <= j1 < k and x3 + j1 * dx == x1 and y3 + j1 * dy == y1 and x1 + dx == x0 and y1 + dy == y0:
                marks |= {(x3 + j * dx, y3 + j * dy, right) for j in range(j1 + 1)}
                break
            marks |= {(x3 + j * dx, y3 + j * dy, right) for j in range(k)}
            x3, y3, s = x3 + k * dx, y3 + k * dy, (s + 4) & 7
            nb3 = _nbrs(img, x3, y3)
            continue
        x4, y4 = x3 + DX[s], y3 + DY[s]
        marks.add((x3, y3, right))
        if s != prev:
            pts.append((x3, y3))
            prev = s
        if (x4, y4, x3, y3) == (x0, y0, x1, y1):
            break
        x3, y3, s = x4, y4, (s + 4) & 7
        nb3 = _nbrs(img, x3, y3)
    return marks, pts


def _masks(rng, n):
    for t in range(n):
        H, W = (int(v) for v in rng.integers(3, 48, 2))
        kind = t % 4
        if kind == 0:
            m = rng.random((H, W)) < rng.uniform(0.2, 0.8)
        elif kind == 1:
            m = np.zeros((H, W), bool)
            for _ in range(int(rng.integers(1, 4))):
                a, b = sorted(rng.integers(0, H, 2))
                c, d = sorted(rng.integers(0, W, 2))
                m[a:b + 1, c:d + 1] = True
        elif kind == 2:
            yy, xx = np.mgrid[:H, :W]
            m = (yy - H / 2) ** 2 / (H / 2.5) ** 2 + (xx - W / 2) ** 2 / (W / 2.5) ** 2 < 1
        else:
            m = np.zeros((H, W), bool)
            for _ in range(int(rng.integers(1, 4))):
                x, y, d = int(rng.integers(0, W)), int(rng.integers(0, H)), int(rng.integers(0, 8))
                for _ in range(int(rng.integers(1, 40))):
                    if 0 <= x < W and 0 <= y < H:
                        m[y, x] = True
                    x, y = x + DX[d], y + DY[d]
        img = np.zeros((H + 2, W + 2), np.uint8)
        img[1:-1, 1:-1] = m
        yield img


def test_run_crossing_equals_step_by_step():
    rng = np.random.default_rng(0)
    n = 0
    for img in _masks(rng, 600):
        ys, xs = np.nonzero(img)
        for y, x in zip(ys, xs):
            if img[y, x - 1] == 0:  # every 0 -> 1 transition as a start
                assert _follow(img, x, y, False) == _follow(img, x, y, True), (x, y)
                n += 1
    assert n > 10000


def _walk(dx, dy):
    err, m, out = dx - 2 * dy, 0, []
    for _ in range(dx + 1):
        out.append(m)
        minor = err < 0
        err += -2 * dy + (2 * dx if minor else 0)
        m += minor
    return out


def test_bresenham_minor_steps_closed_form():
    for dx in range(0, 160):
        for dy in range(0, dx + 1):
            want = _walk(dx, dy)
            got = [(2 * dy * t + dx - 1) // (2 * dx) if dx else 0 for t in range(dx + 1)]
            assert got == want, (dx, dy)

"""Binary instance masks that exercise the mask -> polygon -> cells boundary (FrameProcessor.py:67-97): holes,
several components, an island inside a hole behind a one-pixel wall (RETR_EXTERNAL's lnbd rule), thin diagonal
lines, single pixels, empty masks, masks running off the network input's edges (scale_coords clipping onto the
frame border) and seeded smooth random blobs.  Test data only."""
from __future__ import annotations

import numpy as np
from scipy import ndimage


def blob(rng, H, W, sigma=6.0, thr=0.53):
    return (ndimage.gaussian_filter(rng.random((H, W)), sigma) > thr).astype(np.uint8)


def shapes(H: int, W: int, seed: int = 0) -> list[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = []
    m = np.zeros((H, W), np.uint8)
    m[H // 4:3 * H // 4, W // 5:4 * W // 5] = 1
    m[H // 3:H // 2, W // 3:W // 2] = 0                      # rectangle with a hole
    out.append(m)
    m = np.zeros((H, W), np.uint8)
    m[10:60, 10:200] = 1                                     # a big rectangle (few points) ...
    for k in range(40):                                      # ... and a small jagged strip (many points)
        m[100 + k, 300 + 3 * (k % 2):310 + 2 * (k % 3)] = 1
    out.append(m)
    m = np.zeros((H, W), np.uint8)
    m[50:150, 50:150] = 1
    m[51:149, 51:149] = 0                                    # one-pixel wall ...
    m[90:110, 90:110] = 1                                    # ... around an island
    m[200:300, 200:300] = 1
    m[203:297, 203:297] = 0                                  # three-pixel wall
    m[240:260, 240:260] = 1
    out.append(m)
    m = np.zeros((H, W), np.uint8)
    for k in range(min(H, W) - 40):
        m[20 + k, 20 + k] = 1                                # a one-pixel diagonal line
    m[5, 400 % W] = 1                                        # a single pixel
    out.append(m)
    m = np.zeros((H, W), np.uint8)
    m[H - 40:, W // 3:2 * W // 3] = 1                        # touches the bottom edge
    m[:30, :50] = 1                                          # touches the top-left corner
    out.append(m)
    out.append(np.zeros((H, W), np.uint8))                   # empty
    for _ in range(4):
        out.append(blob(rng, H, W, sigma=float(rng.uniform(3, 9)), thr=float(rng.uniform(0.51, 0.56))))
    return out


def frames_of(H: int, W: int, seed: int = 0, per_frame: int = 3):
    """Batches of instance masks [B, maxn, H, W] + counts: every case alone, and mixed triples (the area choice)."""
    cases = shapes(H, W, seed)
    frames = [[c] for c in cases]
    rng = np.random.default_rng(seed + 1)
    for _ in range(6):
        idx = rng.choice(len(cases), size=per_frame, replace=False)
        frames.append([cases[i] for i in idx])
    maxn = max(len(f) for f in frames)
    arr = np.zeros((len(frames), maxn, H, W), np.uint8)
    n = np.zeros(len(frames), np.int32)
    for b, f in enumerate(frames):
        for k, m in enumerate(f):
            arr[b, k] = m
        n[b] = len(f)
    return arr, n

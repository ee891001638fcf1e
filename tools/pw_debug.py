"""Where does the streaming 1x1 kernel (va_pw.hip) go wrong on multi-tile launches?  Runs one conv through
the test helper and prints the bad pixels by persistent pass (tile // waves-in-grid), by pixel in tile and
by channel."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_seg import _run_single_conv  # noqa: E402

for cin, H, W in ((128, 320, 320), (64, 320, 320), (256, 200, 328)):
    got, ref = _run_single_conv("bf16", cin, 128, 1, 1, H, W, False, False, 0, act=True)
    # [B, C, H, W] -> [M, C]
    g = got.permute(0, 2, 3, 1).reshape(-1, 128)
    r = ref.permute(0, 2, 3, 1).reshape(-1, 128)
    bad = ~((g - r).abs() <= 0.05 * r.abs().max())
    badpix = bad.any(1)
    m = torch.nonzero(badpix).flatten()
    waves = 256 * 8
    tiles = m // 48
    print(f"cin={cin} M={g.shape[0]} ntiles={(g.shape[0] + 47) // 48}: bad pixels {m.numel()}, "
          f"non-finite {int((~torch.isfinite(g)).sum())}", flush=True)
    if m.numel():
        passes = torch.bincount(tiles // waves)
        print("  bad pixels per persistent pass:", passes.tolist())
        print("  per pixel-in-tile:", torch.bincount(m % 48, minlength=48).tolist())
        print("  per channel:", bad.sum(0).tolist())
        print("  first bad tiles:", torch.unique(tiles)[:20].tolist())
        t0 = int(tiles[0])
        print("  tile", t0, "got", g[t0 * 48, :8].tolist(), "ref", r[t0 * 48, :8].tolist())

"""The fused per-frame hot path for a batch of frames, device-resident end to end.

    frames (uint8 BGR, HBM) -> va_seg_run  (preprocess + YOLOv8-seg forward, MFMA)
                            -> va_post_run (decode, NMS, process_mask, mask choice -> cells, rect)
                            -> va_nav_run  (grid, penalties, protrusions, start/end, A*, dedupe)

This is FrameProcessor.__call__ (FrameProcessor.py:301-347) for B frames at
once; PathAnalyser (:349) runs on the host per frame in the FrameProcessor
surface.  Frames of one batch are processed in order for the PathFinder angle
cache (the batch gives exactly the sequential result, see va_nav.hip).
"""
from __future__ import annotations

import torch

from .nav import AngleSeen, NavBatch, NavEngine
from .post import PLANT_IF_NONE, PLANT_NEVER, PostEngine
from .seg import SegNet


class FramePipeline:
    def __init__(self, arch, folded, B: int, H: int, W: int, dtype: str = "bf16", conf: float = 0.5,
                 iou: float = 0.7, max_det: int = 300, device=None, seen: AngleSeen | None = None):
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.B, self.H, self.W = B, H, W
        self.seg = SegNet(arch, folded, dtype=dtype, device=self.device)
        self.plan = self.seg.plan(B, H, W)
        self.post = PostEngine(B, H, W, arch.nc, conf, iou, max_det, device=self.device)
        self.nav = NavEngine(H, W, max_batch=B, device=self.device)
        self.seen = seen if seen is not None else AngleSeen(self.device)

    @property
    def frames(self) -> torch.Tensor:
        """The device frame buffer (uint8 [B, H, W, 3]) the forward reads."""
        return self.plan["frames"]

    def run(self, frames: torch.Tensor | None = None, plant_cells=None, plant_rects=None,
            plant_mode: int = PLANT_NEVER, stream=None) -> NavBatch:
        if frames is not None:
            self.plan["frames"].copy_(frames, non_blocking=True)
        self.seg.run_plan(self.plan, stream)
        out = self.plan["out"]
        if plant_mode != PLANT_NEVER and plant_cells is None:
            raise ValueError("plant_mode needs plant_cells / plant_rects")
        self.post.run(out.levels, out.proto, plant_cells, plant_rects, plant_mode, select=True, stream=stream)
        return self.nav.run(self.post.cells, self.post.rects, self.seen, stream)

    def run_seg_only(self, stream=None) -> None:
        self.seg.run_plan(self.plan, stream)


__all__ = ["FramePipeline", "PLANT_IF_NONE", "PLANT_NEVER"]

"""YOLO model object for FrameProcessor (replaces ``ultralytics.YOLO`` at main.py:43).

``YOLO(weights).to("cuda")`` then ``FrameProcessor(model=...)`` exactly as main.py
does.  The network is YOLOv8-seg (n / s / m) running on the MI355X MFMA kernels
of libva355.so; ``predict`` returns per-frame ``Results`` whose mask has already
been reduced on the device to what FrameProcessor consumes (FrameProcessor.py:67-97):
the chosen instance's cell-lattice samples and bounding rect, plus ``masks.xy`` (the
per-detection polygons, traced on the device as findContours does).

Weights: a ``.safetensors`` file with Ultralytics state-dict names (export one
with ``safetensors.torch.save_file(model.model.state_dict(), path)`` where
ultralytics is available) is folded and packed; a bare model name such as
``yolov8s-seg.pt`` (main.py:14's default, which Ultralytics would download)
gets seeded synthetic weights of that architecture -- nothing is downloaded.
"""
from __future__ import annotations

import os
import re
import warnings

import numpy as np
import torch

from .post import scale_boxes
from .seg_arch import Arch, fold, synthetic_state_dict


class Masks:
    """Device mask summary of one frame (the input of the grid stage) + Results.masks.xy."""

    def __init__(self, cells: torch.Tensor, rect: tuple[int, int, int, int], chosen: int, xy: list | None = None):
        self.cells = cells      # uint8 [H/20, W/20] on the device: fillPoly of the chosen polygon at cell centres
        self.rect = rect        # boundingRect (x, y, w, h) of the chosen polygon
        self.chosen = chosen    # index of the chosen detection (max contourArea), -2 = planted
        self.xy = xy            # per detection: largest external contour in frame pixels, float32 [k, 2] (None: given cells)


class Results:
    def __init__(self, orig_shape, boxes: np.ndarray, masks: Masks | None):
        self.orig_shape = orig_shape
        self.boxes = boxes      # float [k, 6]: x1, y1, x2, y2 (frame pixels), conf, cls (kept, score order)
        self.masks = masks      # None when no mask (FrameProcessor.py:68-69)


class YOLO:
    def __init__(self, model: str = "yolov8s-seg.pt", task: str | None = None, *, dtype: str = "f32", nc: int = 80,
                 seed: int = 0, cls_bias: float | None = None, sparse: int | None = None, solid_masks: bool = False):
        """model: a .safetensors state dict with Ultralytics key names, or a yolov8{n,s,m}-seg name (seeded
        synthetic weights; cls_bias / sparse / solid_masks select the synthetic regime, seg_arch.synthetic_state_dict)."""
        # the constructor's arguments: a FrameDealer worker rebuilds this model on its own GPU (shard.dropin_worker)
        self.spec = (str(model), dict(task=task, dtype=dtype, nc=nc, seed=seed, cls_bias=cls_bias, sparse=sparse,
                                      solid_masks=solid_masks))
        name = os.path.basename(str(model))
        if str(model).endswith(".safetensors") and os.path.exists(model):
            from safetensors.torch import load_file
            sd = load_file(model)
            m = re.search(r"yolov8([nsm])", name)
            scale = m.group(1) if m else "s"
            nc = int(sd["model.22.cv3.0.2.weight"].shape[0]) if "model.22.cv3.0.2.weight" in sd else nc
            self.arch = Arch(scale, nc)
        else:
            m = re.search(r"yolov8([nsm])-seg", name)
            if not m:
                raise ValueError(f"unknown model {model!r}: expected yolov8{{n,s,m}}-seg or a .safetensors state dict")
            self.arch = Arch(m.group(1), nc)
            warnings.warn(f"{model}: no local weights, using seeded synthetic yolov8{m.group(1)}-seg weights "
                          "(nothing is downloaded)")
            sd = synthetic_state_dict(self.arch, seed=seed, cls_bias=cls_bias, sparse=sparse, solid_masks=solid_masks)
        self.folded = fold(self.arch, sd)
        self.dtype = dtype
        self.fp8_calib = None  # fp8: representative frames for the activation scales (SegNet.calibrate_fp8)
        self.device = None
        self._pipes = {}

    def to(self, device):
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        return self

    def pipeline(self, H: int, W: int, conf: float = 0.5, iou: float = 0.7, max_det: int = 300, seen=None,
                 imgsz: int | None = 640):
        """The fused single-frame device pipeline for H x W frames (cached).  imgsz = predict's imgsz (640, the
        Ultralytics default the reference's model.predict(frame, conf=0.5) uses): frames are letterboxed to it
        whenever that changes them; None runs the network at the frame's own size (sides multiples of 32)."""
        from .pipeline import FramePipeline
        key = (H, W, conf, iou, max_det, imgsz)
        if key not in self._pipes:
            self._pipes[key] = FramePipeline(self.arch, self.folded, 1, H, W, dtype=self.dtype, conf=conf, iou=iou,
                                             max_det=max_det, device=self.device, seen=seen, imgsz=imgsz,
                                             fp8_calib=self.fp8_calib, seg=self._segnet())
        return self._pipes[key]

    def stream_batches(self, H: int, W: int, B: int, seen=None, conf: float = 0.5, iou: float = 0.7,
                       max_det: int = 300, imgsz: int | None = 640):
        """A frame stream in device batches of up to B frames (pipeline.StreamBatches, cached), on the same
        weights as ``pipeline`` and predict's defaults: FrameProcessor's batched form (FrameDealer workers)."""
        from .pipeline import StreamBatches
        key = ("batches", H, W, B, conf, iou, max_det, imgsz)
        if key not in self._pipes:
            self._pipes[key] = StreamBatches(self.arch, self.folded, B, H, W, dtype=self.dtype, conf=conf, iou=iou,
                                             max_det=max_det, device=self.device, seen=seen, imgsz=imgsz,
                                             fp8_calib=self.fp8_calib, seg=self._segnet())
        return self._pipes[key]

    def _segnet(self):
        """The packed weights on the device, one SegNet shared by every pipeline of this model."""
        from .seg import SegNet
        if self.device is None:
            self.to("cuda")
        if getattr(self, "_seg", None) is None or self._seg.device != self.device:
            self._seg = SegNet(self.arch, self.folded, dtype=self.dtype, device=self.device)
        return self._seg

    def predict(self, source, conf: float = 0.5, verbose: bool = False, iou: float = 0.7, max_det: int = 300,
                imgsz: int | None = 640):
        frames = source if isinstance(source, (list, tuple)) else [source]
        out = []
        for fr in frames:
            t = torch.as_tensor(fr) if not isinstance(fr, torch.Tensor) else fr
            H, W = int(t.shape[0]), int(t.shape[1])
            pipe = self.pipeline(H, W, conf, iou, max_det, imgsz=imgsz)
            pipe.load(t.reshape(1, H, W, 3))  # pinned-staged H2D, letterboxed to the network input if needed
            pipe.seg.run_plan(pipe.plan)
            o = pipe.plan["out"]
            pipe.post.run(o.levels, o.proto, select=True)
            det, _ = pipe.post.det_tensor(0)
            scale_boxes((pipe.Hn, pipe.Wn), det[:, :4], (H, W))  # Results.boxes in frame pixels (in place)
            chosen = int(pipe.post.chosen[0])
            masks = None
            if chosen >= 0:
                masks = Masks(pipe.post.cells[0].clone(), tuple(int(v) for v in pipe.post.rects[0].cpu()), chosen,
                              pipe.post.polygons(0))
            out.append(Results((H, W), det.numpy(), masks))
        return out

"""Host driver of the segmentation post-processing (libva355.so ``va_post_run``).

Decode -> NMS -> process_mask -> mask choice for B frames, all on the device,
reading the head buffers ``SegNet`` produced (no copies) and writing the
(cells, rects) input of the nav stage.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

VOIDP = ctypes.c_void_p


class PostArgs(ctypes.Structure):
    _fields_ = [
        ("levels", VOIDP * 3), ("proto", VOIDP),
        ("B", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32), ("nc", ctypes.c_int32),
        ("conf", ctypes.c_float), ("iou", ctypes.c_float),
        ("max_det", ctypes.c_int32), ("plant_mode", ctypes.c_int32),
        ("cand", VOIDP), ("cand_count", VOIDP), ("keys", VOIDP),
        ("dets", VOIDP), ("ndet", VOIDP), ("stats", VOIDP),
        ("plant_cells", VOIDP), ("plant_rects", VOIDP),
        ("cells", VOIDP), ("rects", VOIDP), ("chosen", VOIDP),
        ("H0", ctypes.c_int32), ("W0", ctypes.c_int32), ("pad_x", ctypes.c_int32), ("pad_y", ctypes.c_int32),
        ("gain", ctypes.c_float),
        ("max_nms", ctypes.c_int32),
    ]


def letterbox_geometry(H: int, W: int, imgsz: int = 640, stride: int = 32):
    """Ultralytics LetterBox(new_shape=imgsz, auto=True, scaleup=True, center=True) as YOLO.predict applies
    it (data/augment.py; restated, Ultralytics is absent) and the matching scale_coords gain / pad:
    -> (Hn, Wn, top, left, newh, neww, gain, pad_x, pad_y)."""
    r = min(imgsz / H, imgsz / W)
    neww, newh = int(round(W * r)), int(round(H * r))
    dw, dh = (imgsz - neww) % stride, (imgsz - newh) % stride
    dw, dh = dw / 2, dh / 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    Hn, Wn = newh + top + bottom, neww + left + right
    gain = min(Hn / H, Wn / W)  # scale_coords / scale_boxes (ops.py)
    pad_x, pad_y = int(round((Wn - W * gain) / 2 - 0.1)), int(round((Hn - H * gain) / 2 - 0.1))
    return Hn, Wn, top, left, newh, neww, gain, pad_x, pad_y


PLANT_NEVER, PLANT_IF_NONE, PLANT_ALWAYS = 0, 1, 2


class PostEngine:
    """Scratch + outputs for B frames of H x W; one ``run`` per batch."""

    def __init__(self, B: int, H: int, W: int, nc: int, conf: float = 0.5, iou: float = 0.7, max_det: int = 300,
                 device=None, frame=None, max_nms: int = 30000):
        """H x W: the network input.  frame = (H0, W0, gain, pad_x, pad_y) when it is a letterbox of H0 x W0
        frames: the mask choice then reports cells / rects in frame coordinates."""
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        A = int(self.lib.va_post_anchors(H, W))
        if A <= 0:
            raise _lib.VaError(f"va_post_anchors({H}, {W}) = {A}")
        self.B, self.H, self.W, self.nc, self.A = B, H, W, nc, A
        self.conf, self.iou, self.max_det, self.max_nms = conf, iou, max_det, max_nms
        dev = self.device
        self.cand = torch.empty((B, A, 8), dtype=torch.int32, device=dev)
        self.cand_count = torch.empty(B, dtype=torch.int32, device=dev)
        self.keys = torch.empty((B, A), dtype=torch.int64, device=dev)
        self.dets = torch.empty((B, max_det, 8), dtype=torch.int32, device=dev)  # va_det (5 f32 + 3 i32)
        self.ndet = torch.empty(B, dtype=torch.int32, device=dev)
        self.stats = torch.empty((B, max_det, 8), dtype=torch.int32, device=dev)
        self.frame = frame
        H0, W0 = (frame[0], frame[1]) if frame else (H, W)
        self.cells = torch.empty((B, H0 // 20, W0 // 20), dtype=torch.uint8, device=dev)
        self.rects = torch.empty((B, 4), dtype=torch.int32, device=dev)
        self.chosen = torch.empty(B, dtype=torch.int32, device=dev)

    def run(self, levels, proto, plant_cells=None, plant_rects=None, plant_mode=PLANT_NEVER, select=True,
            stream=None) -> None:
        a = PostArgs()
        for i in range(3):
            a.levels[i] = levels[i].data_ptr()
        a.proto = proto.data_ptr()
        a.B, a.H, a.W, a.nc = self.B, self.H, self.W, self.nc
        a.conf, a.iou, a.max_det, a.plant_mode = self.conf, self.iou, self.max_det, plant_mode
        a.max_nms = self.max_nms
        a.cand, a.cand_count, a.keys = self.cand.data_ptr(), self.cand_count.data_ptr(), self.keys.data_ptr()
        a.dets, a.ndet, a.stats = self.dets.data_ptr(), self.ndet.data_ptr(), self.stats.data_ptr()
        if plant_mode != PLANT_NEVER:
            a.plant_cells, a.plant_rects = plant_cells.data_ptr(), plant_rects.data_ptr()
        if select:
            a.cells, a.rects, a.chosen = self.cells.data_ptr(), self.rects.data_ptr(), self.chosen.data_ptr()
        if self.frame:
            a.H0, a.W0, a.gain, a.pad_x, a.pad_y = self.frame
        with torch.cuda.device(self.device):
            _lib.check(self.lib.va_post_run(_lib.stream_ptr(stream, self.device), ctypes.byref(a)), "va_post_run")

    def det_tensor(self, b: int) -> torch.Tensor:
        """Kept detections of frame b as float [k, 6] (x1, y1, x2, y2, score, cls) + anchors [k]."""
        n = int(self.ndet[b])
        raw = self.dets[b, :n].cpu()
        f = raw.view(torch.float32)
        out = torch.cat([f[:, :5], raw[:, 5:6].float()], 1)
        return out, raw[:, 6].clone()

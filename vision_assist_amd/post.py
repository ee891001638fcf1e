"""Host driver of the segmentation post-processing (libva355.so ``va_post_run``).

Decode -> NMS -> process_mask -> mask choice for B frames, all on the device,
reading the head buffers ``SegNet`` produced (no copies) and writing the
(cells, rects) input of the nav stage.
"""
from __future__ import annotations

import ctypes
import os

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
        ("H0", ctypes.c_int32), ("W0", ctypes.c_int32),
        ("sc_gain", ctypes.c_float), ("sc_padx", ctypes.c_float), ("sc_pady", ctypes.c_float),
        ("cscratch", VOIDP), ("cslots", ctypes.c_int32), ("ccap", ctypes.c_int32),
        ("cstats", VOIDP), ("cstatus", VOIDP), ("cpts", VOIDP),
        ("max_nms", ctypes.c_int32), ("cpts_cap", ctypes.c_int32),
    ]


class ContourStat(ctypes.Structure):  # va_contour_stat
    _fields_ = [(n, ctypes.c_int32) for n in ("npts", "ox", "oy", "ncont", "X0", "Y0", "status", "half")] + \
               [("area", ctypes.c_double)]


class MaskSelectArgs(ctypes.Structure):  # va_mask_select_args
    _fields_ = [("masks", VOIDP), ("nmask", VOIDP)] + \
               [(n, ctypes.c_int32) for n in ("B", "maxn", "Hn", "Wn", "H0", "W0")] + \
               [(n, ctypes.c_float) for n in ("gain", "padx", "pady")] + \
               [("scratch", VOIDP), ("nslots", ctypes.c_int32), ("cap", ctypes.c_int32), ("cstats", VOIDP),
                ("cells", VOIDP), ("rects", VOIDP), ("chosen", VOIDP), ("status", VOIDP), ("polys", VOIDP),
                ("poly_n", VOIDP), ("cpts", VOIDP), ("poly_cap", ctypes.c_int32), ("cpts_cap", ctypes.c_int32)]


CSTAT_DTYPE = [("npts", "<i4"), ("ox", "<i4"), ("oy", "<i4"), ("ncont", "<i4"), ("X0", "<i4"), ("Y0", "<i4"),
               ("status", "<i4"), ("half", "<i4"), ("area", "<f8")]
CONTOUR_SLOTS = int(os.environ.get("VA_CT_SLOTS", "1024"))  # contour scratch slots: one wave each, 4 per CU
CONTOUR_CAP = 16384    # points of the fill kernel's buffer per pass (a longer chosen contour takes several passes)
CONTOUR_PTS = 1024     # points kept per instance and buffer half (va_post_args.cpts_cap); longer: followed again


def scale_coords_params(H: int, W: int, H0: int, W0: int) -> tuple[float, float, float]:
    """ops.scale_coords(img1_shape=(H, W), ., img0_shape=(H0, W0)): gain and pad in double, as Ultralytics computes
    them; the kernels use them rounded to float32 (numpy's float32 arithmetic on the float32 polygon)."""
    gain = min(H / H0, W / W0)
    return gain, (W - W0 * gain) / 2, (H - H0 * gain) / 2


def scale_boxes(net_hw: tuple[int, int], boxes: torch.Tensor, frame_hw: tuple[int, int]) -> torch.Tensor:
    """Results.boxes in frame coordinates: Ultralytics' ops.scale_boxes(img1_shape=net, xyxy, img0_shape=frame)
    (reference's vendored ops.py:139-170 + clip_boxes :366-385) on a float32 host tensor, in place: gain in double,
    integer pads round(. - 0.1), float32 arithmetic, clamped to the frame.  Bit-equal to the reference's function
    on its own outputs (tests/test_ops_pinned_cpu.py, tests/golden/ops_goldens.npz)."""
    gain = min(net_hw[0] / frame_hw[0], net_hw[1] / frame_hw[1])
    pad_x = round((net_hw[1] - frame_hw[1] * gain) / 2 - 0.1)
    pad_y = round((net_hw[0] - frame_hw[0] * gain) / 2 - 0.1)
    for c, p in enumerate((pad_x, pad_y, pad_x, pad_y)):
        boxes[..., c] -= p
    boxes[..., :4] /= gain
    for c, hi in enumerate((frame_hw[1], frame_hw[0], frame_hw[1], frame_hw[0])):
        boxes[..., c] = boxes[..., c].clamp(0, hi)
    return boxes


def contour_scratch(H: int, W: int, slots: int = CONTOUR_SLOTS, cap: int = CONTOUR_CAP, device=None) -> torch.Tensor:
    lib = _lib.load()
    sb, io, po = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _lib.check(lib.va_contour_scratch_bytes(H, W, slots, cap, ctypes.byref(sb), ctypes.byref(io), ctypes.byref(po)),
               "va_contour_scratch_bytes")
    return torch.empty(slots * sb.value, dtype=torch.uint8, device=device)


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
        self.H0, self.W0 = H0, W0
        self.cells = torch.empty((B, H0 // 20, W0 // 20), dtype=torch.uint8, device=dev)
        self.rects = torch.empty((B, 4), dtype=torch.int32, device=dev)
        self.chosen = torch.empty(B, dtype=torch.int32, device=dev)
        self.cstats = torch.empty((B, max_det, ctypes.sizeof(ContourStat)), dtype=torch.uint8, device=dev)
        self.cstatus = torch.empty(B, dtype=torch.int32, device=dev)
        self.cscratch = contour_scratch(H, W, device=dev)
        self.cpts = torch.empty((B, max_det, 2, CONTOUR_PTS), dtype=torch.int32, device=dev)

    def run(self, levels, proto, plant_cells=None, plant_rects=None, plant_mode=PLANT_NEVER, select=True,
            stream=None) -> None:
        a = self.args(levels, proto, plant_cells, plant_rects, plant_mode, select)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.va_post_run(_lib.stream_ptr(stream, self.device), ctypes.byref(a)), "va_post_run")

    def args(self, levels, proto, plant_cells=None, plant_rects=None, plant_mode=PLANT_NEVER,
             select=True) -> "PostArgs":
        """The va_post_args of a run on these network outputs (also kept for polygons())."""
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
        self._fill_frame_args(a)
        self._last = (a, levels, proto)  # Results.masks.xy re-reads these buffers (polygons())
        return a

    def _fill_frame_args(self, a: PostArgs) -> None:
        if self.frame:
            a.H0, a.W0 = self.H0, self.W0
            a.sc_gain, a.sc_padx, a.sc_pady = scale_coords_params(self.H, self.W, self.H0, self.W0)
        a.cscratch, a.cslots, a.ccap = self.cscratch.data_ptr(), CONTOUR_SLOTS, CONTOUR_CAP
        a.cstats, a.cstatus = self.cstats.data_ptr(), self.cstatus.data_ptr()
        a.cpts, a.cpts_cap = self.cpts.data_ptr(), CONTOUR_PTS

    def polygons(self, b: int, cap: int = 4096, stream=None) -> list:
        """Results.masks.xy of frame b of the last run: per kept detection its largest external contour in frame
        coordinates (float32 [k, 2], masks2segments 'largest' + scale_coords)."""
        import numpy as np
        a, _levels, _proto = self._last
        pts = self._points_polygons(b)
        if pts is not None:
            return pts
        polys = torch.empty((self.B, self.max_det, cap, 2), dtype=torch.float32, device=self.device)
        pn = torch.zeros((self.B, self.max_det), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.va_post_polygons(_lib.stream_ptr(stream, self.device), ctypes.byref(a), polys.data_ptr(),
                                                 pn.data_ptr(), cap), "va_post_polygons")
        n = int(self.ndet[b])
        cnt = pn[b, :n].cpu().numpy()
        if (cnt > cap).any():  # the kernel reports the full count: rerun with room for the longest
            return self.polygons(b, cap=int(cnt.max()), stream=stream)
        pts = polys[b, :n].cpu().numpy()
        return [np.ascontiguousarray(pts[k, :cnt[k]]) for k in range(n)]

    def _points_polygons(self, b: int):
        """masks.xy from the point buffers the last va_post_run already holds (polygons() used to repeat
        the whole contour pass): each detection's longest contour sits in half cstats.half of its cpts slot as
        network pixels x | y << 16, mapped by the float32 scale_coords the kernel applies (scale_pt: (p - pad) /
        gain, clipped -- IEEE float32 subtract / divide / min / max, the same bits on the host).  None when a contour
        was longer than the buffer (then only a trace from the image has it)."""
        import numpy as np
        n = int(self.ndet[b])
        if n == 0:
            return []
        cs = self.contour_stats(b)
        npts = cs["npts"].astype(np.int64)
        if (npts > CONTOUR_PTS).any():
            return None
        raw = self.cpts[b, :n].cpu().numpy().view(np.uint32)  # [n, 2, CONTOUR_PTS]
        if self.frame:
            g, px, py = (np.float32(v) for v in scale_coords_params(self.H, self.W, self.H0, self.W0))
            W0, H0 = np.float32(self.W0), np.float32(self.H0)
        else:
            g, px, py, W0, H0 = np.float32(1), np.float32(0), np.float32(0), np.float32(self.W), np.float32(self.H)
        out = []
        for k in range(n):
            q = raw[k, int(cs["half"][k]), :int(npts[k])]
            x = (q & 0xFFFF).astype(np.float32)
            y = (q >> 16).astype(np.float32)
            xs = np.minimum(np.maximum((x - px) / g, np.float32(0)), W0)
            ys = np.minimum(np.maximum((y - py) / g, np.float32(0)), H0)
            out.append(np.ascontiguousarray(np.stack([xs, ys], 1).astype(np.float32)))
        return out

    def contour_stats(self, b: int):
        import numpy as np
        n = int(self.ndet[b])
        return self.cstats[b, :n].cpu().numpy().view(np.dtype(CSTAT_DTYPE)).reshape(n)

    def det_tensor(self, b: int) -> torch.Tensor:
        """Kept detections of frame b as float [k, 6] (x1, y1, x2, y2, score, cls) + anchors [k]."""
        n = int(self.ndet[b])
        raw = self.dets[b, :n].cpu()
        f = raw.view(torch.float32)
        out = torch.cat([f[:, :5], raw[:, 5:6].float()], 1)
        return out, raw[:, 6].clone()


def select_masks(masks: torch.Tensor, nmask: torch.Tensor, H0: int, W0: int, poly_cap: int = 4096, stream=None,
                 cap: int = CONTOUR_CAP):
    """The mask -> polygon -> cells boundary (va_post_select_masks) on given binary masks uint8 [B, maxn, Hn, Wn]
    (device) with nmask[b] masks in frame b, mapped onto an H0 x W0 frame as scale_coords does.  cap: points of
    the fill kernel's buffer per pass (a longer chosen contour is taken in several passes; >= CONTOUR_PTS).
    -> dict(cells [B, H0/20, W0/20], rects [B, 4], chosen [B], status [B], cstats [B, maxn], polys list per frame)."""
    import numpy as np
    lib = _lib.load()
    dev = masks.device
    B, maxn, Hn, Wn = masks.shape
    gain, padx, pady = scale_coords_params(Hn, Wn, H0, W0)
    scratch = contour_scratch(Hn, Wn, cap=cap, device=dev)
    cstats = torch.empty((B, maxn, ctypes.sizeof(ContourStat)), dtype=torch.uint8, device=dev)
    cells = torch.empty((B, H0 // 20, W0 // 20), dtype=torch.uint8, device=dev)
    rects = torch.empty((B, 4), dtype=torch.int32, device=dev)
    chosen = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    polys = torch.empty((B, maxn, poly_cap, 2), dtype=torch.float32, device=dev)
    pn = torch.zeros((B, maxn), dtype=torch.int32, device=dev)
    cpts = torch.empty((B, maxn, 2, CONTOUR_PTS), dtype=torch.int32, device=dev)
    nm = nmask.to(dev, torch.int32).contiguous()
    m = masks.contiguous()
    a = MaskSelectArgs(masks=m.data_ptr(), nmask=nm.data_ptr(), B=B, maxn=maxn, Hn=Hn, Wn=Wn, H0=H0, W0=W0,
                       gain=gain, padx=padx, pady=pady, scratch=scratch.data_ptr(), nslots=CONTOUR_SLOTS,
                       cap=cap, cstats=cstats.data_ptr(), cells=cells.data_ptr(), rects=rects.data_ptr(),
                       chosen=chosen.data_ptr(), status=status.data_ptr(), polys=polys.data_ptr(), poly_n=pn.data_ptr(),
                       cpts=cpts.data_ptr(), poly_cap=poly_cap, cpts_cap=CONTOUR_PTS)
    with torch.cuda.device(dev):
        _lib.check(lib.va_post_select_masks(_lib.stream_ptr(stream, dev), ctypes.byref(a)), "va_post_select_masks")
    torch.cuda.synchronize(dev)
    cs = cstats.cpu().numpy().view(np.dtype(CSTAT_DTYPE)).reshape(B, maxn)
    pnh, ph = pn.cpu().numpy(), polys.cpu().numpy()
    nmh = nm.cpu().numpy()
    return {"cells": cells.cpu().numpy(), "rects": rects.cpu().numpy(), "chosen": chosen.cpu().numpy(),
            "status": status.cpu().numpy(), "cstats": cs,
            "polys": [[ph[b, k, :pnh[b, k]] for k in range(nmh[b])] for b in range(B)]}

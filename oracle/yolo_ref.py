"""Plain-PyTorch fp32 (CPU) reference of the segmentation stage (TEST INFRASTRUCTURE).

Checker for the HIP YOLOv8-seg path and the cpu_baseline leg of bench.py;
never imported by the product.  The algorithms live in the third-party
``ultralytics`` package (version evidence 8.3.3:
model/runs/segment/train16/weights/best_saved_model/metadata.yaml:4), absent
from the reference tree and from this image, together with torchvision and
OpenCV; they are restated here from their published definitions and from the
vendored spec copies in the reference:

  preprocess      LetterBox (identity for a 640x640 frame), BGR->RGB, HWC->CHW, /255
                  testing/old/segmenting_using_tflite/just_segmentation_using_tflite_model.py:36-115
  forward         Conv(+BN folded)+SiLU, C2f, SPPF, FPN/PAN, Segment head
  decode          DFL softmax expectation, dist2bbox (xywh) * stride, class sigmoid
  NMS             testing/old/segmenting_using_tflite/ops.py:214-363 (+ torchvision.ops.nms:
                  greedy, IoU > iou_thres suppresses; ties kept in index order here)
  process_mask    ops.py:707-737 (coef @ proto, crop to box/4, bilinear x4, > 0)
  mask -> grid    FrameProcessor.py:67-97 via Results.masks.xy (ops.py:837-859 'largest'):
                  oracle/contours.py restates cv2.findContours / contourArea / boundingRect /
                  fillPoly (PARITY WITH cv2 UNPINNED: OpenCV is not installed).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

REG_MAX = 16
STRIDES = (8, 16, 32)
MAX_WH = 7680


def letterbox_np(frame_bgr_u8: np.ndarray, Hn: int, Wn: int, top: int, left: int, newh: int, neww: int) -> np.ndarray:
    """Ultralytics LetterBox (data/augment.py, restated; Ultralytics and OpenCV are absent, so parity with
    cv2.resize is unpinned): cv2.INTER_LINEAR on uint8 in its fixed-point form -- per axis
    src = (d + 0.5) * (in / out) - 0.5 in float32, clamped at the borders, weights round((1 - f) * 2048) and
    2048 - that, (sum w_y w_x p + 2^21) >> 22 -- placed at (top, left) on a 114 border."""
    H, W, _ = frame_bgr_u8.shape
    out = np.full((Hn, Wn, 3), 114, dtype=np.uint8)
    if (newh, neww) == (H, W):
        out[top:top + H, left:left + W] = frame_bgr_u8
        return out

    def coef(n_out, n_in):
        inv = np.float32(n_in) / np.float32(n_out)
        f = (np.arange(n_out, dtype=np.float32) + np.float32(0.5)) * inv - np.float32(0.5)
        s = np.floor(f).astype(np.int64)
        f = (f - s.astype(np.float32)).astype(np.float32)
        lo = s < 0
        s[lo], f[lo] = 0, 0
        hi = s >= n_in - 1
        s[hi], f[hi] = n_in - 1, 0
        w0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
        return s, np.minimum(s + 1, n_in - 1), w0

    x0, x1, wx0 = coef(neww, W)
    y0, y1, wy0 = coef(newh, H)
    src = frame_bgr_u8.astype(np.int64)
    h0 = src[y0][:, x0] * wx0[None, :, None] + src[y0][:, x1] * (2048 - wx0)[None, :, None]
    h1 = src[y1][:, x0] * wx0[None, :, None] + src[y1][:, x1] * (2048 - wx0)[None, :, None]
    v = (h0 * wy0[:, None, None] + h1 * (2048 - wy0)[:, None, None] + (1 << 21)) >> 22
    out[top:top + newh, left:left + neww] = np.clip(v, 0, 255).astype(np.uint8)
    return out


def preprocess(frames_bgr_u8: torch.Tensor) -> torch.Tensor:
    """uint8 [B, H, W, 3] BGR -> float32 [B, 3, H, W] RGB in [0, 1]."""
    x = frames_bgr_u8[..., [2, 1, 0]].permute(0, 3, 1, 2).contiguous().float()
    return x / 255.0


def forward(arch, fw: dict, x: torch.Tensor):
    """Raw head outputs: (box [B,64,A], cls [B,nc,A], coef [B,32,A], proto [B,32,H/4,W/4]), fp32."""

    def conv(p, t, k, s=1, act=True):
        w, b = fw[p]
        y = F.conv2d(t, w, b, s, k // 2)
        return F.silu(y) if act else y

    def c2f(i, t, n, shortcut):
        y = conv(f"model.{i}.cv1", t, 1)
        ys = list(y.chunk(2, 1))
        for j in range(n):
            u = conv(f"model.{i}.m.{j}.cv1", ys[-1], 3)
            u = conv(f"model.{i}.m.{j}.cv2", u, 3)
            ys.append(ys[-1] + u if shortcut else u)
        return conv(f"model.{i}.cv2", torch.cat(ys, 1), 1)

    plan = {i: (n, sc) for i, _, _, n, sc in arch.c2f_plan()}
    x = conv("model.0", x, 3, 2)
    x = conv("model.1", x, 3, 2)
    x = c2f(2, x, *plan[2])
    x = conv("model.3", x, 3, 2)
    p3 = c2f(4, x, *plan[4])
    x = conv("model.5", p3, 3, 2)
    p4 = c2f(6, x, *plan[6])
    x = conv("model.7", p4, 3, 2)
    x = c2f(8, x, *plan[8])
    # SPPF
    y0 = conv("model.9.cv1", x, 1)
    y1 = F.max_pool2d(y0, 5, 1, 2)
    y2 = F.max_pool2d(y1, 5, 1, 2)
    y3 = F.max_pool2d(y2, 5, 1, 2)
    p5 = conv("model.9.cv2", torch.cat([y0, y1, y2, y3], 1), 1)
    # head
    x = torch.cat([F.interpolate(p5, scale_factor=2, mode="nearest"), p4], 1)
    h12 = c2f(12, x, *plan[12])
    x = torch.cat([F.interpolate(h12, scale_factor=2, mode="nearest"), p3], 1)
    o3 = c2f(15, x, *plan[15])
    x = torch.cat([conv("model.16", o3, 3, 2), h12], 1)
    o4 = c2f(18, x, *plan[18])
    x = torch.cat([conv("model.19", o4, 3, 2), p5], 1)
    o5 = c2f(21, x, *plan[21])
    outs = {"cv2": [], "cv3": [], "cv4": []}
    for l, t in enumerate((o3, o4, o5)):
        for br in outs:
            u = conv(f"model.22.{br}.{l}.0", t, 3)
            u = conv(f"model.22.{br}.{l}.1", u, 3)
            u = conv(f"model.22.{br}.{l}.2", u, 1, act=False)
            outs[br].append(u.flatten(2))
    box = torch.cat(outs["cv2"], 2)
    cls = torch.cat(outs["cv3"], 2)
    coef = torch.cat(outs["cv4"], 2)
    # proto
    u = conv("model.22.proto.cv1", o3, 3)
    w, b = fw["model.22.proto.upsample"]
    u = F.conv_transpose2d(u, w, b, stride=2)
    u = conv("model.22.proto.cv2", u, 3)
    proto = conv("model.22.proto.cv3", u, 1)
    return box, cls, coef, proto


def anchors(H: int, W: int):
    pts, st = [], []
    for s in STRIDES:
        h, w = H // s, W // s
        sy, sx = torch.meshgrid(torch.arange(h, dtype=torch.float32) + 0.5,
                                torch.arange(w, dtype=torch.float32) + 0.5, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), float(s)))
    return torch.cat(pts).T, torch.cat(st).T  # [2, A], [1, A]


def decode(box: torch.Tensor, cls: torch.Tensor, H: int, W: int):
    """Detect inference tail: DFL -> dist2bbox(xywh) * stride; class sigmoid.  -> [B, 4+nc, A]."""
    B, _, A = box.shape
    prob = box.view(B, 4, REG_MAX, A).softmax(2)
    dist = (prob * torch.arange(REG_MAX, dtype=torch.float32).view(1, 1, REG_MAX, 1)).sum(2)
    ap, st = anchors(H, W)
    lt, rb = dist[:, :2], dist[:, 2:]
    x1y1 = ap.unsqueeze(0) - lt
    x2y2 = ap.unsqueeze(0) + rb
    dbox = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * st
    return torch.cat((dbox, cls.sigmoid()), 1)


def nms_candidates(pred: torch.Tensor, coef: torch.Tensor, conf: float = 0.5, max_nms: int = 30000):
    """non_max_suppression for one image up to its torchvision.ops.nms call (ops.py:288-343): pred [4+nc, A],
    coef [32, A] -> det [n, 6 + 32] rows (x1, y1, x2, y2, conf, cls, coef...) -- the conf filter (xc, :288 and
    :322), xywh2xyxy (:463-480), best class only (:319-321), the max_nms cut (:332-333: the max_nms highest
    scores; torch's argsort is not stable, ties are kept lowest anchor first here, the order the device kernel
    uses) -- and the nms inputs: boxes offset by class * max_wh (:336-342) and the scores.  Pinned to the
    reference's own ops.py by tests/golden/ops_goldens.npz (tests/test_ops_pinned_cpu.py)."""
    nc = pred.shape[0] - 4
    x = torch.cat((pred, coef), 0).T  # [A, 4+nc+32]
    xc = x[:, 4:4 + nc].amax(1) > conf
    x = x[xc]
    if not x.shape[0]:
        z = torch.zeros((0, 6 + coef.shape[0]))
        return z, z[:, :4], z[:, 4]
    xy, wh = x[:, :2], x[:, 2:4] / 2
    boxes = torch.cat((xy - wh, xy + wh), 1)
    score, j = x[:, 4:4 + nc].max(1, keepdim=True)
    det = torch.cat((boxes, score, j.float(), x[:, 4 + nc:]), 1)[score.view(-1) > conf]
    if det.shape[0] > max_nms:
        det = det[torch.sort(det[:, 4], descending=True, stable=True).indices[:max_nms]]
    return det, det[:, :4] + det[:, 5:6] * MAX_WH, det[:, 4]


def nms_image(pred: torch.Tensor, coef: torch.Tensor, conf: float = 0.5, iou: float = 0.7, max_det: int = 300,
              max_nms: int = 30000):
    """non_max_suppression for one image (ops.py:214-363): pred [4+nc, A], coef [32, A]
    -> [k, 6 + 32] rows (x1, y1, x2, y2, conf, cls, coef...) in decreasing score order: nms_candidates, then
    the greedy NMS torchvision.ops.nms runs (greedy_nms; torchvision is absent: unpinned) and the max_det cut."""
    det, boxes, scores = nms_candidates(pred, coef, conf, max_nms)
    if not det.shape[0]:
        return det
    keep = greedy_nms(boxes, scores, iou)[:max_det]
    return det[keep]


def scale_boxes(net_hw: tuple[int, int], boxes: torch.Tensor, frame_hw: tuple[int, int]) -> torch.Tensor:
    """ops.scale_boxes(img1_shape=net, boxes xyxy, img0_shape=frame) (ops.py:139-170, then clip_boxes): gain in
    double, integer pads round(. - 0.1), float32 tensor arithmetic, clamp to the frame."""
    gain = min(net_hw[0] / frame_hw[0], net_hw[1] / frame_hw[1])
    px = round((net_hw[1] - frame_hw[1] * gain) / 2 - 0.1)
    py = round((net_hw[0] - frame_hw[0] * gain) / 2 - 0.1)
    b = boxes.clone()
    b[..., 0] -= px
    b[..., 1] -= py
    b[..., 2] -= px
    b[..., 3] -= py
    b[..., :4] /= gain
    b[..., 0] = b[..., 0].clamp(0, frame_hw[1])
    b[..., 1] = b[..., 1].clamp(0, frame_hw[0])
    b[..., 2] = b[..., 2].clamp(0, frame_hw[1])
    b[..., 3] = b[..., 3].clamp(0, frame_hw[0])
    return b


def greedy_nms(boxes: torch.Tensor, scores: torch.Tensor, thr: float) -> torch.Tensor:
    """torchvision.ops.nms semantics (float32 IoU, suppress IoU > thr); stable order for ties."""
    order = torch.sort(scores, descending=True, stable=True).indices
    b = boxes[order]
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    n = b.shape[0]
    sup = torch.zeros(n, dtype=torch.bool)
    keep = []
    for i in range(n):
        if sup[i]:
            continue
        keep.append(int(order[i]))
        xx1 = torch.maximum(b[i, 0], b[i + 1:, 0])
        yy1 = torch.maximum(b[i, 1], b[i + 1:, 1])
        xx2 = torch.minimum(b[i, 2], b[i + 1:, 2])
        yy2 = torch.minimum(b[i, 3], b[i + 1:, 3])
        inter = (xx2 - xx1).clamp(min=0) * (yy2 - yy1).clamp(min=0)
        ovr = inter / (area[i] + area[i + 1:] - inter)
        sup[i + 1:] |= ovr.double() > thr
    return torch.tensor(keep, dtype=torch.long)


def process_mask(proto: torch.Tensor, coef: torch.Tensor, boxes: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """ops.process_mask(upsample=True) (ops.py:707-737): [n,32] @ [32, h*w] -> crop -> bilinear -> > 0."""
    c, mh, mw = proto.shape
    masks = (coef @ proto.float().view(c, -1)).view(-1, mh, mw)
    db = boxes.clone()
    db[:, 0] *= mw / W
    db[:, 2] *= mw / W
    db[:, 3] *= mh / H
    db[:, 1] *= mh / H
    x1, y1, x2, y2 = torch.chunk(db[:, :, None], 4, 1)
    r = torch.arange(mw, dtype=x1.dtype)[None, None, :]
    cc = torch.arange(mh, dtype=x1.dtype)[None, :, None]
    masks = masks * ((r >= x1) * (r < x2) * (cc >= y1) * (cc < y2))
    masks = F.interpolate(masks[None], (H, W), mode="bilinear", align_corners=False)[0]
    return masks.gt_(0.0)


def select_mask(masks: torch.Tensor, frame_hw: tuple[int, int] | None = None):
    """FrameProcessor.py:67-97 on the instance masks of one frame (network resolution): the instance of max
    contourArea of its Results.masks.xy polygon, np.int32, boundingRect, fillPoly -- oracle/contours.py.
    -> (uint8 [H0, W0] image whose cell centres hold the filled polygon's samples, or None when there is no
    detection; rect (x, y, w, h)); frame_hw = the frame the network input was letterboxed from (default: the same)."""
    import numpy as np
    from oracle import contours as C
    H, W = masks.shape[1:] if masks.dim() == 3 else (0, 0)
    frame_hw = frame_hw or (H, W)
    if masks.shape[0] == 0:
        return None, (0, 0, 0, 0)
    k, pts, rect, cells = C.select_cells(masks.numpy().astype(np.uint8), frame_hw)
    img = np.kron(cells, np.ones((20, 20), dtype=np.uint8))
    return torch.from_numpy(img), rect


def select_cells(masks: torch.Tensor, frame_hw: tuple[int, int] | None = None):
    """-> (chosen index or -1, int32 polygon, rect, cells [H0/20, W0/20]) (oracle/contours.select_cells)."""
    import numpy as np
    from oracle import contours as C
    frame_hw = frame_hw or tuple(masks.shape[1:])
    if masks.shape[0] == 0:
        return -1, np.zeros((0, 2), np.int32), (0, 0, 0, 0), np.zeros((frame_hw[0] // 20, frame_hw[1] // 20), np.uint8)
    return C.select_cells(masks.numpy().astype(np.uint8), frame_hw)


def predict(arch, fw, frames_bgr_u8: torch.Tensor, conf=0.5, iou=0.7, max_det=300, max_nms=30000):
    """Full segmentation stage for a batch: -> list of (det [k, 38], masks [k, H, W] bool)."""
    B, H, W, _ = frames_bgr_u8.shape
    x = preprocess(frames_bgr_u8)
    box, cls, coef, proto = forward(arch, fw, x)
    pred = decode(box, cls, H, W)
    out = []
    for b in range(B):
        det = nms_image(pred[b], coef[b], conf, iou, max_det, max_nms)
        if det.shape[0]:
            masks = process_mask(proto[b], det[:, 6:], det[:, :4], H, W)
        else:
            masks = torch.zeros((0, H, W))
        out.append((det, masks))
    return out

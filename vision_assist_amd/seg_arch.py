"""YOLOv8-seg architecture (n / s / m) and seeded synthetic weights.

The reference calls Ultralytics' ``YOLO(weights).predict`` (main.py:43,
FrameProcessor.py:322); Ultralytics and every weight file are absent here
(SURVEY.md §8c), so the architecture is restated from the yolov8-seg model
definition (verified by exact parameter counts: n 3.40 M,
s 11.81 M, m 27.27 M) and weights are synthetic and seeded:
He-normal conv weights, BN gamma ~ U[.5, 1.5], beta, mean ~ N(0, .1),
var ~ U[.5, 1.5], eps 1e-3, one ``torch.Generator(seed + layer_index)`` per
parameterised module.  Parameter names follow the Ultralytics state-dict
(``model.<i>.cv1.conv.weight``, ``model.22.cv3.<l>.2.bias`` ...) so a real
checkpoint exported to safetensors loads through ``fold()`` unchanged.

``fold()`` folds every Conv+BN into (weight, bias) exactly like
``fuse_conv_and_bn`` (the ``fuse`` frame of the reference's profile.svg).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

SCALES = {  # depth, width, max_channels
    "n": (0.33, 0.25, 1024),
    "s": (0.33, 0.50, 1024),
    "m": (0.67, 0.75, 768),
}
BN_EPS = 1e-3
REG_MAX = 16
NM = 32  # mask coefficients
STRIDES = (8, 16, 32)
# the 'sparse' regime (synthetic_state_dict(sparse=640 | 1280)): per (scale, network side, seed) and head level, the
# class-0 logit (bias 0, solid masks) that one anchor per frame exceeds on average over seeded uniform-noise
# frames (tools/sparse_calib.py, on the oracle forward); class 0's weights are scaled by SPARSE_GAIN and its
# bias set to -SPARSE_GAIN * threshold, every other class is off, so a frame keeps ~1-5 detections
SPARSE_GAIN = 10.0
SPARSE_THRESHOLDS = {
    ("s", 640, 0): (0.234166, 0.323434, 0.273133),
    ("n", 640, 0): (0.553922, 56.835182, 18.296261),
    ("m", 1280, 0): (287.544861, 125.099106, 66.233734),
}


def _make_div(x: float, d: int = 8) -> int:
    return int(math.ceil(x / d) * d)


@dataclass
class Arch:
    scale: str = "s"
    nc: int = 80

    def __post_init__(self):
        self.depth, self.width, self.max_ch = SCALES[self.scale]

    def ch(self, c: int) -> int:
        return _make_div(min(c, self.max_ch) * self.width, 8)

    def rep(self, n: int) -> int:
        return max(round(n * self.depth), 1) if n > 1 else n

    # channel plan
    @property
    def c1(self):  # layer 0
        return self.ch(64)

    @property
    def c2(self):  # P2
        return self.ch(128)

    @property
    def c3(self):  # P3
        return self.ch(256)

    @property
    def c4(self):  # P4
        return self.ch(512)

    @property
    def c5(self):  # P5
        return self.ch(1024)

    @property
    def npr(self):  # proto channels
        return self.ch(256)

    @property
    def head_c2(self):  # box branch
        return max(16, self.c3 // 4, REG_MAX * 4)

    @property
    def head_c3(self):  # cls branch
        return max(self.c3, min(self.nc, 100))

    @property
    def head_c4(self):  # mask-coefficient branch
        return max(self.c3 // 4, NM)

    @property
    def no(self):
        return 4 * REG_MAX + self.nc

    def c2f_plan(self):
        """(layer index, c_in, c_out, n, shortcut) for the 8 C2f blocks."""
        return [
            (2, self.c2, self.c2, self.rep(3), True),
            (4, self.c3, self.c3, self.rep(6), True),
            (6, self.c4, self.c4, self.rep(6), True),
            (8, self.c5, self.c5, self.rep(3), True),
            (12, self.c5 + self.c4, self.c4, self.rep(3), False),
            (15, self.c4 + self.c3, self.c3, self.rep(3), False),
            (18, self.c3 + self.c4, self.c4, self.rep(3), False),
            (21, self.c4 + self.c5, self.c5, self.rep(3), False),
        ]

    STRIDE2 = ("model.0", "model.1", "model.3", "model.5", "model.7", "model.16", "model.19")

    def stride_of(self, prefix: str) -> int:
        """The stride of a conv_specs module: the backbone's downsampling Convs and the neck's two (yolov8-seg.yaml)."""
        return 2 if prefix in self.STRIDE2 else 1

    def conv_specs(self):
        """Every parameterised module in state-dict order:
        (prefix, kind, c_in, c_out, k) with kind in {'conv' (Conv+BN+SiLU), 'conv2d' (plain, bias), 'deconv'}."""
        s = []
        s.append(("model.0", "conv", 3, self.c1, 3))
        s.append(("model.1", "conv", self.c1, self.c2, 3))
        c2f = {i: (ci, co, n, sc) for i, ci, co, n, sc in self.c2f_plan()}

        def add_c2f(i):
            ci, co, n, _ = c2f[i]
            c = co // 2
            s.append((f"model.{i}.cv1", "conv", ci, 2 * c, 1))
            s.append((f"model.{i}.cv2", "conv", (2 + n) * c, co, 1))
            for j in range(n):
                s.append((f"model.{i}.m.{j}.cv1", "conv", c, c, 3))
                s.append((f"model.{i}.m.{j}.cv2", "conv", c, c, 3))

        add_c2f(2)
        s.append(("model.3", "conv", self.c2, self.c3, 3))
        add_c2f(4)
        s.append(("model.5", "conv", self.c3, self.c4, 3))
        add_c2f(6)
        s.append(("model.7", "conv", self.c4, self.c5, 3))
        add_c2f(8)
        s.append(("model.9.cv1", "conv", self.c5, self.c5 // 2, 1))
        s.append(("model.9.cv2", "conv", 4 * (self.c5 // 2), self.c5, 1))
        add_c2f(12)
        add_c2f(15)
        s.append(("model.16", "conv", self.c3, self.c3, 3))
        add_c2f(18)
        s.append(("model.19", "conv", self.c4, self.c4, 3))
        add_c2f(21)
        chs = (self.c3, self.c4, self.c5)
        for br, cm, cout in (("cv2", self.head_c2, 4 * REG_MAX), ("cv3", self.head_c3, self.nc), ("cv4", self.head_c4, NM)):
            for l, cx in enumerate(chs):
                s.append((f"model.22.{br}.{l}.0", "conv", cx, cm, 3))
                s.append((f"model.22.{br}.{l}.1", "conv", cm, cm, 3))
                s.append((f"model.22.{br}.{l}.2", "conv2d", cm, cout, 1))
        s.append(("model.22.proto.cv1", "conv", self.c3, self.npr, 3))
        s.append(("model.22.proto.upsample", "deconv", self.npr, self.npr, 2))
        s.append(("model.22.proto.cv2", "conv", self.npr, self.npr, 3))
        s.append(("model.22.proto.cv3", "conv", self.npr, NM, 1))
        return s

    def n_params(self) -> int:
        n = 0
        for _, kind, ci, co, k in self.conv_specs():
            n += ci * co * k * k
            n += 4 * co if kind == "conv" else co  # BN (w, b, mean, var) are 2 learnable + 2 buffers; count learnable
        return n


def learnable_params(arch: Arch) -> int:
    """Ultralytics' reported parameter count (learnable: conv weights, BN gamma/beta, biases)."""
    n = 0
    for _, kind, ci, co, k in arch.conv_specs():
        n += ci * co * k * k
        n += 2 * co if kind == "conv" else co
    return n


def synthetic_state_dict(arch: Arch, seed: int = 0, cls_bias: float | None = None, solid_masks: bool = False,
                         sparse: int | None = None) -> dict:
    """Seeded synthetic weights in Ultralytics state-dict layout (fp32, CPU).

    cls_bias: None -> Ultralytics' prior (Detect.bias_init: log(5 / nc / (640 / stride)^2));
    a number -> every class bias set to it (the 'dense' regime uses +4).
    solid_masks: the prototypes made constant (proto.cv3's BN scale 0: channel 0 = SiLU(3), the others SiLU(0) = 0)
    and mask coefficient 0 fixed at +5, so every instance mask is its whole box -- one compact blob per detection,
    as a trained model's masks are, instead of the random weights' noise (the 'dense_box' regime).
    sparse: the network side (640 / 1280) of a 'sparse' regime -- solid masks, one live class whose per-level
    bias leaves ~1-5 detections per noise frame (SPARSE_THRESHOLDS), the rest off: a trained model's
    few-object frames."""
    sd = {}
    for idx, (prefix, kind, ci, co, k) in enumerate(arch.conv_specs()):
        g = torch.Generator().manual_seed(seed * 100003 + idx)
        if kind == "deconv":
            fan_in = ci * k * k
            sd[f"{prefix}.weight"] = torch.randn(ci, co, k, k, generator=g) * math.sqrt(2.0 / fan_in)
            sd[f"{prefix}.bias"] = torch.randn(co, generator=g) * 0.1
            continue
        fan_in = ci * k * k
        w = torch.randn(co, ci, k, k, generator=g) * math.sqrt(2.0 / fan_in)
        if kind == "conv":
            sd[f"{prefix}.conv.weight"] = w
            sd[f"{prefix}.bn.weight"] = torch.rand(co, generator=g) + 0.5
            sd[f"{prefix}.bn.bias"] = torch.randn(co, generator=g) * 0.1
            sd[f"{prefix}.bn.running_mean"] = torch.randn(co, generator=g) * 0.1
            sd[f"{prefix}.bn.running_var"] = torch.rand(co, generator=g) + 0.5
        else:
            sd[f"{prefix}.weight"] = w
            parts = prefix.split(".")
            br, lvl = parts[2], int(parts[3])
            if br == "cv2":
                b = torch.full((co,), 1.0)
            elif br == "cv3":
                prior = math.log(5 / arch.nc / (640 / STRIDES[lvl]) ** 2)
                b = torch.full((co,), prior if cls_bias is None else float(cls_bias))
            else:
                b = torch.randn(co, generator=g) * 0.1
            sd[f"{prefix}.bias"] = b
    if sparse is not None:
        key = (arch.scale, int(sparse), seed)
        if key not in SPARSE_THRESHOLDS:
            raise KeyError(f"no sparse calibration for {key}: run tools/sparse_calib.py")
        for lvl, t in enumerate(SPARSE_THRESHOLDS[key]):
            q = f"model.22.cv3.{lvl}.2"
            sd[f"{q}.weight"][0].mul_(SPARSE_GAIN)
            sd[f"{q}.weight"][1:].zero_()
            sd[f"{q}.bias"][0] = -SPARSE_GAIN * t
            sd[f"{q}.bias"][1:] = -50.0
        solid_masks = True
    if solid_masks:
        p = "model.22.proto.cv3"
        sd[f"{p}.bn.weight"] = torch.zeros_like(sd[f"{p}.bn.weight"])
        beta = torch.zeros_like(sd[f"{p}.bn.bias"])
        beta[0] = 3.0
        sd[f"{p}.bn.bias"] = beta
        for lvl in range(3):
            q = f"model.22.cv4.{lvl}.2"
            sd[f"{q}.weight"][0].zero_()
            sd[f"{q}.bias"][0] = 5.0
    return sd


def fold(arch: Arch, sd: dict) -> dict:
    """prefix -> (weight fp32, bias fp32) with BN folded (fuse_conv_and_bn)."""
    out = {}
    for prefix, kind, ci, co, k in arch.conv_specs():
        if kind == "conv":
            w = sd[f"{prefix}.conv.weight"].float()
            gamma = sd[f"{prefix}.bn.weight"].float()
            beta = sd[f"{prefix}.bn.bias"].float()
            mean = sd[f"{prefix}.bn.running_mean"].float()
            var = sd[f"{prefix}.bn.running_var"].float()
            scale = gamma.div(torch.sqrt(var + BN_EPS))
            wf = torch.mm(torch.diag(scale), w.view(co, -1)).view_as(w)
            bf = beta - gamma.mul(mean).div(torch.sqrt(var + BN_EPS))
            out[prefix] = (wf.contiguous(), bf.contiguous())
        else:
            out[prefix] = (sd[f"{prefix}.weight"].float().contiguous(), sd[f"{prefix}.bias"].float().contiguous())
    return out

"""YOLOv8-seg on MI355X: weight packing, buffer planning and the forward op list.

``SegNet(arch, folded, dtype)`` packs the folded Conv weights once (K ordered
(ky, kx, ci), zero padded to the MFMA tile), and ``plan(B, H, W)`` lays out
every activation of a forward as NHWC channel slices of a few buffers so that
C2f chunk/cat, SPPF cat and the FPN/PAN concats are free, then emits the list
of ops (``va_seg_op``) that ``va_seg_run`` executes in ONE C call.

Output of a forward (``SegOutputs``): per pyramid level a float32 NHWC buffer
[B, h, w, 64 + nc + 32] = (DFL box logits, class logits, mask coefficients) --
the tensors Ultralytics' Segment head concatenates before decoding -- and the
proto masks float32 [B, H/4, W/4, 32].
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import torch

from . import _lib
from .seg_arch import NM, REG_MAX, Arch

VA_DTYPE_BF16, VA_DTYPE_F32, VA_DTYPE_FP8 = 1, 2, 3
F8_KS = 128        # K-step of the fp8 kernel (va_fp8.hip): fp8 weights are padded to it
F8_MAX = 448.0     # largest OCP e4m3 value
FP8_HEADROOM = 8.0  # calibration amax x this x the buffer scale lands in [224, 448] (SegNet.calibrate_fp8)
VA_OP_CONV, VA_OP_SPPF, VA_OP_UPSAMPLE, VA_OP_PREPROCESS, VA_OP_CONV0, VA_OP_C2F, VA_OP_STEM = 1, 2, 3, 4, 5, 6, 7
VA_OP_FORK, VA_OP_JOIN = 8, 9  # lanes of a branch-parallel list (va355.h)
C2FB_MAX_B = 1      # va_seg_c2fb for batches up to this (SegNet.c2fb_max_b)
C2FB_MIN_TILES = 96  # SegNet._c2fb_tile: the fewest workgroups a tile side may leave (f32)
C2FB_CUS = 256       # SegNet._c2fb_tile_bf16: workgroups per round (one per CU)
C2FB_FIXED = 16_000_000  # SegNet._c2fb_tile_bf16: a tile's fixed latency, in MACs
SPLITK_WS_BYTES, SPLITK_NCNT = 32 << 20, 128  # per-plan split-K slabs / arrival counters (va_conv_args.ws)
BK = 64  # K padding: the bf16 kernels step K by 64, the f32 ones by 32 (SegNet.bk)
NPAD = 128


# The planner's A/B switches, read from the environment when a SegNet is built or a plan is made --
# every default is the measured-best form; "0" turns a fusion off for a same-box comparison (tools/plan_ab.py).  The
# library's own switches (VA_F32_SPLIT, VA_CONV3H, ...) are read in csrc/va_handle.hip.
PLANNER_SWITCHES = {
    "VA_CONV0": "1",        # 0: model.0 as preprocess + a conv (no fused first layer)
    "VA_CONV0_F32M": "1",   # 0: f32 model.0 on the VALU kernel instead of the MFMA one
    "VA_STEM": "1",         # 0: model.0 and model.1 as two launches (bf16 and f32 stems)
    "VA_STEM_TAIL": "1",    # 0: model.2.cv1 a launch of its own instead of the f32 stem's epilogue
    "VA_C2F": "1",          # 0: the bf16 model.2 C2f's four convs apart
    "VA_C2FB": "1",         # 0: the batch-1 C2f blocks' layers apart
    "VA_FOLD_PROTO": "1",   # 0: proto's upsample + cv2 unfolded
    "VA_FUSE_UP": "1",      # 0: the FPN upsample materialised instead of read in place
    "VA_FUSE_TAIL": "1",    # 0: no fused 1x1 tails
    "VA_LANES": "1",        # 0: no branch-parallel lanes at small batches
    "VA_LANES_MAX_B": "8",  # the largest batch planned with lanes
    "VA_W8": "1",           # 0: w8a16 plans on the host-dequantized bf16 weights (round 5's form) instead of e4m3 bytes
    "VA_CONV3H": "1",       # (the library's switch, read here too: a fused f32 tail needs conv3h)
    "VA_CONV3Q": "1",       # (likewise: the f32 32-channel tail needs conv3q)
}


def switch(name: str) -> str:
    """The planner switch ``name`` (PLANNER_SWITCHES: its documented default unless the environment sets it)."""
    return os.environ.get(name, PLANNER_SWITCHES[name])


def switch_on(name: str) -> bool:
    return switch(name) != "0"


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("N", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32), ("Cin", ctypes.c_int32),
        ("ldx", ctypes.c_int32),
        ("kh", ctypes.c_int32), ("kw", ctypes.c_int32), ("stride", ctypes.c_int32), ("pad", ctypes.c_int32),
        ("Ho", ctypes.c_int32), ("Wo", ctypes.c_int32),
        ("w", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("Cout", ctypes.c_int32), ("Npad", ctypes.c_int32), ("K", ctypes.c_int32), ("Kpad", ctypes.c_int32),
        ("y", ctypes.c_void_p), ("ldy", ctypes.c_int32),
        ("res", ctypes.c_void_p), ("ldr", ctypes.c_int32),
        ("act", ctypes.c_int32), ("mode", ctypes.c_int32), ("M", ctypes.c_int32), ("dtype", ctypes.c_int32),
        ("out_f32", ctypes.c_int32), ("bias4", ctypes.c_int32),
        ("w2", ctypes.c_void_p), ("b2", ctypes.c_void_p), ("c2", ctypes.c_int32), ("act2", ctypes.c_int32),
        ("xu", ctypes.c_void_p), ("ldu", ctypes.c_int32), ("cu", ctypes.c_int32),
        ("wscale", ctypes.c_void_p), ("xscale", ctypes.c_float), ("x8", ctypes.c_int32),
        ("yscale", ctypes.c_float), ("rscale", ctypes.c_float),
        ("w3", ctypes.c_void_p),
        ("ws", ctypes.c_void_p),
        ("ws_bytes", ctypes.c_int64),
        ("wcnt", ctypes.c_void_p),
        ("ncnt", ctypes.c_int32),
        ("w8", ctypes.c_int32),
    ]


class SegOp(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("lane", ctypes.c_int32), ("a", ConvArgs)]


def _ceil(a, b):
    return (a + b - 1) // b * b


def _cdiv(a, b):
    return (a + b - 1) // b


@dataclass
class Packed:
    w: torch.Tensor
    b: torch.Tensor
    cin: int       # padded input channels the packed K assumes
    cout: int
    k: int
    K: int
    Kpad: int
    Npad: int
    deconv: bool = False
    w3: torch.Tensor | None = None  # f32 mode: the weights as three exact bf16 terms (split3_bf16, va_conv_args.w3)


def quantize_weights_e4m3(folded: dict) -> dict:
    """The folded weights with every conv but model.0 rounded to e4m3 values times one f32 scale per output channel
    (the channel's largest |w| maps to 448, round to nearest even: _pack_fp8's quantization), returned in float32."""
    out = {}
    for k, v in folded.items():
        w, b = v
        if k == "model.0" or w.dim() != 4:
            out[k] = v
            continue
        wf = w.float()
        amax = wf.abs().flatten(1).amax(1) if not k.endswith("upsample") else wf.abs().transpose(0, 1).flatten(1).amax(1)
        sw = torch.where(amax > 0, amax / F8_MAX, torch.ones_like(amax))
        shape = (-1, 1, 1, 1) if not k.endswith("upsample") else (1, -1, 1, 1)
        q = (wf / sw.view(shape)).clamp(-F8_MAX, F8_MAX).to(torch.float8_e4m3fn).float()
        out[k] = (q * sw.view(shape), b)
    return out


W8_CHUNKS = (0, 4, 1, 5, 2, 6, 3, 7)  # the stored order of the eight 8-element chunks of a 64-element K block


def w8_order(q: torch.Tensor, inverse: bool = False) -> torch.Tensor:
    """e4m3 weight rows [..., Kpad] (Kpad % 64 == 0) in the bf16 kernels' K order (va355.h va_conv_args.w8): per 64-
    element block the chunks 0, 4, 1, 5, 2, 6, 3, 7, so a lane's two MFMA K halves are one 16-byte piece; inverse: back
    to natural order."""
    g = q.reshape(*q.shape[:-1], q.shape[-1] // 64, 8, 8)
    idx = torch.tensor(W8_CHUNKS, device=q.device)
    if inverse:
        idx = torch.argsort(idx)
    return g.index_select(-2, idx).reshape(q.shape).contiguous()


def split3_bf16(w: torch.Tensor) -> torch.Tensor:
    """f32 [..., K] (K % 8 == 0) -> bf16 [..., K / 8, 3, 8]: per 8-element group the round-to-nearest bf16 h of each
    value, then m = bf16(x - h), then l = bf16(x - h - m) -- x == h + m + l exactly (both subtractions are exact in
    f32, l has at most 8 significant bits; tests/test_split_cpu.py), the planes conv3t_kernel / conv3h_kernel stage (w3_rows orders their K)."""
    w = w.float()
    h = w.to(torch.bfloat16)
    r = w - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    g = w.shape[:-1] + (w.shape[-1] // 8, 8)
    return torch.stack([h.reshape(g), m.reshape(g), lo.reshape(g)], -2).contiguous()


def w3_group(stride: int, taps: int, cin: int) -> int:
    """Input channels per K group of a layer's w3 planes (w3_rows): 32 for the stride-2 multi-tap convs with Cin % 32
    == 0 (conv3t then reads both 64-byte halves of an input pixel's 128-byte line in consecutive K-steps), else 16.
    va_seg.hip conv3t_kernel applies the same rule to the layer's va_conv_args."""
    return 32 if stride == 2 and taps > 1 and cin % 32 == 0 else 16


def w3_rows(w: torch.Tensor, taps: int, cin: int, g: int = 16) -> torch.Tensor:
    """The pre-split planes' K order (va_conv_args.w3): f32 rows [..., K = taps x cin] (K = tap cin + c, the im2col
    order) re-ordered group-major -- g-channel group, then tap, then channel (K' = (c // g) taps g + g tap + c % g; g =
    w3_group: 16, or 32 on the stride-2 3x3s) -- and split (split3_bf16): a K-step's 96-byte run is 16 channels of one
    (group, tap), so conv3t walks all taps of a group in a row (the group's input footprint stays in L2 across its taps;
    tap-major, a stride-2 layer re-read its input from HBM) and conv3h's per-chunk tap loop reads consecutive runs."""
    lead = w.shape[:-1]
    w = w.float().reshape(*lead, taps, cin // g, g).transpose(-3, -2).reshape(*lead, taps * cin)
    return split3_bf16(w)


class Slice:
    """A channel slice of an NHWC buffer: (buffer, channel offset, channels)."""

    def __init__(self, buf: torch.Tensor, off: int, c: int):
        self.buf, self.off, self.c = buf, off, c

    @property
    def ld(self):
        return self.buf.shape[-1]

    @property
    def ptr(self):
        return self.buf.data_ptr() + self.off * self.buf.element_size()

    def sub(self, off, c):
        return Slice(self.buf, self.off + off, c)

    @property
    def e4m3(self) -> bool:
        """An fp8-mode activation buffer: e4m3 bytes (with one power-of-two scale per buffer)."""
        return self.buf.dtype == torch.uint8


@dataclass
class SegOutputs:
    levels: list   # 3 x float32 [B, h, w, 64 + nc + 32]
    proto: torch.Tensor  # float32 [B, H/4, W/4, 32]
    strides: tuple = (8, 16, 32)


class SegNet:
    def __init__(self, arch: Arch, folded: dict, dtype: str = "bf16", device=None, c2fb_f32: bool = True):
        """c2fb_f32: the batch-1 C2f blocks of f32 plans on va_seg_c2fb's f32 form where its layout keeps the
        intermediates as term planes (_c2fb_tile); False keeps them apart (A/B)."""
        _lib.require_gpu()
        self.lib = _lib.load()
        self.arch = arch
        if dtype not in ("bf16", "f32", "fp8", "w8a16"):
            raise ValueError(f"dtype {dtype!r}: bf16, f32, fp8 or w8a16")
        # w8a16 (C5's weight-only form): every conv's weights as e4m3 BYTES with one f32 scale per output channel (per
        # GEMM row: _pack_e4m3), bf16 activations; the bf16 kernels convert the bytes exactly to bf16 in their A stage
        # and scale the f32 accumulator (va355.h va_conv_args.w8) -- HBM holds 1 byte per weight.  model.0 stays bf16
        # (as in the fp8 mode), and so do the weights of the kernels with no A stage to convert in: the fused 1x1
        # tails' w2 and the s / n-only fused blocks (stem, C2f, c2fb) -- those take the e4m3 values dequantized on the
        # host, rounded to bf16 (quantize_weights_e4m3)
        self.form = dtype
        folded_f = folded
        if dtype == "w8a16":
            folded = quantize_weights_e4m3(folded)
            dtype = "bf16"
        self.dtype = dtype
        self.tdtype = torch.bfloat16 if self.store == "bf16" else torch.float32
        self.va_dtype = VA_DTYPE_BF16 if self.store == "bf16" else VA_DTYPE_F32
        self.vec = 8 if self.store == "bf16" else 4
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.w = {}
        self.w8w = {}  # w8a16: prefix -> (e4m3 bytes [Npad][Kpad], per-row scale float [Npad])
        for prefix, kind, ci, co, k in arch.conv_specs():
            w, b = folded[prefix]
            self.w[prefix] = self._pack(w, b, deconv=(kind == "deconv"), stride=arch.stride_of(prefix))
            if self.form == "w8a16":
                self.w8w[prefix] = self._pack_e4m3(self._rows(folded_f[prefix][0], deconv=(kind == "deconv")))
        # the three head branches' first 3x3 convs share their input: one GEMM per level
        for l in range(3):
            for src, fw_ in ((folded, False), (folded_f, True)):
                if fw_ and self.form != "w8a16":
                    continue
                parts = [src[f"model.22.{br}.{l}.0"] for br in ("cv2", "cv3", "cv4")]
                w = torch.cat([p[0] for p in parts], 0)
                b = torch.cat([p[1] for p in parts], 0)
                if fw_:
                    self.w8w[f"head.{l}.0"] = self._pack_e4m3(self._rows(w))
                else:
                    self.w[f"head.{l}.0"] = self._pack(w, b)
        # model.0 for the fused bf16 first layer: [Cout][32], k = (ky*3 + kx)*3 + c (RGB), zero padded
        w0, b0 = folded["model.0"]
        w0p = torch.zeros(w0.shape[0], 32, dtype=torch.float32)
        w0p[:, :27] = w0.permute(0, 2, 3, 1).reshape(w0.shape[0], 27)
        self.w0 = (w0p.to(self.device, self.tdtype).contiguous(), b0.float().to(self.device).contiguous())
        self.fuse_first = w0.shape[0] % 16 == 0 and w0.shape[0] <= 64 and switch_on("VA_CONV0")
        self.w0_3 = None
        # small batches: head levels + proto on lanes beside the neck (plan() laned; VA_LANES=0 off, A/B)
        self.lanes = switch_on("VA_LANES")
        self.lanes_max_b = int(switch("VA_LANES_MAX_B"))
        if dtype == "f32":  # va_seg_conv0_f32: [Cout][27], k = (ky*3 + kx)*3 + c (RGB)
            self.w0 = (w0.permute(0, 2, 3, 1).reshape(w0.shape[0], 27).float().to(self.device).contiguous(),
                       b0.float().to(self.device).contiguous())
            # va_seg_conv0_f32m: the K-padded rows as three exact bf16 terms (VA_CONV0_F32M=0: the VALU form, A/B)
            if switch_on("VA_CONV0_F32M"):
                self.w0_3 = split3_bf16(w0p).to(self.device).contiguous()
        # bf16: the fold runs with proto.cv3 as its fused tail (npr 128); f32: fold, then cv3 as its own 1x1
        # (bf16 wider protos -- m's 192 -- fold without the tail: conv2's plain mode-2 epilogue, then cv3 as a 1x1)
        fold_ok = arch.npr >= 128 and arch.npr % 64 == 0 and dtype in ("bf16", "f32")
        # (w8a16: the fold of the float weights -- its bias table too -- whose rows proto_fold8 quantizes)
        self.proto_fold = self._fold_proto(folded_f if self.form == "w8a16" else folded) \
            if (fold_ok and switch_on("VA_FOLD_PROTO")) else None
        self.proto_fold8 = None  # w8a16: the fold of the float weights, quantized per (class, row)
        if self.proto_fold is not None and self.form == "w8a16":
            wm = self._fold_rows(folded_f)
            q, sw = zip(*(self._pack_e4m3(wm[c]) for c in range(4)))
            self.proto_fold8 = (torch.stack(q).contiguous(), torch.stack(sw).contiguous())
            # VA_W8=0 (A/B): the same e4m3 values dequantized into bf16 rows
            self.proto_fold8_bf16 = (w8_order(self.proto_fold8[0], inverse=True).view(torch.float8_e4m3fn).float()
                                     * self.proto_fold8[1][..., None]).to(torch.bfloat16).contiguous()
        # the fused stem (va355.h va_seg_stem): preprocess + model.0 + model.1 with 32 -> 64 channels ('s')
        self.stem = None
        if dtype == "bf16" and self.fuse_first and w0.shape[0] == 32 and switch_on("VA_STEM"):
            w1, b1 = folded["model.1"]
            if tuple(w1.shape) == (64, 32, 3, 3):
                self.stem = self._pack_stem(w0p, b0, w1, b1)
        # f32: the same fusion in the f32 arithmetic (va355.h va_seg_stem_f32): model.0's three-term weights and
        # model.1's packed f32 weights; VA_STEM=0 keeps the two layers apart (A/B)
        self.stem32 = (dtype == "f32" and self.fuse_first and self.w0_3 is not None and w0.shape[0] == 32 and
                       tuple(folded["model.1"][0].shape) == (64, 32, 3, 3) and switch_on("VA_STEM"))
        # ... with model.2.cv1 (the C2f's 1x1, 64 -> 64) in its epilogue, so model.1's map never reaches HBM either;
        # VA_STEM_TAIL=0 keeps cv1 a launch of its own (A/B).  b2 = [model.1 bias | cv1 bias]
        self.stem32_b2 = None
        pc1 = self.w.get("model.2.cv1")
        if (self.stem32 and pc1 is not None and pc1.k == 1 and pc1.cin == 64 and pc1.cout == 64 and
                pc1.Kpad == 64 and switch_on("VA_STEM_TAIL")):
            self.stem32_b2 = torch.cat([self.w["model.1"].b[:64], pc1.b[:64]]).contiguous()
        # C2f blocks the fused kernel covers (va355.h va_seg_c2f): n = 1, shortcut, 64 -> 64 (model.2 of 's')
        self.c2f_fused = {}
        if dtype == "bf16" and switch_on("VA_C2F"):
            for i, ci, co, n, shortcut in arch.c2f_plan():
                if ci == 64 and co == 64 and n == 1 and shortcut:
                    self.c2f_fused[i] = self._pack_c2f(folded, i)
        # small batches (bf16): every C2f block as one launch, intermediates on the chip and the 3x3s' halo recomputed
        # per tile (va355.h va_seg_c2fb), for B <= c2fb_max_b; VA_C2FB=0 keeps the blocks' layers apart (A/B).  f32
        # plans take the f32 form of the same kernel for the blocks whose intermediates fit the LDS as bf16 term
        # planes (split once per value, not per read): s-seg's batch-1 forward 1.28 -> 1.21 ms, n-seg's 1.05 ->
        # 0.70.  c2fb_tile: per block index a tile side overriding _c2fb_tile's choice (tools / tests)
        on = switch_on("VA_C2FB") and (dtype == "bf16" or (dtype == "f32" and c2fb_f32))
        self.c2fb_max_b = C2FB_MAX_B if on else 0
        self.c2fb = {}
        self.c2fb_tile = {}
        self._plans = {}
        # fp8: e4m3 weights with per-output-channel scales (the convs whose input channels come in 16s), and
        # the per-conv activation scales of calibrate_fp8
        self.w8 = {}
        self.xscale = None   # per fp8 conv: its input's scale (calibrate_fp8)
        self.bscale = None   # per activation buffer of the plan, in creation order (calibrate_fp8)
        # fp8 calibration: frames to calibrate on (uint8 [n, H, W, 3]; None = 2 seeded noise frames) and the
        # headroom factor above the calibration amax: real frames exceed the noise calibration frames' amax by
        # 2.3-2.8x from model.3 on (tools/m_condition.py --real); 8 keeps the calibration amax in [28, 56], three
        # binades below e4m3's 448, and costs nothing above e4m3's normal range (2^-6)
        self.fp8_calib_frames = None
        self.fp8_headroom = FP8_HEADROOM
        if dtype == "fp8":
            for prefix, p in self.w.items():
                if p.cin % 16 == 0:
                    self.w8[prefix] = self._pack_fp8(p)

    def _pack_c2fb(self, i: int, n: int, s2: str | None = None):
        """(weight blob, bias blob) of va_seg_c2fb for C2f block ``model.{i}`` with n Bottlenecks: per conv (cv1,
        m.j.cv1 / m.j.cv2, cv2) the packed rows [Cout][K] (the unfused layers' own weights, K ordered (ky, kx,
        ci)) zero padded to 16 x 32 tiles, tile order [Cout / 16][K / 32], each tile as MFMA A fragment lanes
        (lane 16 q + r: row r, columns 8 q .. 8 q + 7) -- bf16, or in f32 mode three fragments per tile, the exact
        bf16 terms h, m, l of the f32 weights (split3_bf16's split); biases zero padded to 16 per conv.  s2: the
        stride-2 conv fused as the block's prologue (va355.h va_seg_c2fb), its tiles and biases last."""
        if (i, s2) in self.c2fb:
            return self.c2fb[(i, s2)]
        names = [f"model.{i}.cv1"] + [f"model.{i}.m.{j}.cv{k}" for j in range(n) for k in (1, 2)] + [f"model.{i}.cv2"]
        names += [s2] if s2 else []
        frags, biases = [], []
        for nm in names:
            p = self.w[nm]
            ncb, ks = _cdiv(p.cout, 16), _cdiv(p.K, 32)
            wm = torch.zeros(16 * ncb, 32 * ks, dtype=p.w.dtype, device=p.w.device)
            wm[:p.cout, :p.K] = p.w[:p.cout, :p.K]
            if self.store == "f32":
                h = wm.to(torch.bfloat16)
                r = wm - h.float()
                m = r.to(torch.bfloat16)
                t3 = torch.stack([h, m, (r - m.float()).to(torch.bfloat16)])  # [3][16 ncb][32 ks]
                frags.append(t3.reshape(3, ncb, 16, ks, 4, 8).permute(1, 3, 0, 4, 2, 5).reshape(-1))
            else:
                frags.append(wm.reshape(ncb, 16, ks, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1))
            b = torch.zeros(16 * ncb, dtype=torch.float32, device=p.b.device)
            b[:p.cout] = p.b[:p.cout].float()
            biases.append(b)
        self.c2fb[(i, s2)] = (torch.cat(frags).contiguous(), torch.cat(biases).contiguous())
        return self.c2fb[(i, s2)]

    def _c2fb_tile_bf16(self, B: int, h: int, w: int, ci: int, co: int, n: int, c: int, cs: int, cis: int) -> int:
        """bf16 (C2's latency plan): any side 2 .. 16 whose layout fits (with the stride-2 prologue's source region
        when cs), at the least (workgroup rounds of C2FB_CUS) x (per-tile MACs with the halos + C2FB_FIXED): a tile
        count just past a multiple of the CUs costs a whole round, and 100 tiles leave most CUs idle.  n-seg batch 1:
        model.2 / 4 / 6 / 12 / 15 / 18 at T = 10 / 5 / 3 / 3 / 5 / 3 instead of 16 / 8 / 4 / 4 / 8 / 4 (all five
        stride-2 prologues fused), C2 seg-only 0.362 -> 0.346 ms (profiles/r05/c2fb_tiles/bf16_n/).  (The f32 form
        keeps the 96-tile rule: with several frames in flight on other streams its full-chip launches cost C4 5 %,
        DESIGN.md §4.1.)"""
        best, bcost = 0, None
        for T in range(16, 1, -1):
            if self.c2fb_layout(c, n, ci, co, T, cs, cis)[0] <= 0:
                continue
            S0 = T + 4 * n
            macs = (S0 * S0 + T * T) * ci * c + T * T * (2 + n) * c * co + S0 * S0 * 9 * cis * cs
            macs += sum(((S0 - 4 * j - 2) ** 2 + (S0 - 4 * j - 4) ** 2) * 9 * c * c for j in range(n))
            cost = _cdiv(B * _cdiv(h, T) * _cdiv(w, T), C2FB_CUS) * (macs + C2FB_FIXED)
            if bcost is None or cost < bcost:
                best, bcost = T, cost
        return best

    def c2fb_layout(self, c: int, n: int, ci: int, co: int, T: int, cs: int = 0, cis: int = 0):
        """(LDS bytes or -1, A fragments, bias floats, f32 term planes 1 / 0) of va_seg_c2fb's layout (va355.h
        va_c2fb_layout); cs / cis: the stride-2 prologue's output / input channels (0: none)."""
        out = (ctypes.c_int64 * 4)()
        rc = self.lib.va_c2fb_layout(c, n, ci, co, T, self.va_dtype, cs, cis, out)
        return (int(out[0]) if rc == 0 else -1, int(out[1]), int(out[2]), int(out[3]))

    def _c2fb_tile(self, i: int, B: int, h: int, w: int, ci: int, co: int, n: int, cs: int = 0, cis: int = 0) -> int:
        """va_seg_c2fb's tile side for block i at B x h x w (bf16: _c2fb_tile_bf16): the largest of 16 / 8 / 4 / 2
        whose launch has at least C2FB_MIN_TILES workgroups (a batch-1 layer fills a few dozen of the 256 CUs, so a smaller tile's
        larger halo share costs less than idle CUs) and whose LDS layout fits; 0 when none fits.  f32: only layouts
        with the intermediates as term planes and hidden widths up to 128 -- the f32-region form (a split per read)
        and s's 256-wide blocks at T = 2 measured slower than the blocks' layers apart."""
        if i in self.c2fb_tile:
            return self.c2fb_tile[i]
        c = co // 2
        if self.store == "bf16":
            return self._c2fb_tile_bf16(B, h, w, ci, co, n, c, cs, cis)
        lay = {T: self.c2fb_layout(c, n, ci, co, T, cs, cis) for T in (16, 8, 4, 2)}
        fits = [T for T, l in lay.items() if l[0] > 0 and (self.store == "bf16" or (l[3] and c <= 128))]
        for T in fits:
            if B * _cdiv(h, T) * _cdiv(w, T) >= C2FB_MIN_TILES:
                return T
        return fits[-1] if fits else 0

    def _pack_fp8(self, p: Packed):
        """(e4m3 bytes [Npad][Kpad128], per-output-channel scale float [Npad]) of a packed bf16 conv: the
        channel's largest |w| maps to 448, values rounded to nearest even (torch.float8_e4m3fn)."""
        wf = p.w.float().cpu()
        Kp = _ceil(p.K, F8_KS)
        amax = wf.abs().amax(1)
        sw = torch.where(amax > 0, amax / F8_MAX, torch.ones_like(amax))
        w8 = torch.zeros(p.Npad, Kp, dtype=torch.float32)
        w8[:, :p.K] = (wf[:, :p.K] / sw[:, None]).clamp(-F8_MAX, F8_MAX)
        q = w8.to(torch.float8_e4m3fn).view(torch.uint8)
        return q.to(self.device).contiguous(), sw.to(self.device).contiguous(), Kp

    def calibrate_fp8(self, H: int, W: int, frames_u8: torch.Tensor | None = None, seed: int = 0,
                      headroom: float | None = None) -> dict:
        """Static scales of the fp8 mode: one forward of this network in bf16 (same weights, the same buffers in
        the same order) on `frames_u8` (default: self.fp8_calib_frames, else 2 seeded uniform uint8 frames, the
        bench's input distribution).  Every activation buffer gets the power of two s with amax * headroom * s in
        [224, 448] (headroom default self.fp8_headroom), amax the largest |x| it held there; buffers an upsample
        copies between share one scale (the copy moves bytes).  Values are stored as sat(x * s) in e4m3, so the
        accuracy depends on how well the calibration frames cover the deployment's activations: pass
        representative frames (FramePipeline / YOLO fp8_calib).  -> {conv prefix: its input's scale}."""
        hr = float(self.fp8_headroom if headroom is None else headroom)
        if frames_u8 is None:
            frames_u8 = self.fp8_calib_frames
        if frames_u8 is None:
            g = torch.Generator().manual_seed(seed)
            frames_u8 = torch.randint(0, 256, (2, H, W, 3), generator=g, dtype=torch.uint8)
        if tuple(frames_u8.shape[1:]) != (H, W, 3):
            raise _lib.VaError(f"fp8 calibration frames {tuple(frames_u8.shape)} for a {H}x{W} network")
        B = frames_u8.shape[0]
        p = self.plan(B, H, W, tag=-1, _calib=True)
        p["frames"].copy_(frames_u8.to(self.device), non_blocking=True)
        self.run_plan(p)
        torch.cuda.synchronize(self.device)
        bufs = p["bufs"]
        amax = [float(t.float().abs().max()) for t in bufs]
        parent = list(range(len(bufs)))

        def find(i):
            while parent[i] != i:
                parent[i] = parent[parent[i]]
                i = parent[i]
            return i

        for i, j in p["links"]:
            parent[find(i)] = find(j)
        gmax = {}
        for i, m in enumerate(amax):
            r = find(i)
            gmax[r] = max(gmax.get(r, 0.0), m)
        # a power of two (exact in the kernels' conversions): amax lands in [224, 448]
        self.bscale = [2.0 ** math.floor(math.log2(F8_MAX / (hr * gmax[find(i)]))) if gmax[find(i)] > 0 else 1.0
                       for i in range(len(bufs))]
        index = {t.data_ptr(): i for i, t in enumerate(bufs)}
        self.xscale = {m["prefix"]: self.bscale[index[m["src"].buf.data_ptr()]] for m in p["meta"]
                       if m.get("src") is not None and m["prefix"] in self.w8}
        self._plans = {k: v for k, v in self._plans.items() if k[3:5] != (-1, True)}
        return self.xscale

    def _pack_stem(self, w0p: torch.Tensor, b0: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor):
        """Weight blob + bias vector of va_seg_stem: bf16 MFMA A fragments (see _pack_c2f) W0 = model.0
        [2 row groups][2 K-steps] (K = (ky*3 + kx)*4 + channel, channels R, G, B, 0), then W1 = model.1
        [9 taps][4 row groups] with K in P32 order inside the tap (the channel order model.0's C fragments
        leave in LDS) and rows permuted so a lane's two row groups are 8 consecutive output channels."""
        p32 = torch.tensor([4 * (k >> 3) + (k & 3) + 16 * ((k >> 2) & 1) for k in range(32)])

        def frag(a):  # [16][32] -> [64][8]
            return a.reshape(16, 4, 8).permute(1, 0, 2).reshape(64, 8)

        # model.0 with k = tap * 4 + c (c = R, G, B, 0), 36 of 64: from w0p's k = tap * 3 + c
        w0k = torch.zeros(w0p.shape[0], 64)
        for tap in range(9):
            w0k[:, 4 * tap:4 * tap + 3] = w0p[:, 3 * tap:3 * tap + 3].float()
        f0 = [frag(w0k[16 * q:16 * q + 16, 32 * s:32 * s + 32]) for q in range(2) for s in range(2)]
        f1 = []
        for t in range(9):
            for q in range(4):
                rows = torch.tensor([32 * (q >> 1) + 8 * (r >> 2) + 4 * (q & 1) + (r & 3) for r in range(16)])
                f1.append(frag(w1[rows][:, :, t // 3, t % 3].float()[:, p32]))
        blob = torch.stack(f0 + f1).reshape(-1)
        assert blob.numel() == 20480
        bias = torch.cat([b0.float(), b1.float()])
        return (blob.to(self.device, self.tdtype).contiguous(), bias.to(self.device).contiguous())

    def _pack_c2f(self, folded: dict, i: int):
        """Weight blob + bias vector of va_seg_c2f for C2f block ``model.{i}`` (block.py C2f / Bottleneck).

        The blob is bf16 MFMA A fragments (64 lanes x 8 values; lane l = 16 fq + fr holds row fr, K
        8 fq .. 8 fq + 7 of a 16 x 32 tile) in the order F1 cv1 [4 row groups][2 K-steps], F2 m.0.cv1
        [9 taps][2], F3 m.0.cv2 [9][2], F4 cv2 [4][3].  K inside every 32-channel chunk that the kernel
        hands over in registers or LDS is in P32 order (the channel a C fragment puts at position k),
        and cv2's rows are permuted so a lane's two row groups are 8 consecutive output channels."""
        w1, b1 = folded[f"model.{i}.cv1"]
        wm1, bm1 = folded[f"model.{i}.m.0.cv1"]
        wm2, bm2 = folded[f"model.{i}.m.0.cv2"]
        w2, b2 = folded[f"model.{i}.cv2"]
        p32 = torch.tensor([4 * (k >> 3) + (k & 3) + 16 * ((k >> 2) & 1) for k in range(32)])

        def frag(a):  # [16][32] -> [64][8]
            return a.reshape(16, 4, 8).permute(1, 0, 2).reshape(64, 8)

        w1m = w1[:, :, 0, 0].float()  # [64 co][64 ci]
        f1 = [frag(w1m[16 * q:16 * q + 16, 32 * s:32 * s + 32]) for q in range(4) for s in range(2)]
        f2 = [frag(wm1[16 * q:16 * q + 16, :, t // 3, t % 3].float()[:, p32]) for t in range(9) for q in range(2)]
        f3 = [frag(wm2[16 * q:16 * q + 16, :, t // 3, t % 3].float()[:, p32]) for t in range(9) for q in range(2)]
        w2m = w2[:, :, 0, 0].float()  # [64 co][96 ci]
        f4 = []
        for q in range(4):
            rows = torch.tensor([32 * (q >> 1) + 8 * (r >> 2) + 4 * (q & 1) + (r & 3) for r in range(16)])
            for s in range(3):
                f4.append(frag(w2m[rows][:, 32 * s + p32]))
        blob = torch.stack(f1 + f2 + f3 + f4).reshape(-1)
        assert blob.numel() == 28672
        bias = torch.cat([b1, bm1, bm2, b2]).float()
        return (blob.to(self.device, self.tdtype).contiguous(), bias.to(self.device).contiguous())

    def _fold_proto(self, folded: dict) -> Packed:
        """Packed weights of the sub-pixel fold of proto's upsample + cv2 (see fold_proto_weights), and its
        border bias table (va355.h va_conv_args.bias4): the deconv bias reaches an output pixel through
        the taps that fall inside the low-res map, so it is folded into a per-(class, row border, column
        border) bias instead of riding on a constant-1 input channel -- K stays 4 x 128 (the FK
        addressing of conv2 applies, 6 % fewer MACs)."""
        wd, bd = folded["model.22.proto.upsample"]
        w2, b2 = folded["model.22.proto.cv2"]
        wfull = fold_proto_weights(wd, bd, w2)  # [4][O][2][2][Ci + 8], deconv-bias taps at channel Ci
        ci = wd.shape[0]
        wb = wfull[..., ci]  # per-tap bias contributions [4][O][2][2]
        o = wfull.shape[1]
        K = 4 * ci
        Kpad, Npad = _ceil(K, self.bk), _ceil(o, NPAD)
        wm = self._fold_rows(folded, wfull)
        bt = torch.zeros(4, 2, 2, Npad, dtype=torch.float64)
        for c in range(4):
            dy, dx = c >> 1, c & 1
            fy_out, fx_out = (0 if dy == 0 else 1), (0 if dx == 0 else 1)  # the tap that leaves the map
            for rf in range(2):
                for cf in range(2):
                    acc = b2.double().clone()
                    for fy in range(2):
                        for fx in range(2):
                            if (rf and fy == fy_out) or (cf and fx == fx_out):
                                continue
                            acc += wb[c, :, fy, fx]
                    bt[c, rf, cf, :o] = acc
        p = Packed(wm.to(self.device, self.tdtype).contiguous(),
                   bt.float().reshape(-1).to(self.device).contiguous(), ci, o, 2, K, Kpad, Npad)
        if self.store == "f32" and ci % 16 == 0 and K == Kpad:
            p.w3 = w3_rows(p.w, 4, ci)
        return p

    def _fold_rows(self, folded: dict, wfull: torch.Tensor | None = None) -> torch.Tensor:
        """The sub-pixel fold's weight rows, float64 [4 classes][Npad][Kpad] (K = (fy, fx, ci), zero padded)."""
        wd, bd = folded["model.22.proto.upsample"]
        if wfull is None:
            wfull = fold_proto_weights(wd, bd, folded["model.22.proto.cv2"][0])
        ci = wd.shape[0]
        o = wfull.shape[1]
        K = 4 * ci
        wm = torch.zeros(4, _ceil(o, NPAD), _ceil(K, self.bk), dtype=torch.float64)
        wm[:, :o, :K] = wfull[..., :ci].reshape(4, o, K)
        return wm

    def _pack_e4m3(self, wm: torch.Tensor):
        """(e4m3 bytes [Npad][Kpad], scale float32 [Npad]) of packed weight rows wm [Npad][Kpad] for the bf16 kernels'
        w8 form (va355.h va_conv_args.w8): per row the largest |w| maps to 448 (scale amax / 448, 1 for an empty row),
        values rounded to nearest even and saturated (torch.float8_e4m3fn) -- w ~= e4m3 x scale -- in the kernels' K
        order (w8_order)."""
        wf = wm.double()
        amax = wf.abs().amax(1)
        sw = torch.where(amax > 0, amax / F8_MAX, torch.ones_like(amax)).float()
        q = (wf / sw.double()[:, None]).clamp(-F8_MAX, F8_MAX).float().to(torch.float8_e4m3fn).view(torch.uint8)
        return w8_order(q).to(self.device).contiguous(), sw.to(self.device).contiguous()

    @property
    def store(self) -> str:
        """Activation storage of the f32 / bf16 kernels: f32 in the f32 mode, else bf16.  The fp8 mode
        (BASELINE.json configs[4], e4m3 MFMA -- va_fp8.hip) keeps its activations as e4m3 bytes with one scale per
        buffer (plan(), calibrate_fp8); only model.0's output (and its weights' padding) stays bf16."""
        return "f32" if self.dtype == "f32" else "bf16"

    @property
    def bk(self) -> int:
        """K padding of the packed weights: the conv2 K-step (64 bf16 / 32 f32)."""
        return BK if self.store == "bf16" else 32

    # ------------------------------------------------------------------ packing
    def _rows(self, w: torch.Tensor, deconv: bool = False) -> torch.Tensor:
        """A conv's weights as the GEMM rows _pack lays out, float32 [Npad][Kpad]: K ordered (ky, kx, ci) with the
        input channels padded to the kernels' vector width, zero padded; ConvTranspose2d(2, 2) as the 1x1 GEMM with
        rows q * Cout + co (q = 2 dy + dx)."""
        if deconv:
            cin, cout = w.shape[0], w.shape[1]
            return self._rows(w.permute(2, 3, 1, 0).reshape(4 * cout, cin).view(4 * cout, cin, 1, 1))
        cout, cin, kh, kw = w.shape
        cin_p = max(_ceil(cin, self.vec), 8) if cin < 8 else _ceil(cin, self.vec)
        wp = torch.zeros(cout, kh, kw, cin_p, dtype=torch.float32)
        wp[..., :cin] = w.float().permute(0, 2, 3, 1)
        K = kh * kw * cin_p
        wm = torch.zeros(_ceil(cout, NPAD), _ceil(K, self.bk), dtype=torch.float32)
        wm[:cout, :K] = wp.reshape(cout, K)
        return wm

    def _pack(self, w: torch.Tensor, b: torch.Tensor, deconv: bool = False, stride: int = 1) -> Packed:
        if deconv:  # ConvTranspose2d weight [Cin, Cout, 2, 2] -> 1x1 GEMM rows q*Cout + co, q = dy*2 + dx
            cin, cout = w.shape[0], w.shape[1]
            wg = w.permute(2, 3, 1, 0).reshape(4 * cout, cin)  # [dy, dx, co, ci]
            bg = b.repeat(4)
            p = self._pack(wg.view(4 * cout, cin, 1, 1), bg)
            p.deconv = True
            return p
        cout, cin, kh, kw = w.shape
        cin_p = max(_ceil(cin, self.vec), 8) if cin < 8 else _ceil(cin, self.vec)
        K = kh * kw * cin_p
        Kpad = _ceil(K, self.bk)
        Npad = _ceil(cout, NPAD)
        wm = self._rows(w)
        bm = torch.zeros(Npad, dtype=torch.float32)
        bm[:cout] = b
        p = Packed(wm.to(self.device, self.tdtype).contiguous(), bm.to(self.device).contiguous(), cin_p, cout, kh, K,
                   Kpad, Npad)
        if self.store == "f32" and cin_p % 16 == 0 and K == Kpad:
            p.w3 = w3_rows(p.w, kh * kw, cin_p, w3_group(stride, kh * kw, cin_p))
        return p

    # ------------------------------------------------------------------ planning
    def _buf(self, B, h, w, c, dtype=None):
        return torch.empty((B, h, w, c), dtype=dtype or self.tdtype, device=self.device)

    def plan(self, B: int, H: int, W: int, tag: int = 0, _calib: bool = False, lanes: bool | None = None):
        """Op list + buffers for B frames of H x W (``tag`` gives independent buffer sets, e.g. for
        double-buffered batches that overlap on two streams).  fp8: calibrated on first use (calibrate_fp8);
        _calib = the bf16 plan that calibration runs.  ``lanes``: the branch-parallel list (laned(); default
        self.lanes for B <= self.lanes_max_b) -- off for callers that already overlap whole forwards."""
        if lanes is None:
            lanes = self.lanes and B <= self.lanes_max_b
        key = (B, H, W, tag, _calib, lanes)
        if key in self._plans:
            return self._plans[key]
        fp8 = self.dtype == "fp8" and not _calib
        use_w8 = self.form == "w8a16" and switch_on("VA_W8")  # e4m3 weight bytes (else their bf16 dequantization)
        if fp8 and self.bscale is None:
            self.calibrate_fp8(H, W)
        if H % 32 or W % 32:
            raise _lib.VaError(f"frame {H}x{W}: the network needs multiples of 32 (pad/letterbox first)")
        a = self.arch
        ops = []
        meta = []  # per op: name, kind, GEMM M/N/K (algorithmic), bytes moved
        keep = []  # buffers referenced by the op list
        bufs = []  # activation buffers in creation order (fp8: one scale each, calibrate_fp8)
        links = []  # (i, j): buffers an upsample copies between (one scale)
        scale = {}  # fp8: buffer data_ptr -> its scale
        # split-K workspace of this plan (va355.h va_conv_args.ws; its ops run in order on one stream)
        ws = torch.empty(SPLITK_WS_BYTES, dtype=torch.uint8, device=self.device)
        wcnt = torch.zeros(SPLITK_NCNT, dtype=torch.int32, device=self.device)
        keep += [ws, wcnt]

        def with_ws(args: ConvArgs) -> ConvArgs:
            args.ws, args.ws_bytes, args.wcnt, args.ncnt = ws.data_ptr(), ws.numel(), wcnt.data_ptr(), wcnt.numel()
            return args

        def new(h, w, c, dtype=None):
            # fp8: activations as e4m3 bytes, except the float outputs and the bf16 map model.0 writes
            t = self._buf(B, h, w, c, dtype if dtype is not None or not fp8 else torch.uint8)
            keep.append(t)
            if fp8:
                scale[t.data_ptr()] = self.bscale[len(bufs)]
            bufs.append(t)
            return Slice(t, 0, c)

        def bidx(sl: Slice) -> int:
            return next(i for i, t in enumerate(bufs) if t.data_ptr() == sl.buf.data_ptr())

        def conv(prefix, src: Slice, dst: Slice, h, w, stride=1, act=True, res: Slice | None = None,
                 out_f32=False, tail: str | None = None, act2=False, up: Slice | None = None):
            """One conv op; with ``tail`` the named 1x1 conv (the only consumer of this one) runs fused in
            its epilogue and ``dst`` / ``out_f32`` describe the tail's output.  With ``up`` the first
            ``up.c`` input channels are the nearest-x2 upsample of that half-resolution slice, read in
            place (va355.h va_conv_args.xu) instead of from ``src``."""
            p = self.w[prefix]
            p2 = self.w[tail] if tail else None
            k = p.k
            pad = k // 2
            ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
            if src.c != p.cin and not (src.c < p.cin and src.ld >= p.cin):
                raise _lib.VaError(f"{prefix}: input has {src.c} channels, packed for {p.cin}")
            args = with_ws(ConvArgs(
                x=src.ptr, N=B, H=h, W=w, Cin=p.cin, ldx=src.ld, kh=k, kw=k, stride=stride, pad=pad, Ho=ho, Wo=wo,
                w=p.w.data_ptr(), bias=p.b.data_ptr(), Cout=p.cout, Npad=p.Npad, K=p.K, Kpad=p.Kpad,
                y=dst.ptr, ldy=dst.ld, res=res.ptr if res is not None else None, ldr=res.ld if res is not None else 0,
                act=1 if act else 0, mode=1 if p.deconv else 0, M=B * ho * wo, dtype=self.va_dtype,
                out_f32=1 if (out_f32 and self.store == "bf16") else 0))
            on_fp8 = fp8 and prefix in self.w8 and tail is None and up is None and self._fp8_fits(p, src, dst, res,
                                                                                                  out_f32)
            if fp8 and not on_fp8:
                raise _lib.VaError(f"{prefix}: the fp8 mode's e4m3 buffers need the fp8 kernel's operand rules")
            if on_fp8:  # va_fp8.hip: e4m3 weights; input, output and residual with their buffers' scales
                w8, sw, Kp = self.w8[prefix]
                xs = scale[src.buf.data_ptr()]
                ws = (sw / xs).contiguous()
                keep.append(ws)
                args.dtype, args.w, args.Kpad, args.wscale, args.xscale = VA_DTYPE_FP8, w8.data_ptr(), Kp, \
                    ws.data_ptr(), xs
                args.x8 = 1 if src.e4m3 else 0
                args.yscale = scale[dst.buf.data_ptr()] if dst.e4m3 else 0.0
                args.rscale = scale[res.buf.data_ptr()] if res is not None and res.e4m3 else 0.0
            if up is not None:
                args.xu, args.ldu, args.cu = up.ptr, up.ld, up.c
            w8 = use_w8 and prefix in self.w8w
            if w8:  # w8a16: the e4m3 bytes and their per-row scales (va355.h va_conv_args.w8)
                q8, sw8 = self.w8w[prefix]
                args.w, args.wscale, args.w8 = q8.data_ptr(), sw8.data_ptr(), 1
            if p.w3 is not None and self.store == "f32" and up is None:
                args.w3 = p.w3.data_ptr()  # the three-plane kernel takes the layers it fits (va_seg.hip use_conv3t)
            cout = p.cout
            if p2 is not None:
                if p2.cin != p.cout or p2.k != 1:
                    raise _lib.VaError(f"{prefix}+{tail}: tail must be a 1x1 conv over all {p.cout} channels")
                if self.store == "f32":  # the tail's weights as three exact bf16 terms, rows in 32-channel blocks
                    w2 = split3_bf16(p2.w[:32 * ((p2.cout + 31) // 32), :p.cout])
                else:
                    w2 = p2.w[:, :p.cout].contiguous()  # [Npad][Cout]: the tail reads rows of exactly Cout
                keep.append(w2)
                args.w2, args.b2, args.c2, args.act2 = w2.data_ptr(), p2.b.data_ptr(), p2.cout, 1 if act2 else 0
                cout = p2.cout
            if dst.c != (cout // 4 if p.deconv else cout):
                raise _lib.VaError(f"{prefix}: output slice has {dst.c} channels, conv gives {cout}")
            ops.append(SegOp(kind=VA_OP_CONV, a=args))
            es = 2 if self.store == "bf16" else 4
            xe, ye = src.buf.element_size(), (4 if out_f32 else dst.buf.element_size())
            flops = 2 * B * ho * wo * p.cout * k * k * src.c + (2 * B * ho * wo * p.cout * cout if p2 else 0)
            meta.append({"name": prefix + (f"+{tail}" if tail else ""), "kind": "conv", "M": B * ho * wo,
                         "N": p.cout, "K": k * k * src.c, "k": k, "stride": stride, "flops": flops,
                         "bytes": xe * B * h * w * src.c + (1 if on_fp8 or w8 else es) * p.cout * k * k * src.c
                         + B * ho * wo * cout * ye,
                         "prefix": prefix, "src": src, "fp8": on_fp8})
            return ho, wo

        def c2f(i, src: Slice, dst: Slice, h, w, up: Slice | None = None, pre: Slice | None = None,
                s2: tuple | None = None):
            """pre: the block's concat buffer with cv1's output already in it (cv1 fused into the producer).
            s2 = (prefix, source slice): the stride-2 conv that writes the block's first input channels (src's first
            cs), run as the fused block's prologue where va_seg_c2fb takes the block, else as its own op first."""
            _, ci, co, n, shortcut = next(p for p in a.c2f_plan() if p[0] == i)
            cs = cis = 0
            if s2 is not None:
                ps2 = self.w[s2[0]]
                cs, cis = ps2.cout, ps2.cin
            if pre is not None:
                c = co // 2
                t = pre
            c = co // 2
            if (pre is None and B <= self.c2fb_max_b and c in (16, 32, 64, 128, 256) and n in (1, 2) and ci % 8 == 0 and
                    co % 16 == 0 and src.ld % 8 == 0 and dst.ld % 8 == 0 and (up is None or up.ld % 8 == 0) and
                    src.c == ci):
                T = self._c2fb_tile(i, B, h, w, ci, co, n)
                # the stride-2 prologue where its source region still leaves the block its tile side (a smaller tile
                # recomputes more of the block than the prologue saves: model.5 + model.6 of n-seg at T = 2 took 74 us
                # against 15 + 30 apart, profiles/r05/c2fb/ab_b1_s2.log; at T = 3, 38 against 15 + 27)
                if s2 is not None and not (self.store == "bf16" and up is None and s2[1].ld % 8 == 0 and
                                           s2[1].c == cis and cis >= 8 and cis & (cis - 1) == 0 and cs % 16 == 0 and
                                           T and self._c2fb_tile(i, B, h, w, ci, co, n, cs, cis) == T):
                    conv(s2[0], s2[1], src.sub(0, cs), 2 * h, 2 * w, stride=2)
                    s2 = None
                if T:
                    blob, bias = self._pack_c2fb(i, n, s2[0] if s2 else None)
                    args = ConvArgs(x=src.ptr, N=B, H=h, W=w, Cin=ci, ldx=src.ld, w=blob.data_ptr(),
                                    bias=bias.data_ptr(), Cout=co, y=dst.ptr, ldy=dst.ld, dtype=self.va_dtype, mode=3,
                                    kh=n, kw=1 if shortcut else 0, Npad=c, stride=T)
                    if up is not None:
                        args.xu, args.ldu, args.cu = up.ptr, up.ld, up.c
                    macs = ci * 2 * c + n * 2 * 9 * c * c + (2 + n) * c * co  # per output pixel, without the halo
                    name = f"model.{i} (fused C2f, T={T})"
                    es = 2 if self.store == "bf16" else 4
                    nbytes = es * B * h * w * (ci + co)
                    if s2 is not None:  # va355.h va_seg_c2fb: a.res / ldr = the prologue's source, c2 = cs, K = cis
                        args.res, args.ldr, args.c2, args.K = s2[1].ptr, s2[1].ld, cs, cis
                        macs += 9 * cis * cs
                        name = f"{s2[0]}+model.{i} (fused C2f, T={T})"
                        nbytes += es * B * 4 * h * w * cis - es * B * h * w * cs
                    ops.append(SegOp(kind=VA_OP_C2F, a=args))
                    meta.append({"name": name, "kind": "conv", "M": B * h * w, "N": co, "K": macs // co, "k": 1,
                                 "stride": 1, "flops": 2 * B * h * w * macs, "bytes": nbytes})
                    return
            if s2 is not None:
                conv(s2[0], s2[1], src.sub(0, cs), 2 * h, 2 * w, stride=2)
            if pre is None and i in self.c2f_fused and src.c == 64 and src.ld % 8 == 0 and dst.ld % 8 == 0:
                blob, bias = self.c2f_fused[i]
                ops.append(SegOp(kind=VA_OP_C2F, a=with_ws(ConvArgs(x=src.ptr, N=B, H=h, W=w, Cin=64, ldx=src.ld,
                                                                     w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                                                                     y=dst.ptr, ldy=dst.ld, dtype=self.va_dtype))))
                macs = 64 * 64 + 2 * 32 * 288 + 64 * 96  # per pixel, the four convs
                meta.append({"name": f"model.{i} (fused C2f)", "kind": "conv", "M": B * h * w, "N": 64,
                             "K": macs // 64, "k": 1, "stride": 1, "flops": 2 * B * h * w * macs,
                             "bytes": 2 * B * h * w * 128})
                return
            if pre is None:
                c = co // 2
                t = new(h, w, (2 + n) * c)
                conv(f"model.{i}.cv1", src, t.sub(0, 2 * c), h, w, up=up)
            tmp = new(h, w, c)
            for j in range(n):
                x_in = t.sub((1 + j) * c, c)
                conv(f"model.{i}.m.{j}.cv1", x_in, tmp, h, w)
                conv(f"model.{i}.m.{j}.cv2", tmp, t.sub((2 + j) * c, c), h, w, res=x_in if shortcut else None)
            conv(f"model.{i}.cv2", t, dst, h, w)

        def upsample(src: Slice, dst: Slice, h, w):
            links.append((bidx(src), bidx(dst)))
            ops.append(SegOp(kind=VA_OP_UPSAMPLE, a=ConvArgs(x=src.ptr, ldx=src.ld, y=dst.ptr, ldy=dst.ld, N=B, H=h, W=w,
                                                              Cin=src.c,
                                                              dtype=VA_DTYPE_FP8 if src.e4m3 else self.va_dtype)))
            meta.append({"name": "upsample", "kind": "upsample"})

        def finish(proto: Slice):
            nonlocal ops, meta
            marks["P"] = len(ops)
            if lanes:
                ops, meta = laned(ops, meta)
            assert len(meta) == len(ops)
            plan = {"ops": (SegOp * len(ops))(*ops), "n": len(ops), "meta": meta, "keep": keep, "frames": frames,
                    "bufs": bufs, "links": links, "out": SegOutputs(levels=levels, proto=proto.buf)}
            self._plans[key] = plan
            return plan

        def laned(ops, meta):
            """Small batches: the head's levels and proto overlap the rest of the neck (va355.h VA_OP_FORK).
            Lane 1 runs head level 0 then proto once model.15 (o3) is out, lane 2 head level 1 once model.18
            (o4) is, the calling stream model.16 .. model.21 then head.2.0, whose three branches (box / cls /
            coef, independent 3x3 + 1x1 pairs) then run on the calling stream, lane 3 and lane 2 (f32): the
            critical path drops from the whole list to backbone + neck + head.2.0 + one branch.  Each lane gets its own
            split-K workspace (the kernels' slabs and arrival counters must not be shared by launches that can
            overlap)."""
            m = marks
            rng = {"A": (0, m["A"]), "B": (m["A"], m["B"]), "C": (m["B"], m["C"]), "H0": (m["C"], m["H0"]),
                   "H1": (m["H0"], m["H1"]), "H2.0": (m["H1"], m["H2.0"]), "H2.cv2": (m["H2.0"], m["H2.cv2"]),
                   "H2.cv3": (m["H2.cv2"], m["H2.cv3"]), "H2.cv4": (m["H2.cv3"], m["H2.cv4"]),
                   "P": (m["H2"], m["P"])}
            assert m["H2.cv4"] == m["H2"]
            # a fork + join costs a few us of cross-queue signalling: worth it for the f32 branches (~40 us each,
            # f32 s batch 1: 1302 -> 1282 us), not for the bf16 ones (~15 us: 714 -> 728 us)
            split_h2 = self.store == "f32"
            out_ops, out_meta = [], []

            def take(part, lane):
                for i in range(*rng[part]):
                    op = ops[i]
                    op.lane = lane
                    if lane and op.kind == VA_OP_CONV and op.a.ws:
                        lws, lcnt = lane_ws[lane]
                        op.a.ws, op.a.wcnt = lws.data_ptr(), lcnt.data_ptr()
                    out_ops.append(op)
                    out_meta.append(meta[i])

            def sync(kind, lane):
                out_ops.append(SegOp(kind=kind, a=ConvArgs(N=lane)))
                out_meta.append({"name": f"{'fork' if kind == VA_OP_FORK else 'join'} lane {lane}", "kind": "sync"})

            lane_ws = {}
            for lane in (1, 2, 3) if split_h2 else (1, 2):
                lane_ws[lane] = (torch.empty(SPLITK_WS_BYTES, dtype=torch.uint8, device=self.device),
                                 torch.zeros(SPLITK_NCNT, dtype=torch.int32, device=self.device))
                keep.extend(lane_ws[lane])
            take("A", 0)
            sync(VA_OP_FORK, 1)
            take("H0", 1)
            take("P", 1)
            take("B", 0)
            sync(VA_OP_FORK, 2)
            take("H1", 2)
            take("C", 0)
            take("H2.0", 0)
            if split_h2:
                sync(VA_OP_FORK, 3)
                take("H2.cv3", 3)
                sync(VA_OP_FORK, 2)  # lane 2 is through head level 1 by now (model.19 .. head.2.0 ran meanwhile)
                take("H2.cv4", 2)
                take("H2.cv2", 0)
            else:
                for br in ("cv2", "cv3", "cv4"):
                    take(f"H2.{br}", 0)
            for lane in (1, 2, 3) if split_h2 else (1, 2):
                sync(VA_OP_JOIN, lane)
            return out_ops, out_meta


        frames = torch.empty((B, H, W, 3), dtype=torch.uint8, device=self.device)
        h1, w1 = H // 2, W // 2
        h2, w2 = H // 4, W // 4
        h3, w3 = H // 8, W // 8
        h4, w4 = H // 16, W // 16
        h5, w5 = H // 32, W // 32
        if self.stem is not None and W % 16 == 0:
            a1 = new(h2, w2, a.c2)
            blob, bias = self.stem
            ops.append(SegOp(kind=VA_OP_STEM, a=with_ws(ConvArgs(x=frames.data_ptr(), N=B, H=H, W=W, Cin=32,
                                                                  w=blob.data_ptr(), bias=bias.data_ptr(), Cout=64,
                                                                  y=a1.ptr, ldy=a1.ld, dtype=self.va_dtype))))
            macs = 27 * 32 * 4 + 288 * 64  # per model.1 output pixel: 4 model.0 pixels + model.1
            meta.append({"name": "model.0+model.1 (fused stem)", "kind": "conv", "M": B * h2 * w2, "N": 64,
                         "K": macs // 64, "k": 3, "stride": 2, "flops": 2 * B * h2 * w2 * macs,
                         "bytes": B * H * W * 3 + 2 * B * h2 * w2 * 64})
        elif self.stem32 and (W * 3) % 16 == 0:
            p1 = self.w["model.1"]
            sa = with_ws(ConvArgs(x=frames.data_ptr(), N=B, H=H, W=W, Cin=32, Cout=64, w3=self.w0_3.data_ptr(),
                                  bias=self.w0[1].data_ptr(), w=p1.w.data_ptr(), b2=p1.b.data_ptr(), Npad=p1.Npad,
                                  K=p1.K, Kpad=p1.Kpad, dtype=VA_DTYPE_F32))  # wcnt: the work-queue schedule
            macs = 27 * 32 * 4 + 288 * 64  # per model.1 output pixel: 4 model.0 pixels + model.1
            name = "model.0+model.1 (fused f32 stem)"
            if self.stem32_b2 is not None:  # + model.2.cv1: the stem writes cv1's output into model.2's concat buffer
                n2 = next(p for p in a.c2f_plan() if p[0] == 2)[3]
                t2 = new(h2, w2, (2 + n2) * 32)
                a1 = t2.sub(0, 64)
                sa.w2, sa.b2, sa.c2, sa.act2 = self.w["model.2.cv1"].w.data_ptr(), self.stem32_b2.data_ptr(), 64, 1
                macs += 64 * 64
                name = "model.0+model.1+model.2.cv1 (fused f32 stem)"
            else:
                t2 = None
                a1 = new(h2, w2, a.c2)
            sa.y, sa.ldy = a1.ptr, a1.ld
            ops.append(SegOp(kind=VA_OP_STEM, a=sa))
            meta.append({"name": name, "kind": "conv", "M": B * h2 * w2, "N": 64,
                         "K": macs // 64, "k": 3, "stride": 2, "flops": 2 * B * h2 * w2 * macs,
                         "flops_c0": 2 * B * h2 * w2 * 27 * 32 * 4,  # model.0's share (three term products, once)
                         "bytes": B * H * W * 3 + 4 * B * h2 * w2 * 64})
        else:
            # fp8: e4m3 straight from the fused model.0 (else bf16, and model.1 quantizes it while staging)
            a0 = new(h1, w1, a.c1, None if self.fuse_first else self.tdtype)
            if self.fuse_first:
                c0 = ConvArgs(x=frames.data_ptr(), N=B, H=H, W=W, w=self.w0[0].data_ptr(), bias=self.w0[1].data_ptr(),
                              Cout=a.c1, y=a0.ptr, ldy=a0.ld, dtype=self.va_dtype)
                if self.w0_3 is not None and (W * 3) % 16 == 0:
                    c0.w3 = self.w0_3.data_ptr()
                if a0.e4m3:
                    c0.dtype, c0.yscale = VA_DTYPE_FP8, scale[a0.buf.data_ptr()]
                ops.append(SegOp(kind=VA_OP_CONV0, a=c0))
                meta.append({"name": "model.0", "kind": "conv", "M": B * h1 * w1, "N": a.c1, "K": 27, "k": 3,
                             "stride": 2, "bytes": B * H * W * 3 + (2 if self.store == "bf16" else 4) * B * h1 * w1 * a.c1})
            else:
                x0 = new(H, W, 8, self.tdtype)
                ops.append(SegOp(kind=VA_OP_PREPROCESS, a=ConvArgs(x=frames.data_ptr(), y=x0.ptr, N=B, H=H, W=W,
                                                                    dtype=self.va_dtype)))
                meta.append({"name": "preprocess", "kind": "preprocess"})
                conv("model.0", x0, a0, H, W, stride=2)
            a1 = new(h2, w2, a.c2)
            conv("model.1", a0, a1, h1, w1, stride=2)
        p2 = new(h2, w2, a.c2)
        c2f(2, a1, p2, h2, w2, pre=t2 if self.stem32 and (W * 3) % 16 == 0 else None)
        # each stride-2 conv feeds only the C2f block after it: c2f() runs it first, or as the fused block's prologue
        a3 = new(h3, w3, a.c3)
        cat14 = new(h3, w3, a.c4 + a.c3)          # [up(h12) | P3]
        P3 = cat14.sub(a.c4, a.c3)
        c2f(4, a3, P3, h3, w3, s2=("model.3", p2))
        a5 = new(h4, w4, a.c4)
        cat11 = new(h4, w4, a.c5 + a.c4)          # [up(P5) | P4]
        P4 = cat11.sub(a.c5, a.c4)
        c2f(6, a5, P4, h4, w4, s2=("model.5", P3))
        a7 = new(h5, w5, a.c5)
        b8 = new(h5, w5, a.c5)
        c2f(8, a7, b8, h5, w5, s2=("model.7", P4))
        cs = a.c5 // 2
        sp = new(h5, w5, 4 * cs)
        conv("model.9.cv1", b8, sp.sub(0, cs), h5, w5)
        ops.append(SegOp(kind=VA_OP_SPPF, a=ConvArgs(y=sp.ptr, N=B, H=h5, W=w5, Cin=cs, ldy=sp.ld,
                                                      dtype=VA_DTYPE_FP8 if sp.e4m3 else self.va_dtype)))
        meta.append({"name": "sppf_pool", "kind": "sppf"})
        cat20 = new(h5, w5, a.c4 + a.c5)          # [conv19(o4) | P5]
        P5 = cat20.sub(a.c4, a.c5)
        conv("model.9.cv2", sp, P5, h5, w5)
        # the FPN's Upsample + Concat: read in place by the consumer's 1x1 cv1 (bf16) or materialised
        ks = 64 if self.dtype == "bf16" else 32  # the conv2 K-step the upsampled prefix must align to
        fuse_up = self.dtype != "fp8" and switch_on("VA_FUSE_UP") and a.c5 % ks == 0 \
            and a.c4 % ks == 0 and (a.c5 + a.c4) % ks == 0 and (a.c4 + a.c3) % ks == 0
        if not fuse_up:
            upsample(P5, cat11.sub(0, a.c5), h5, w5)
        cat17 = new(h4, w4, a.c3 + a.c4)          # [conv16(o3) | h12]
        h12 = cat17.sub(a.c3, a.c4)
        c2f(12, cat11, h12, h4, w4, up=P5 if fuse_up else None)
        if not fuse_up:
            upsample(h12, cat14.sub(0, a.c4), h4, w4)
        o3 = new(h3, w3, a.c3)
        c2f(15, cat14, o3, h3, w3, up=h12 if fuse_up else None)
        marks = {"A": len(ops)}  # op index ranges of the branches finish() may put on lanes
        o4 = new(h4, w4, a.c4)
        c2f(18, cat17, o4, h4, w4, s2=("model.16", o3))
        marks["B"] = len(ops)
        o5 = new(h5, w5, a.c5)
        c2f(21, cat20, o5, h5, w5, s2=("model.19", o4))
        marks["C"] = len(ops)
        # Segment head: per level [box 64 | cls nc | coef 32] float32
        cb, cc, cm = a.head_c2, a.head_c3, a.head_c4
        no = 4 * REG_MAX + a.nc + NM
        levels = []
        for l, (src, hh, ww) in enumerate(((o3, h3, w3), (o4, h4, w4), (o5, h5, w5))):
            hb = new(hh, ww, cb + cc + cm)
            conv(f"head.{l}.0", src, hb, hh, ww)
            marks[f"H{l}.0"] = len(ops)
            hb2 = new(hh, ww, cb + cc + cm)
            out = new(hh, ww, no, torch.float32)
            levels.append(out.buf)
            for br, off, cw, ooff, oc in (("cv2", 0, cb, 0, 4 * REG_MAX), ("cv3", cb, cc, 4 * REG_MAX, a.nc),
                                           ("cv4", cb + cc, cm, 4 * REG_MAX + a.nc, NM)):
                if self._can_fuse_tail(f"model.22.{br}.{l}.1", f"model.22.{br}.{l}.2", B * hh * ww):
                    conv(f"model.22.{br}.{l}.1", hb.sub(off, cw), out.sub(ooff, oc), hh, ww, out_f32=True,
                         tail=f"model.22.{br}.{l}.2", act2=False)
                else:
                    conv(f"model.22.{br}.{l}.1", hb.sub(off, cw), hb2.sub(off, cw), hh, ww)
                    conv(f"model.22.{br}.{l}.2", hb2.sub(off, cw), out.sub(ooff, oc), hh, ww, act=False,
                         out_f32=True)
                marks[f"H{l}.{br}"] = len(ops)
            marks[f"H{l}"] = len(ops)
        # Proto
        if self.proto_fold is not None and self.dtype == "f32":
            # the sub-pixel fold (mode 2, border bias table) into the 4x map, then cv3 as its own 1x1 GEMM
            pf = self.proto_fold
            pr1 = new(h3, w3, a.npr)
            conv("model.22.proto.cv1", o3, pr1, h3, w3)
            p3 = self.w["model.22.proto.cv3"]
            if pf.w3 is not None and self._fuse_tail_f32(pf.cout, p3, 4 * B * h3 * w3, fold=True):
                # cv3 in the fold's epilogue (va_seg.hip conv_tail32): one launch, the 4x map never written
                proto = new(h2, w2, NM, torch.float32)
                w3c = split3_bf16(p3.w[:32 * ((p3.cout + 31) // 32), :pf.cout])
                keep.append(w3c)
                ops.append(SegOp(kind=VA_OP_CONV, a=with_ws(ConvArgs(
                    x=pr1.ptr, N=B, H=h3, W=w3, Cin=pf.cin, ldx=pr1.ld, kh=2, kw=2, stride=1, pad=1, Ho=h3, Wo=w3,
                    w=pf.w.data_ptr(), bias=pf.b.data_ptr(), Cout=pf.cout, Npad=pf.Npad, K=pf.K, Kpad=pf.Kpad,
                    y=proto.ptr, ldy=proto.ld, act=1, mode=2, M=B * h3 * w3, dtype=self.va_dtype, bias4=1,
                    w3=pf.w3.data_ptr(), w2=w3c.data_ptr(), b2=p3.b.data_ptr(), c2=p3.cout, act2=1))))
                meta.append({"name": "model.22.proto.upsample+cv2+cv3 (sub-pixel fold)", "kind": "conv",
                             "M": 4 * B * h3 * w3, "N": pf.cout, "K": pf.K, "k": 2, "stride": 1,
                             "flops": 2 * 4 * B * h3 * w3 * pf.cout * (pf.K + p3.cout),
                             "bytes": 4 * B * h3 * w3 * pf.cin + 4 * pf.w.numel() + 4 * B * h2 * w2 * NM})
                return finish(proto)
            pr3 = new(h2, w2, a.npr)
            ops.append(SegOp(kind=VA_OP_CONV, a=with_ws(ConvArgs(
                x=pr1.ptr, N=B, H=h3, W=w3, Cin=pf.cin, ldx=pr1.ld, kh=2, kw=2, stride=1, pad=1, Ho=h3, Wo=w3,
                w=pf.w.data_ptr(), bias=pf.b.data_ptr(), Cout=pf.cout, Npad=pf.Npad, K=pf.K, Kpad=pf.Kpad,
                y=pr3.ptr, ldy=pr3.ld, act=1, mode=2, M=B * h3 * w3, dtype=self.va_dtype, bias4=1,
                w3=pf.w3.data_ptr() if pf.w3 is not None else None))))
            meta.append({"name": "model.22.proto.upsample+cv2 (sub-pixel fold)", "kind": "conv",
                         "M": 4 * B * h3 * w3, "N": pf.cout, "K": pf.K, "k": 2, "stride": 1,
                         "flops": 2 * 4 * B * h3 * w3 * pf.cout * pf.K,
                         "bytes": 4 * B * h3 * w3 * pf.cin + 4 * pf.w.numel() + 4 * B * h2 * w2 * pf.cout})
            proto = new(h2, w2, NM, torch.float32)
            conv("model.22.proto.cv3", pr3, proto, h2, w2, out_f32=True)
            return finish(proto)
        if self.proto_fold is not None and self.proto_fold.cout != 128:
            # bf16, a wider proto (m: 192 channels): the fold alone into the 4x map, then cv3 as its own 1x1 -- 40 % of
            # the unfolded pair's MACs (the ConvTranspose GEMM + the 3x3 on the 4x map)
            pf = self.proto_fold
            pr1 = new(h3, w3, a.npr)
            conv("model.22.proto.cv1", o3, pr1, h3, w3)
            pr3 = new(h2, w2, a.npr)
            fa = with_ws(ConvArgs(
                x=pr1.ptr, N=B, H=h3, W=w3, Cin=pf.cin, ldx=pr1.ld, kh=2, kw=2, stride=1, pad=1, Ho=h3, Wo=w3,
                w=pf.w.data_ptr(), bias=pf.b.data_ptr(), Cout=pf.cout, Npad=pf.Npad, K=pf.K, Kpad=pf.Kpad,
                y=pr3.ptr, ldy=pr3.ld, act=1, mode=2, M=B * h3 * w3, dtype=self.va_dtype, bias4=1))
            if self.proto_fold8 is not None:  # w8a16: [4][Npad][Kpad] e4m3 bytes, [4][Npad] scales
                if use_w8:
                    fa.w, fa.wscale, fa.w8 = self.proto_fold8[0].data_ptr(), self.proto_fold8[1].data_ptr(), 1
                else:
                    fa.w = self.proto_fold8_bf16.data_ptr()
            ops.append(SegOp(kind=VA_OP_CONV, a=fa))
            meta.append({"name": "model.22.proto.upsample+cv2 (sub-pixel fold)", "kind": "conv",
                         "M": 4 * B * h3 * w3, "N": pf.cout, "K": pf.K, "k": 2, "stride": 1,
                         "flops": 2 * 4 * B * h3 * w3 * pf.cout * pf.K,
                         "bytes": 2 * B * h3 * w3 * pf.cin + (1 if fa.w8 else 2) * pf.w.numel()
                         + 2 * B * h2 * w2 * pf.cout})
            proto = new(h2, w2, NM, torch.float32)
            conv("model.22.proto.cv3", pr3, proto, h2, w2, out_f32=True)
            return finish(proto)
        if self.proto_fold is not None:
            pf = self.proto_fold
            pr1 = new(h3, w3, a.npr)
            conv("model.22.proto.cv1", o3, pr1, h3, w3)
            proto = new(h2, w2, NM, torch.float32)
            p3 = self.w["model.22.proto.cv3"]
            w3c = p3.w[:, :pf.cout].contiguous()
            keep.append(w3c)
            fa = with_ws(ConvArgs(
                x=pr1.ptr, N=B, H=h3, W=w3, Cin=pf.cin, ldx=pr1.ld, kh=2, kw=2, stride=1, pad=1, Ho=h3, Wo=w3,
                w=pf.w.data_ptr(), bias=pf.b.data_ptr(), Cout=pf.cout, Npad=pf.Npad, K=pf.K, Kpad=pf.Kpad,
                y=proto.ptr, ldy=proto.ld, act=1, mode=2, M=B * h3 * w3, dtype=self.va_dtype, out_f32=1, bias4=1,
                w2=w3c.data_ptr(), b2=p3.b.data_ptr(), c2=p3.cout, act2=1))
            if self.proto_fold8 is not None:  # w8a16: the fold's e4m3 rows (the tail's w2 stays bf16)
                if use_w8:
                    fa.w, fa.wscale, fa.w8 = self.proto_fold8[0].data_ptr(), self.proto_fold8[1].data_ptr(), 1
                else:
                    fa.w = self.proto_fold8_bf16.data_ptr()
            ops.append(SegOp(kind=VA_OP_CONV, a=fa))
            meta.append({"name": "model.22.proto.upsample+cv2+cv3 (sub-pixel fold)", "kind": "conv",
                         "M": 4 * B * h3 * w3, "N": pf.cout, "K": pf.K, "k": 2, "stride": 1,
                         "flops": 2 * 4 * B * h3 * w3 * pf.cout * (pf.K + p3.cout),
                         "bytes": 2 * B * h3 * w3 * pf.cin + 2 * pf.w.numel() + 4 * B * h2 * w2 * NM})
            return finish(proto)
        pr1 = new(h3, w3, a.npr)
        conv("model.22.proto.cv1", o3, pr1, h3, w3)
        pr2 = new(h2, w2, a.npr)
        conv("model.22.proto.upsample", pr1, pr2, h3, w3, act=False)
        proto = new(h2, w2, NM, torch.float32)
        if self._can_fuse_tail("model.22.proto.cv2", "model.22.proto.cv3"):
            conv("model.22.proto.cv2", pr2, proto, h2, w2, out_f32=True, tail="model.22.proto.cv3", act2=True)
        else:
            pr3 = new(h2, w2, a.npr)
            conv("model.22.proto.cv2", pr2, pr3, h2, w2)
            conv("model.22.proto.cv3", pr3, proto, h2, w2, out_f32=True)
        return finish(proto)

    @staticmethod
    def _fp8_fits(p: Packed, src: Slice, dst: Slice, res, out_f32: bool) -> bool:
        """va_fp8.hip's operand rules (va_fp8_conv_ok): input rows in 16-byte runs of 16 channels (e4m3 or bf16),
        outputs and residuals in 8-element runs (4 for a float output, which takes no residual)."""
        xe = src.buf.element_size()
        ok = (src.ld * xe) % 16 == 0 and (src.off * xe) % 16 == 0 and p.cin % 16 == 0
        if out_f32:
            return ok and p.cout % 4 == 0 and dst.ld % 4 == 0 and res is None
        cd = p.cout // 4 if p.deconv else p.cout
        ye = dst.buf.element_size()
        ok = ok and cd % 8 == 0 and dst.ld % 8 == 0 and (dst.off * ye) % (8 * ye) == 0
        if res is not None:
            re = res.buf.element_size()
            ok = ok and res.ld % 8 == 0 and (res.off * re) % (8 * re) == 0
        return ok

    def _fuse_tail_f32(self, cout: int, p2: Packed, M: int, fold: bool = False) -> bool:
        """f32: the tail runs in conv3h's epilogue (va_seg.hip conv_tail32) when the whole channel set is one of its
        tiles (Cout 64 or 128; the fold: 128), the tail has <= 96 channels, and the launch has >= 128 tiles --
        below that conv2 would split the conv over K (batch-1 shapes), which a fused launch cannot, so the pair
        stays unfused there.  VA_FUSE_TAIL=0 / VA_CONV3H=0 turn it off."""
        if not switch_on("VA_FUSE_TAIL") or not switch_on("VA_CONV3H"):
            return False
        if p2.k != 1 or p2.cin != cout or p2.cout % 4 or p2.cout > 96 or cout not in ((128,) if fold else (64, 128)):
            return False
        return (M + 127) // 128 >= 128

    def _can_fuse_tail(self, prefix: str, tail: str, M: int = 0) -> bool:
        """Whether the 1x1 conv ``tail`` (sole consumer of ``prefix``) can run in prefix's epilogue: bf16,
        a 128-channel main conv with <= 80 tail channels or a 32 / 64-channel one with <= 64 (va355.h
        va_conv_args.w2); f32, a stride-1 3x3 conv on conv3h (_fuse_tail_f32; M = its output pixels).
        VA_FUSE_TAIL=0 turns it off (A/B timing)."""
        p, p2 = self.w[prefix], self.w[tail]
        if self.dtype == "f32" and p.cin == 32 and p.cout == 32:
            # the 32-channel 3x3 (the head's cv4.l.1) on conv3q with the tail in its epilogue, where the launch has
            # four 16 x 16 tiles per CU (va_seg.hip Q3_MIN_TILES_PER_CU; M / 256 is a lower bound of its tiles)
            if not switch_on("VA_FUSE_TAIL") or not switch_on("VA_CONV3Q"):
                return False
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            return (p.k == 3 and not p.deconv and p2.k == 1 and p2.cin == 32 and p2.cout <= 32 and p2.cout % 4 == 0
                    and M // 256 >= 4 * cus)
        if self.dtype == "f32":
            return p.k == 3 and not p.deconv and p.w3 is not None and self._fuse_tail_f32(p.cout, p2, M)
        if self.dtype != "bf16" or not switch_on("VA_FUSE_TAIL"):
            return False
        if p.deconv or p2.k != 1 or p2.cin != p.cout or p2.cout % 4:
            return False
        if p.cout == 128:
            return p2.cout <= 80
        return p.cout in (32, 64) and p.cin >= 32 and p2.cout <= 64 and p.cout * (p.Kpad + 8) * 2 <= 120 * 1024

    def forward(self, frames_u8: torch.Tensor, stream=None) -> SegOutputs:
        """frames_u8: uint8 [B, H, W, 3] BGR on the device."""
        B, H, W, _ = frames_u8.shape
        p = self.plan(B, H, W)
        p["frames"].copy_(frames_u8, non_blocking=True)
        self.run_plan(p, stream)
        return p["out"]

    def run_plan(self, p, stream=None) -> None:
        with torch.cuda.device(self.device):
            _lib.check(self.lib.va_seg_run(_lib.stream_ptr(stream, self.device), p["ops"], p["n"]), "va_seg_run")

    @staticmethod
    def plan_gflop(plan) -> float:
        """GFLOPs the plan's GEMMs execute per call (2 x MACs, unpadded; folded / fused ops counted as run)."""
        return sum(m.get("flops", 2.0 * m["M"] * m["N"] * m["K"]) for m in plan["meta"] if m["kind"] == "conv") / 1e9

    def gflop_per_frame(self, H: int, W: int) -> float:
        """Algorithmic FLOPs (2 x MACs of every conv, unpadded) per frame."""
        total = 0
        for prefix, kind, ci, co, k in self.arch.conv_specs():
            total += 2 * ci * co * k * k * _spatial(prefix, H, W)
        return total / 1e9


def fold_proto_weights(wd: torch.Tensor, bd: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """ConvTranspose2d(k2, s2) (weight wd [Ci, C, 2, 2], bias bd [C]) followed by a 3x3 / pad 1 conv
    (weight w2 [O, C, 3, 3]) as 4 sub-pixel 2x2 convs over the low-res input: float64
    [4 classes (2 dy + dx)][O][2][2][Ci + 8] (va355.h va_conv_args.mode 2).

    Output pixel (2Y + dy, 2X + dx) sees upsampled rows 2Y + dy + ky - 1 (ky = 0..2), i.e. low-res
    row Y + floor((dy + ky - 1) / 2) through deconv tap (dy + ky - 1) mod 2 -- two low-res rows per
    class, likewise columns; summing the 3x3 taps through the deconv weights gives each class a 2x2
    kernel whose tap (fy, fx) reads low-res pixel (Y + dy - 1 + fy, X + dx - 1 + fx): K = 4 x Ci
    instead of 9 x C at 4x the pixels plus the deconv (2.3x fewer MACs for proto, and no 4x-size
    intermediate map).  The deconv bias rides on input channel Ci, which the caller holds at 1 inside
    the map (0 in the zero padding), so border pixels get exactly the taps inside the upsampled map."""
    wd, bd, w2 = wd.double(), bd.double(), w2.double()
    ci, o = wd.shape[0], w2.shape[0]
    wc = torch.zeros(4, o, 2, 2, ci + 8, dtype=torch.float64)
    for dy in range(2):
        for dx in range(2):
            for ky in range(3):
                t = dy + ky - 1
                fy, ta = t // 2 - (dy - 1), t % 2
                for kx in range(3):
                    u = dx + kx - 1
                    fx, tb = u // 2 - (dx - 1), u % 2
                    wc[2 * dy + dx, :, fy, fx, :ci] += w2[:, :, ky, kx] @ wd[:, :, ta, tb].T
                    wc[2 * dy + dx, :, fy, fx, ci] += w2[:, :, ky, kx] @ bd
    return wc


def _spatial(prefix: str, H: int, W: int) -> int:
    """Output pixels of the module `prefix` for an H x W input."""
    parts = prefix.split(".")
    i = int(parts[1])
    if i == 22:
        if parts[2] == "proto":  # cv1 and the deconv GEMM run at stride 8, cv2/cv3 at stride 4
            return (H // 8) * (W // 8) if parts[3] in ("cv1", "upsample") else (H // 4) * (W // 4)
        l = int(parts[3])
        s = (8, 16, 32)[l]
        return (H // s) * (W // s)
    stride = {0: 2, 1: 4, 2: 4, 3: 8, 4: 8, 5: 16, 6: 16, 7: 32, 8: 32, 9: 32, 12: 16, 15: 8, 16: 16, 18: 16,
              19: 32, 21: 32}[i]
    return (H // stride) * (W // stride)

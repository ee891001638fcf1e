"""What v_cvt_scalef32_pk_fp8_bf16 does with its scale (multiply or divide) and out of range, against the staging
path's explicit x * s, clamp, v_cvt_pk_fp8_f32 and torch.float8_e4m3fn.  Debug tool; prints one JSON line."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vision_assist_amd import _lib  # noqa: E402

lib = _lib.load()
lib.va_fp8_cvt_probe.restype = ctypes.c_int
lib.va_fp8_cvt_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                                 ctypes.c_int]
vals = [0.0, 0.5, 1.0, 1.3, -2.7, 3.0, 100.0, 300.0, 447.0, 448.0, 460.0, 500.0, 1000.0, -1000.0, 1e-3, 0.0137]
x = torch.tensor(vals, dtype=torch.bfloat16).cuda()
res = {}
for mode in (0, 1):
    for s in (1.0, 2.0, 0.5):
        out = torch.zeros(len(vals), dtype=torch.uint8, device="cuda")
        _lib.check(lib.va_fp8_cvt_probe(_lib.stream_ptr(), x.data_ptr(), out.data_ptr(), len(vals), s, mode), "probe")
        torch.cuda.synchronize()
        dec = out.cpu().view(torch.float8_e4m3fn).float().tolist()
        res[f"mode{mode}_s{s}"] = dec
for s in (1.0, 2.0, 0.5):
    res[f"torch_mul_s{s}"] = (x.float().cpu() * s).clamp(-448, 448).to(torch.float8_e4m3fn).float().tolist()
print(json.dumps(res))

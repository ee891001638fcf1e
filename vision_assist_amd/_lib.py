"""ctypes binding of libva355.so (the HIP/gfx950 C-ABI, include/va355.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
vision_assist_amd/csrc``).  There is NO fallback: if the shared object is
missing or a GPU is absent, every entry point raises.  torch is imported first
so that the process has exactly one HIP runtime (torch's bundled
libamdhip64.so.7 satisfies the library's DT_NEEDED of the same soname).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

HERE = os.path.dirname(os.path.abspath(__file__))
# VA355_LIB: load another build of the same C-ABI (same-box A/B timing of kernel variants, tools/)
LIB_PATH = os.environ.get("VA355_LIB") or os.path.join(HERE, "libva355.so")

VA_OK = 0
VA_ERR_ARG, VA_ERR_HIP, VA_ERR_RANGE = -1, -2, -3
VA_FRAME_OK, VA_FRAME_EMPTY, VA_FRAME_INDEX_ERROR, VA_FRAME_NO_MASK = 0, 1, 2, 3
VA_QUERY_NONE, VA_QUERY_FOUND, VA_QUERY_NO_PATH = 0, 1, 2
VA_CELL_EMPTY, VA_CELL_ARTIFICIAL = 1, 2
VA_NODE_EXISTS, VA_NODE_NONEMPTY, VA_NODE_IN_GRIDS, VA_NODE_MULT_SHIFT, VA_NODE_ARTIFICIAL = 1, 2, 4, 3, 32


class VaNavDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("H", "W", "LR", "LC", "start_y", "NART", "PMAX", "MAXPK", "NODES", "pad")] + \
               [(n, ctypes.c_int64) for n in
                ("frame_bytes", "off_hdr", "off_peaks", "off_pos_obj", "off_pos_y", "off_pos_attr",
                 "off_cell_flags", "off_cell_pen", "off_node_flags", "off_node_pen",
                 "query_bytes", "off_q_hdr", "off_q_path", "off_queries_per_frame")]


class VaError(RuntimeError):
    pass


_LIB = None

# (name, restype, argtypes) for every symbol include/va355.h declares
P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
SIGNATURES = [
    ("va_nav_dims_for", I32, [I32, I32, ctypes.POINTER(VaNavDims)]),
    ("va_nav_workspace_bytes", I64, [I32, I32, I32]),
    ("va_nav_sample_cells", I32, [P, P, I64, I32, I32, I32, P]),
    ("va_nav_run", I32, [P, P, P, I32, I32, I32, P, P, ctypes.POINTER(I32)]),
    ("va_nav_records_bytes", I64, [I32, I32, I32]),
    ("va_nav_run_rb", I32, [P, P, P, I32, I32, I32, P, P, ctypes.POINTER(I32), P, I64]),
    ("va_nav_query_bytes", I64, [I32]),
    ("va_astar_workspace_bytes", I64, [I32, I32]),
    ("va_astar_run", I32, [P, P, P, I32, I32, P, P, I32, P, P, ctypes.POINTER(I32)]),
    ("va_seg_conv", I32, [P, P]),
    ("va_seg_c2f", I32, [P, P]),
    ("va_seg_c2fb", I32, [P, P]),
    ("va_c2fb_layout", I32, [I32, I32, I32, I32, I32, I32, I32, I32, ctypes.POINTER(I64)]),
    ("va_seg_stem", I32, [P, P]),
    ("va_seg_stem_f32", I32, [P, P]),
    ("va_c2f_trace", I32, [P]),
    ("va_c2fb_trace", I32, [P]),
    ("va_stem_trace", I32, [P]),
    ("va_seg_preprocess", I32, [P, P, I32, I32, I32, I32, P]),
    ("va_seg_conv0", I32, [P, P, I32, I32, I32, P, P, I32, P, I32]),
    ("va_seg_conv0_f32", I32, [P, P, I32, I32, I32, P, P, I32, P, I32]),
    ("va_seg_conv0_f32m", I32, [P, P, I32, I32, I32, P, P, I32, P, I32]),
    ("va_seg_conv0_e4m3", I32, [P, P, I32, I32, I32, P, P, I32, P, I32, ctypes.c_float]),
    ("va_create", I32, [I32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    ("va_destroy", I32, [P]),
    ("va_handle_device", I32, [P, ctypes.POINTER(ctypes.c_int32)]),
    ("va_frame", I32, [P, P, P, I32, P, I32, I32, P, P, ctypes.POINTER(ctypes.c_int32)]),
    ("va_frame_rb", I32, [P, P, P, I32, P, I32, I32, P, P, ctypes.POINTER(ctypes.c_int32), P, I64]),
    ("va_seg_sppf_pool", I32, [P, P, I32, I32, I32, I32, I32, I32]),
    ("va_seg_upsample2x", I32, [P, P, I32, P, I32, I32, I32, I32, I32, I32]),
    ("va_seg_run", I32, [P, P, I32]),
    ("va_prof_start", I32, [I32]),
    ("va_prof_stop", I32, [P, P, I32]),
    ("va_prof_stop_ops", I32, [P, I32]),
    ("va_prof_enable", I32, [I32]),
    ("va_post_anchors", I32, [I32, I32]),
    ("va_post_run", I32, [P, P]),
    ("va_contour_scratch_bytes", I32, [I32, I32, I32, I32, P, P, P]),
    ("va_post_select_masks", I32, [P, P]),
    ("va_post_polygons", I32, [P, P, P, P, I32]),
    ("va_letterbox", I32, [P, P, I32, I32, I32, P, I32, I32, I32, I32, I32, I32]),
    ("va_abi_struct_sizes", I32, [P, I32]),
    ("va_diag", I32, [P, I32, I32]),
    ("va_switches_reload", I32, []),
    ("va_version", ctypes.c_char_p, []),
]


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes handle.  Raises if the .so is absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise VaError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "(the HIP extension is required; there is no CPU fallback)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != VA_OK:
        raise VaError(f"{what} failed with status {rc}")


def reload_switches() -> None:
    """Re-read the library's A/B switches from the environment (va_switches_reload; they are read once per process
    otherwise).  For tests that hold two kernel forms against each other inside one process."""
    if _LIB is not None:
        check(_LIB.va_switches_reload(), "va_switches_reload")


DIAG_UNITS = ("post", "contour", "nav")


def diag(clear: bool = True) -> dict:
    """Out-of-range state the kernels rejected instead of faulting since the last clear (va_diag; codes in
    csrc/va_diag.h): {unit: (first code, v0, v1, count)} for the units that recorded any (synchronises the device)."""
    w = (ctypes.c_uint32 * 12)()
    check(load().va_diag(w, 12, int(clear)), "va_diag")
    return {u: tuple(int(v) for v in w[4 * i:4 * i + 4]) for i, u in enumerate(DIAG_UNITS) if w[4 * i + 3]}


def nav_dims(H: int, W: int) -> VaNavDims:
    d = VaNavDims()
    check(load().va_nav_dims_for(H, W, ctypes.byref(d)), f"va_nav_dims_for({H}, {W})")
    return d


def stream_ptr(stream=None, device=None) -> int:
    """The HIP stream handle to launch on: ``stream``, else the current stream of ``device`` (default: the
    current device).  Launches go to the current HIP device, so callers run under torch.cuda.device(device)."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    if device is not None and s.device != torch.device(device):
        raise VaError(f"stream of {s.device} used for work on {device}")
    return int(s.cuda_stream)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise VaError("vision_assist_amd needs a ROCm GPU (MI355X); torch.cuda.is_available() is False")


class Handle:
    """A va_create handle bound to one HIP device (va355.h: va_frame runs a whole batch on it)."""

    _by_device: dict = {}

    def __init__(self, device: int):
        lib = load()
        h = ctypes.c_void_p()
        check(lib.va_create(int(device), 0, ctypes.byref(h)), f"va_create({device})")
        self.ptr, self.device, self._lib = h.value, int(device), lib

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.va_destroy(self.ptr)
            self.ptr = None

    @classmethod
    def for_device(cls, device) -> "Handle":
        """The process's handle for `device` (created on first use)."""
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
        if idx not in cls._by_device:
            cls._by_device[idx] = cls(idx)
        return cls._by_device[idx]


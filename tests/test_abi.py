"""CPU checks of the C-ABI library: it loads, exports every symbol include/va355.h
declares, and its host-side layout functions agree with the python decoders.
(No compute entry point is called here: there is no GPU in the build container.)"""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "va355.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(va_\w+)\s*\(", src, re.M)))


def test_header_declares_symbols():
    syms = _declared_symbols()
    assert "va_nav_run" in syms and "va_astar_run" in syms and len(syms) >= 8


def test_library_exports_every_declared_symbol():
    from vision_assist_amd import _lib
    lib = _lib.load()
    for s in _declared_symbols():
        assert hasattr(lib, s), f"libva355.so does not export {s}"
    assert {s for s, _, _ in _lib.SIGNATURES} >= set(_declared_symbols())


@pytest.mark.parametrize("H,W", [(640, 640), (1280, 1280), (1280, 720)])
def test_nav_dims(H, W):
    from vision_assist_amd import _lib
    d = _lib.nav_dims(H, W)
    assert (d.LR, d.LC) == (H // 20, W // 20)
    sy = int(H * 0.875)
    sy = sy + (20 - sy % 20) % 20
    assert d.start_y == sy and d.NART == (H - sy) // 20
    assert d.frame_bytes % 16 == 0 and d.query_bytes % 16 == 0
    assert _lib.load().va_nav_workspace_bytes(4, H, W) >= 4 * d.frame_bytes


def test_nav_dims_rejects_bad_shapes():
    from vision_assist_amd import _lib
    d = _lib.VaNavDims()
    lib = _lib.load()
    assert lib.va_nav_dims_for(630, 640, ctypes.byref(d)) != 0
    assert lib.va_nav_dims_for(640, 2000, ctypes.byref(d)) != 0
    assert lib.va_nav_workspace_bytes(0, 640, 640) < 0


def test_angle_table_header_matches_reference():
    """va_angle_table.h (baked into the library) == the reference-generated table."""
    from tests.golden_io import load_goldens
    txt = open(os.path.join(REPO, "vision_assist_amd", "csrc", "va_angle_table.h")).read()
    pens = re.search(r"VA_ANGLE_PEN\[128\] = \{([^}]*)\}", txt).group(1).split(",")
    degs = re.search(r"VA_ANGLE_DEG\[128\] = \{([^}]*)\}", txt).group(1).split(",")
    golden = load_goldens()["angle_table"]
    assert len(pens) == len(degs) == len(golden) == 128
    for (a, b, c, dd, gdeg, gpen), deg, pen in zip(golden, degs, pens):
        assert float.fromhex(deg.strip()).hex() == gdeg
        want = 0.0 if gpen.startswith("i") else float.fromhex(gpen)
        assert float.fromhex(pen.strip()) == want


def test_struct_layouts_match_python_mirrors():
    """Every ctypes / numpy mirror of a va355.h struct has the C sizeof."""
    import numpy as np
    from vision_assist_amd import _lib
    from vision_assist_amd.nav import FRAME_HDR, QUERY_HDR
    from vision_assist_amd.post import CSTAT_DTYPE, ContourStat, MaskSelectArgs, PostArgs
    from vision_assist_amd.seg import ConvArgs, SegOp
    lib = _lib.load()
    out = (ctypes.c_int64 * 11)()
    assert lib.va_abi_struct_sizes(out, 11) == 11
    want = [ctypes.sizeof(_lib.VaNavDims), FRAME_HDR.itemsize, QUERY_HDR.itemsize, ctypes.sizeof(ConvArgs),
            ctypes.sizeof(SegOp), 32, 32, 32, ctypes.sizeof(PostArgs), ctypes.sizeof(ContourStat),
            ctypes.sizeof(MaskSelectArgs)]
    assert np.dtype(CSTAT_DTYPE).itemsize == ctypes.sizeof(ContourStat)
    assert list(out) == want
    del np


def test_seg_run_rejects_bad_lanes():
    """va_seg_run's lane checks (va355.h VA_OP_FORK) fail before any launch: a lane out of range, a join or an
    op on a lane never forked, a fork of lane 0.  The failing op's index is encoded as rc - 1000 * (i + 1)."""
    from vision_assist_amd import _lib
    from vision_assist_amd.seg import VA_OP_CONV, VA_OP_FORK, VA_OP_JOIN, ConvArgs, SegOp
    lib = _lib.load()

    def run(*ops):
        arr = (SegOp * len(ops))(*ops)
        return lib.va_seg_run(None, arr, len(ops))

    err = -1  # VA_ERR_ARG
    assert run(SegOp(kind=VA_OP_CONV, lane=4)) == err - 1000
    assert run(SegOp(kind=VA_OP_CONV, lane=-1)) == err - 1000
    assert run(SegOp(kind=VA_OP_JOIN, a=ConvArgs(N=1))) == err - 1000
    assert run(SegOp(kind=VA_OP_FORK, a=ConvArgs(N=0))) == err - 1000
    assert run(SegOp(kind=VA_OP_FORK, a=ConvArgs(N=4))) == err - 1000
    assert run(SegOp(kind=VA_OP_FORK, lane=1, a=ConvArgs(N=2))) == err - 1000
    assert run(SegOp(kind=VA_OP_CONV, lane=2)) == err - 1000
    assert lib.va_seg_run(None, (SegOp * 1)(), 0) == 0


def _c2fb_expect(c, n, ci, co, cs=0, cis=0, f32=False):
    """va_seg_c2fb's blob sizes restated (seg.py SegNet._pack_c2fb): per conv ceil(Cout / 16) x ceil(K / 32) tiles
    of one A fragment (three in f32) and 16 ceil(Cout / 16) biases."""
    convs = [(2 * c, ci)] + [(c, 9 * c)] * (2 * n) + [(co, (2 + n) * c)] + ([(cs, 9 * cis)] if cs else [])
    tiles = sum(-(-o // 16) * -(-k // 32) for o, k in convs)
    return tiles * (3 if f32 else 1), sum(16 * -(-o // 16) for o, _ in convs)


@pytest.mark.parametrize("c,n,ci,co,T,cs,cis,f32,planes", [
    (16, 1, 32, 32, 16, 0, 0, False, 0), (32, 2, 64, 64, 8, 64, 32, False, 0), (64, 2, 128, 128, 4, 0, 0, False, 0),
    (128, 1, 256, 256, 2, 256, 128, False, 0), (64, 1, 384, 128, 4, 0, 0, False, 0),
    (64, 1, 192, 128, 4, 64, 64, False, 0), (128, 1, 384, 256, 2, 128, 128, False, 0),
    (256, 1, 512, 512, 2, 0, 0, True, 1), (64, 2, 128, 128, 4, 0, 0, True, 1), (128, 2, 256, 256, 2, 0, 0, True, 0),
    (64, 1, 192, 128, 8, 0, 0, True, 1)])
def test_c2fb_layout_matches_packing(c, n, ci, co, T, cs, cis, f32, planes):
    """va_c2fb_layout (host side of va_seg_c2fb): the LDS of the planner's tile sides for YOLOv8n's blocks (bf16, with
    the stride-2 prologues it fuses) and s's (f32) fits 160 KiB, the blob sizes equal the packing's, and the f32 form
    keeps its intermediates as bf16 term planes where they fit (s's model.6, c 128 with two Bottlenecks, stays f32)."""
    from vision_assist_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_int64 * 4)()
    rc = lib.va_c2fb_layout(c, n, ci, co, T, 2 if f32 else 1, cs, cis, out)  # va355.h VA_DTYPE_F32 / _BF16
    assert rc == 0 and 0 < out[0] <= 160 * 1024, (rc, out[0])
    assert (out[1], out[2]) == _c2fb_expect(c, n, ci, co, cs, cis, f32)
    assert out[3] == planes


@pytest.mark.parametrize("c,n,ci,co,T,lds", [
    (64, 1, 384, 128, 8, 150336),   # s's model.15: cv1's staged chunk inside the regions (R1 on), biases after them
    (64, 1, 192, 128, 4, 59136),    # the staged chunk past the regions: the biases move up behind it
    (128, 1, 768, 256, 4, 106560)])
def test_c2fb_f32_layout_with_cv1_staging(c, n, ci, co, T, lds):
    """va_c2fb_layout's f32 LDS with cv1's operand staged (va_c2fb.hip xf_stage: 64-channel chunks of the tile's
    S0 x S0 pixels as three bf16 planes, 400 bytes a pixel, from R1's offset): the regions R0b | R0a | R1 .. at 6C + 16
    bytes a pixel, then the chunk where it reaches past them, then the biases."""
    from vision_assist_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_int64 * 4)()
    assert lib.va_c2fb_layout(c, n, ci, co, T, 2, 0, 0, out) == 0 and out[3] == 1
    S0, ps = T + 4 * n, 6 * c + 16
    regions = [S0 * S0, T * T] + [(T + 2 * (2 * n - j)) ** 2 for j in range(1, 2 * n + 1)]
    off_r1 = (regions[0] + regions[1]) * ps
    end = max(sum(regions) * ps, off_r1 + S0 * S0 * 400)
    assert out[0] == end + 4 * out[2] == lds


def test_c2fb_layout_rejects_what_the_kernel_does_not_cover():
    from vision_assist_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_int64 * 4)()
    assert lib.va_c2fb_layout(48, 1, 96, 96, 4, 1, 0, 0, out) != 0        # hidden width 48
    assert lib.va_c2fb_layout(64, 3, 128, 128, 4, 1, 0, 0, out) != 0      # three Bottlenecks
    assert lib.va_c2fb_layout(128, 2, 256, 256, 16, 1, 0, 0, out) != 0    # past the LDS
    assert lib.va_c2fb_layout(64, 1, 128, 128, 4, 1, 64, 24, out) != 0    # prologue input not a power of two
    assert lib.va_c2fb_layout(64, 1, 128, 128, 4, 2, 64, 64, out) != 0    # no f32 prologue

"""The device-bound handle of the C ABI (va355.h va_create / va_destroy / va_handle_device / va_frame, SURVEY.md
§8b): argument checks, and one va_frame call giving exactly the records of the three stages called one by one."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_handle_create_checks():
    from vision_assist_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.va_create(0, 1, ctypes.byref(h)) == _lib.VA_ERR_ARG          # flags must be 0
    assert lib.va_create(torch.cuda.device_count(), 0, ctypes.byref(h)) == _lib.VA_ERR_ARG  # no such device
    assert lib.va_create(0, 0, ctypes.byref(h)) == _lib.VA_OK
    d = ctypes.c_int32(-1)
    assert lib.va_handle_device(h, ctypes.byref(d)) == _lib.VA_OK and d.value == 0
    assert lib.va_destroy(h) == _lib.VA_OK


def test_va_frame_equals_stage_by_stage():
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_IF_NONE
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from workloads.corridors import cells_rect, corridor_cells
    arch = Arch("s")
    fw = fold(arch, synthetic_state_dict(arch, seed=0, cls_bias=0.0))
    B = 3
    frames = torch.randint(0, 256, (B, 640, 640, 3), generator=torch.Generator().manual_seed(4),
                           dtype=torch.uint8).cuda()
    grids = [corridor_cells(900 + i, 32, 32) for i in range(B)]
    pc = torch.tensor(np.stack(grids).astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g) for g in grids], dtype=np.int32)).cuda()
    fused = FramePipeline(arch, fw, B, 640, 640, dtype="bf16")
    split = FramePipeline(arch, fw, B, 640, 640, dtype="bf16", seg=fused.seg, tag=1)
    a = fused.run(frames, pc, pr, PLANT_IF_NONE)      # va_frame
    split.load(frames)
    split.seg_post(pc, pr, PLANT_IF_NONE)
    b = split.nav_run()                              # va_seg_run, va_post_run, va_nav_run
    for i in range(B):
        fa, fb = a.frame(i), b.frame(i)
        assert fa.status == fb.status and fa.peaks == fb.peaks and fa.start == fb.start
        if fa.status == 0:
            assert np.array_equal(fa.cell_pen, fb.cell_pen) and np.array_equal(fa.node_flags, fb.node_flags)
        assert [(q["path"], float(q["cost"]).hex()) for q in fa.queries] == \
            [(q["path"], float(q["cost"]).hex()) for q in fb.queries]
    assert torch.equal(fused.post.cells, split.post.cells) and torch.equal(fused.seen.t, split.seen.t)

"""Real-weight import (main.py:43 `YOLO(weights)`): a state dict saved with Ultralytics key names as .safetensors
(the route a trained checkpoint takes here: export `model.model.state_dict()` with safetensors.torch.save_file where
ultralytics is available; no .pt is unpickled) loads through YOLO(path) into exactly the folded weights the same
dict gives directly, with the architecture (scale from the file name, nc from the class head) recovered."""
import os

import pytest
import torch


@pytest.mark.parametrize("scale,nc", [("n", 80), ("s", 3)])
def test_safetensors_round_trip(tmp_path, scale, nc):
    from safetensors.torch import save_file

    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from vision_assist_amd.yolo import YOLO
    arch = Arch(scale, nc)
    sd = synthetic_state_dict(arch, seed=7, sparse=None, cls_bias=0.5)
    path = os.path.join(tmp_path, f"best_yolov8{scale}-seg.safetensors")
    save_file({k: v.contiguous() for k, v in sd.items()}, path)
    m = YOLO(path)
    assert m.arch.scale == scale and m.arch.nc == nc
    want = fold(arch, sd)
    assert sorted(m.folded) == sorted(want)
    for k, (w, b) in want.items():
        assert torch.equal(m.folded[k][0], w) and torch.equal(m.folded[k][1], b), k


def test_unknown_weights_name_raises():
    from vision_assist_amd.yolo import YOLO
    with pytest.raises(ValueError):
        YOLO("resnet50.pt")

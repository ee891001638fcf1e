"""Saves a network's head outputs (GPU, given dtype) for one seeded frame as .npz, to compare offline against
float32 / float64 CPU references (tools/f64_check.py).  Debug tool."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    scale, res, seed_w, seed_f, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    arch = Arch(scale)
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=seed_w)), dtype="f32")
    fr = torch.randint(0, 256, (1, res, res, 3), generator=torch.Generator().manual_seed(seed_f), dtype=torch.uint8)
    o = net.forward(fr.cuda())
    torch.cuda.synchronize()
    lv = torch.cat([t.float().cpu().flatten(1, 2) for t in o.levels], 1).permute(0, 2, 1).numpy()
    np.savez_compressed(out, levels=lv, proto=o.proto.float().cpu().permute(0, 3, 1, 2).numpy())


if __name__ == "__main__":
    main()
